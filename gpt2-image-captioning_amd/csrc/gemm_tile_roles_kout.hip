#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// Variant 31 (round 6): the K-outer weight-gradient products (dW = dY^T X over token rows, icap_gemm_args.trans_ab) on
// the split-role ring of gemm_tile.h: 4 MFMA waves of 64 x 64 reading ds_read_b64_tr_b16 fragments from the T10 (b)
// images + 4 LDS-DMA waves, 4 stages of 32 KiB, one block per CU walking tiles x splits; splits go through the slabs
// and the reduce pass.
void launch_tile_roles_kout(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
#define ICAP_GKK(TC, KIND) \
  hipLaunchKernelGGL((gemm_kernel<bf16_t, TC, 4, 1, 2, 2, 4, 4, true, KIND, true>), grid, block, 0, s, p, tn, sp, nks, thr, inv_keep)
  if (p.c_dtype != ICAP_BF16) {
    if (pl.actk == ACT_OFF) ICAP_GKK(float, ACT_OFF);
    else ICAP_GKK(float, ACT_ANY);
  } else {
    if (pl.actk == ACT_OFF) ICAP_GKK(bf16_t, ACT_OFF);
    else ICAP_GKK(bf16_t, ACT_ANY);
  }
#undef ICAP_GKK
}

// A group of K-outer products in ONE launch (icap_gemm_group, round 6): every block walks the concatenated tile list of
// the group (product i owns tile ids [tstart[i], tstart[i + 1])) with the variant-31 body, unsplit — so a layer's four
// weight-gradient products fill the chip together (432 tiles at the mapper's shape) without split-K slabs or a reduce
// pass. Each output tile is the variant-31 (and the K-outer tile kernel's) unsplit MFMA chain: bitwise equal to
// running the products one by one with split_k = 1.
__global__ __launch_bounds__(512, 2) void gemm_group_kernel(GemmGroup g) {
  const int total = g.tstart[g.n];
  for (int b = blockIdx.x; b < total; b += gridDim.x) {
    int i = 0;
    while (i + 1 < g.n && b >= g.tstart[i + 1]) ++i;
    const icap_gemm_args p = g.a[i];
    const int tn = g.tiles_n[i];
    const int tm = (g.tstart[i + 1] - g.tstart[i]) / tn;
    gemm_body<bf16_t, float, 4, 1, 2, 2, 4, 4, true, ACT_OFF, true>(p, tn, 1, g.nk[i], 0u, 1.f, b - g.tstart[i], tm, p.M);
  }
}

void launch_group_kout(const GemmGroup& g, int cus, hipStream_t s) {
  const int total = g.tstart[g.n];
  hipLaunchKernelGGL(gemm_group_kernel, dim3((unsigned)(total < cus ? total : cus)), dim3(2 * GNT), 0, s, g);
}

}  // namespace icap

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

}  // namespace icap

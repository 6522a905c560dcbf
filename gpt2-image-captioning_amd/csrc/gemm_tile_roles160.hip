#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// Variant 32 (round 6): 160 x 128 tiles on the split-role ring (gemm_tile.h ROLES): 4 MFMA waves of 80 x 64 + 4 LDS-DMA
// waves, 4 stages of 36 KiB (two in flight), one block per CU. For the N <= 1024 products of more rows than one round of
// 96 x 128 tiles holds: CLIP-B/32's 6400 x 768 out_proj / fc2 are 40 x 6 = 240 tiles (96 x 128: 402, 1.6 rounds).
void launch_tile_roles160(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
#define ICAP_GKW(TC, KIND) \
  hipLaunchKernelGGL((gemm_kernel<bf16_t, TC, 4, 1, 2, 2, 5, 4, false, KIND, true>), grid, block, 0, s, p, tn, sp, nks, thr, inv_keep)
  if (p.c_dtype != ICAP_BF16) {
    if (pl.actk == ACT_OFF) ICAP_GKW(float, ACT_OFF);
    else ICAP_GKW(float, ACT_ANY);
    return;
  }
  switch (pl.actk) {
    case ACT_OFF: ICAP_GKW(bf16_t, ACT_OFF); break;
    case ACT_LNS + ACT_OFF: ICAP_GKW(bf16_t, ACT_LNS + ACT_OFF); break;
    default: ICAP_GKW(bf16_t, ACT_ANY); break;
  }
#undef ICAP_GKW
}

}  // namespace icap

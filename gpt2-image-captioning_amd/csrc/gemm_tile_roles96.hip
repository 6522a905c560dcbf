#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// Variant 27 (round 6): 96 x 128 tiles on the split-role ring (gemm_tile.h ROLES): 4 MFMA waves of 48 x 64 + 4 LDS-DMA
// waves, 5 stages of 28 KiB (three in flight), one block per CU. For the N <= 1024 products: 3584 x 768 is 38 x 6 = 228
// tiles, one round over 256 CUs with no split of K (GPT-2's N = 768 products at K = 768 / 2304 / 3072).
void launch_tile_roles96(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
#define ICAP_GKW(TC, KIND) \
  hipLaunchKernelGGL((gemm_kernel<bf16_t, TC, 5, 1, 2, 2, 3, 4, false, KIND, true>), grid, block, 0, s, p, tn, sp, nks, thr, inv_keep)
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

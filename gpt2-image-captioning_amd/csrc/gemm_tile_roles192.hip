#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// Variant 28 (round 6): 192 x 256 tiles on the split-role ring (gemm_tile.h ROLES) with 8 MFMA waves (2 x 4, 96 x 64
// each, two per SIMD) + 4 LDS-DMA waves, 2 stages of 56 KiB, one block per CU: for the N = 3072 products of the step
// (3584 x 3072 is 19 x 12 = 228 tiles, one round; 128 x 256 tiles make 336, two rounds).
void launch_tile_roles192(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
#define ICAP_GKW(TC, KIND) \
  hipLaunchKernelGGL((gemm_kernel<bf16_t, TC, 2, 1, 2, 4, 6, 4, false, KIND, true>), grid, block, 0, s, p, tn, sp, nks, thr, inv_keep)
  if (p.c_dtype != ICAP_BF16) {
    if (pl.actk == ACT_OFF) ICAP_GKW(float, ACT_OFF);
    else ICAP_GKW(float, ACT_ANY);
    return;
  }
  switch (pl.actk) {
    case ACT_OFF: ICAP_GKW(bf16_t, ACT_OFF); break;
    case ACT_FWD + ICAP_ACT_GELU_NEW: ICAP_GKW(bf16_t, ACT_FWD + ICAP_ACT_GELU_NEW); break;
    case ACT_BWD + ICAP_ACT_GELU_NEW: ICAP_GKW(bf16_t, ACT_BWD + ICAP_ACT_GELU_NEW); break;
    case ACT_FWD + ICAP_ACT_QUICK_GELU: ICAP_GKW(bf16_t, ACT_FWD + ICAP_ACT_QUICK_GELU); break;
    case ACT_FWD + ICAP_ACT_RELU: ICAP_GKW(bf16_t, ACT_FWD + ICAP_ACT_RELU); break;
    case ACT_BWD + ICAP_ACT_RELU: ICAP_GKW(bf16_t, ACT_BWD + ICAP_ACT_RELU); break;
    case ACT_LNS + ACT_OFF: ICAP_GKW(bf16_t, ACT_LNS + ACT_OFF); break;
    case ACT_LNF + ACT_OFF: ICAP_GKW(bf16_t, ACT_LNF + ACT_OFF); break;
    case ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW: ICAP_GKW(bf16_t, ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW); break;
    case ACT_LNF + ACT_FWD + ICAP_ACT_QUICK_GELU: ICAP_GKW(bf16_t, ACT_LNF + ACT_FWD + ICAP_ACT_QUICK_GELU); break;
    default: ICAP_GKW(bf16_t, ACT_ANY); break;
  }
#undef ICAP_GKW
}

}  // namespace icap

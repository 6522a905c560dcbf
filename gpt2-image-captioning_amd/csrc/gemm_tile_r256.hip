#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// Variant 22: 256 x 128 tiles of 8 waves (4 x 2, 64 x 64 each) on the 3-stage LDS-DMA ring, one block per CU
// (gemm_tile.h, NST >= 3), bf16 inputs, every epilogue form the plan may give it (round 5).
void launch_tile_r256(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
#define ICAP_GKR(TC, KIND) \
  hipLaunchKernelGGL((gemm_kernel<bf16_t, TC, 3, 1, 4, 2, 4, 4, false, KIND>), grid, block, 0, s, p, tn, sp, nks, thr, inv_keep)
  if (p.c_dtype != ICAP_BF16) {
    if (pl.actk == ACT_OFF) ICAP_GKR(float, ACT_OFF);
    else ICAP_GKR(float, ACT_ANY);
    return;
  }
  switch (pl.actk) {
    case ACT_OFF: ICAP_GKR(bf16_t, ACT_OFF); break;
    case ACT_FWD + ICAP_ACT_GELU_NEW: ICAP_GKR(bf16_t, ACT_FWD + ICAP_ACT_GELU_NEW); break;
    case ACT_BWD + ICAP_ACT_GELU_NEW: ICAP_GKR(bf16_t, ACT_BWD + ICAP_ACT_GELU_NEW); break;
    case ACT_FWD + ICAP_ACT_QUICK_GELU: ICAP_GKR(bf16_t, ACT_FWD + ICAP_ACT_QUICK_GELU); break;
    case ACT_LNS + ACT_OFF: ICAP_GKR(bf16_t, ACT_LNS + ACT_OFF); break;
    case ACT_LNF + ACT_OFF: ICAP_GKR(bf16_t, ACT_LNF + ACT_OFF); break;
    case ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW: ICAP_GKR(bf16_t, ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW); break;
    case ACT_LNF + ACT_FWD + ICAP_ACT_QUICK_GELU: ICAP_GKR(bf16_t, ACT_LNF + ACT_FWD + ICAP_ACT_QUICK_GELU); break;
    default: ICAP_GKR(bf16_t, ACT_ANY); break;
  }
#undef ICAP_GKR
}

}  // namespace icap

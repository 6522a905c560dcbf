#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// Activation-specialised epilogues (gemm_plan: bf16 in / out, variants 0, 4, 5, 13)
void launch_tile_act(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
#define ICAP_GKS(NST, MINB, TM_, TN_, KIND) \
  hipLaunchKernelGGL((gemm_kernel<bf16_t, bf16_t, NST, MINB, 2, 2, TM_, TN_, false, KIND>), grid, block, 0, s, p, tn, sp, \
                     nks, thr, inv_keep)
  switch (pl.actk) {
    case ACT_FWD + ICAP_ACT_GELU_NEW:  // (variant 0: GPT-2 large / medium c_fc, K = 1280 / 1024 > 16 stages)
      if (pl.variant == 0) ICAP_GKS(2, 2, 4, 4, ACT_FWD + ICAP_ACT_GELU_NEW);
      else if (pl.variant == 4) ICAP_GKS(1, 3, 4, 4, ACT_FWD + ICAP_ACT_GELU_NEW);
      else ICAP_GKS(1, 4, 4, 4, ACT_FWD + ICAP_ACT_GELU_NEW);
      break;
    case ACT_BWD + ICAP_ACT_GELU_NEW:
      if (pl.variant == 0) ICAP_GKS(2, 2, 4, 4, ACT_BWD + ICAP_ACT_GELU_NEW);
      else if (pl.variant == 4) ICAP_GKS(1, 3, 4, 4, ACT_BWD + ICAP_ACT_GELU_NEW);
      else ICAP_GKS(1, 4, 4, 4, ACT_BWD + ICAP_ACT_GELU_NEW);
      break;
    case ACT_FWD + ICAP_ACT_QUICK_GELU: ICAP_GKS(1, 3, 4, 4, ACT_FWD + ICAP_ACT_QUICK_GELU); break;
    case ACT_FWD + ICAP_ACT_GELU_ERF: ICAP_GKS(1, 3, 4, 4, ACT_FWD + ICAP_ACT_GELU_ERF); break;
    case ACT_FWD + ICAP_ACT_RELU: ICAP_GKS(1, 4, 4, 2, ACT_FWD + ICAP_ACT_RELU); break;
    default: ICAP_GKS(1, 4, 4, 2, ACT_BWD + ICAP_ACT_RELU); break;
  }
#undef ICAP_GKS
}

}  // namespace icap

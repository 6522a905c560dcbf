#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// The LayerNorm statistics hand-off forms (bf16 in / out; gemm_plan lists the combinations): producers (ACT_LNS, no
// activation) and consumers (ACT_LNF: no activation, gelu_new, quick_gelu; 128 x 64 tiles with the dispatching form)
void launch_tile_ln(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
#define ICAP_GKL(NST, MINB, TM_, TN_, KIND) \
  hipLaunchKernelGGL((gemm_kernel<bf16_t, bf16_t, NST, MINB, 2, 2, TM_, TN_, false, KIND>), grid, block, 0, s, p, tn, sp, \
                     nks, thr, inv_keep)
#define ICAP_GKL_V(KIND)                                     \
  switch (pl.variant) {                                      \
    case 0: ICAP_GKL(2, 2, 4, 4, KIND); break;               \
    case 4: ICAP_GKL(1, 3, 4, 4, KIND); break;               \
    case 5: ICAP_GKL(1, 4, 4, 4, KIND); break;               \
    case 12: ICAP_GKL(2, 3, 4, 2, KIND); break;              \
    default: ICAP_GKL(1, 4, 4, 2, KIND); break;              \
  }
  switch (pl.actk) {
    case ACT_LNS + ACT_OFF: ICAP_GKL_V(ACT_LNS + ACT_OFF) break;
    case ACT_LNF + ACT_OFF: ICAP_GKL_V(ACT_LNF + ACT_OFF) break;
    case ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW:
      if (pl.variant == 0) ICAP_GKL(2, 2, 4, 4, ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW);
      else if (pl.variant == 4) ICAP_GKL(1, 3, 4, 4, ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW);
      else ICAP_GKL(1, 4, 4, 4, ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW);
      break;
    case ACT_LNF + ACT_FWD + ICAP_ACT_QUICK_GELU: ICAP_GKL(1, 3, 4, 4, ACT_LNF + ACT_FWD + ICAP_ACT_QUICK_GELU); break;
    default:  // ACT_LNF + ACT_ANY, 128 x 64
      if (pl.variant == 12) ICAP_GKL(2, 3, 4, 2, ACT_LNF + ACT_ANY);
      else ICAP_GKL(1, 4, 4, 2, ACT_LNF + ACT_ANY);
      break;
  }
#undef ICAP_GKL_V
#undef ICAP_GKL
}

}  // namespace icap

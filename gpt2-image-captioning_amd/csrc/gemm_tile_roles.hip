#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// Variant 26 (round 6): 128 x 256 tiles, the split-role ring of gemm_tile.h (ROLES): 4 MFMA waves of 64 x 128 (one per
// SIMD) + 4 LDS-DMA waves, 3 stages of 48 KiB, one block per CU. For the products with N >= 2048 whose 128 x 256 tiles
// fill about one round (GPT-2's 3584 x 2304 x 768 c_attn: 252 tiles). Every epilogue form the plan may give it.
void launch_tile_roles(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
#define ICAP_GKW(TC, KIND) \
  hipLaunchKernelGGL((gemm_kernel<bf16_t, TC, 3, 1, 2, 2, 4, 8, false, KIND, true>), grid, block, 0, s, p, tn, sp, nks, thr, inv_keep)
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
    case ACT_LNS + ACT_OFF: ICAP_GKW(bf16_t, ACT_LNS + ACT_OFF); break;
    case ACT_LNF + ACT_OFF: ICAP_GKW(bf16_t, ACT_LNF + ACT_OFF); break;
    case ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW: ICAP_GKW(bf16_t, ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW); break;
    case ACT_LNF + ACT_FWD + ICAP_ACT_QUICK_GELU: ICAP_GKW(bf16_t, ACT_LNF + ACT_FWD + ICAP_ACT_QUICK_GELU); break;
    default: ICAP_GKW(bf16_t, ACT_ANY); break;
  }
#undef ICAP_GKW
}

}  // namespace icap

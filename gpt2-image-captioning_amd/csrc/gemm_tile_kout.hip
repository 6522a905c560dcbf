#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// K-outer operands (trans_ab; bf16 inputs): double-buffered (14) / single-stage (15)
void launch_tile_kout(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
  if (p.c_dtype == ICAP_BF16) {
    if (pl.variant == 14) ICAP_GK(bf16_t, bf16_t, 2, 2, 4, 4, true);
    else ICAP_GK(bf16_t, bf16_t, 1, 3, 4, 4, true);
  } else {
    if (pl.variant == 14) ICAP_GK(bf16_t, float, 2, 2, 4, 4, true);
    else ICAP_GK(bf16_t, float, 1, 3, 4, 4, true);
  }
}

}  // namespace icap

#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// MX block-scaled fp8 inputs: variants 0 / 4 only (gemm_plan)
void launch_tile_mx(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
  if (p.c_dtype == ICAP_BF16) {
    if (pl.variant == 0) ICAP_GK(fp8_t, bf16_t, 2, 2, 4, 4, false);
    else ICAP_GK(fp8_t, bf16_t, 1, 3, 4, 4, false);
  } else {
    if (pl.variant == 0) ICAP_GK(fp8_t, float, 2, 2, 4, 4, false);
    else ICAP_GK(fp8_t, float, 1, 3, 4, 4, false);
  }
}

}  // namespace icap

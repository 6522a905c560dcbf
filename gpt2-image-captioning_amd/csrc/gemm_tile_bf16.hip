#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// bf16 inputs, runtime-dispatch (ACT_ANY) or activation-free (ACT_OFF) epilogues: 128 x 128 (variants 0 / 4 / 5),
// the 4-stage ring (16), 128 x 64 (12 / 13)
void launch_tile_bf16(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
  if (pl.variant == 16) {  // 4-stage ring
    if (p.c_dtype == ICAP_BF16) ICAP_GK(bf16_t, bf16_t, 4, 1, 4, 4, false);
    else ICAP_GK(bf16_t, float, 4, 1, 4, 4, false);
  } else if (pl.variant == 12 || pl.variant == 13) {  // 128 x 64
    if (p.c_dtype == ICAP_BF16) {
      if (pl.variant == 12) ICAP_GK(bf16_t, bf16_t, 2, 3, 4, 2, false);
      else ICAP_GK(bf16_t, bf16_t, 1, 4, 4, 2, false);
    } else {
      if (pl.variant == 12) ICAP_GK(bf16_t, float, 2, 3, 4, 2, false);
      else ICAP_GK(bf16_t, float, 1, 4, 4, 2, false);
    }
  } else if (p.c_dtype == ICAP_BF16) {
    ICAP_GEMM_LAUNCH(bf16_t, bf16_t)
  } else {
    ICAP_GEMM_LAUNCH(bf16_t, float)
  }
}

}  // namespace icap

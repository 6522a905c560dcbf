#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// fp32 inputs (the parity mode: exact-fp32 16x16x4 MFMA chains): variants 0 / 4 / 5
void launch_tile_f32(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
  if (p.c_dtype == ICAP_BF16) {
    ICAP_GEMM_LAUNCH(float, bf16_t)
  } else {
    ICAP_GEMM_LAUNCH(float, float)
  }
}

}  // namespace icap

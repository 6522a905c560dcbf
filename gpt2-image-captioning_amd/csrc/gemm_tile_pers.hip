#include "gemm_pers.h"
#include "gemm_plan.h"

namespace icap {

// Variant 30 (round 6): the persistent split-role GEMM with the overlapped epilogue (gemm_pers.h): 96 x 128 tiles,
// 4 MFMA + 4 LDS-DMA + 4 epilogue waves, a 3-stage ring and an fp32 C buffer, one block per CU walking its tiles.
// For products of several rounds of tiles, where the one-tile-at-a-time forms pay every tile's epilogue in series.
void launch_tile_pers(const GemmPlan& pl, const icap_gemm_args& p, int nk, hipStream_t s) {
  const dim3 grid = pl.grid, block(768);
  const int tn = pl.tiles_n;
  const uint32_t thr = pl.thr;
  const float inv_keep = pl.inv_keep;
#define ICAP_GKP(TC, KIND) \
  hipLaunchKernelGGL((gemm_pers_kernel<TC, 3, 3, 4, KIND>), grid, block, 0, s, p, tn, nk, thr, inv_keep)
  if (p.c_dtype != ICAP_BF16) {
    if (pl.actk == ACT_OFF) ICAP_GKP(float, ACT_OFF);
    else ICAP_GKP(float, ACT_ANY);
    return;
  }
  switch (pl.actk) {
    case ACT_OFF: ICAP_GKP(bf16_t, ACT_OFF); break;
    case ACT_FWD + ICAP_ACT_GELU_NEW: ICAP_GKP(bf16_t, ACT_FWD + ICAP_ACT_GELU_NEW); break;
    case ACT_BWD + ICAP_ACT_GELU_NEW: ICAP_GKP(bf16_t, ACT_BWD + ICAP_ACT_GELU_NEW); break;
    case ACT_FWD + ICAP_ACT_QUICK_GELU: ICAP_GKP(bf16_t, ACT_FWD + ICAP_ACT_QUICK_GELU); break;
    case ACT_FWD + ICAP_ACT_RELU: ICAP_GKP(bf16_t, ACT_FWD + ICAP_ACT_RELU); break;
    case ACT_BWD + ICAP_ACT_RELU: ICAP_GKP(bf16_t, ACT_BWD + ICAP_ACT_RELU); break;
    case ACT_LNS + ACT_OFF: ICAP_GKP(bf16_t, ACT_LNS + ACT_OFF); break;
    case ACT_LNF + ACT_OFF: ICAP_GKP(bf16_t, ACT_LNF + ACT_OFF); break;
    case ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW: ICAP_GKP(bf16_t, ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW); break;
    case ACT_LNF + ACT_FWD + ICAP_ACT_QUICK_GELU: ICAP_GKP(bf16_t, ACT_LNF + ACT_FWD + ICAP_ACT_QUICK_GELU); break;
    default: ICAP_GKP(bf16_t, ACT_ANY); break;
  }
#undef ICAP_GKP
}

}  // namespace icap

#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// Variant 24: 192 x 64 tiles of 4 waves stacked in M (4 x 1, 48 x 64 each), double-buffered LDS-DMA at 2 blocks per
// CU (gemm_tile.h, NST 2), bf16 inputs (round 5). For the N = 768 products of the packed step: 3584 x 768 is 19 x 12
// = 228 tiles, one round over 256 CUs, where 128 x 64 tiles make 336 (1.3 rounds) and 128 x 128 make 168 (two thirds
// of the CUs). hipBLASLt runs those shapes on one round of 128 x 96 tiles (profiles/r05_blaslt_kernels.txt); 96
// columns per tile do not split into the 32-column groups of the LayerNorm statistics epilogue, 64 do.
// Variant 25: the same tiles on the LDS-DMA ring (gemm_tile.h NST 4: three stages in flight, one
// block per CU) for long K. (Round 5 also measured a fragment prefetch across the ring's stages and a register-staged
// double buffer on these tiles — bitwise equal, neither faster: profiles/r05_w192_ab.txt; removed.)
void launch_tile_w192(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s) {
  ICAP_TILE_PRELUDE;
#define ICAP_GKW(TC, KIND)                                                                                                 \
  do {                                                                                                                     \
    if (pl.variant == 25)                                                                                                  \
      hipLaunchKernelGGL((gemm_kernel<bf16_t, TC, 4, 1, 4, 1, 3, 4, false, KIND>), grid, block, 0, s, p, tn, sp, nks, thr, inv_keep); \
    else                                                                                                                   \
      hipLaunchKernelGGL((gemm_kernel<bf16_t, TC, 2, 2, 4, 1, 3, 4, false, KIND>), grid, block, 0, s, p, tn, sp, nks, thr, inv_keep); \
  } while (0)
  if (p.c_dtype != ICAP_BF16) {
    if (pl.actk == ACT_OFF) ICAP_GKW(float, ACT_OFF);
    else ICAP_GKW(float, ACT_ANY);
    return;
  }
  switch (pl.actk) {
    case ACT_OFF: ICAP_GKW(bf16_t, ACT_OFF); break;
    case ACT_LNS + ACT_OFF: ICAP_GKW(bf16_t, ACT_LNS + ACT_OFF); break;
    default: ICAP_GKW(bf16_t, ACT_ANY); break;
  }
#undef ICAP_GKW
}

}  // namespace icap

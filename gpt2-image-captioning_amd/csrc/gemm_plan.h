// The launch plan icap_gemm makes for one call (gemm.hip: gemm_plan) and the per-form launchers of the tile
// kernel (gemm_tile_*.hip: one translation unit per input form, so their instantiations compile in parallel).
#pragma once
#include "gemm_common.h"

namespace icap {
// What icap_gemm launches for one call (shared by the launcher and icap_gemm_kernel_name).
struct GemmPlan {
  bool skinny = false;
  bool g256 = false;     // the 256 x 256 8-phase kernel (gemm256.hip)
  int g8p = 0;           // the 256-row 8-phase kernel (gemm8p.hip): its tile width BN (128 / 256), 0 = not taken
  int nt = 1;            // skinny: 16-column slabs per block
  int sku = 3;           // skinny: k-steps in flight per wave
  int variant = 0;       // tile kernel (see ICAP_GEMM_LAUNCH)
  int splits = 1, nk_split = 0, tiles_n = 0;
  bool fused = false;    // split-K combined inside the launch (tickets), no reduce pass
  int actk = ACT_ANY;    // tile kernels: the epilogue's activation instantiation (ACT_OFF / ACT_ANY / a specialised one)
  dim3 grid, block;
  uint32_t thr = 0;
  float inv_keep = 1.f;
};

// Launch the tile-kernel instantiation pl selects (grid pl.grid, block pl.block); nks = nk_split | skew / diag bits.
void launch_tile_bf16(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s);  // variants 0/4/5/12/13/16
void launch_tile_act(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s);   // specialised epilogues
void launch_tile_kout(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s);  // K-outer (14 / 15)
void launch_tile_mx(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s);    // MX fp8 (0 / 4)
void launch_tile_f32(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s);   // fp32 parity (0 / 4 / 5)
void launch_tile_ln(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s);    // LN statistics hand-off
void launch_tile_r256(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s);  // 256 x 128 ring (22)
void launch_tile_w192(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s);  // 192 x 64 (24)
void launch_tile_roles(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s);    // roles 128 x 256 (26)
void launch_tile_roles96(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s);  // roles 96 x 128 (27)
void launch_tile_roles192(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s); // roles 192 x 256 (28)
void launch_tile_roles_kout(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s); // roles K-outer (31)
void launch_tile_roles160(const GemmPlan& pl, const icap_gemm_args& p, int nks, hipStream_t s);  // roles 160 x 128 (32)
// a group of K-outer weight-gradient products run in one launch (icap_gemm_group)
constexpr int ICAP_GEMM_GROUP_MAX = 8;
struct GemmGroup {
  icap_gemm_args a[ICAP_GEMM_GROUP_MAX];
  int tiles_n[ICAP_GEMM_GROUP_MAX];
  int nk[ICAP_GEMM_GROUP_MAX];
  int tstart[ICAP_GEMM_GROUP_MAX + 1];
  int n;
};
void launch_group_kout(const GemmGroup& g, int cus, hipStream_t s);

}  // namespace icap

// The launch helpers of the gemm_tile_*.hip units (each defines its launcher with these).
#define ICAP_TILE_PRELUDE                                       \
  const dim3 grid = pl.grid, block = pl.block;                  \
  const int sp = pl.splits, tn = pl.tiles_n;                    \
  const uint32_t thr = pl.thr;                                  \
  const float inv_keep = pl.inv_keep
#define ICAP_GK(TI, TC, NST, MINB, TM_, TN_, KOUT)                                                              \
  do {                                                                                                       \
    if (pl.actk == ACT_ANY) hipLaunchKernelGGL((gemm_kernel<TI, TC, NST, MINB, 2, 2, TM_, TN_, KOUT, ACT_ANY>), grid, block, 0, s, p, tn, sp, nks, thr, inv_keep); \
    else hipLaunchKernelGGL((gemm_kernel<TI, TC, NST, MINB, 2, 2, TM_, TN_, KOUT, ACT_OFF>), grid, block, 0, s, p, tn, sp, nks, thr, inv_keep); \
  } while (0)
#define ICAP_GEMM_LAUNCH(TI, TC)                                    \
  switch (pl.variant) {                                             \
    case 0: ICAP_GK(TI, TC, 2, 2, 4, 4, false); break;              \
    case 4: ICAP_GK(TI, TC, 1, 3, 4, 4, false); break;              \
    default: ICAP_GK(TI, TC, 1, 4, 4, 4, false); break;             \
  }

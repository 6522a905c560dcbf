// The 128-row tile GEMM kernel template (included by gemm.hip and the gemm_tile_*.hip translation units,
// which instantiate and launch its forms; split so the instantiations compile in parallel).
// MFMA GEMM for gfx950: C[M,N] = epi(alpha * A[M,K] . B[N,K]^T).
//
// Both operands are K-contiguous in HBM ("weights stored [out,in]"), which is
// the layout every forward/backward product of the captioning path is brought
// into (frozen GPT-2 weights are kept in both orientations, trainable ones get
// their transposed bf16 copy refreshed after each optimizer step, dW products
// transpose their activation operands first).
//
// Tiling: 128x128 output tile per 256-thread workgroup (4 waves in 2x2, each a
// 64x64 sub-tile = 4x4 MFMA 16x16 tiles). One pipeline stage holds 128 bytes
// of K per row (bf16: 64 K, f32: 32 K) for A and B in LDS (16 KiB each), two
// stages double-buffered (64 KiB). LDS rows are 128 B with the 16-byte chunk
// index XOR-swizzled by (row & 7) so the ds_read_b128 fragment reads and the
// ds_write_b128 staging writes are bank-conflict free
// (cdna_hip_programming.md §5.5 T2). Global->LDS goes through registers
// (loads for stage k+1 are issued before the MFMAs of stage k: T14) with
// buffer loads whose hardware range check zero-fills out-of-range rows and
// K-tail chunks, so the main loop has no per-load branches (§5 trap (c)).
//
// Epilogue: each wave stages its 64x64 fp32 accumulators through LDS (two
// 32-row halves) and re-reads them 4 consecutive columns per lane, so bias /
// activation / dropout / residual / aux / beta are applied on coalesced 8- or
// 16-byte vectors (16 lanes cover one 64-column row segment).
//
// bf16: v_mfma_f32_16x16x32_bf16 — lane l supplies row (l&15), k = 8(l>>4)..+7.
// f32 (parity mode): v_mfma_f32_16x16x4_f32 (exact fp32 FMA chain) — one
// 16-byte chunk per lane = 4 K values, consumed by four MFMAs; lane group g
// supplies k = 4g+s in MFMA s for both operands, so the K permutation is
// identical on A and B and the product is exact.
// C/D map (both): col = lane&15, row = 4*(lane>>4) + reg.
#pragma once
#include "gemm_common.h"

// Diagnostic builds only (make stamps: -DICAP_STAMPS): phase timestamps per workgroup into icap_gemm_args.diag_stamps
// (8 uint64 per blockIdx.x; s_memrealtime, 100 MHz): [0] split | order << 8 | tile << 32, [1] start, [2] first stage
// landed, [3] main loop done, [4] split-K publish / combine done, [5] epilogue done. Not compiled otherwise.
#ifdef ICAP_STAMPS
#define ICAP_STAMP(i, v)                                                                                         \
  do {                                                                                                         \
    if (p.diag_stamps && threadIdx.x == 0) p.diag_stamps[(int64_t)blockIdx.x * 8 + (i)] = (uint64_t)(v);       \
  } while (0)
#define ICAP_NOW() __builtin_amdgcn_s_memrealtime()
#else
#define ICAP_STAMP(i, v) do {} while (0)
#define ICAP_NOW() 0ull
#endif

namespace icap {

// ---- K-outer operand images (trans_ab): [64 k-rows][128 columns] bf16, 256-byte rows, 16-byte chunk ch of row r
// stored at chunk ch ^ kout_swz(r) (cdna_hip_programming.md T10 layout (b)) so the transposed reads below are
// at most 2-way bank conflicted.
__device__ __forceinline__ int kout_swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int kout_off(int r, int ch) { return r * 256 + ((ch ^ kout_swz(r)) << 4); }
typedef short kv4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) kv4s_t* kout_lds_ptr;
// MFMA 16x16x32 operand (lane: column c0 + (lane & 15)) over k-rows r0..r0+31 of a K-outer image, as two
// ds_read_b64_tr_b16: lane 4q+p of 16-lane group g addresses row r0 + kb(g) + q (then + 16), columns 4p..4p+3 of
// the 16-column block, kb(g) = 8 (g & 1) + 4 (g >> 1); element j of the result = k-row r0 + kb(g) + j (j < 4),
// r0 + 16 + kb(g) + j - 4 (j >= 4). The two 16-lane groups of a 32-lane half (g, g ^ 1) read blocks 8 rows apart
// in the same columns, which the image's XOR makes conflict-free (cdna_hip_programming.md T10); with adjacent
// blocks (kb = 4g) every read was 2-way (SQ_LDS_BANK_CONFLICT = 0.47 of the kernel's LDS cycles,
// profiles/r04_pmc_lds.txt). Any k order works as long as both operands use the same one.
__device__ __forceinline__ uint4 kout_frag(const char* img, int r0, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int ch = (c0 >> 3) + (pp >> 1), half = (pp & 1) * 8;
  const int kb = 8 * (g & 1) + 4 * (g >> 1);
  const char* a0 = img + kout_off(r0 + kb + q, ch) + half;
  const char* a1 = img + kout_off(r0 + 16 + kb + q, ch) + half;
  const kv4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((kout_lds_ptr)(a0));
  const kv4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((kout_lds_ptr)(a1));
  uint4 r;
  r.x = (uint32_t)(uint16_t)lo[0] | ((uint32_t)(uint16_t)lo[1] << 16);
  r.y = (uint32_t)(uint16_t)lo[2] | ((uint32_t)(uint16_t)lo[3] << 16);
  r.z = (uint32_t)(uint16_t)hi[0] | ((uint32_t)(uint16_t)hi[1] << 16);
  r.w = (uint32_t)(uint16_t)hi[2] | ((uint32_t)(uint16_t)hi[3] << 16);
  return r;
}

// N fragment reads of 16 rows each (ds_read_b128, 2048 bytes apart) from LDS byte address a + BASE, as inline asm:
// hipcc would wait vmcnt(0) for any in-flight LDS-DMA before an LDS read it can see (the roles / ring main loops
// retire these reads with counted lgkmcnt waits instead)
typedef uint32_t frag_u32x4_t __attribute__((ext_vector_type(4)));
template <int I, int N, int BASE>
struct lds_frags {
  static __device__ __forceinline__ void run(frag_u32x4_t* f, uint32_t a) {
    if constexpr (I < N) {
      asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(f[I]) : "v"(a), "n"(BASE + I * 2048));
      lds_frags<I + 1, N, BASE>::run(f, a);
    }
  }
};

// Block geometry: WM x WN waves, each owning a (16 TM) x (16 TN) sub-tile of MFMA 16x16 accumulators, so the
// block tile is BM = 16 WM TM by BN = 16 WN TN. One pipeline stage holds 128 bytes of K per row (bf16: 64 K,
// f32: 32 K) for the BM rows of A and the BN rows of B in LDS.
// NST: LDS stages (2 = double-buffered: the LDS-DMA of stage k+1 overlaps the MFMAs of stage k; 1 = single
// buffer, two barriers per K step, latency hidden by MINB co-resident blocks per CU).
// Configurations in use: 128x128 / 4 waves (NST 1 or 2) and 256x256 / 8 waves (NST 2, 128 KiB, 1 block per CU:
// 4x the MFMA work per staged byte and per exposed load latency).
// KOUT: both operands K-outer (icap_gemm_args.trans_ab): A stored [K][lda] (m contiguous), B [K][ldb] — the dW
// products dY^T X over token rows, read without transposing either. A stage is then 64 k-rows x 128 m (n)
// columns, 256-byte LDS rows in the T10 (b) XOR image (cdna_hip_programming.md T10), written by LDS-DMA with the
// swizzle on the source address; fragments come from ds_read_b64_tr_b16 pairs (k order {kb..kb+3, 16+kb..},
// the same on both operands, so the contraction is unchanged). bf16 inputs, 128 x 128 tiles only.
// ACT: false for launches with no activation (act == dact == NONE: most of the step's products): the epilogue's
// activation code is then not compiled into the kernel at all. Measured (profiles/r03_k768_counters.txt): with it
// present, the plain 8320 x 2304 x 768 product ran 53.7 vs 45.0 us — the same memory instructions, +7 % VALU and
// +22 % SQ_WAIT_ANY (the larger function scheduled its main loop worse), SQ_WAIT_INST_ANY +1 % (not instruction fetch).
// ROLES (round 6; variants 26 / 27 / 28): the block has 4 more waves; waves 0 .. NW-1 read fragments and issue MFMAs
// only (NW = 4: one per SIMD; NW = 8: two per SIMD), waves NW .. NW+3 issue the LDS-DMA of the NST-stage ring and wait
// for it (one per SIMD), so the DMA's issue cost runs beside the MFMA stream instead of in front of it.
// epilogue prefetch groups of a ROLES block: the fewest (a divisor of the NH staging passes) that keep a wave's
// prefetched rows (passes per group x rows per pass / the NHALF waves sharing them) at <= 4 16-byte rows
constexpr int roles_prefetch_groups(int nh, int rows_per_pass, int nhalf) {
  for (int g = 1; g < nh; ++g)
    if (nh % g == 0 && (nh / g) * rows_per_pass / nhalf <= 4) return g;
  return nh;
}

template <typename TI, typename TC, int NST, int MINB, int WM, int WN, int TM, int TN, bool KOUT = false, int ACT = ACT_ANY,
          bool ROLES = false>
// The body of one tile (gemm_kernel below runs it once per block, or, for ROLES, once per live tile of a grid-stride
// loop): bid = the tile's block id in the capacity grid of tiles_m x tiles_n x splits blocks, Mv = the device row count.
__device__ __forceinline__ void gemm_body(icap_gemm_args p, int tiles_n, int splits, int nk_split, uint32_t drop_thresh,
                                          float inv_keep, const int bid, const int tiles_m, const int64_t Mv) {
  static_assert(!KOUT || (sizeof(TI) == 2 && 16 * WM * TM == 128 && 16 * WN * TN == 128),
                "K-outer operands: bf16, 128 x 128 tiles");
  static_assert(!ROLES || (sizeof(TI) == 2 && MINB == 1 &&
                            ((WM == 2 && WN == 2 && NST >= 3 && (!KOUT || (TM == 4 && TN == 4))) ||
                             (!KOUT && WM * WN == 8 && NST >= 2))),
                "roles: bf16 operands, 4 MFMA waves on a ring of >= 3 stages (K-outer: 128 x 128 tiles) or 8 on >= 2 "
                "(row-major), one block per CU");
  // MX block-scaled fp8 (TI = fp8_t): a stage's 128-byte LDS row is one 128-deep K step of
  // v_mfma_scale_f32_16x16x128_f8f6f4 (twice the bf16 flops per staged byte and per fragment byte read); the
  // per-32 E8M0 scales of the wave's 4 fragment rows of A and of B come in one 16-byte load each per stage
  constexpr bool MX = sizeof(TI) == 1;
  constexpr int AK = ACT & 0xFF;   // the epilogue's activation kind (ACT_OFF / ACT_ANY / ACT_FWD + a / ACT_BWD + a)
  constexpr int LNX = ACT >> 8;    // LayerNorm statistics hand-off: 1 = producer (ACT_LNS), 2 = consumer (ACT_LNF)
  static_assert(!MX || (!KOUT && TM == 4 && TN == 4 && WM == 2 && WN == 2), "MX fp8: 128 x 128 tiles of 4 waves");
  constexpr int NW = WM * WN;
  constexpr int BM = 16 * WM * TM, BN = 16 * WN * TN;
  constexpr int STB = (BM + BN) * GROWB;    // bytes per stage
  // rows per LDS-staged epilogue pass (16 where a wave's 16 TM rows are no multiple of 32: the 192-row tiles)
  constexpr int EPR = (NST >= 2 && (16 * TM) % 32 == 0) ? 32 : 16;
  constexpr int ELD = 16 * TN + 4;          // fp32 row stride of the epilogue staging tile
  static_assert(NW * EPR * ELD * 4 <= NST * STB, "epilogue staging must fit the stage buffers");
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "each wave stages whole 8-row DMA pieces");
  constexpr int APW = BM / (8 * NW), BPW = BN / (8 * NW);  // DMA instructions per wave per stage
  // (+ the consumer's LayerNorm row table, LNX == 2: its own 8 BM bytes past the stage buffers)
  __shared__ __attribute__((aligned(16))) char smem[NST * STB + (LNX == 2 ? 8 * BM : 0)];
  constexpr int ES = sizeof(TI);
  constexpr int EPC = 16 / ES;         // elements per 16-byte chunk
  constexpr int BKE = GROWB / ES;      // K elements per stage

  int tid = threadIdx.x;
  // (ROLES runs this body in a loop over tiles: an opaque thread index keeps hipcc from hoisting the lane-dependent
  // offsets of both roles out of the loop, where they would stay live through the whole body and spill)
  if constexpr (ROLES) asm volatile("" : "+v"(tid));
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave - wm * WN;

  const int64_t M = p.M, N = p.N, K = p.K;
  // bijective XCD-aware remap over the LIVE blocks: blocks sharing an XCD get consecutive tiles (consecutive
  // tiles share the A row panel). With a device row count the grid is sized for M but only the first
  // nlive = (row tiles of Mv) x tiles_n x splits blocks work: they are the lowest block ids, which the dispatcher
  // hands out first and round-robin over the XCDs, so the live tiles land one per CU before any CU takes a second
  // (the dead blocks exit at once), and the remap over nlive keeps every XCD's share contiguous.
  const int tiles_mv = p.m_dev ? (int)((Mv + BM - 1) / BM) : tiles_m;
  const int nwg = tiles_mv * tiles_n * splits;
  if (bid >= nwg) return;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  // split-K: split-major order, so the blocks of one split (same K range) sit together on an XCD
  const int tiles = tiles_mv * tiles_n;
  const int split = wgid / tiles, tile = wgid - split * tiles;
  const int tm = tile / tiles_n, tn = tile - tm * tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  if (m0 >= Mv) return;
  ICAP_STAMP(1, ICAP_NOW());
  // tile-relative buffer descriptors: rows past M / N fall beyond num_records and load zeros
  // (K-outer: k-rows past K do; columns past M / N read neighbouring data that only reaches unstored outputs)
  const char* Ab = reinterpret_cast<const char*>(p.A) + (KOUT ? m0 : m0 * p.lda) * ES;
  const char* Bb = reinterpret_cast<const char*>(p.B) + (KOUT ? n0 : n0 * p.ldb) * ES;
  const int64_t mrows = Mv - m0 < BM ? Mv - m0 : BM;
  const int64_t nrows = N - n0 < BN ? N - n0 : BN;
  // (K-outer: the last row's range ends on a whole 16-byte chunk — the hardware zeroes a dword that crosses
  // num_records — which lda % 8 == 0, lda >= M keeps inside the allocation)
  // timing diagnostic only (ICAP_GEMM_DIAG, never set in a real run): bits 28-29 of nk_split give the A / B
  // descriptor zero records, so the range check drops that operand's staging loads (cdna_hip_programming.md §7:
  // pricing one buffer's traffic) while the instruction stream, waits and barriers stay
  const int diag = (nk_split >> 28) & 3;
  const bool acq = (nk_split >> 30) & 1;  // fused split-K: acquire fence after the ticket poll (gemm_acquire())
  const __amdgpu_buffer_rsrc_t ra_rsrc = make_rsrc(
      Ab, (diag & 1) ? 0 : (uint64_t)(KOUT ? (K - 1) * p.lda + ((mrows + 7) & ~7ll) : (mrows - 1) * p.lda + K) * ES);
  const __amdgpu_buffer_rsrc_t rb_rsrc = make_rsrc(
      Bb, (diag & 2) ? 0 : (uint64_t)(KOUT ? (K - 1) * p.ldb + ((nrows + 7) & ~7ll) : (nrows - 1) * p.ldb + K) * ES);
  // LDS-DMA staging (buffer_load_dwordx4 ... lds): one wave-instruction writes 1 KiB = 8 LDS rows of
  // 128 B linearly (lane l -> row l>>3, physical chunk l&7). The XOR swizzle therefore goes on the SOURCE:
  // physical chunk pc of row r holds logical K-chunk pc ^ (r & 7) (cdna_hip_programming.md §5.4 rule 21).
  const int lrow = lane >> 3;
  const int lchunk = ((lane & 7) ^ lrow) * EPC;  // logical K offset (elements) of this lane's 16 B
  uint32_t a_off[APW], b_off[BPW];
  if constexpr (KOUT) {
    // one wave-instruction = 4 k-rows of 256 B: lane l -> row 4 i' + (l >> 4), physical chunk l & 15 holding
    // logical chunk (l & 15) ^ kout_swz(row)
    const int krow = lane >> 4;
#pragma unroll
    for (int i = 0; i < APW; ++i) {
      const int row = (wave * APW + i) * 4 + krow;
      a_off[i] = (uint32_t)(row * p.lda + (((lane & 15) ^ kout_swz(row)) << 3)) * ES;
    }
#pragma unroll
    for (int i = 0; i < BPW; ++i) {
      const int row = (wave * BPW + i) * 4 + krow;
      b_off[i] = (uint32_t)(row * p.ldb + (((lane & 15) ^ kout_swz(row)) << 3)) * ES;
    }
  } else {
#pragma unroll
    for (int i = 0; i < APW; ++i) a_off[i] = (uint32_t)(((wave * APW + i) * 8 + lrow) * p.lda + lchunk) * ES;
#pragma unroll
    for (int i = 0; i < BPW; ++i) b_off[i] = (uint32_t)(((wave * BPW + i) * 8 + lrow) * p.ldb + lchunk) * ES;
  }
  auto load_stage = [&](int64_t k0, int s) {
    if constexpr (KOUT) {  // k-rows past K lie beyond num_records (zeros)
      char* As = smem + s * STB;
      char* Bs = As + BM * GROWB;
      const uint32_t ka = (uint32_t)(k0 * p.lda * ES), kb2 = (uint32_t)(k0 * p.ldb * ES);
#pragma unroll
      for (int i = 0; i < APW; ++i) dma16(ra_rsrc, As + (wave * APW + i) * 8 * GROWB, a_off[i] + ka);
#pragma unroll
      for (int i = 0; i < BPW; ++i) dma16(rb_rsrc, Bs + (wave * BPW + i) * 8 * GROWB, b_off[i] + kb2);
      return;
    }
    const uint32_t kb = (uint32_t)(k0 * ES);
    const bool kin = k0 + lchunk < K;
    char* As = smem + s * STB;
    char* Bs = As + BM * GROWB;
#pragma unroll
    for (int i = 0; i < APW; ++i) dma16(ra_rsrc, As + (wave * APW + i) * 8 * GROWB, kin ? a_off[i] + kb : OOB);
#pragma unroll
    for (int i = 0; i < BPW; ++i) dma16(rb_rsrc, Bs + (wave * BPW + i) * 8 * GROWB, kin ? b_off[i] + kb : OOB);
  };

  // ---- LayerNorm fold (consumer, LNX == 2): the row statistics of A from the producer's per-32-column (mean, M2)
  // pairs, two threads per row: the mean of the group means, then M2 = sum M2_g + 32 (mean_g - mean)^2 (two passes
  // over the loaded pairs, no E[x^2] - mean^2 cancellation); rstd = 1 / sqrt(M2 / K + eps). Computed in the prologue,
  // right after the first stage's DMA is issued (its loads overlap that DMA instead of adding a dependent round
  // trip to the epilogue), into an LDS table of its own that the epilogue rows read after the main loop's barriers.
  float* lnr = reinterpret_cast<float*>(smem + NST * STB);
  auto ln_prologue = [&]() __attribute__((always_inline)) {
    if constexpr (LNX == 2) {
      static_assert(NW * 64 >= 2 * BM, "two threads per LN table row");
      if (tid >= 2 * BM) return;  // (8 MFMA waves over 192 rows: the first 384 threads)
      // each thread of the pair holds one half of the row's G pairs: G / 4 16-byte loads issued together (the host
      // guarantees G % 4 == 0 and G <= 4 LNQ), both passes from registers
      constexpr int LNQ = 10;  // 16-byte loads per thread at most: K <= 1280
      const int rr = tid >> 1, hf = tid & 1;
      const int64_t grow = m0 + rr < Mv ? m0 + rr : Mv - 1;
      const int G = (int)(K >> 5), nq = G >> 2;
      const float4* st = reinterpret_cast<const float4*>(p.ln_stats_in) + grow * (G >> 1) + hf * nq;
      float4 v[LNQ];
#pragma unroll
      for (int q = 0; q < LNQ; ++q)
        if (q < nq) v[q] = st[q];
      float sm = 0.f;
#pragma unroll
      for (int q = 0; q < LNQ; ++q)
        if (q < nq) sm += v[q].x + v[q].z;
      sm += __shfl_xor(sm, 1, 64);
      const float mean = sm / (float)G;
      float m2 = 0.f;
#pragma unroll
      for (int q = 0; q < LNQ; ++q)
        if (q < nq) {
          const float d0 = v[q].x - mean, d1 = v[q].z - mean;
          m2 += (v[q].y + 32.f * d0 * d0) + (v[q].w + 32.f * d1 * d1);
        }
      m2 += __shfl_xor(m2, 1, 64);
      const float rs = 1.f / sqrtf(m2 / (float)K + p.ln_eps);
      if (hf == 0) {
        lnr[2 * rr] = mean;
        lnr[2 * rr + 1] = rs;
        if (p.ln_mean_out && tn == 0 && split == 0 && m0 + rr < Mv) {  // for the LayerNorm backward (one block)
          p.ln_mean_out[m0 + rr] = mean;
          p.ln_rstd_out[m0 + rr] = rs;
        }
      }
    }
  };

  f32x4_t acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  // K-skew (host: kskew_for): bits 20-27 of nk_split rotate this tile's k-step order within its K range
  const int kskew = (nk_split >> 20) & 0xFF;
  nk_split &= 0xFFFFF;
  const int nk_all = (int)((K + BKE - 1) / BKE);
  const int kt0 = split * nk_split;
  const int nk = (nk_all - kt0 < nk_split ? nk_all - kt0 : nk_split);  // >= 1 by the host's choice of splits
  const int64_t kbase = (int64_t)kt0 * BKE;
  const int fr = lane & 15, fg = lane >> 4;
  const int koff = kskew ? (int)(((int64_t)(tm * 7 + tn) * kskew) % nk) : 0;
  auto kstep = [&](int kt) -> int64_t { const int j = kt + koff; return (int64_t)(j >= nk ? j - nk : j) * BKE; };

  // MX scales (mx_scale_off layout): this lane's 16 bytes per stage = the scales of rows i*16 + fr (i = 0..3) of the
  // wave's 64-row group, blocks 0..3; the lane's own block is fg (byte 8 fg of each word after the shift below)
  const int64_t rga = MX ? (M + 63) / 64 : 0, rgb = MX ? (N + 63) / 64 : 0;
  const __amdgpu_buffer_rsrc_t rsa = make_rsrc(MX ? p.a_scale : nullptr, MX ? (uint64_t)(K / 32) * rga * 64 : 0);
  const __amdgpu_buffer_rsrc_t rsb = make_rsrc(MX ? p.b_scale : nullptr, MX ? (uint64_t)(K / 32) * rgb * 64 : 0);
  auto load_scales = [&](int st, uint4& sa, uint4& sb) {
    if constexpr (MX) {
      sa = bload(rsa, (uint32_t)((((int64_t)st * rga + (m0 >> 6) + wm) * 16 + fr) * 16));
      sb = bload(rsb, (uint32_t)((((int64_t)st * rgb + (n0 >> 6) + wn) * 16 + fr) * 16));
    }
  };
  uint4 sca_cur{}, scb_cur{}, sca_nxt{}, scb_nxt{};

  // fragments of one stage: bf16 / f32 two 16-byte k-steps per row fragment; MX one 32-byte operand
  constexpr int KS = MX ? 1 : 2;
  typedef typename std::conditional<MX, i32x8_t, uint4>::type frag_t;
  auto read_frags = [&](const char* As, frag_t (&af)[KS][TM], frag_t (&bfr)[KS][TN]) {
    const char* Bs = As + BM * GROWB;
    if constexpr (MX) {  // lane (fr, fg): chunks fg and 4 + fg of its row = k 16 fg.. and 64 + 16 fg..
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * 16 * TM + i * 16 + fr;
        af[0][i] = ld_mx_frag(As + lds_off(row, fg), As + lds_off(row, 4 + fg));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * 16 * TN + j * 16 + fr;
        bfr[0][j] = ld_mx_frag(Bs + lds_off(row, fg), Bs + lds_off(row, 4 + fg));
      }
      return;
    }
    if constexpr (KOUT) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
#pragma unroll
        for (int i = 0; i < TM; ++i) af[ks][i] = kout_frag(As, ks * 32, wm * 16 * TM + i * 16, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bfr[ks][j] = kout_frag(Bs, ks * 32, wn * 16 * TN + j * 16, lane);
      }
      return;
    }
    if constexpr (!MX) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fg;  // chunks fg and 4 + fg: two MFMA k-steps
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[ks][i] = *reinterpret_cast<const uint4*>(As + lds_off(wm * 16 * TM + i * 16 + fr, ch));
#pragma unroll
      for (int j = 0; j < TN; ++j)
        bfr[ks][j] = *reinterpret_cast<const uint4*>(Bs + lds_off(wn * 16 * TN + j * 16 + fr, ch));
    }
    }
  };
  auto mfmas = [&](const frag_t (&af)[KS][TM], const frag_t (&bfr)[KS][TN]) {
    if constexpr (MX) {
      const uint32_t wa[4] = {sca_cur.x, sca_cur.y, sca_cur.z, sca_cur.w};
      const uint32_t wb[4] = {scb_cur.x, scb_cur.y, scb_cur.z, scb_cur.w};
      const int sh = 8 * fg;
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mfma_mx(acc[i][j], af[0][i], bfr[0][j], wa[i] >> sh, wb[j] >> sh);
    } else {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) mfma_chunk<TI>(acc[i][j], af[ks][i], bfr[ks][j]);  // lane = col, regs = 4 rows
    }
  };

  if constexpr (ROLES) {
    // Split roles over an NST-stage LDS-DMA ring, one barrier per 64-deep k-step (tools/microbench/gemm_lab.hip,
    // profiles/r06_gemm_lab.txt). Barrier B_k (k = 0 .. nk) is reached by
    //   a loader wave after its DMA of stage k has landed (counted vmcnt: stages k+1 .. k+NST-2 stay in flight);
    //   an MFMA wave after every fragment read of stage k-1 has retired (lgkmcnt(0)).
    // After B_k the loaders issue stage k+NST-1 into the slot stage k-1 used (free: its reads retired before B_k), the
    // MFMA waves read stage k. The MFMA waves read each 32-deep substep's fragments while the previous substep's MFMAs
    // issue, so B_{k+1} falls between the two substeps of stage k: [wait F0] [read F1 of k] [MFMAs F0] [wait F1] B_{k+1}
    // [read F0 of k+1] [MFMAs F1]. Loader waves never read LDS and MFMA waves never issue DMA, so no wave ever waits
    // for LDS-DMA it did not issue except through a barrier.
    // Stages past K are issued with out-of-range offsets (nothing is fetched, zeros land in a free slot), so every
    // loop iteration has the same DMA count and the same vmcnt.
    constexpr int NLW = 4;                    // loader waves
    constexpr int P = (BM + BN) / (8 * NLW);  // 1-KiB DMA pieces per loader wave per stage
    constexpr int PA = BM / (8 * NLW);        // of them A rows (pieces i < PA)
    static_assert((BM + BN) % (8 * NLW) == 0 && BM % (8 * NLW) == 0 && (NST - 2) * P < 64, "roles: stage split");
    const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>(smem);
    if (wave >= NW) {
      const int lw = wave - NW;
      uint32_t voff[P];
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const int q = i * NLW + lw;  // 1-KiB piece of the [A image; B image] stack
        if constexpr (KOUT) {
          // K-outer (round 6): 4 k-rows of 256 B per piece, lane l -> k-row 4 q' + (l >> 4), physical chunk l & 15
          // holding logical chunk (l & 15) ^ kout_swz(row) (the tile kernel's T10 (b) image)
          const int krow = (i < PA ? q : q - BM / 8) * 4 + (lane >> 4);
          voff[i] = (uint32_t)((int64_t)krow * (i < PA ? p.lda : p.ldb) + (((lane & 15) ^ kout_swz(krow)) << 3)) * ES;
        } else {
          const int row = (i < PA ? q : q - BM / 8) * 8 + lrow;  // 8-row piece
          voff[i] = (uint32_t)((int64_t)row * (i < PA ? p.lda : p.ldb) + lchunk) * ES;
        }
      }
      auto issue = [&](int kt, int slot) __attribute__((always_inline)) {
        const bool live = kt < nk;
        const int64_t k0 = live ? kbase + kstep(kt) : 0;
        if constexpr (KOUT) {  // k-rows past K lie beyond num_records (zeros)
          const uint32_t ka = (uint32_t)(k0 * p.lda * ES), kb2 = (uint32_t)(k0 * p.ldb * ES);
#pragma unroll
          for (int i = 0; i < P; ++i) {
            const uint32_t lds = __builtin_amdgcn_readfirstlane(sbase + (uint32_t)(slot * STB + (i * NLW + lw) * 1024));
            dma16a(i < PA ? ra_rsrc : rb_rsrc, lds, live ? voff[i] + (i < PA ? ka : kb2) : OOB);
          }
          return;
        }
        const uint32_t kb = (uint32_t)(k0 * ES);
        const bool kin = live && k0 + lchunk < K;
#pragma unroll
        for (int i = 0; i < P; ++i) {
          const uint32_t lds = __builtin_amdgcn_readfirstlane(sbase + (uint32_t)(slot * STB + (i * NLW + lw) * 1024));
          dma16a(i < PA ? ra_rsrc : rb_rsrc, lds, kin ? voff[i] + kb : OOB);
        }
      };
#pragma unroll
      for (int s = 0; s < NST - 1; ++s) issue(s, s);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * P) : "memory");
      __builtin_amdgcn_s_barrier();  // B_0
      for (int kt = 0; kt < nk; ++kt) {
        issue(kt + NST - 1, (kt + NST - 1) % NST);
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * P) : "memory");  // stage kt + 1 landed
        __builtin_amdgcn_s_barrier();                                        // B_{kt+1}
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the past-K stages' zeros, before the epilogue reuses LDS
    } else {
    typedef frag_u32x4_t u32x4_t;
    uint32_t la[2], lb[2];  // this lane's fragment row in a stage (A row / B row), swizzled chunk of substep ks
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint32_t sw = (uint32_t)(((ks * 4 + fg) ^ (fr & 7)) << 4);
      la[ks] = (uint32_t)((wm * 16 * TM + fr) * GROWB) + sw;
      lb[ks] = (uint32_t)((wn * 16 * TN + fr) * GROWB) + sw;
    }
    u32x4_t fa0[TM], fb0[TN], fa1[TM], fb1[TN];
    auto rd = [&](u32x4_t (&fa)[TM], u32x4_t (&fb)[TN], uint32_t a, uint32_t b) __attribute__((always_inline)) {
      lds_frags<0, TM, 0>::run(fa, a);
      lds_frags<0, TN, BM * GROWB>::run(fb, b);
    };
    // retire every outstanding fragment read; the empty asm ties make the MFMAs that use them wait here
    auto retire = [&](u32x4_t (&fa)[TM], u32x4_t (&fb)[TN]) __attribute__((always_inline)) {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(fa[i]));
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(fb[j]));
      __builtin_amdgcn_sched_barrier(0);
    };
    auto mm = [&](const u32x4_t (&fa)[TM], const u32x4_t (&fb)[TN]) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          mfma_chunk<TI>(acc[i][j], __builtin_bit_cast(uint4, fa[i]), __builtin_bit_cast(uint4, fb[j]));
    };
    ln_prologue();  // (its loads are the MFMA waves' only vector-memory operations)
    __builtin_amdgcn_s_barrier();  // B_0
    __builtin_amdgcn_sched_barrier(0);
    ICAP_STAMP(2, ICAP_NOW());
    if constexpr (KOUT) {
      // K-outer (round 6, the mapper's weight gradients): fragments by ds_read_b64_tr_b16 pairs from the T10 (b)
      // images (kout_frag), the same k order on both operands; double-buffered by 32-deep substep like the row-major
      // loop below, every read of stage kt retired (lgkmcnt(0) + ties) before B_{kt+1}
      auto rdk = [&](uint32_t sb, int ks, u32x4_t(&fa)[TM], u32x4_t(&fb)[TN]) __attribute__((always_inline)) {
        const char* As = smem + (sb - sbase);
#pragma unroll
        for (int i = 0; i < TM; ++i) fa[i] = __builtin_bit_cast(u32x4_t, kout_frag(As, ks * 32, wm * 16 * TM + i * 16, lane));
#pragma unroll
        for (int j = 0; j < TN; ++j)
          fb[j] = __builtin_bit_cast(u32x4_t, kout_frag(As + BM * GROWB, ks * 32, wn * 16 * TN + j * 16, lane));
      };
      rdk(sbase, 0, fa0, fb0);
      for (int kt = 0; kt < nk; ++kt) {
        const uint32_t sb = sbase + (uint32_t)((kt % NST) * STB);
        retire(fa0, fb0);
        rdk(sb, 1, fa1, fb1);
        mm(fa0, fb0);
        retire(fa1, fb1);
        __builtin_amdgcn_s_barrier();  // B_{kt+1}
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 1 < nk) rdk(sbase + (uint32_t)(((kt + 1) % NST) * STB), 0, fa0, fb0);
        mm(fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else if constexpr (NW == 8) {
      // two MFMA waves per SIMD (variant 28, 96 x 64 per wave): one fragment set each (the 168-register budget of
      // three waves per SIMD), read right before its MFMAs — the partner wave's MFMAs cover the read latency
      for (int kt = 0; kt < nk; ++kt) {
        const uint32_t sb = sbase + (uint32_t)((kt % NST) * STB);
        rd(fa0, fb0, sb + la[0], sb + lb[0]);
        retire(fa0, fb0);
        mm(fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        rd(fa0, fb0, sb + la[1], sb + lb[1]);
        retire(fa0, fb0);
        mm(fa0, fb0);
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_barrier();  // B_{kt+1}: every read of stage kt retired (retire above)
      }
    } else {
    rd(fa0, fb0, sbase + la[0], sbase + lb[0]);
    for (int kt = 0; kt < nk; ++kt) {
      const uint32_t sb = sbase + (uint32_t)((kt % NST) * STB);
      retire(fa0, fb0);
      rd(fa1, fb1, sb + la[1], sb + lb[1]);
      mm(fa0, fb0);
      retire(fa1, fb1);
      __builtin_amdgcn_s_barrier();  // B_{kt+1}
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nk) {
        const uint32_t sn = sbase + (uint32_t)(((kt + 1) % NST) * STB);
        rd(fa0, fb0, sn + la[0], sn + lb[0]);
      }
      mm(fa1, fb1);
      __builtin_amdgcn_sched_barrier(0);
    }
    }
    }
    __syncthreads();  // every MFMA wave is done reading the ring and the loaders' DMA has drained
  } else if constexpr (NST >= 3) {
    // Deep ring for launches with about one tile per CU (the packed step's N = 768 products, round 3: 128 x 128
    // tiles, 4 LDS stages = 128 KiB) and for the 256 x 128 tiles of 8 waves (round 5: 3 stages of 48 KiB = 144 KiB):
    // one block per CU, NST - 2 stages in flight while stage kt is read and stage kt + NST - 1 is issued. The round-5
    // form exists because a CU's LDS-DMA intake, not the MFMA, bounds the main loop (≈ 70 GB/s per CU from the XCD's
    // L2: MI355X_MICROARCH.md "Indexed rows: gather into LDS"): a 256 x 128 tile fetches 48 KiB per 64-deep k-step
    // for the MFMA work two 128 x 128 tiles fetch 64 KiB for, and it needs >= 72 KiB in flight to reach that rate.
    // The fragment reads are inline asm (hipcc would otherwise drain the DMA queue, vmcnt(0), in front of every LDS
    // read), retired by counted lgkmcnt waits tied to their registers; the DMA waits are counted vmcnt (never 0 in
    // the steady state) and the barriers raw s_barrier (cdna_hip_programming.md "Pipelining across barriers", T3+T4).
    //   RAW: stage kt is read after this wave's vmcnt wait for it and a barrier every wave passed after its own.
    //   WAR: stage kt+NST-1 is written into the slot read in iteration kt-1, whose reads every wave retired
    //        (lgkmcnt) before that iteration's MFMAs, i.e. before the barrier of iteration kt.
    static_assert(!KOUT && !MX && sizeof(TI) == 2 && (TM == 4 || TM == 3) && TN == 4,
                  "ring: bf16 row-major operands, 64 x 64 or 48 x 64 per wave");
    constexpr int D = APW + BPW;  // DMA instructions per wave per stage
    typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
    const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>(smem);
    uint32_t la[2], lb[2];  // byte offsets in a stage of this lane's fragment rows (A row / B row + 16 i)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint32_t sw = (uint32_t)(((ks * 4 + fg) ^ (fr & 7)) << 4);
      la[ks] = (uint32_t)((wm * 16 * TM + fr) * GROWB) + sw;
      lb[ks] = (uint32_t)(BM * GROWB + (wn * 16 * TN + fr) * GROWB) + sw;
    }
#pragma unroll
    for (int s = 0; s < NST - 1; ++s)
      if (s < nk) load_stage(kbase + kstep(s), s);
    ln_prologue();  // (its loads are waited for at their first use, which drains the prologue's DMA once)
#define ICAP_RING_RD(dst, addr, off) asm volatile("ds_read_b128 %0, %1 offset:" #off : "=v"(dst) : "v"(addr))
    for (int kt = 0; kt < nk; ++kt) {
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (NST == 4) {
        if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * D) : "memory");  // kt+1, kt+2 stay in flight
        else if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(D) : "memory");  // kt+1 stays in flight
        else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kt + NST - 1 < nk) load_stage(kbase + kstep(kt + NST - 1), (kt + NST - 1) % NST);
      __builtin_amdgcn_sched_barrier(0);
      const uint32_t sb = sbase + (uint32_t)((kt % NST) * STB);
      u32x4_t fa0[4], fb0[4], fa1[4], fb1[4];
      {
        const uint32_t a0 = sb + la[0], b0 = sb + lb[0], a1 = sb + la[1], b1 = sb + lb[1];
        ICAP_RING_RD(fa0[0], a0, 0); ICAP_RING_RD(fa0[1], a0, 2048); ICAP_RING_RD(fa0[2], a0, 4096);
        if constexpr (TM == 4) ICAP_RING_RD(fa0[3], a0, 6144);
        ICAP_RING_RD(fb0[0], b0, 0); ICAP_RING_RD(fb0[1], b0, 2048); ICAP_RING_RD(fb0[2], b0, 4096); ICAP_RING_RD(fb0[3], b0, 6144);
        ICAP_RING_RD(fa1[0], a1, 0); ICAP_RING_RD(fa1[1], a1, 2048); ICAP_RING_RD(fa1[2], a1, 4096);
        if constexpr (TM == 4) ICAP_RING_RD(fa1[3], a1, 6144);
        ICAP_RING_RD(fb1[0], b1, 0); ICAP_RING_RD(fb1[1], b1, 2048); ICAP_RING_RD(fb1[2], b1, 4096); ICAP_RING_RD(fb1[3], b1, 6144);
      }
      // the first half's TM + 4 reads retired, the second half's TM + 4 still in flight
      if constexpr (TM == 4)
        asm volatile("s_waitcnt lgkmcnt(8)"
                     : "+v"(fa0[0]), "+v"(fa0[1]), "+v"(fa0[2]), "+v"(fa0[3]), "+v"(fb0[0]), "+v"(fb0[1]), "+v"(fb0[2]),
                       "+v"(fb0[3]));
      else
        asm volatile("s_waitcnt lgkmcnt(7)"
                     : "+v"(fa0[0]), "+v"(fa0[1]), "+v"(fa0[2]), "+v"(fb0[0]), "+v"(fb0[1]), "+v"(fb0[2]), "+v"(fb0[3]));
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (NW > 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          mfma_chunk<TI>(acc[i][j], __builtin_bit_cast(uint4, fa0[i]), __builtin_bit_cast(uint4, fb0[j]));
      if constexpr (NW > 4) __builtin_amdgcn_s_setprio(0);
      if constexpr (TM == 4)
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(fa1[0]), "+v"(fa1[1]), "+v"(fa1[2]), "+v"(fa1[3]), "+v"(fb1[0]), "+v"(fb1[1]), "+v"(fb1[2]),
                       "+v"(fb1[3]));
      else
        asm volatile("s_waitcnt lgkmcnt(0)"
                     : "+v"(fa1[0]), "+v"(fa1[1]), "+v"(fa1[2]), "+v"(fb1[0]), "+v"(fb1[1]), "+v"(fb1[2]), "+v"(fb1[3]));
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (NW > 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          mfma_chunk<TI>(acc[i][j], __builtin_bit_cast(uint4, fa1[i]), __builtin_bit_cast(uint4, fb1[j]));
      if constexpr (NW > 4) __builtin_amdgcn_s_setprio(0);
    }
#undef ICAP_RING_RD
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();  // (no DMA outstanding) every wave is done reading the ring before the epilogue reuses it
  } else if (NST == 2) {
    load_stage(kbase + kstep(0), 0);
    load_scales(kt0, sca_cur, scb_cur);
    ln_prologue();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    ICAP_STAMP(2, ICAP_NOW());
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = kt & 1;
      // all fragment reads of this stage first: hipcc waits vmcnt(0) before any LDS read that follows an
      // LDS-DMA issue, so the next stage's DMA is issued only after the reads (and overlaps the MFMAs)
      frag_t af[KS][TM], bfr[KS][TN];
      read_frags(smem + cur * STB, af, bfr);
      // the other buffer was last read in iteration kt-1, which every wave finished before the barrier below
      if (kt + 1 < nk) {
        load_stage(kbase + kstep(kt + 1), cur ^ 1);
        load_scales(kt0 + kt + 1, sca_nxt, scb_nxt);
      }
      mfmas(af, bfr);
      // keep the MFMAs above the wait: they are register-only, so without this fence hipcc sinks them below the
      // vmcnt/barrier and the DMA is waited for right after it is issued (cdna_hip_programming.md §5.4 rule 18)
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of stage kt+1 has landed
      __syncthreads();                                      // ... and every other wave's
      if constexpr (MX) {
        sca_cur = sca_nxt;
        scb_cur = scb_nxt;
      }
    }
  } else {
    for (int kt = 0; kt < nk; ++kt) {
      if (kt > 0) __syncthreads();  // every wave has finished reading the previous stage
      load_stage(kbase + kstep(kt), 0);
      load_scales(kt0 + kt, sca_cur, scb_cur);
      if (kt == 0) ln_prologue();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (kt == 0) ICAP_STAMP(2, ICAP_NOW());
      frag_t af[KS][TM], bfr[KS][TN];
      read_frags(smem, af, bfr);
      mfmas(af, bfr);
    }
  }

  // ---- split-K combine inside the launch (p.tickets): the splits of a tile take a ticket when their K range is
  // done; every split but the last publishes its fp32 accumulators (write-through sc1 stores, in register order: lane
  // l of wave w stores acc[i][j] at ((w TM TN + i TN + j) 64 + l) 16 bytes of its slot) and counts itself done; the
  // last arriver waits for that count, adds the partials in split order (its own from registers: a fixed order,
  // so the sum is deterministic), resets the tile's two counters for the next launch, and runs the whole epilogue.
  // Nobody waits on a block that has not taken its ticket, so there is no residency assumption
  // (cdna_hip_programming.md §5 "In-launch split-K reduction", §6 Guideline 16 R1 with sc1 loads).
  ICAP_STAMP(3, ICAP_NOW());
  const bool fused = !ROLES && splits > 1 && p.tickets != nullptr;  // (roles: one K range per tile, host rule)
  if (fused) {
    typedef uint32_t u32x4f_t __attribute__((ext_vector_type(4)));
    int* sflag = reinterpret_cast<int*>(smem);
    __syncthreads();  // every wave is done with the stage buffers (NST 1 reads them up to its last MFMA)
    int32_t* cnt = p.tickets + 2 * (int64_t)tile;
    if (tid == 0) sflag[0] = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int order = sflag[0];
    constexpr uint32_t PB = (uint32_t)NW * TM * TN * 64 * 16;  // bytes of one split's partial tile
    char* pbase = reinterpret_cast<char*>(p.workspace) + (int64_t)tile * splits * PB;
    const uint32_t lofs = (uint32_t)((wave * TM * TN * 64 + lane) * 16);
    if (order < splits - 1) {
      const __amdgpu_buffer_rsrc_t rs = make_rsrc(pbase + (int64_t)split * PB, PB);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4f_t, acc[i][j]), rs,
                                                 lofs + (uint32_t)((i * TN + j) * 1024), 0, 16 /* sc1 */);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave: its payload has left
      __syncthreads();
      if (tid == 0) __hip_atomic_fetch_add(cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ICAP_STAMP(0, (uint64_t)split | ((uint64_t)order << 8) | ((uint64_t)tile << 32));
      ICAP_STAMP(4, ICAP_NOW());
      return;
    }
    if (tid == 0) {
      while (__hip_atomic_load(cnt + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < splits - 1)
        __builtin_amdgcn_s_sleep(2);
      if (acq) {  // (bit 30 of nk_split) agent-scope acquire: invalidate this CU's vector L1 / the XCD's stale lines
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      }
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(cnt + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    // Visibility without an agent-scope acquire (MI355X_MICROARCH.md "Valid forms", sc1 hand-off): every payload
    // byte was stored sc1 (write-through, dropped from the producer XCD's L2) and drained (vmcnt(0)) by every storing
    // wave before that block's barrier and its relaxed agent-scope add; every load below is an sc1 buffer load to
    // registers (L1 bypassed), issued after the relaxed poll matched (lane 0) and the barrier above (other waves).
    // A stale copy could only sit in THIS XCD's L2 if something on it had read the slot during this launch before
    // the poll matched: nothing does (a slot is read only by its tile's last arriver, after the poll), and the
    // dispatch of a launch invalidates the L2's copies from earlier launches. The alternative, an agent acquire
    // fence (buffer_inv sc1 + vmcnt(0)), costs the last arriver ~1.7 us (x2 at 2 blocks / CU) on a ~36 us launch;
    // a release add costs every publishing split a buffer_wbl2. tests/test_fused_splitk_gpu.py checks every output
    // word (eager, graph, concurrent streams). If a launch faults, the tickets may be left non-zero: the HIP context
    // is unusable after a device fault anyway; a new process (or re-zeroed tickets) starts clean.
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(pbase, (uint64_t)PB * splits);
    // the other splits' partials, GI accumulator rows at a time (all loads of a group in flight together; one row
    // at 3-4 blocks per CU, whose register budget is 170 / 128)
    constexpr int GI = (MINB >= 3 || TM % 2 != 0) ? 1 : 2;
#pragma unroll
    for (int i0 = 0; i0 < TM; i0 += GI) {
      f32x4_t v[3][GI][TN];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        if (q < splits - 1) {
          const int sq = q < split ? q : q + 1;  // the q-th other split, in split order
#pragma unroll
          for (int ii = 0; ii < GI; ++ii)
#pragma unroll
            for (int j = 0; j < TN; ++j)
              v[q][ii][j] = __builtin_bit_cast(f32x4_t, __builtin_amdgcn_raw_buffer_load_b128(
                  rs, (uint32_t)sq * PB + lofs + (uint32_t)(((i0 + ii) * TN + j) * 1024), 0, 16 /* sc1 */));
        }
      }
#pragma unroll
      for (int ii = 0; ii < GI; ++ii)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const f32x4_t own = acc[i0 + ii][j];
          f32x4_t t = split == 0 ? own : v[0][ii][j];
#pragma unroll
          for (int pos = 1; pos < 4; ++pos) {
            if (pos < splits) {
              const f32x4_t x = pos < split ? v[pos][ii][j] : (pos == split ? own : v[pos - 1][ii][j]);
#pragma unroll
              for (int c = 0; c < 4; ++c) t[c] += x[c];  // per component: no packed-FP32 op
            }
          }
          acc[i0 + ii][j] = t;
        }
    }
  }
  ICAP_STAMP(0, (uint64_t)split | ((uint64_t)(fused ? splits - 1 : 0) << 8) | ((uint64_t)tile << 32));
  ICAP_STAMP(4, ICAP_NOW());
  const bool whole = splits == 1 || fused;  // this block applies the full epilogue (else: its split's slab)

  uint64_t seed = 0;
  if (whole && drop_thresh != 0u) seed = eff_seed(p.seed, p.seed_ptr);
  // split-K partial slab of this split (separate reduce pass): raw fp32 [M, N] (N % 4 == 0 is guaranteed by the host)
  float* slab = !whole ? reinterpret_cast<float*>(p.workspace) + (int64_t)split * M * N : nullptr;

  // ---- LDS-staged epilogue: each wave re-reads its accumulators EW = 8 consecutive columns per lane, so every
  // global access of the epilogue is 16 bytes (bf16) — the store tail is issue-bound (cdna_hip_programming.md T21)
  // ROLES: both waves of a SIMD store the tile of its MFMA wave (ew), which stages its accumulators; the rows of
  // even / odd t go to the MFMA / loader wave (half), so the epilogue's VALU and stores run on twice the waves
  // (8 MFMA waves: each stores its own tile, the loader waves only pass the barriers)
  constexpr int NHALF = (ROLES && NW == 4) ? 2 : 1;
  const int ew = NHALF == 2 ? (wave & (NW - 1)) : wave;
  const int ewm = ew / WN, ewn = ew - ewm * WN;
  const int half = NHALF == 2 ? wave / NW : 0;
  const bool stager = !ROLES || wave < NW;
  const bool storer = !ROLES || NHALF == 2 || wave < NW;
  float* cs = reinterpret_cast<float*>(smem) + ew * (EPR * ELD);
  constexpr int EW = 8;
  constexpr int LPR = 16 * TN / EW;  // lanes per staged row (EW columns each)
  constexpr int RPI = 64 / LPR;     // rows per wave instruction
  const int er = lane / LPR;
  const int ec = (lane - er * LPR) * EW;
  const int64_t col = n0 + ewn * 16 * TN + ec;
  const bool fullw = col + EW <= N;
  float biasw[EW];
#pragma unroll
  for (int e = 0; e < EW; ++e) biasw[e] = 0.f;
  if (whole && p.bias && p.dact == ICAP_ACT_NONE) {
#pragma unroll
    for (int e = 0; e < EW; ++e) biasw[e] = (col + e < N) ? p.bias[col + e] : 0.f;
  }
  // Prefetch of the epilogue's input operand (bf16 C: dact_src in the backward form, resid in the forward form):
  // the rows this lane stores, issued before the LDS staging (all of them, or in two halves at 4 blocks/CU) so one
  // memory latency is exposed per group instead of one dependent round trip per staged row pair (on the N = 768
  // launches a CU holds 1-2 tiles, so nothing else hides it). Out-of-range rows read row Mv-1 (no branch per
  // load: cdna_hip_programming.md §5 trap (c)) and are never stored.
  constexpr int NH = 16 * TM / EPR;              // staging passes
  // prefetch groups: half the rows at a time at 128 VGPRs; ROLES (round 6): at most 4 rows per wave at a time —
  // the 128 x 256 / 192 x 256 tiles held 8 / 12 and the compiler demoted the array to scratch, each load then waited
  // for its own round trip before its scratch store (192 x 256 dgelu epilogue: 22.7 us)
  constexpr int NPG = ROLES ? roles_prefetch_groups(NH, EPR / RPI, NHALF) : (MINB >= 4 && NH >= 2 ? 2 : 1);
  constexpr int HPG = NH / NPG;                  // passes per prefetch group
  constexpr int NEP = HPG * (EPR / RPI);         // prefetched rows of a group (this wave: NEP / NHALF of them)
  typedef typename rawbf<EW>::T pre_t;
  static_assert(NHALF == 1 || (EPR / RPI) % NHALF == 0, "roles: a wave's prefetched rows alternate");
  pre_t pre[NEP / NHALF];  // (roles, NHALF = 2: row i of the group is this wave's when i % 2 == half, held at i / 2)
  bool want_pre = false;  // block-uniform: this launch has a bf16 dact_src / resid operand
  const bf16_t* esrc = nullptr;
  int64_t eld = 0;
  const int64_t rb = m0 + ewm * 16 * TM + er;  // row of (pass h, row t) = rb + h EPR + t RPI
  auto prefetch = [&](auto gc) __attribute__((always_inline)) {  // rows of passes [g HPG, g HPG + HPG)
    constexpr int g = decltype(gc)::value;
    if (want_pre && fullw && storer) {
#pragma unroll
      for (int i = 0; i < NEP; ++i) {
        if (NHALF > 1 && (i % (EPR / RPI)) % NHALF != half) continue;  // (roles: the other wave's rows)
        const int64_t r0 = rb + (int64_t)(g * NEP + i) * RPI;
        const int64_t row = r0 < Mv ? r0 : Mv - 1;
        pre[i / NHALF] = *reinterpret_cast<const pre_t*>(esrc + row * eld + col);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the loads here: hipcc would sink each to its use
  };
  if constexpr (std::is_same<TC, bf16_t>::value) {
    if (whole) {
      if (AK >= ACT_BWD || (AK == ACT_ANY && p.dact != ICAP_ACT_NONE)) {
        esrc = reinterpret_cast<const bf16_t*>(p.dact_src);
        eld = p.ld_dact;
      } else if (p.resid) {
        esrc = reinterpret_cast<const bf16_t*>(p.resid);
        eld = p.ldr;
      }
    }
    want_pre = esrc != nullptr && (eld % EW) == 0 && (reinterpret_cast<uintptr_t>(esrc) & 15) == 0 &&
               (p.ldc % EW) == 0 && (reinterpret_cast<uintptr_t>(p.C) & 15) == 0;
    prefetch(std::integral_constant<int, 0>{});
  }
  // the consumer's epilogue factor: wsum of W gamma per output column (its row table came from the prologue)
  float wsumw[EW];
  if constexpr (LNX == 2) {
#pragma unroll
    for (int e = 0; e < EW; ++e) wsumw[e] = (col + e < N) ? p.ln_wsum[col + e] : 0.f;
  }
  if (NST == 1) __syncthreads();  // the single stage buffer is still being read by other waves
  // rows [EPR h, EPR h + EPR) of this wave's accumulator tile -> LDS (h compile-time: it indexes acc[])
  auto stage_rows = [&](auto hc) __attribute__((always_inline)) {
    constexpr int h = decltype(hc)::value;
#pragma unroll
    for (int ii = 0; ii < EPR / 16; ++ii)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v)
          cs[(ii * 16 + fg * 4 + v) * ELD + j * 16 + fr] = acc[(EPR / 16) * h + ii][j][v];
  };
  auto store_row = [&](int h, int t, const pre_t* pq) __attribute__((always_inline)) {
    const int lr = t * RPI + er;  // 0..EPR-1
    const int64_t row = m0 + ewm * 16 * TM + h * EPR + lr;
    float x[EW];
#pragma unroll
    for (int q = 0; q < EW / 4; ++q)
      *reinterpret_cast<float4*>(x + 4 * q) = *reinterpret_cast<const float4*>(cs + lr * ELD + ec + 4 * q);
    const bool ok = row < Mv && col < N;
    if constexpr (LNX == 2) {  // rstd (A.B^T - mean wsum); the host passed bias = b + W . beta
      const int br = ewm * 16 * TM + h * EPR + lr;
      const float mean = lnr[2 * br], rs = lnr[2 * br + 1];
#pragma unroll
      for (int e = 0; e < EW; ++e) x[e] = rs * (x[e] - mean * wsumw[e]);
    }
    if (ok) {
      if (slab) {  // N % 4 == 0 (host check): whole float4 pieces
#pragma unroll
        for (int q = 0; q < EW / 4; ++q)
          if (col + 4 * q < N)
            *reinterpret_cast<float4*>(slab + row * N + col + 4 * q) = *reinterpret_cast<const float4*>(x + 4 * q);
      } else {
        epiw<TC, EW, AK>(p, row, col, x, biasw, fullw, seed, drop_thresh, inv_keep, pq);
      }
    }
    if constexpr (LNX == 1) {
      // producer: (mean, M2) of the STORED (rounded) values over this row's 32-column group = 4 lanes x EW
      // (every lane runs the shuffles; rows / columns out of range count as zeros and are not written)
      float xr[EW], sm = 0.f;
#pragma unroll
      for (int e = 0; e < EW; ++e) {
        xr[e] = ok ? bf2f(f2bf(x[e])) : 0.f;
        sm += xr[e];
      }
      sm += __shfl_xor(sm, 1, 64);
      sm += __shfl_xor(sm, 2, 64);
      const float mg = sm * (1.f / 32.f);
      float q2 = 0.f;
#pragma unroll
      for (int e = 0; e < EW; ++e) {
        const float d = xr[e] - mg;
        q2 += d * d;
      }
      q2 += __shfl_xor(q2, 1, 64);
      q2 += __shfl_xor(q2, 2, 64);
      if (ok && (lane & 3) == 0)
        reinterpret_cast<float2*>(p.ln_stats_out)[row * (N >> 5) + (col >> 5)] = make_float2(mg, q2);
    }
  };
  if (want_pre || MINB >= 4) {  // (at 4 blocks/CU one path: a second one made the 128-VGPR build spill)
    // passes h / rows t as compile-time indices (static_for) so pre[] stays in registers (the unroller refuses
    // a full unroll of this body by size); a separate path, so launches without the operand keep the compact
    // loop below (the fully unrolled copy cost the plain launches 5-15 % in instruction fetch)
    static_for<0, NH>([&](auto hc) {
      constexpr int h = decltype(hc)::value;
      if constexpr (h > 0 && h % HPG == 0) prefetch(std::integral_constant<int, h / HPG>{});
      if (stager) stage_rows(hc);
      __syncthreads();
      static_for<0, EPR / RPI>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        if ((NHALF == 1 || t % NHALF == half) && storer)
          store_row(h, t, (want_pre && fullw) ? &pre[((h % HPG) * (EPR / RPI) + t) / NHALF] : nullptr);
      });
      __syncthreads();
    });
  } else {
    static_for<0, NH>([&](auto hc) {  // h compile-time: acc[] is indexed by it
      constexpr int h = decltype(hc)::value;
      if (stager) stage_rows(hc);
      __syncthreads();
      if (storer) {
#pragma unroll 2
        for (int t = half; t < EPR / RPI; t += NHALF) store_row(h, t, nullptr);
      }
      __syncthreads();
    });
  }
  ICAP_STAMP(5, ICAP_NOW());
}

template <typename TI, typename TC, int NST, int MINB, int WM, int WN, int TM, int TN, bool KOUT = false, int ACT = ACT_ANY,
          bool ROLES = false>
// (hip-clang reads launch_bounds' second argument as waves per SIMD: MINB blocks of NWT waves per CU is MINB NWT / 4
// rounded up — for the 4-wave blocks the same number)
__global__ __launch_bounds__(64 * (WM * WN + (ROLES ? 4 : 0)), (MINB * (WM * WN + (ROLES ? 4 : 0)) + 3) / 4) void gemm_kernel(icap_gemm_args p, int tiles_n, int splits,
                                                                  int nk_split, uint32_t drop_thresh, float inv_keep) {
  const int64_t Mv = p.m_dev && (int64_t)*p.m_dev < p.M ? (int64_t)*p.m_dev : p.M;  // device row count
  if constexpr (ROLES) {
    // a grid of at most one block per CU walks the live tiles (host: grid = min(tiles, CUs)): with the capacity grid
    // of the packed step (65 row tiles for 28 live ones) the dead blocks — 147 KiB of LDS each, so never co-resident
    // with a live one — were dispatched only as the live ones finished and delayed the launch's end
    // (K-outer: split-K over slabs, the blocks of every split walked the same way; the reduce pass follows)
    constexpr int BM = 16 * WM * TM;
    const int tiles_m = (int)((p.M + BM - 1) / BM);
    const int nlive = (int)((Mv + BM - 1) / BM) * tiles_n * splits;
    for (int b = blockIdx.x; b < nlive; b += gridDim.x)
      gemm_body<TI, TC, NST, MINB, WM, WN, TM, TN, KOUT, ACT, ROLES>(p, tiles_n, splits, nk_split, drop_thresh, inv_keep,
                                                                       b, tiles_m, Mv);
  } else {
    gemm_body<TI, TC, NST, MINB, WM, WN, TM, TN, KOUT, ACT, ROLES>(p, tiles_n, splits, nk_split, drop_thresh, inv_keep,
                                                                     blockIdx.x, (int)(gridDim.x / splits) / tiles_n, Mv);
  }
}

}  // namespace icap

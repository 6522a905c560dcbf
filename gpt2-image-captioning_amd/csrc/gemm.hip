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
#include "gemm_common.h"

namespace icap {

// ---- K-outer operand images (trans_ab): [64 k-rows][128 columns] bf16, 256-byte rows, 16-byte chunk ch of row r
// stored at chunk ch ^ kout_swz(r) (cdna_hip_programming.md T10 layout (b)) so the transposed reads below are
// at most 2-way bank conflicted.
__device__ __forceinline__ int kout_swz(int r) { return ((r & 3) << 2) | ((r >> 2) & 3); }
__device__ __forceinline__ int kout_off(int r, int ch) { return r * 256 + ((ch ^ kout_swz(r)) << 4); }
typedef short kv4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) kv4s_t* kout_lds_ptr;
// MFMA 16x16x32 operand (lane: column c0 + (lane & 15)) over k-rows r0..r0+31 of a K-outer image, as two
// ds_read_b64_tr_b16: lane 4q+p of 16-lane group g addresses row r0 + 4g + q (then + 16), columns 4p..4p+3 of
// the 16-column block; element j of the result = k-row r0 + 4g + j (j < 4), r0 + 16 + 4g + j - 4 (j >= 4)
__device__ __forceinline__ uint4 kout_frag(const char* img, int r0, int c0, int lane) {
  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  const int ch = (c0 >> 3) + (pp >> 1), half = (pp & 1) * 8;
  const char* a0 = img + kout_off(r0 + 4 * g + q, ch) + half;
  const char* a1 = img + kout_off(r0 + 16 + 4 * g + q, ch) + half;
  const kv4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((kout_lds_ptr)(a0));
  const kv4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((kout_lds_ptr)(a1));
  uint4 r;
  r.x = (uint32_t)(uint16_t)lo[0] | ((uint32_t)(uint16_t)lo[1] << 16);
  r.y = (uint32_t)(uint16_t)lo[2] | ((uint32_t)(uint16_t)lo[3] << 16);
  r.z = (uint32_t)(uint16_t)hi[0] | ((uint32_t)(uint16_t)hi[1] << 16);
  r.w = (uint32_t)(uint16_t)hi[2] | ((uint32_t)(uint16_t)hi[3] << 16);
  return r;
}

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
// swizzle on the source address; fragments come from ds_read_b64_tr_b16 pairs (k order {4g..4g+3, 16+4g..},
// the same on both operands, so the contraction is unchanged). bf16 inputs, 128 x 128 tiles only.
// ACT: false for launches with no activation (act == dact == NONE: most of the step's products): the epilogue's
// activation code is then not compiled into the kernel at all. Measured (profiles/r03_k768_counters.txt): with it
// present, the plain 8320 x 2304 x 768 product ran 53.7 vs 45.0 us — the same memory instructions, +7 % VALU and
// +22 % SQ_WAIT_ANY (the larger function scheduled its main loop worse), SQ_WAIT_INST_ANY +1 % (not instruction fetch).
template <typename TI, typename TC, int NST, int MINB, int WM, int WN, int TM, int TN, bool KOUT = false, int ACT = ACT_ANY>
__global__ __launch_bounds__(64 * WM * WN, MINB) void gemm_kernel(icap_gemm_args p, int tiles_n, int splits,
                                                                  int nk_split, uint32_t drop_thresh, float inv_keep) {
  static_assert(!KOUT || (sizeof(TI) == 2 && 16 * WM * TM == 128 && 16 * WN * TN == 128),
                "K-outer operands: bf16, 128 x 128 tiles");
  // MX block-scaled fp8 (TI = fp8_t): a stage's 128-byte LDS row is one 128-deep K step of
  // v_mfma_scale_f32_16x16x128_f8f6f4 (twice the bf16 flops per staged byte and per fragment byte read); the
  // per-32 E8M0 scales of the wave's 4 fragment rows of A and of B come in one 16-byte load each per stage
  constexpr bool MX = sizeof(TI) == 1;
  static_assert(!MX || (!KOUT && TM == 4 && TN == 4 && WM == 2 && WN == 2), "MX fp8: 128 x 128 tiles of 4 waves");
  constexpr int NW = WM * WN;
  constexpr int BM = 16 * WM * TM, BN = 16 * WN * TN;
  constexpr int STB = (BM + BN) * GROWB;    // bytes per stage
  constexpr int EPR = NST >= 2 ? 32 : 16;   // rows per LDS-staged epilogue pass
  constexpr int ELD = 16 * TN + 4;          // fp32 row stride of the epilogue staging tile
  static_assert(NW * EPR * ELD * 4 <= NST * STB, "epilogue staging must fit the stage buffers");
  static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0, "each wave stages whole 8-row DMA pieces");
  constexpr int APW = BM / (8 * NW), BPW = BN / (8 * NW);  // DMA instructions per wave per stage
  __shared__ __attribute__((aligned(16))) char smem[NST * STB];
  constexpr int ES = sizeof(TI);
  constexpr int EPC = 16 / ES;         // elements per 16-byte chunk
  constexpr int BKE = GROWB / ES;      // K elements per stage

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WN, wn = wave - wm * WN;

  const int64_t M = p.M, N = p.N, K = p.K;
  const int64_t Mv = p.m_dev && (int64_t)*p.m_dev < M ? (int64_t)*p.m_dev : M;  // device row count
  // bijective XCD-aware remap over the LIVE blocks: blocks sharing an XCD get consecutive tiles (consecutive
  // tiles share the A row panel). With a device row count the grid is sized for M but only the first
  // nlive = (row tiles of Mv) x tiles_n x splits blocks work: they are the lowest block ids, which the dispatcher
  // hands out first and round-robin over the XCDs, so the live tiles land one per CU before any CU takes a second
  // (the dead blocks exit at once), and the remap over nlive keeps every XCD's share contiguous.
  const int bid = blockIdx.x;
  const int tiles_m = (int)(gridDim.x / splits) / tiles_n;
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

  if constexpr (NST == 4) {
    // Deep ring for launches with about one tile per CU and long K (the packed step's N = 768 products): 4 LDS
    // stages (128 KiB, one block per CU), stages kt+1..kt+2 in flight while stage kt is read and stage kt+3 is
    // issued, so three DMA round trips overlap each stage's MFMAs (the double-buffered loop leaves one: at one block
    // per CU it waited ~0.6 of every k-step on the DMA). The fragment reads are inline asm (hipcc would otherwise
    // drain the DMA queue, vmcnt(0), in front of every LDS read), retired by counted lgkmcnt waits tied to their
    // registers; the DMA waits are counted vmcnt (never 0 in the steady state) and the barriers raw s_barrier
    // (cdna_hip_programming.md "Pipelining across barriers", T3+T4).
    //   RAW: stage kt is read after this wave's vmcnt wait for it and a barrier every wave passed after its own.
    //   WAR: stage kt+3 is written into the slot read in iteration kt-1, whose reads every wave retired (lgkmcnt)
    //        before that iteration's MFMAs, i.e. before the barrier of iteration kt.
    static_assert(!KOUT && !MX && sizeof(TI) == 2 && TM == 4 && TN == 4 && APW + BPW == 8,
                  "ring: bf16 row-major operands, 128 x 128 tiles of 4 waves");
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
    for (int s = 0; s < 3; ++s)
      if (s < nk) load_stage(kbase + kstep(s), s);
#define ICAP_RING_RD(dst, addr, off) asm volatile("ds_read_b128 %0, %1 offset:" #off : "=v"(dst) : "v"(addr))
    for (int kt = 0; kt < nk; ++kt) {
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 2 < nk) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");      // stages kt+1, kt+2 stay in flight
      else if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 3 < nk) load_stage(kbase + kstep(kt + 3), (kt + 3) & 3);
      __builtin_amdgcn_sched_barrier(0);
      const uint32_t sb = sbase + (uint32_t)((kt & 3) * STB);
      u32x4_t fa0[4], fb0[4], fa1[4], fb1[4];
      {
        const uint32_t a0 = sb + la[0], b0 = sb + lb[0], a1 = sb + la[1], b1 = sb + lb[1];
        ICAP_RING_RD(fa0[0], a0, 0); ICAP_RING_RD(fa0[1], a0, 2048); ICAP_RING_RD(fa0[2], a0, 4096); ICAP_RING_RD(fa0[3], a0, 6144);
        ICAP_RING_RD(fb0[0], b0, 0); ICAP_RING_RD(fb0[1], b0, 2048); ICAP_RING_RD(fb0[2], b0, 4096); ICAP_RING_RD(fb0[3], b0, 6144);
        ICAP_RING_RD(fa1[0], a1, 0); ICAP_RING_RD(fa1[1], a1, 2048); ICAP_RING_RD(fa1[2], a1, 4096); ICAP_RING_RD(fa1[3], a1, 6144);
        ICAP_RING_RD(fb1[0], b1, 0); ICAP_RING_RD(fb1[1], b1, 2048); ICAP_RING_RD(fb1[2], b1, 4096); ICAP_RING_RD(fb1[3], b1, 6144);
      }
      asm volatile("s_waitcnt lgkmcnt(8)"
                   : "+v"(fa0[0]), "+v"(fa0[1]), "+v"(fa0[2]), "+v"(fa0[3]), "+v"(fb0[0]), "+v"(fb0[1]), "+v"(fb0[2]),
                     "+v"(fb0[3]));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          mfma_chunk<TI>(acc[i][j], __builtin_bit_cast(uint4, fa0[i]), __builtin_bit_cast(uint4, fb0[j]));
      asm volatile("s_waitcnt lgkmcnt(0)"
                   : "+v"(fa1[0]), "+v"(fa1[1]), "+v"(fa1[2]), "+v"(fa1[3]), "+v"(fb1[0]), "+v"(fb1[1]), "+v"(fb1[2]),
                     "+v"(fb1[3]));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          mfma_chunk<TI>(acc[i][j], __builtin_bit_cast(uint4, fa1[i]), __builtin_bit_cast(uint4, fb1[j]));
    }
#undef ICAP_RING_RD
    __builtin_amdgcn_sched_barrier(0);
    __syncthreads();  // (no DMA outstanding) every wave is done reading the ring before the epilogue reuses it
  } else if (NST == 2) {
    load_stage(kbase + kstep(0), 0);
    load_scales(kt0, sca_cur, scb_cur);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
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
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
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
  const bool fused = splits > 1 && p.tickets != nullptr;
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
      return;
    }
    if (tid == 0) {
      while (__hip_atomic_load(cnt + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < splits - 1)
        __builtin_amdgcn_s_sleep(2);
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
    constexpr int GI = MINB >= 3 ? 1 : 2;
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
              t += x;
            }
          }
          acc[i0 + ii][j] = t;
        }
    }
  }
  const bool whole = splits == 1 || fused;  // this block applies the full epilogue

  uint64_t seed = 0;
  if (whole && drop_thresh != 0u) seed = eff_seed(p.seed, p.seed_ptr);
  // split-K partial slab of this split (separate reduce pass): raw fp32 [M, N] (N % 4 == 0 is guaranteed by the host)
  float* slab = !whole ? reinterpret_cast<float*>(p.workspace) + (int64_t)split * M * N : nullptr;

  // ---- LDS-staged epilogue: each wave re-reads its accumulators EW = 8 consecutive columns per lane, so every
  // global access of the epilogue is 16 bytes (bf16) — the store tail is issue-bound (cdna_hip_programming.md T21)
  float* cs = reinterpret_cast<float*>(smem) + wave * (EPR * ELD);
  constexpr int EW = 8;
  constexpr int LPR = 16 * TN / EW;  // lanes per staged row (EW columns each)
  constexpr int RPI = 64 / LPR;     // rows per wave instruction
  const int er = lane / LPR;
  const int ec = (lane - er * LPR) * EW;
  const int64_t col = n0 + wn * 16 * TN + ec;
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
  constexpr int NPG = MINB >= 4 && NH >= 2 ? 2 : 1;  // prefetch groups: half the rows at a time at 128 VGPRs
  constexpr int HPG = NH / NPG;                  // passes per prefetch group
  constexpr int NEP = HPG * (EPR / RPI);         // prefetched rows held at once
  typedef typename rawbf<EW>::T pre_t;
  pre_t pre[NEP];
  bool want_pre = false;  // block-uniform: this launch has a bf16 dact_src / resid operand
  const bf16_t* esrc = nullptr;
  int64_t eld = 0;
  const int64_t rb = m0 + wm * 16 * TM + er;  // row of (pass h, row t) = rb + h EPR + t RPI
  auto prefetch = [&](auto gc) __attribute__((always_inline)) {  // rows of passes [g HPG, g HPG + HPG)
    constexpr int g = decltype(gc)::value;
    if (want_pre && fullw) {
#pragma unroll
      for (int i = 0; i < NEP; ++i) {
        const int64_t r0 = rb + (int64_t)(g * NEP + i) * RPI;
        const int64_t row = r0 < Mv ? r0 : Mv - 1;
        pre[i] = *reinterpret_cast<const pre_t*>(esrc + row * eld + col);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the loads here: hipcc would sink each to its use
  };
  if constexpr (std::is_same<TC, bf16_t>::value) {
    if (whole) {
      if (ACT >= ACT_BWD || (ACT == ACT_ANY && p.dact != ICAP_ACT_NONE)) {
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
    const int64_t row = m0 + wm * 16 * TM + h * EPR + lr;
    float x[EW];
#pragma unroll
    for (int q = 0; q < EW / 4; ++q)
      *reinterpret_cast<float4*>(x + 4 * q) = *reinterpret_cast<const float4*>(cs + lr * ELD + ec + 4 * q);
    if (row < Mv && col < N) {
      if (slab) {  // N % 4 == 0 (host check): whole float4 pieces
#pragma unroll
        for (int q = 0; q < EW / 4; ++q)
          if (col + 4 * q < N)
            *reinterpret_cast<float4*>(slab + row * N + col + 4 * q) = *reinterpret_cast<const float4*>(x + 4 * q);
      } else {
        epiw<TC, EW, ACT>(p, row, col, x, biasw, fullw, seed, drop_thresh, inv_keep, pq);
      }
    }
  };
  if (want_pre || MINB >= 4) {  // (at 4 blocks/CU one path: a second one made the 128-VGPR build spill)
    // passes h / rows t as compile-time indices (static_for) so pre[] stays in registers (the unroller refuses
    // a full unroll of this body by size); a separate path, so launches without the operand keep the compact
    // loop below (the fully unrolled copy cost the plain launches 5-15 % in instruction fetch)
    static_for<0, NH>([&](auto hc) {
      constexpr int h = decltype(hc)::value;
      if constexpr (h > 0 && h % HPG == 0) prefetch(std::integral_constant<int, h / HPG>{});
      stage_rows(hc);
      __syncthreads();
      static_for<0, EPR / RPI>([&](auto tc) {
        constexpr int t = decltype(tc)::value;
        store_row(h, t, (want_pre && fullw) ? &pre[(h % HPG) * (EPR / RPI) + t] : nullptr);
      });
      __syncthreads();
    });
  } else {
    static_for<0, NH>([&](auto hc) {  // h compile-time: acc[] is indexed by it
      constexpr int h = decltype(hc)::value;
      stage_rows(hc);
      __syncthreads();
#pragma unroll 2
      for (int t = 0; t < EPR / RPI; ++t) store_row(h, t, nullptr);
      __syncthreads();
    });
  }
}

// Skinny-M GEMM (M <= 128: greedy-decode steps over the batch, CLIP projection, mapper input Linear).
// A weight-streaming, latency-bound problem: block = 8 waves over a 16*NT-column slab of B (= W rows) and a
// 16*MT-row slab of A (grid.y walks M, so no block streams all of A through its CU: per-CU L2 bandwidth, not
// HBM, bounded the all-rows form); the waves split the K steps round-robin and keep SK_U steps of MFMA
// fragments in flight each (range-checked buffer loads straight from HBM/L2). The fp32 partial tiles are reduced
// through LDS in two rounds before the shared epilogue. One launch, no slabs.
// Accumulators use the C layout (lane = column, 4 consecutive rows per lane).
// one 16-byte A chunk -> LayerNorm-ed chunk in the input dtype
template <typename TI>
__device__ __forceinline__ uint4 ln_chunk(const uint4 a, float mean, float rs, const float* g, const float* bt);
template <>
__device__ __forceinline__ uint4 ln_chunk<bf16_t>(const uint4 a, float mean, float rs, const float* g, const float* bt) {
  const uint32_t w[4] = {a.x, a.y, a.z, a.w};
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float v0 = (__uint_as_float(w[q] << 16) - mean) * rs * g[2 * q] + bt[2 * q];
    const float v1 = (__uint_as_float(w[q] & 0xffff0000u) - mean) * rs * g[2 * q + 1] + bt[2 * q + 1];
    o[q] = f2bf2(v0, v1);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}
template <>
__device__ __forceinline__ uint4 ln_chunk<float>(const uint4 a, float mean, float rs, const float* g, const float* bt) {
  return make_uint4(__float_as_uint((__uint_as_float(a.x) - mean) * rs * g[0] + bt[0]),
                    __float_as_uint((__uint_as_float(a.y) - mean) * rs * g[1] + bt[1]),
                    __float_as_uint((__uint_as_float(a.z) - mean) * rs * g[2] + bt[2]),
                    __float_as_uint((__uint_as_float(a.w) - mean) * rs * g[3] + bt[3]));
}

constexpr int SK_WAVES = 8;
constexpr int SK_LNK = 1280;  // LN-fused launches up to this K stage gamma / beta in LDS
// NT: 16-column slabs per block (the host picks the fewest that fit the grid in one pass over the CUs);
// SKU: k-steps in flight per wave (the host picks enough for one memory round trip over all of K where the
// registers allow). Neither changes the arithmetic: every wave accumulates its steps in step order and the waves
// are summed in a fixed order, so all (NT, SKU) instantiations store bitwise-identical outputs.
template <typename TI, typename TC, int NT, int MT, int SKU>
__global__ __launch_bounds__(64 * SK_WAVES) void gemm_skinny_kernel(icap_gemm_args p, uint32_t drop_thresh,
                                                                  float inv_keep) {
  constexpr int ES = sizeof(TI);
  constexpr int EPC = 16 / ES;        // K elements per lane chunk
  constexpr int KSTEP = 4 * EPC;      // K elements per MFMA chunk step (4 lane groups)
  constexpr int BN = 16 * NT;
  constexpr int RLD = BN + 4;         // fp32 stride of the LDS partial tiles
  constexpr int HALF = SK_WAVES / 2;
  constexpr int BM = 16 * MT;
  constexpr int QPR = BN / 4;         // 4-column epilogue quads per row
  static_assert(BM * QPR <= 64 * SK_WAVES, "one epilogue quad per thread");
  __shared__ __attribute__((aligned(16))) float red[HALF][BM * RLD];
  __shared__ __attribute__((aligned(16))) float lngb[2 * SK_LNK];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t N = p.N, K = p.K;
  const int64_t n0 = (int64_t)blockIdx.x * BN, m0 = (int64_t)blockIdx.y * BM;
  const int64_t M = p.m_dev && (int64_t)*p.m_dev < p.M ? (int64_t)*p.m_dev : p.M;  // device row count
  if (m0 >= M) return;
  const int64_t nrows = N - n0 < BN ? N - n0 : BN;
  const int64_t mrows = M - m0 < BM ? M - m0 : BM;
  const __amdgpu_buffer_rsrc_t ra =
      make_rsrc(reinterpret_cast<const char*>(p.A) + m0 * p.lda * ES, (uint64_t)((mrows - 1) * p.lda + K) * ES);
  const __amdgpu_buffer_rsrc_t rb =
      make_rsrc(reinterpret_cast<const char*>(p.B) + n0 * p.ldb * ES, (uint64_t)((nrows - 1) * p.ldb + K) * ES);
  f32x4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  // rows past M / N lie beyond the descriptor range (zero-filled); K-tail chunks and steps past the end are
  // redirected out of range (zero fragments: the MFMAs on them add nothing)
  uint32_t aoff[MT], boff[NT];
#pragma unroll
  for (int i = 0; i < MT; ++i) aoff[i] = (uint32_t)(((i * 16 + fr) * p.lda + fg * EPC) * ES);
#pragma unroll
  for (int j = 0; j < NT; ++j) boff[j] = (uint32_t)(((j * 16 + fr) * p.ldb + fg * EPC) * ES);
  const int64_t nks = (K + KSTEP - 1) / KSTEP;
  uint4 af[SKU][MT], bfr[SKU][NT];
  auto load_steps = [&](int64_t base) {  // steps past the end load zero fragments (the MFMAs add nothing)
#pragma unroll
    for (int u = 0; u < SKU; ++u) {
      const int64_t k0 = (base + (int64_t)u * SK_WAVES) * KSTEP;
      const bool kin = k0 + fg * EPC < K;
      const uint32_t kb = (uint32_t)(k0 * ES);
#pragma unroll
      for (int j = 0; j < NT; ++j) bfr[u][j] = bload(rb, kin ? boff[j] + kb : OOB);
#pragma unroll
      for (int i = 0; i < MT; ++i) af[u][i] = bload(ra, kin ? aoff[i] + kb : OOB);
    }
  };
  // LN gamma / beta (K <= SK_LNK) are loaded first, so storing them to LDS waits for these loads only, not for
  // the fragment loads behind them
  const bool fuse_ln = p.ln_gamma != nullptr;
  const bool ln_lds = fuse_ln && K <= SK_LNK;
  constexpr int LNS = (SK_LNK + 64 * SK_WAVES - 1) / (64 * SK_WAVES);  // gamma (and beta) values per thread
  float lg[LNS], lb[LNS];
  if (ln_lds) {
#pragma unroll
    for (int q = 0; q < LNS; ++q) {
      const int k = threadIdx.x + q * 64 * SK_WAVES;
      lg[q] = k < K ? p.ln_gamma[k] : 0.f;
      lb[q] = k < K ? p.ln_beta[k] : 0.f;
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  // every wave runs at least one (possibly all-zero) pass, so the LN-stats barrier below is block-uniform
  load_steps(wave);
  __builtin_amdgcn_sched_barrier(0);
  if (ln_lds) {
#pragma unroll
    for (int q = 0; q < LNS; ++q) {
      const int k = threadIdx.x + q * 64 * SK_WAVES;
      if (k < K) {
        lngb[k] = lg[q];
        lngb[SK_LNK + k] = lb[q];
      }
    }
  }

  // Epilogue operands, fetched now so their latency hides under the main loop's: one 4-column quad per thread
  // (bias; the bf16 residual, or dact_src in the backward form, for full quads).
  const int er = threadIdx.x / QPR, ec = (threadIdx.x - er * QPR) * 4;
  const int64_t erow = m0 + er, ecol = n0 + ec;
  const bool eact = threadIdx.x < BM * QPR && erow < M && ecol < N;
  float bias4[4] = {0.f, 0.f, 0.f, 0.f};
  uint2 pre = make_uint2(0u, 0u);
  bool use_pre = false;
  if (eact) {
    if (p.bias && p.dact == ICAP_ACT_NONE) {
#pragma unroll
      for (int e = 0; e < 4; ++e) bias4[e] = (ecol + e < N) ? p.bias[ecol + e] : 0.f;
    }
    if constexpr (sizeof(TC) == 2) {
      const bf16_t* src = reinterpret_cast<const bf16_t*>(p.dact != ICAP_ACT_NONE ? p.dact_src : p.resid);
      const int64_t lds_ = p.dact != ICAP_ACT_NONE ? p.ld_dact : p.ldr;
      if (src && ecol + 4 <= N && (lds_ & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 7) == 0) {
        pre = *reinterpret_cast<const uint2*>(src + erow * lds_ + ecol);
        use_pre = true;
      }
    }
  }

  // LayerNorm-fused A (icap_gemm_args.ln_gamma): mean / rstd of the block's rows over all K (two passes: mean,
  // then the centred sum of squares), then (x - mean) * rstd * gamma + beta -> input dtype per fragment.
  // bf16 with every k-step in registers (nks <= 8 SKU, the decode launches): the statistics come from the
  // fragments themselves (lane sums -> the 4 lane groups -> the 8 waves through LDS, fixed order), so LN costs no
  // extra global reads; otherwise the loop form (16 threads per row, the order and rounding of ln_fwd8_kernel).
  // gamma / beta are staged in LDS when K <= SK_LNK (above); the barriers below publish them.
  __shared__ float ln_mr[BM][2];
  __shared__ float lnp[SK_WAVES][BM];
  __shared__ float lnp2[SK_WAVES][BM];
  // (instantiations with few fragment registers only: the others would spill; LN-fused launches have K = D)
  constexpr bool LN_FRAG = ES == 2 && SKU * (MT + NT) <= 24;
  // folded LayerNorm (icap_gemm_args.ln_wsum): the same row statistics, but only the epilogue needs them
  // (C = rstd (A.B^T - mean wsum) + bias), so the MFMAs run on the raw fragments without waiting for them: the
  // wave partials go to LDS here and are summed by the epilogue threads after the partial-tile reduction barrier
  const bool fold = p.ln_wsum != nullptr;
  const bool ln_frag = LN_FRAG && (fuse_ln || fold) && nks <= (int64_t)SK_WAVES * SKU;
  float ln_mean[MT], ln_rs[MT];
  if (LN_FRAG && ln_frag) {
    // one pass over the fragments: per-row sums of (x - x0) and (x - x0)^2 with x0 the row's first element (the
    // shifted-data form: no cancellation between E[x^2] and mean^2 when |mean| >> std), reduced together (lane
    // groups by shuffles, the 8 waves through LDS in a fixed order); mean = x0 + E[d], var = E[d^2] - E[d]^2
    auto chunk_in = [&](int u) { return (int64_t)(wave + u * SK_WAVES) * KSTEP + fg * EPC < K; };
    float part[MT], part2[MT], x0[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v0[8];
      unpack_bf16(bload(ra, (uint32_t)((i * 16 + fr) * p.lda * ES)), v0);  // rows past M: zero
      x0[i] = v0[0];
      part[i] = 0.f;
      part2[i] = 0.f;
#pragma unroll
      for (int u = 0; u < SKU; ++u) {
        if (chunk_in(u)) {
          const int64_t kc = (int64_t)(wave + u * SK_WAVES) * KSTEP + fg * EPC;
          float v[8];
          unpack_bf16(af[u][i], v);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = kc + e < K ? v[e] - x0[i] : 0.f;
            part[i] += d;
            part2[i] += d * d;
          }
        }
      }
      part[i] += __shfl_xor(part[i], 16, 64);
      part[i] += __shfl_xor(part[i], 32, 64);
      part2[i] += __shfl_xor(part2[i], 16, 64);
      part2[i] += __shfl_xor(part2[i], 32, 64);
      if (fg == 0) {
        lnp[wave][i * 16 + fr] = part[i];
        lnp2[wave][i * 16 + fr] = part2[i];
        if (fold && wave == 0) ln_mr[i * 16 + fr][0] = x0[i];
      }
    }
    if (fuse_ln) {  // (fold: the partials are published by the reduction barrier below)
      __syncthreads();
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        float t = 0.f, t2 = 0.f;
#pragma unroll
        for (int w = 0; w < SK_WAVES; ++w) {
          t += lnp[w][i * 16 + fr];
          t2 += lnp2[w][i * 16 + fr];
        }
        const float dm = t / (float)K;
        ln_mean[i] = x0[i] + dm;
        const float var = t2 / (float)K - dm * dm;
        ln_rs[i] = 1.f / sqrtf((var > 0.f ? var : 0.f) + p.ln_eps);
      }
    }
  } else if (fuse_ln || fold) {
    const int t = threadIdx.x & 15;
    for (int rr = threadIdx.x >> 4; rr < BM; rr += 64 * SK_WAVES / 16) {
      const int64_t row = m0 + rr < M ? m0 + rr : M - 1;
      const TI* xr = reinterpret_cast<const TI*>(p.A) + row * p.lda;
      float s = 0.f;
      for (int64_t k = (int64_t)t * EPC; k < K; k += 16 * EPC) {
        float v[EPC];
        if constexpr (EPC == 8) io<TI>::ld8(xr + k, v); else io<TI>::ld4(xr + k, v);
#pragma unroll
        for (int e = 0; e < EPC; ++e) s += v[e];
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      const float mean = s / (float)K;
      float s2 = 0.f;
      for (int64_t k = (int64_t)t * EPC; k < K; k += 16 * EPC) {
        float v[EPC];
        if constexpr (EPC == 8) io<TI>::ld8(xr + k, v); else io<TI>::ld4(xr + k, v);
#pragma unroll
        for (int e = 0; e < EPC; ++e) s2 += (v[e] - mean) * (v[e] - mean);
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
      if (t == 0) {
        ln_mr[rr][0] = mean;
        ln_mr[rr][1] = 1.f / sqrtf(s2 / (float)K + p.ln_eps);
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      ln_mean[i] = ln_mr[i * 16 + fr][0];
      ln_rs[i] = ln_mr[i * 16 + fr][1];
    }
  }
  for (int64_t base = wave;;) {
    // all SKU steps' loads are issued before the first MFMA waits (without this fence hipcc sinks each load
    // to its use and every MFMA waits out a full memory latency)
    __builtin_amdgcn_sched_barrier(0);
    if (fuse_ln) {
#pragma unroll
      for (int u = 0; u < SKU; ++u) {
        const int64_t k0 = (base + (int64_t)u * SK_WAVES) * KSTEP + fg * EPC;
        if (k0 < K) {  // K-tail / past-the-end chunks stay zero
          float g[EPC], bt[EPC];
          if (ln_lds) {
#pragma unroll
            for (int e = 0; e < EPC; e += 4) {
              const float4 gv = *reinterpret_cast<const float4*>(&lngb[k0 + e]);
              const float4 bv = *reinterpret_cast<const float4*>(&lngb[SK_LNK + k0 + e]);
              g[e] = gv.x; g[e + 1] = gv.y; g[e + 2] = gv.z; g[e + 3] = gv.w;
              bt[e] = bv.x; bt[e + 1] = bv.y; bt[e + 2] = bv.z; bt[e + 3] = bv.w;
            }
          } else if constexpr (EPC == 8) {
            io<float>::ld8(p.ln_gamma + k0, g); io<float>::ld8(p.ln_beta + k0, bt);
          } else {
            io<float>::ld4(p.ln_gamma + k0, g); io<float>::ld4(p.ln_beta + k0, bt);
          }
#pragma unroll
          for (int i = 0; i < MT; ++i) af[u][i] = ln_chunk<TI>(af[u][i], ln_mean[i], ln_rs[i], g, bt);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < SKU; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) mfma_chunk<TI>(acc[i][j], af[u][i], bfr[u][j]);
    base += SK_WAVES * SKU;
    if (base >= nks) break;
    load_steps(base);
  }
  // round 1: waves [HALF, 2 HALF) park their partials, waves [0, HALF) add them; round 2: the HALF sums -> LDS
  auto park = [&](float* dst) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) dst[(i * 16 + fg * 4 + v) * RLD + j * 16 + fr] = acc[i][j][v];
  };
  if (wave >= HALF) park(red[wave - HALF]);
  __syncthreads();
  if (wave < HALF) {
    const float* src = red[wave];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[i][j][v] += src[(i * 16 + fg * 4 + v) * RLD + j * 16 + fr];
    park(red[wave]);  // same addresses this lane just read: no cross-lane hazard
  }
  __syncthreads();
  if (!eact) return;
  const uint64_t seed = drop_thresh != 0u ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  float x[4];
  *reinterpret_cast<float4*>(x) = *reinterpret_cast<const float4*>(&red[0][er * RLD + ec]);
#pragma unroll
  for (int w = 1; w < HALF; ++w) {
    const float4 v = *reinterpret_cast<const float4*>(&red[w][er * RLD + ec]);
    x[0] += v.x; x[1] += v.y; x[2] += v.z; x[3] += v.w;
  }
  if (fold) {  // rstd (acc - mean wsum); the host passed bias = b + W . beta
    float mean, rs;
    if (ln_frag) {  // the wave partials in wave order (the order of the LN-fused form above)
      float t = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < SK_WAVES; ++w) {
        t += lnp[w][er];
        t2 += lnp2[w][er];
      }
      const float dm = t / (float)K;
      mean = ln_mr[er][0] + dm;
      const float var = t2 / (float)K - dm * dm;
      rs = 1.f / sqrtf((var > 0.f ? var : 0.f) + p.ln_eps);
    } else {
      mean = ln_mr[er][0];
      rs = ln_mr[er][1];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = ecol + e < N ? rs * (x[e] - mean * p.ln_wsum[ecol + e]) : x[e];
  }
  // two call sites rather than a selected pointer (a pointer select on a local puts it in scratch)
  if (use_pre) epiw<TC, 4>(p, erow, ecol, x, bias4, ecol + 4 <= N, seed, drop_thresh, inv_keep, &pre);
  else epiw<TC, 4>(p, erow, ecol, x, bias4, ecol + 4 <= N, seed, drop_thresh, inv_keep);
}

// Split-K reduction: sum the fp32 partial slabs of `splits` K-ranges in a fixed order (deterministic) and
// apply the full epilogue. One thread per 4 consecutive columns.
template <typename TC>
__global__ __launch_bounds__(256) void gemm_splitk_reduce(icap_gemm_args p, int splits, uint32_t drop_thresh,
                                                         float inv_keep) {
  const int64_t M = p.M, N = p.N;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n4 = N >> 2;
  if (q >= M * n4) return;
  const int64_t row = q / n4, col = (q - row * n4) * 4;
  if (p.m_dev && row >= (int64_t)*p.m_dev) return;
  const float* ws = reinterpret_cast<const float*>(p.workspace) + row * N + col;
  float x[4];
  *reinterpret_cast<float4*>(x) = *reinterpret_cast<const float4*>(ws);
  for (int s = 1; s < splits; ++s) {
    const float4 v = *reinterpret_cast<const float4*>(ws + (int64_t)s * M * N);
    x[0] += v.x; x[1] += v.y; x[2] += v.z; x[3] += v.w;
  }
  float bias4[4] = {0.f, 0.f, 0.f, 0.f};
  if (p.bias && p.dact == ICAP_ACT_NONE) {
#pragma unroll
    for (int e = 0; e < 4; ++e) bias4[e] = p.bias[col + e];  // flat-parameter views: only 4-byte aligned
  }
  const uint64_t seed = drop_thresh != 0u ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  epi4<TC>(p, row, col, x, bias4, true, seed, drop_thresh, inv_keep);
}


// ---------------------------------------------------------------------------------------------------------------
}  // namespace icap

using namespace icap;

// Tile-kernel variant. Measured on MI355X (tools/gemm_bench.py, profiles/r01_gemm_variants.txt): short K (<= 16 stages) is
// bound by the per-block prologue/epilogue, which co-resident blocks hide -> single LDS buffer, 3-4 blocks/CU (4
// when the epilogue moves a second M x N tensor: dact_src read / aux store); long K favours the double-buffered
// main loop at 2 blocks/CU.
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
static int gemm_variant(const icap_gemm_args& p, int64_t nk_per_block) {
  if (nk_per_block > 16) return 0;
  const bool heavy = p.dact != ICAP_ACT_NONE || p.aux;
  const bool act = p.act != ICAP_ACT_NONE || p.dact != ICAP_ACT_NONE;
  // (A/B) ICAP_VAR_HEAVY / ICAP_VAR_ACT / ICAP_VAR_LIGHT: variant for short-K launches with dact / aux, with an
  // activation only, and with neither
  static const int vh = env_int("ICAP_VAR_HEAVY", 5), va = env_int("ICAP_VAR_ACT", 4), vl = env_int("ICAP_VAR_LIGHT", 4);
  return heavy ? vh : act ? va : vl;
}

// compute units of the current device (the skinny-GEMM grid rule, the 256 x 256 kernel's pick)
static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

namespace icap {
int gemm256_launch(const icap_gemm_args& p, uint32_t thr, float inv_keep, hipStream_t s);
}

// ICAP_GEMM256: 0 = never, 2 = wherever eligible, default = the shape rule below (A/B measurements only)
static int g256_mode() {
  static const int m = [] {
    const char* e = getenv("ICAP_GEMM256");
    return e && (e[0] == '0' || e[0] == '2') ? e[0] - '0' : 1;
  }();
  return m;
}

// The 256 x 256 kernel's preconditions, and when it is the automatic choice. It runs one block per CU, so a
// tile's prologue (first DMA round trip) and epilogue do not overlap other tiles' MFMAs: it beats the 128-row
// tile kernels (2-3 blocks per CU) on long K (4096^3: 1.09-1.22 vs 0.95 PF) and on many full tile rounds (LM
// head 8320 x 50304 x 768: 758 vs 835 us), not on the train step's 2-round K = 768 products (8320 x 3072 x 768:
// 84 vs 80 us) (profiles/r02_gemm256_bench.txt). path 3 forces it where eligible.
static bool g256_pick(const icap_gemm_args& p) {
  if (p.path == 1) return false;
  if (p.in_dtype != ICAP_BF16 || p.trans_ab || p.ln_gamma || p.beta != 0.f || p.m_dev || p.split_k > 1) return false;
  if (p.M < 256 || p.N < 256 || p.K < 64) return false;
  if (p.path == 3 || g256_mode() == 2) return true;
  if (g256_mode() == 0) return false;
  const int64_t tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  const int64_t cus = device_cus();
  const int64_t rounds = (tiles + cus - 1) / cus;
  const bool full = tiles * 10 >= rounds * cus * 7;  // rounds at least 70 % occupied
  return (p.K >= 2048 && tiles * 4 >= cus * 3 && full) || (rounds >= 4 && tiles * 10 >= rounds * cus * 8);
}

static bool al16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

// A/B switches for the in-launch split-K (read once): ICAP_FUSED_S = forced split count, ICAP_FUSED_NST = 1 gives
// its K ranges the variant rule (default: the double-buffered kernel)
static int fused_s_override() {
  static const int v = [] { const char* e = getenv("ICAP_FUSED_S"); return e ? atoi(e) : 0; }();
  return v;
}
// K-skew: tile (tm, tn) walks its K range starting at step ((7 tm + tn) * skew) mod nk and wraps, so the tiles of
// one XCD that share an A row panel (consecutive tn) or a B panel do not request the same lines in lockstep (a
// line they all miss on is fetched once and waited for by every one of them). Measured over the packed train step
// (eager per-shape table, profiles/r03_kskew_ab.txt): skew 1 took the N = 768 products 5-15 % shorter and the step
// 11.3 -> 10.9 ms; skew 2-4 less; launches over more than 64 k-steps per split (the LM-head dX, K = 50304) ran
// longer, so they keep the natural order. ICAP_KSKEW overrides the skew (0 = off; A/B only); path 1 (tile_only)
// keeps the natural order (the path-equality tests compare it bitwise with the 256 x 256 kernel).
static int kskew_for(const icap_gemm_args& p, int64_t nk_split) {
  static const int v = [] { const char* e = getenv("ICAP_KSKEW"); return e ? atoi(e) : 1; }();
  if (p.path == 1 || p.in_dtype == ICAP_FP8_MX || nk_split > 64) return 0;
  return v > 0 && v < 256 ? v : 0;
}
// ICAP_GEMM_DIAG = 1 / 2 / 3: drop the A / B / both operands' staging loads of the tile kernels (zero-record
// descriptors) — a timing diagnostic for what the operand traffic costs; the outputs are wrong. Never in a real run.
static int gemm_diag() {  // (read per launch: an A/B driver toggles it in one process)
  const char* e = getenv("ICAP_GEMM_DIAG");
  return e ? (atoi(e) & 3) : 0;
}
static bool spec_act_on() {  // ICAP_SPEC_ACT=0: the runtime-dispatch epilogue everywhere (A/B only)
  static const bool v = [] { const char* e = getenv("ICAP_SPEC_ACT"); return !(e && e[0] == '0'); }();
  return v;
}
static int fused_nst_override() {
  static const int v = [] { const char* e = getenv("ICAP_FUSED_NST"); return e ? atoi(e) : 0; }();
  return v;
}

namespace {
// What icap_gemm launches for one call (shared by the launcher and icap_gemm_kernel_name).
struct GemmPlan {
  bool skinny = false;
  bool g256 = false;     // the 256 x 256 8-phase kernel (gemm256.hip)
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
}  // namespace

static int gemm_plan(const icap_gemm_args& p, GemmPlan& pl) {
  ICAP_REQUIRE(p.M >= 0 && p.N >= 0 && p.K >= 0, "icap_gemm: negative size");
  ICAP_REQUIRE(p.path == 0 || p.path == 1 || p.path == 3, "icap_gemm: path must be 0, 1 or 3");
  ICAP_REQUIRE(p.A && p.B && p.C, "icap_gemm: null operand");
  ICAP_REQUIRE(p.in_dtype == ICAP_F32 || p.in_dtype == ICAP_BF16 || p.in_dtype == ICAP_FP8_MX,
               "icap_gemm: bad in_dtype");
  ICAP_REQUIRE(p.c_dtype == ICAP_F32 || p.c_dtype == ICAP_BF16, "icap_gemm: bad c_dtype");
  const bool mx = p.in_dtype == ICAP_FP8_MX;
  if (mx) {
    ICAP_REQUIRE(p.K % 128 == 0 && p.lda % 16 == 0 && p.ldb % 16 == 0,
                 "icap_gemm: FP8_MX needs K % 128 == 0 and lda, ldb multiples of 16");
    ICAP_REQUIRE(p.a_scale && p.b_scale && al16(p.a_scale) && al16(p.b_scale),
                 "icap_gemm: FP8_MX needs 16-byte aligned a_scale / b_scale");
    ICAP_REQUIRE(!p.trans_ab && !p.ln_gamma && p.path != 3, "icap_gemm: FP8_MX takes no trans_ab / ln / path 3");
    ICAP_REQUIRE((p.K / 32) * ((p.M + 63) / 64) * 64 < 0x7fffffffll && (p.K / 32) * ((p.N + 63) / 64) * 64 < 0x7fffffffll,
                 "icap_gemm: FP8_MX scale arrays must stay below 2 GiB");
  }
  const int epc = p.in_dtype == ICAP_BF16 ? 8 : mx ? 16 : 4;
  ICAP_REQUIRE(p.trans_ab || p.K % epc == 0, "icap_gemm: K must be a multiple of 8 (bf16) / 4 (f32)");
  ICAP_REQUIRE(p.lda % epc == 0 && p.ldb % epc == 0, "icap_gemm: lda/ldb must be multiples of 8 (bf16) / 4 (f32)");
  ICAP_REQUIRE((p.trans_ab || (p.lda >= p.K && p.ldb >= p.K)) && p.ldc >= p.N, "icap_gemm: leading dimension too small");
  ICAP_REQUIRE((reinterpret_cast<uintptr_t>(p.A) & 15) == 0 && (reinterpret_cast<uintptr_t>(p.B) & 15) == 0,
               "icap_gemm: A and B must be 16-byte aligned");
  const int es = p.in_dtype == ICAP_BF16 ? 2 : mx ? 1 : 4;
  ICAP_REQUIRE((int64_t)256 * p.lda * es < 0x7fffffffll && (int64_t)256 * p.ldb * es < 0x7fffffffll,
               "icap_gemm: a 256-row operand panel must stay below 2 GiB");
  ICAP_REQUIRE(p.beta == 0.f || p.c_dtype == ICAP_F32, "icap_gemm: beta != 0 requires f32 C");
  ICAP_REQUIRE(p.dact == ICAP_ACT_NONE || p.dact_src != nullptr, "icap_gemm: dact requires dact_src");
  ICAP_REQUIRE(p.act >= ICAP_ACT_NONE && p.act <= ICAP_ACT_GELU_ERF && p.dact >= ICAP_ACT_NONE &&
                   p.dact <= ICAP_ACT_GELU_ERF, "icap_gemm: unknown activation");
  ICAP_REQUIRE(p.drop_p >= 0.f && p.drop_p < 1.f, "icap_gemm: drop_p out of range");
  if (p.trans_ab) {
    ICAP_REQUIRE(p.in_dtype == ICAP_BF16, "icap_gemm: trans_ab needs bf16 inputs");
    ICAP_REQUIRE(p.lda >= p.M && p.ldb >= p.N, "icap_gemm: trans_ab needs lda >= M, ldb >= N");
    ICAP_REQUIRE(p.m_dev == nullptr, "icap_gemm: trans_ab does not take m_dev");
    ICAP_REQUIRE((int64_t)(p.K + 64) * p.lda * 2 < 0x7fffffffll && (int64_t)(p.K + 64) * p.ldb * 2 < 0x7fffffffll,
                 "icap_gemm: trans_ab operands must stay below 2 GiB");
  }
  const int64_t tiles_m = (p.M + GBM - 1) / GBM;
  int64_t tiles_n = (p.N + GBN - 1) / GBN;
  int64_t tiles = tiles_m * tiles_n;
  ICAP_REQUIRE(tiles < (1ll << 26), "icap_gemm: too many tiles");
  ICAP_REQUIRE(p.split_k >= 0, "icap_gemm: split_k must be >= 0");
  pl.thr = p.drop_p > 0.f ? drop_threshold(p.drop_p) : 0u;
  pl.inv_keep = p.drop_p > 0.f ? 1.f / (1.f - p.drop_p) : 1.f;
  const bool fuse_ln = p.ln_gamma != nullptr;
  ICAP_REQUIRE(!fuse_ln || (p.ln_beta && p.M <= 128 && p.split_k == 0 && !p.trans_ab && p.K <= 4096),
               "icap_gemm: ln_gamma needs ln_beta, M <= 128, K <= 4096, no split_k / trans_ab");
  const bool fold_ln = p.ln_wsum != nullptr;
  ICAP_REQUIRE(!fold_ln || (!fuse_ln && p.M <= 128 && p.split_k == 0 && !p.trans_ab && !mx && p.K <= 4096),
               "icap_gemm: ln_wsum needs M <= 128, no ln_gamma / split_k / trans_ab / FP8_MX, K <= 4096");
  if (p.M <= 128 && p.split_k == 0 && (tiles <= 128 || fuse_ln || fold_ln) && !p.trans_ab && !mx) {
    pl.skinny = true;
    // the fewest 16-column slabs per block that keep the grid within one pass over the CUs (every CU streams one
    // block's A rows + W slab; a second block on a CU doubles its bytes), then enough k-steps in flight per wave
    // to cover K in one round trip where the fragment registers allow (SKU in {3, 4, 6}; 12 for one-slab blocks)
    const int64_t gy = (p.M + 31) / 32;
    const int cus = device_cus();
    pl.nt = 4;
    for (int nt = 1; nt <= 4; ++nt)
      if ((p.N + 16 * nt - 1) / (16 * nt) * gy <= cus) { pl.nt = nt; break; }
    if (p.in_dtype == ICAP_BF16) {
      const int64_t need = ((p.K + 31) / 32 + SK_WAVES - 1) / SK_WAVES;
      pl.sku = need <= 3 ? 3 : need <= 4 ? 4 : (need <= 6 || pl.nt > 1) ? 6 : 12;
    } else {
      pl.sku = 6;
    }
    pl.grid = dim3((unsigned)((p.N + 16 * pl.nt - 1) / (16 * pl.nt)), (unsigned)gy);
    pl.block = dim3(64 * SK_WAVES);
    return ICAP_OK;
  }
  // 256 x 256 8-phase kernel (gemm256.hip) for wide products whose 256-tiles fill the chip in few, full rounds
  if (g256_pick(p)) {
    pl.g256 = true;
    return ICAP_OK;
  }
  // split-K over K stages for launches that cannot fill the chip (decode-time M = batch, small projections):
  // fp32 partial slabs in the caller's workspace + one deterministic reduce/epilogue pass — or, with tickets, the
  // in-launch combine (long K over fewer tiles than CUs: the packed step's N = 768 products, the mapper's M = 3200
  // products and weight gradients): S = 2 * CUs / tiles rounded, 2..4, so the tile x split blocks fill the chip
  // about twice, and no slab round trip or extra launch.
  const int64_t bke = 128 / es;
  const int64_t nk = (p.K + bke - 1) / bke;
  const int64_t slab = p.M * p.N * (int64_t)sizeof(float);
  const int64_t cus = device_cus();
  // with a device row count the kernel choice follows the expected count (m_hint)
  const int64_t m_plan = (p.m_dev && p.m_hint > 0 && p.m_hint < p.M) ? p.m_hint : p.M;
  const int64_t tiles_plan = ((m_plan + GBM - 1) / GBM) * tiles_n;
  // The split count is a function of the shape (M, N, K, dtype, trans_ab; with a device row count, the caller's
  // expected count m_hint) alone — never of the workspace size or of whether tickets are attached — so the partial
  // sums are always added in the same order. Tickets only choose HOW the splits combine (inside the launch or in a
  // reduce pass over slabs); both add the partials in split order starting from split 0 and apply the same epilogue
  // formula, so the two mechanisms store bitwise-identical outputs (tests/test_fused_splitk_gpu.py). A NULL workspace
  // turns the automatic split off (documented: include/icap.h); a given one too small for the shape's split is an error.
  int64_t splits = 1;
  pl.fused = false;
  bool fusable = false;  // the long-K / few-tiles rule below (the splits may combine inside the launch)
  // (not for the K-outer weight-gradient products: measured, their in-launch combine ran 6-7 µs slower than the
  // slab + reduce pass — 768x3072x3200 53 vs 47 µs, profiles/r03_gemm_detail_fused.txt — since the last arriver of
  // a 3-block-per-CU tile reads its partials one accumulator row at a time)
  if (p.split_k == 0 && p.workspace && !p.trans_ab && (p.N & 3) == 0 && nk >= 24 && tiles_plan < cus) {
    int64_t sf = (2 * cus + tiles_plan / 2) / tiles_plan;
    if (sf > 4) sf = 4;
    while (sf > 2 && nk / sf < 8) --sf;
    // A/B measurements only (ICAP_FUSED_S): the in-launch combine reads at most 3 other partials (4 splits)
    if (fused_s_override() > 1) sf = fused_s_override() < 4 ? fused_s_override() : 4;
    if (sf >= 2) {
      splits = sf;
      fusable = true;
    }
  }
  if (fusable) {
    const int64_t pbytes = (int64_t)GBM * GBN * (int64_t)sizeof(float);
    const int64_t sfin = splits;
    const int64_t nks_ = (nk + sfin - 1) / sfin;
    const int64_t sreal = (nk + nks_ - 1) / nks_;  // the split count after every split got >= 1 stage (below)
    // with a device row count the grid still covers every row tile of M, so tickets / partials for all of them
    pl.fused = p.tickets && p.tickets_len >= 2 * tiles && p.workspace_bytes >= tiles * sreal * pbytes;
  } else if (p.split_k > 1) {
    splits = p.split_k;
  } else if (p.split_k == 0 && p.workspace && p.trans_ab && (p.N & 3) == 0 && nk >= 16 && tiles < 320) {
    // K-outer weight gradients over the token rows (the mapper's 3200-row products): about 320 blocks, at most 6
    // splits — measured 31.8 / 23.3 / 35.4 / 35.8 us for 2304x768 / 768x768 / 3072x768 / 768x3072 over 3200 rows
    // against 33.9 / 24.7 / 40.3 / 40.2 with the 512-block rule below (profiles/r03_dw_bench.txt)
    splits = (320 + tiles - 1) / tiles;
    if (splits > 6) splits = 6;
  } else if (p.split_k == 0 && p.workspace && (p.N & 3) == 0 && nk >= 2 && (tiles <= 64 || (tiles < 256 && nk >= 16))) {
    // the count depends on the shape alone — never on the workspace a caller passes — so a product computed on
    // another stream with its own scratch sums its K ranges in the same order and rounds identically (a
    // workspace too small for the shape's split is an error below, not a silent change of the summation order)
    splits = (512 + tiles - 1) / tiles;
    if (tiles > 64 && splits > nk / 4) splits = nk / 4;
    if (splits > 32) splits = 32;
  }
  if (splits > nk) splits = nk;
  if (splits < 1) splits = 1;
  const int64_t nk_split = nk > 0 ? (nk + splits - 1) / splits : 0;
  if (nk_split > 0) splits = (nk + nk_split - 1) / nk_split;  // every split gets >= 1 stage
  if (splits > 1 && !pl.fused) {
    ICAP_REQUIRE((p.N & 3) == 0, "icap_gemm: split-K requires N % 4 == 0");
    ICAP_REQUIRE(p.workspace && (reinterpret_cast<uintptr_t>(p.workspace) & 15) == 0 &&
                     p.workspace_bytes >= splits * slab,
                 "icap_gemm: split-K workspace missing, misaligned or too small");
  }
  if (pl.fused)
    ICAP_REQUIRE((reinterpret_cast<uintptr_t>(p.workspace) & 15) == 0 && (reinterpret_cast<uintptr_t>(p.tickets) & 7) == 0,
                 "icap_gemm: split-K workspace / tickets misaligned");
  // Short-K launches (<= 16 stages) of fewer than 4 tiles of 128 x 128 per CU (the N = 768 products, the mapper's
  // M = 3200 and CLIP's M = 6400 ones) run faster on 128 x 64 tiles: twice the blocks, so a CU holds more of them
  // to hide each one's prologue / epilogue; longer K keeps 128 x 128 (profiles/r01_gemm_narrow.txt).
  const bool narrow = p.in_dtype == ICAP_BF16 && p.M > 128 && !p.trans_ab && tiles < 1024 && nk <= 16 && splits == 1;
  pl.splits = (int)splits;
  pl.nk_split = (int)nk_split;
  pl.variant = gemm_variant(p, nk_split);
  // in-launch split-K: the double-buffered main loop at 2 blocks per CU for every split's K range (measured on the
  // packed 3584 x 768 x 3072 / x 2304 products: 36.6 / 30.4 vs 40.1 / 32.4 µs with the single-stage form the
  // per-split K of 16 stages would pick; profiles/r03_fused_ab.txt); ICAP_FUSED_NST=1 restores the variant rule
  if (pl.fused && fused_nst_override() != 1) pl.variant = 0;
  // Long K over at most one 128 x 128 tile per CU and no split (no tickets given): the 4-stage ring at one block per
  // CU (the double-buffered loop at 2 blocks per CU only pays when a CU holds two tiles).
  if (p.in_dtype == ICAP_BF16 && !p.trans_ab && splits == 1 && nk_split > 16 && tiles_plan <= cus)
    pl.variant = 16;
  if (mx && pl.variant == 5) pl.variant = 4;  // MX at 4 blocks / CU (128 VGPRs) spills: 3 blocks / CU
  if (narrow) {
    tiles_n = (p.N + 63) / 64;
    tiles = tiles_m * tiles_n;
    pl.variant = tiles < 256 ? 12 : 13;
  }
  if (p.trans_ab) pl.variant = nk_split > 16 ? 14 : 15;  // K-outer forms of variants 0 / 4
  pl.tiles_n = (int)tiles_n;
  const bool any_act = (splits == 1 || pl.fused) && (p.act != ICAP_ACT_NONE || p.dact != ICAP_ACT_NONE);
  pl.actk = any_act ? ACT_ANY : ACT_OFF;
  // the step's activated products get an epilogue compiled for their one activation (gemm_common.h ACT_FWD /
  // ACT_BWD): GPT-2 c_fc gelu_new (+ aux) and its dgelu, CLIP c_fc quick_gelu, ViT / DINOv3 c_fc erf gelu, the
  // mapper's relu / drelu (128 x 64 tiles). Measured over the packed step (tools/specact_ab.sh, profiles/
  // r03_specact_ab.txt): 10.98 -> 10.61 ms; the mapper's 3200x3072x768 relu 36.4 -> 29.1 µs, CLIP's quick_gelu
  // 68.6 -> 64.0, gelu + aux 64.5 -> 57.6 — the runtime dispatch over five activations (libm erff / tanhf / expf
  // inlined per case) cost registers and scratch in the epilogue of every activated launch.
  if (any_act && p.in_dtype == ICAP_BF16 && p.c_dtype == ICAP_BF16 && !p.trans_ab && spec_act_on()) {
    const int fa = p.dact == ICAP_ACT_NONE ? p.act : -1, ba = p.act == ICAP_ACT_NONE ? p.dact : -1;
    const bool v045 = pl.variant == 0 || pl.variant == 4 || pl.variant == 5;
    if (v045 && fa == ICAP_ACT_GELU_NEW) pl.actk = ACT_FWD + ICAP_ACT_GELU_NEW;
    else if (v045 && ba == ICAP_ACT_GELU_NEW) pl.actk = ACT_BWD + ICAP_ACT_GELU_NEW;
    else if (pl.variant == 4 && fa == ICAP_ACT_QUICK_GELU) pl.actk = ACT_FWD + ICAP_ACT_QUICK_GELU;
    else if (pl.variant == 4 && fa == ICAP_ACT_GELU_ERF) pl.actk = ACT_FWD + ICAP_ACT_GELU_ERF;
    else if (pl.variant == 13 && fa == ICAP_ACT_RELU) pl.actk = ACT_FWD + ICAP_ACT_RELU;
    else if (pl.variant == 13 && ba == ICAP_ACT_RELU) pl.actk = ACT_BWD + ICAP_ACT_RELU;
  }
  pl.block = dim3(GNT);
  pl.grid = dim3((unsigned)(tiles * splits));
  return ICAP_OK;
}

// "TI, TC, template ints" of each tile variant (keep in sync with the launch switch below); %%d = ACT kind
static const char* variant_kernel(int v) {
  switch (v) {
    case 0: return "gemm_kernel<%s, %s, 2, 2, 2, 2, 4, 4, false, %d>";
    case 4: return "gemm_kernel<%s, %s, 1, 3, 2, 2, 4, 4, false, %d>";
    case 5: return "gemm_kernel<%s, %s, 1, 4, 2, 2, 4, 4, false, %d>";
    case 12: return "gemm_kernel<%s, %s, 2, 3, 2, 2, 4, 2, false, %d>";
    case 13: return "gemm_kernel<%s, %s, 1, 4, 2, 2, 4, 2, false, %d>";
    case 14: return "gemm_kernel<%s, %s, 2, 2, 2, 2, 4, 4, true, %d>";
    case 16: return "gemm_kernel<%s, %s, 4, 1, 2, 2, 4, 4, false, %d>";
    default: return "gemm_kernel<%s, %s, 1, 3, 2, 2, 4, 4, true, %d>";
  }
}

extern "C" const char* icap_gemm_kernel_name(const icap_gemm_args* a) {
  static thread_local char buf[160];
  if (a == nullptr) return nullptr;
  GemmPlan pl;
  if (gemm_plan(*a, pl) != ICAP_OK) return nullptr;
  const char* ti = a->in_dtype == ICAP_BF16 ? "unsigned short" : a->in_dtype == ICAP_FP8_MX ? "icap::fp8_t" : "float";
  const char* tc = a->c_dtype == ICAP_BF16 ? "unsigned short" : "float";
  char fmt[96];
  if (pl.g256) {
    snprintf(buf, sizeof buf, "icap::gemm256_kernel<%s>", tc);
    return buf;
  }
  char inner[128];
  if (pl.skinny) {
    snprintf(fmt, sizeof fmt, "gemm_skinny_kernel<%%s, %%s, %d, 2, %d>", pl.nt, pl.sku);
    snprintf(inner, sizeof inner, fmt, ti, tc);
  } else {
    snprintf(inner, sizeof inner, variant_kernel(pl.variant), ti, tc, pl.actk);
  }
  snprintf(buf, sizeof buf, "icap::%s", inner);
  return buf;
}

extern "C" int icap_gemm_plan_info(const icap_gemm_args* a, int32_t* splits, int32_t* fused) {
  ICAP_REQUIRE(a != nullptr && splits != nullptr && fused != nullptr, "icap_gemm_plan_info: null pointer");
  GemmPlan pl;
  const int rc = gemm_plan(*a, pl);
  if (rc != ICAP_OK) return rc;
  *splits = pl.skinny || pl.g256 ? 1 : pl.splits;
  *fused = pl.fused ? 1 : 0;
  return ICAP_OK;
}

extern "C" int icap_gemm(const icap_gemm_args* a, void* stream) {
  ICAP_REQUIRE(a != nullptr, "icap_gemm: null args");
  if (a->M == 0 || a->N == 0) return ICAP_OK;
  GemmPlan pl;
  const int prc = gemm_plan(*a, pl);
  if (prc != ICAP_OK) return prc;
  // the kernels take the in-launch combine exactly when tickets reach them: only for the plan that chose it (a
  // reduce-pass split must write its slabs, whatever the caller passed)
  icap_gemm_args pk = *a;
  if (!pl.fused) pk.tickets = nullptr;
  const icap_gemm_args& p = pk;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint32_t thr = pl.thr;
  const float inv_keep = pl.inv_keep;
  if (pl.skinny) {
    const dim3 sgrid = pl.grid, sblock = pl.block;
#define ICAP_SK(TI, TC, NT, U) hipLaunchKernelGGL((gemm_skinny_kernel<TI, TC, NT, 2, U>), sgrid, sblock, 0, s, p, thr, inv_keep)
#define ICAP_SKINNY_BF(TC)                                                                 \
  switch (pl.nt * 100 + pl.sku) {                                                          \
    case 103: ICAP_SK(bf16_t, TC, 1, 3); break;                                            \
    case 104: ICAP_SK(bf16_t, TC, 1, 4); break;                                            \
    case 106: ICAP_SK(bf16_t, TC, 1, 6); break;                                            \
    case 112: ICAP_SK(bf16_t, TC, 1, 12); break;                                           \
    case 203: ICAP_SK(bf16_t, TC, 2, 3); break;                                            \
    case 204: ICAP_SK(bf16_t, TC, 2, 4); break;                                            \
    case 206: ICAP_SK(bf16_t, TC, 2, 6); break;                                            \
    case 303: ICAP_SK(bf16_t, TC, 3, 3); break;                                            \
    case 304: ICAP_SK(bf16_t, TC, 3, 4); break;                                            \
    case 306: ICAP_SK(bf16_t, TC, 3, 6); break;                                            \
    case 403: ICAP_SK(bf16_t, TC, 4, 3); break;                                            \
    case 404: ICAP_SK(bf16_t, TC, 4, 4); break;                                            \
    default: ICAP_SK(bf16_t, TC, 4, 6); break;                                             \
  }
#define ICAP_SKINNY_F32(TC)                                                                \
  switch (pl.nt) {                                                                         \
    case 1: ICAP_SK(float, TC, 1, 6); break;                                               \
    case 2: ICAP_SK(float, TC, 2, 6); break;                                               \
    case 3: ICAP_SK(float, TC, 3, 6); break;                                               \
    default: ICAP_SK(float, TC, 4, 6); break;                                              \
  }
    if (p.in_dtype == ICAP_BF16) {
      if (p.c_dtype == ICAP_BF16) { ICAP_SKINNY_BF(bf16_t) } else { ICAP_SKINNY_BF(float) }
    } else {
      if (p.c_dtype == ICAP_BF16) { ICAP_SKINNY_F32(bf16_t) } else { ICAP_SKINNY_F32(float) }
    }
#undef ICAP_SKINNY_BF
#undef ICAP_SKINNY_F32
#undef ICAP_SK
    return check_launch("icap_gemm(skinny)");
  }
  if (pl.g256) return gemm256_launch(p, thr, inv_keep, s);
  const dim3 grid = pl.grid, block = pl.block;
  const int sp = pl.splits, tn = pl.tiles_n;
  const int nks = pl.nk_split | (kskew_for(p, pl.nk_split) << 20) | (gemm_diag() << 28);
  const dim3 rgrid((unsigned)((p.M * (p.N / 4) + 255) / 256));
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
#define ICAP_GKS(NST, MINB, TM_, TN_, KIND) \
  hipLaunchKernelGGL((gemm_kernel<bf16_t, bf16_t, NST, MINB, 2, 2, TM_, TN_, false, KIND>), grid, block, 0, s, p, tn, sp, \
                     nks, thr, inv_keep)
  if (pl.actk >= ACT_FWD) {  // specialised activation epilogues (gemm_plan: bf16 in / out, variants 0, 4, 5, 13)
    switch (pl.actk) {
      case ACT_FWD + ICAP_ACT_GELU_NEW:  // (variant 0: GPT-2 large / medium c_fc, K = 1280 / 1024 > 16 stages)
        if (pl.variant == 0) ICAP_GKS(2, 2, 4, 4, ACT_FWD + ICAP_ACT_GELU_NEW);
        else if (pl.variant == 4) ICAP_GKS(1, 3, 4, 4, ACT_FWD + ICAP_ACT_GELU_NEW);
        else ICAP_GKS(1, 4, 4, 4, ACT_FWD + ICAP_ACT_GELU_NEW);
        break;
      case ACT_BWD + ICAP_ACT_GELU_NEW:
        if (pl.variant == 0) ICAP_GKS(2, 2, 4, 4, ACT_BWD + ICAP_ACT_GELU_NEW);
        else if (pl.variant == 4) ICAP_GKS(1, 3, 4, 4, ACT_BWD + ICAP_ACT_GELU_NEW);
        else ICAP_GKS(1, 4, 4, 4, ACT_BWD + ICAP_ACT_GELU_NEW);
        break;
      case ACT_FWD + ICAP_ACT_QUICK_GELU: ICAP_GKS(1, 3, 4, 4, ACT_FWD + ICAP_ACT_QUICK_GELU); break;
      case ACT_FWD + ICAP_ACT_GELU_ERF: ICAP_GKS(1, 3, 4, 4, ACT_FWD + ICAP_ACT_GELU_ERF); break;
      case ACT_FWD + ICAP_ACT_RELU: ICAP_GKS(1, 4, 4, 2, ACT_FWD + ICAP_ACT_RELU); break;
      default: ICAP_GKS(1, 4, 4, 2, ACT_BWD + ICAP_ACT_RELU); break;
    }
#undef ICAP_GKS
  } else if (pl.variant == 14 || pl.variant == 15) {  // K-outer operands (bf16 inputs only)
    if (p.c_dtype == ICAP_BF16) {
      if (pl.variant == 14) ICAP_GK(bf16_t, bf16_t, 2, 2, 4, 4, true);
      else ICAP_GK(bf16_t, bf16_t, 1, 3, 4, 4, true);
    } else {
      if (pl.variant == 14) ICAP_GK(bf16_t, float, 2, 2, 4, 4, true);
      else ICAP_GK(bf16_t, float, 1, 3, 4, 4, true);
    }
  } else if (pl.variant == 16) {  // 4-stage ring (bf16 inputs only)
    if (p.c_dtype == ICAP_BF16) ICAP_GK(bf16_t, bf16_t, 4, 1, 4, 4, false);
    else ICAP_GK(bf16_t, float, 4, 1, 4, 4, false);
  } else if (pl.variant == 12 || pl.variant == 13) {  // 128 x 64 (bf16 inputs only)
    if (p.c_dtype == ICAP_BF16) {
      if (pl.variant == 12) ICAP_GK(bf16_t, bf16_t, 2, 3, 4, 2, false);
      else ICAP_GK(bf16_t, bf16_t, 1, 4, 4, 2, false);
    } else {
      if (pl.variant == 12) ICAP_GK(bf16_t, float, 2, 3, 4, 2, false);
      else ICAP_GK(bf16_t, float, 1, 4, 4, 2, false);
    }
  } else if (p.in_dtype == ICAP_BF16) {
    if (p.c_dtype == ICAP_BF16) { ICAP_GEMM_LAUNCH(bf16_t, bf16_t) } else { ICAP_GEMM_LAUNCH(bf16_t, float) }
  } else if (p.in_dtype == ICAP_FP8_MX) {  // variants 0 / 4 only (gemm_plan)
    if (p.c_dtype == ICAP_BF16) {
      if (pl.variant == 0) ICAP_GK(fp8_t, bf16_t, 2, 2, 4, 4, false);
      else ICAP_GK(fp8_t, bf16_t, 1, 3, 4, 4, false);
    } else {
      if (pl.variant == 0) ICAP_GK(fp8_t, float, 2, 2, 4, 4, false);
      else ICAP_GK(fp8_t, float, 1, 3, 4, 4, false);
    }
  } else {
    if (p.c_dtype == ICAP_BF16) { ICAP_GEMM_LAUNCH(float, bf16_t) } else { ICAP_GEMM_LAUNCH(float, float) }
  }
#undef ICAP_GEMM_LAUNCH
#undef ICAP_GK
  if (sp > 1 && !pl.fused) {
    if (p.c_dtype == ICAP_BF16)
      hipLaunchKernelGGL((gemm_splitk_reduce<bf16_t>), rgrid, dim3(256), 0, s, p, sp, thr, inv_keep);
    else
      hipLaunchKernelGGL((gemm_splitk_reduce<float>), rgrid, dim3(256), 0, s, p, sp, thr, inv_keep);
  }
  return check_launch("icap_gemm");
}

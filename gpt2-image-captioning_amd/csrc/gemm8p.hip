// 256-row tile bf16 GEMM on the 8-phase schedule, for the packed train step's products (round 5).
// C[M,N] = epi(alpha * A[M,K] . B[N,K]^T), both operands K-contiguous, C bf16 or f32; BN = 128 or 256 columns.
//
// Why: the 128 x 128 tile kernel (gemm_tile.h) runs two barriers per K-step with the next stage's LDS-DMA waited for
// (vmcnt(0)) inside the step; on the packed step's 3584-row products (one round of tiles) it reached 0.2 of the
// bf16 peak, and hipBLASLt ran the same plain products 1.3-1.65x faster (tools/ab/launch_probe.py,
// profiles/r05_tile_graph_ab.txt). The 8-phase schedule (cdna_hip_programming.md §5 "The 256² 8-phase template",
// gemm256.hip) keeps a half K-tile of DMA in flight across every barrier and overlaps one wave's MFMAs with the
// other wave's fragment reads on each SIMD; gemm256.hip runs it on 256 x 256 tiles, which the step's shapes fill
// only half (3584 x 2304: 126 tiles for 256 CUs). Here the same schedule on 256 x 128 tiles (252 tiles: one per
// CU) or 256 x 256, with the tile kernel's epilogue forms: the device row count (m_dev: packed rows), bias /
// activation / aux / dact / residual / dropout (epiw), and the LayerNorm statistics hand-off (producer: (mean, M2)
// per row and 32-column group of the stored C; consumer: rstd (A.B^T - mean wsum) + b from the producer's groups).
//
// Geometry: 8 waves as 2 (M) x 4 (N); wave (wr, wc) owns rows wr*128 + [0,128) and columns wc*WCN + [0,WCN)
// (WCN = BN / 4), as 8 x (WCN / 16) MFMA 16x16x32 accumulators. K advances 64 per tile (BK).
// LDS: NBUF K-tile buffers (3 at BN 128: the DMA runs two K-tiles ahead; 2 at BN 256: one ahead, gemm256.hip's
// schedule); a K-tile is four half-tiles of 128-byte rows (64 K):
//   h0 A-qm0: A rows {0..63} u {128..191}      (the first 64 rows of each wave-row's 128)
//   h1 B-qn0: B rows wc*WCN + [0, QN), wc = 0..3  (QN = WCN / 2: the first half of each wave-column)
//   h2 B-qn1: B rows wc*WCN + [QN, WCN)
//   h3 A-qm1: A rows {64..127} u {192..255}
// chunk index XOR-swizzled by (row & 7) (conflict-free ds_read_b128); the LDS-DMA writes lane-linear 1 KiB pieces
// and the swizzle lives on the per-lane source address (rule 21).
// Phases of one K-tile (one output quadrant each) and the DMA / wait schedule are gemm256.hip's (its header has the
// RAW / WAR argument), shifted by LA = NBUF - 1 K-tiles: half-tile h0 / h1 of K-tile u is issued at phase p2 / p3 of
// K-tile u - LA - 1, h2 / h3 at p0 / p1 of K-tile u - LA. Every issue still lands in the buffer of a K-tile whose
// same half was read two or more phases earlier (buffer (u mod NBUF): for h0 at p2 of K-tile t, u = t + LA + 1 ≡ t),
// so the WAR argument is unchanged; the RAW wait at p3 of K-tile t retires K-tile t + 1 and leaves everything issued
// after its last half in flight (counted per wave: an A half-tile is 2 DMA instructions, a B half-tile BN / 128).
#include "gemm_common.h"

namespace icap {
namespace g8p {
constexpr int BM = 256;
constexpr int HTA = 128 * GROWB;  // A half-tile bytes (128 rows)
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
template <int BN>
struct Geo {
  static constexpr int WCN = BN / 4;             // columns per wave
  static constexpr int QN = WCN / 2;             // columns per quadrant
  static constexpr int NJ = QN / 16;             // 16-column MFMA tiles per quadrant
  static constexpr int HTB = (BN / 2) * GROWB;   // B half-tile bytes
  static constexpr int TB = 2 * HTA + 2 * HTB;   // one 64-deep K-tile
  static constexpr int BPW = BN / 128;           // B DMA pieces per wave per half-tile
  static constexpr int ELD = WCN + 4;            // fp32 row stride of the epilogue staging
  static constexpr int EW = 64 * ELD * 4;        // staging bytes per wave (64 rows)
  // K-tile buffers: three for 128-column tiles (144 KiB: two K-tiles in flight, the >= 72 KiB a CU needs in flight
  // to reach its LDS-DMA intake rate), two for 256 columns (128 KiB)
  static constexpr int NBUF = BN == 128 ? 3 : 2;
  static constexpr int SMEM = (NBUF * TB > 8 * EW) ? NBUF * TB : 8 * EW;
  static constexpr int LPR = WCN / 8;            // epilogue lanes per row (8 columns each)
  static constexpr int RPI = 64 / LPR;           // rows per epilogue wave instruction
};
}  // namespace g8p

#define G8P_RD(dst, addr, off) asm volatile("ds_read_b128 %0, %1 offset:" #off : "=v"(dst) : "v"(addr))

template <typename TC, int BN, int ACT>
__global__ __launch_bounds__(512, 1) void gemm8p_kernel(icap_gemm_args p, int tiles_n, uint32_t drop_thresh,
                                                       float inv_keep) {
  using namespace g8p;
  using G = Geo<BN>;
  constexpr int AK = ACT & 0xFF;  // the epilogue's activation kind
  constexpr int LNX = ACT >> 8;   // 1 = LayerNorm statistics producer, 2 = consumer
  constexpr int NJ = G::NJ, WCN = G::WCN, QN = G::QN, BPW = G::BPW, TB = G::TB, HTB = G::HTB, NBUF = G::NBUF;
  constexpr int LA = NBUF - 1;  // K-tiles the DMA runs ahead: half-tile h of K-tile u is issued in K-tile u - LA
  __shared__ __attribute__((aligned(16))) char smem[G::SMEM + (LNX == 2 ? 8 * BM : 0)];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t M = p.M, N = p.N, K = p.K;
  const int64_t Mv = p.m_dev && (int64_t)*p.m_dev < M ? (int64_t)*p.m_dev : M;  // device row count
  // bijective XCD-aware remap over the LIVE tiles (gemm_tile.h): the grid covers M's row tiles, the first
  // ceil(Mv / BM) x tiles_n block ids work and the rest exit before any barrier
  const int bid = blockIdx.x;
  const int tiles_mv = (int)((Mv + BM - 1) / BM);
  const int nwg = tiles_mv * tiles_n;
  if (bid >= nwg) return;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = wg / tiles_n, tn = wg - tm * tiles_n;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t mr = Mv - m0 < BM ? Mv - m0 : BM, nr = N - n0 < BN ? N - n0 : BN;
  const int nk = (int)((K + 63) / 64);
  const bf16_t* Ag = reinterpret_cast<const bf16_t*>(p.A);
  const bf16_t* Bg = reinterpret_cast<const bf16_t*>(p.B);
  const __amdgpu_buffer_rsrc_t ra = make_rsrc_u(Ag + m0 * p.lda, (uint64_t)((mr - 1) * p.lda + K) * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc_u(Bg + n0 * p.ldb, (uint64_t)((nr - 1) * p.ldb + K) * 2);

  // ---- LDS-DMA: piece (i, wave) of a half-tile = LDS rows (8 i + wave) * 8 + l / 8; lane l's slot l % 8 holds
  // source chunk c = (l & 7) ^ (l >> 3) of tile row map_h(lr)
  const int c = (lane & 7) ^ (lane >> 3);
  uint32_t voa[2][2], vob[2][BPW];  // [A half (h0, h3) | B half (h1, h2)][piece]
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int lr = (i * 8 + wave) * 8 + (lane >> 3);
    const int trow = (lr & 63) + (lr >> 6) * 128;
    voa[0][i] = (uint32_t)((trow * p.lda + c * 8) * 2);
    voa[1][i] = (uint32_t)(((trow + 64) * p.lda + c * 8) * 2);
  }
#pragma unroll
  for (int i = 0; i < BPW; ++i) {
    const int lr = (i * 8 + wave) * 8 + (lane >> 3);
    const int trow = (lr / QN) * WCN + (lr % QN);
    vob[0][i] = (uint32_t)((trow * p.ldb + c * 8) * 2);
    vob[1][i] = (uint32_t)(((trow + QN) * p.ldb + c * 8) * 2);
  }
  auto issue = [&](auto hc, int u) __attribute__((always_inline)) {
    constexpr int H = decltype(hc)::value;
    if (u >= nk) return;  // block-uniform
    const int64_t k0 = (int64_t)u * 64;
    const bool kin = k0 + c * 8 < K;  // K % 8 == 0: a 16-byte chunk is wholly inside or outside
    constexpr int off = H == 0 ? 0 : H == 1 ? HTA : H == 2 ? HTA + HTB : HTA + 2 * HTB;
    char* dst = smem + (u % NBUF) * TB + off;
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(k0 * 2));
    if constexpr (H == 0 || H == 3) {
#pragma unroll
      for (int i = 0; i < 2; ++i) dma16s(ra, dst + (i * 8 + wave) * 1024, kin ? voa[H == 3][i] : OOB, so);
    } else {
#pragma unroll
      for (int i = 0; i < BPW; ++i) dma16s(rb, dst + (i * 8 + wave) * 1024, kin ? vob[H == 2][i] : OOB, so);
    }
  };

  // ---- LayerNorm fold (consumer): the row statistics of A from the producer's per-32-column (mean, M2) groups,
  // two threads per row (gemm_tile.h ln_prologue: same formula and order), into an LDS table past the stages
  float* lnr = reinterpret_cast<float*>(smem + G::SMEM);
  auto ln_prologue = [&]() __attribute__((always_inline)) {
    if constexpr (LNX == 2) {
      constexpr int LNQ = 10;  // 16-byte loads per thread at most: K <= 1280
      const int rr = tid >> 1, hf = tid & 1;
      const int64_t grow = m0 + rr < Mv ? m0 + rr : Mv - 1;
      const int Gk = (int)(K >> 5), nq = Gk >> 2;
      const float4* st = reinterpret_cast<const float4*>(p.ln_stats_in) + grow * (Gk >> 1) + hf * nq;
      float4 v[LNQ];
#pragma unroll
      for (int q = 0; q < LNQ; ++q)
        if (q < nq) v[q] = st[q];
      float sm = 0.f;
#pragma unroll
      for (int q = 0; q < LNQ; ++q)
        if (q < nq) sm += v[q].x + v[q].z;
      sm += __shfl_xor(sm, 1, 64);
      const float mean = sm / (float)Gk;
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
        if (p.ln_mean_out && tn == 0 && m0 + rr < Mv) {  // for the LayerNorm backward (one block per row)
          p.ln_mean_out[m0 + rr] = mean;
          p.ln_rstd_out[m0 + rr] = rs;
        }
      }
    }
  };

  // ---- fragment addressing: A rows wr*64 + mi*16 + fr of an A half, B rows wc*QN + nj*16 + fr of a B half
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>(smem);
  uint32_t la[2], lb[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const uint32_t sw = (uint32_t)(((ks * 4 + fg) ^ (fr & 7)) << 4);
    la[ks] = (uint32_t)((wr * 64 + fr) * GROWB) + sw;
    lb[ks] = (uint32_t)((wc * QN + fr) * GROWB) + sw;
  }
  u32x4_t RA[2][4], RB0[2][NJ], RB1[2][NJ];
  f32x4_t acc[8][2 * NJ];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 2 * NJ; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto read_a = [&](uint32_t half_base) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint32_t a = half_base + la[ks];
      G8P_RD(RA[ks][0], a, 0);
      G8P_RD(RA[ks][1], a, 2048);
      G8P_RD(RA[ks][2], a, 4096);
      G8P_RD(RA[ks][3], a, 6144);
    }
  };
  auto read_b = [&](u32x4_t (&R)[2][NJ], uint32_t half_base) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint32_t a = half_base + lb[ks];
      G8P_RD(R[ks][0], a, 0);
      if constexpr (NJ == 2) G8P_RD(R[ks][1], a, 2048);
    }
  };
  auto quad = [&](int am, int bn, u32x4_t (&RB)[2][NJ]) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < NJ; ++nj)
          mfma_chunk<bf16_t>(acc[am + mi][bn + nj], __builtin_bit_cast(uint4, RA[ks][mi]),
                             __builtin_bit_cast(uint4, RB[ks][nj]));
    __builtin_amdgcn_s_setprio(0);
  };
  // lgkmcnt(0) waits tied to the registers the asm reads wrote (hipcc does not see those reads)
  auto wait_a = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)"
                 : "+v"(RA[0][0]), "+v"(RA[0][1]), "+v"(RA[0][2]), "+v"(RA[0][3]), "+v"(RA[1][0]), "+v"(RA[1][1]),
                   "+v"(RA[1][2]), "+v"(RA[1][3]));
  };
  auto wait_b = [&](u32x4_t (&R)[2][NJ]) __attribute__((always_inline)) {
    if constexpr (NJ == 2)
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(R[0][0]), "+v"(R[0][1]), "+v"(R[1][0]), "+v"(R[1][1]));
    else
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(R[0][0]), "+v"(R[1][0]));
  };
#define G8P_FENCE() __builtin_amdgcn_sched_barrier(0)
  // counted waits: DMA instructions per wave of an A / B half-tile = 2 / BPW, a K-tile = 4 + 2 BPW
  constexpr int DH = 2 + BPW, DT = 4 + 2 * BPW;
  // retire K-tile t+1 at the end of K-tile t (or tile 0 in the prologue), leaving the later issues in flight:
  // tile t+2's first two half-tiles (LA 1), or all of tile t+2 and tile t+3's first two (LA 2), as far as issued
  auto retire_next = [&](int t) __attribute__((always_inline)) {
    if constexpr (LA == 1) {
      if (t + 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DH) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      if (t + 3 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DT + DH) : "memory");
      else if (t + 2 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(DT) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
  };

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  // prologue: tiles 0 .. LA-1 whole and the first two half-tiles of tile LA in flight; the LN row table; wait for
  // tile 0
#pragma unroll
  for (int u = 0; u < LA; ++u) {
    issue(I0{}, u); issue(I1{}, u); issue(I2{}, u); issue(I3{}, u);
  }
  issue(I0{}, LA); issue(I1{}, LA);
  G8P_FENCE();
  ln_prologue();  // (its loads are waited for at their first use, inside the prologue; that drains the DMA once)
  G8P_FENCE();
  retire_next(-1);
  __builtin_amdgcn_s_barrier();
  // wave-row 1 runs one barrier behind wave-row 0: on every SIMD one wave's MFMAs overlap the other's reads
  if (wr == 1) __builtin_amdgcn_s_barrier();
  G8P_FENCE();

  for (int t = 0; t < nk; ++t) {
    const uint32_t tb = sbase + (uint32_t)((t % NBUF) * TB);
    // p0: (qm0, qn0); DMA tile t+LA h2
    read_a(tb);
    read_b(RB0, tb + HTA);
    G8P_FENCE();
    issue(I2{}, t + LA);
    G8P_FENCE();
    __builtin_amdgcn_s_barrier();
    wait_a();
    wait_b(RB0);
    G8P_FENCE();
    quad(0, 0, RB0);
    G8P_FENCE();
    __builtin_amdgcn_s_barrier();
    G8P_FENCE();
    // p1: (qm0, qn1); DMA tile t+LA h3
    read_b(RB1, tb + HTA + HTB);
    G8P_FENCE();
    issue(I3{}, t + LA);
    G8P_FENCE();
    __builtin_amdgcn_s_barrier();
    wait_b(RB1);
    G8P_FENCE();
    quad(0, NJ, RB1);
    G8P_FENCE();
    __builtin_amdgcn_s_barrier();
    G8P_FENCE();
    // p2: (qm1, qn1); DMA tile t+LA+1 h0
    read_a(tb + HTA + 2 * HTB);
    G8P_FENCE();
    issue(I0{}, t + LA + 1);
    G8P_FENCE();
    __builtin_amdgcn_s_barrier();
    wait_a();
    G8P_FENCE();
    quad(4, NJ, RB1);
    G8P_FENCE();
    __builtin_amdgcn_s_barrier();
    G8P_FENCE();
    // p3: (qm1, qn0); DMA tile t+LA+1 h1; retire tile t+1
    issue(I1{}, t + LA + 1);
    G8P_FENCE();
    retire_next(t);
    __builtin_amdgcn_s_barrier();
    G8P_FENCE();
    quad(4, 0, RB0);
    G8P_FENCE();
    __builtin_amdgcn_s_barrier();
    G8P_FENCE();
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // equal barrier counts: wave-row 0 waits for row 1's last phase
#undef G8P_FENCE

  // ---- epilogue: no DMA outstanding (the last wait was vmcnt(0)); every wave is past the last barrier ----------
  // Each wave stages 64 of its 128 rows at a time through its own LDS slice and re-reads 8 consecutive columns per
  // lane (16-byte stores), then applies the shared epilogue (epiw) / the LayerNorm forms of the tile kernel.
  float* st = reinterpret_cast<float*>(smem + wave * G::EW);
  constexpr int LPR = G::LPR, RPI = G::RPI, ELD = G::ELD;
  const int er = lane / LPR, ec = (lane - er * LPR) * 8;
  const int64_t gcol = n0 + wc * WCN + ec;
  const bool fullw = gcol + 8 <= N;
  float bias8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (p.bias && p.dact == ICAP_ACT_NONE) {
#pragma unroll
    for (int e = 0; e < 8; ++e) bias8[e] = gcol + e < N ? p.bias[gcol + e] : 0.f;
  }
  float wsum8[8];
  if constexpr (LNX == 2) {
#pragma unroll
    for (int e = 0; e < 8; ++e) wsum8[e] = gcol + e < N ? p.ln_wsum[gcol + e] : 0.f;
  }
  const uint64_t seed = drop_thresh != 0u ? eff_seed(p.seed, p.seed_ptr) : 0ull;
#pragma unroll
  for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 2 * NJ; ++nj)
#pragma unroll
        for (int v = 0; v < 4; ++v) st[(mi * 16 + fg * 4 + v) * ELD + nj * 16 + fr] = acc[qm * 4 + mi][nj][v];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll 2
    for (int it = 0; it < 64 / RPI; ++it) {
      const int row = it * RPI + er;
      const int brow = wr * 128 + qm * 64 + row;  // row within the block tile
      const int64_t grow = m0 + brow;
      float x[8];
      const float4 v0 = *reinterpret_cast<const float4*>(st + row * ELD + ec);
      const float4 v1 = *reinterpret_cast<const float4*>(st + row * ELD + ec + 4);
      x[0] = v0.x; x[1] = v0.y; x[2] = v0.z; x[3] = v0.w;
      x[4] = v1.x; x[5] = v1.y; x[6] = v1.z; x[7] = v1.w;
      const bool ok = grow < Mv && gcol < N;
      if constexpr (LNX == 2) {  // rstd (A.B^T - mean wsum); the host passed bias = b + W . beta
        const float mean = lnr[2 * brow], rs = lnr[2 * brow + 1];
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = rs * (x[e] - mean * wsum8[e]);
      }
      if (ok) epiw<TC, 8, AK>(p, grow, gcol, x, bias8, fullw, seed, drop_thresh, inv_keep);
      if constexpr (LNX == 1) {
        // producer: (mean, M2) of the STORED (rounded) values over this row's 32-column group = 4 lanes x 8
        float xr[8], sm = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          xr[e] = ok ? bf2f(f2bf(x[e])) : 0.f;
          sm += xr[e];
        }
        sm += __shfl_xor(sm, 1, 64);
        sm += __shfl_xor(sm, 2, 64);
        const float mg = sm * (1.f / 32.f);
        float q2 = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = xr[e] - mg;
          q2 += d * d;
        }
        q2 += __shfl_xor(q2, 1, 64);
        q2 += __shfl_xor(q2, 2, 64);
        if (ok && (lane & 3) == 0)
          reinterpret_cast<float2*>(p.ln_stats_out)[grow * (N >> 5) + (gcol >> 5)] = make_float2(mg, q2);
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
}
#undef G8P_RD

// host side: the forms the plan may pick (gemm.hip gemm8p_ok); BN 128 or 256
int gemm8p_launch(const icap_gemm_args& p, int bn, int actk, uint32_t thr, float inv_keep, hipStream_t s) {
  const int tiles_m = (int)((p.M + 255) / 256), tiles_n = (int)((p.N + bn - 1) / bn);
  const dim3 grid((unsigned)(tiles_m * tiles_n)), block(512);
#define G8P_GO(TC, BNV, A) hipLaunchKernelGGL((gemm8p_kernel<TC, BNV, A>), grid, block, 0, s, p, tiles_n, thr, inv_keep)
#define G8P_ACT(TC, BNV)                                                                                  \
  switch (actk) {                                                                                        \
    case ACT_OFF: G8P_GO(TC, BNV, ACT_OFF); break;                                                       \
    case ACT_FWD + ICAP_ACT_GELU_NEW: G8P_GO(TC, BNV, ACT_FWD + ICAP_ACT_GELU_NEW); break;               \
    case ACT_BWD + ICAP_ACT_GELU_NEW: G8P_GO(TC, BNV, ACT_BWD + ICAP_ACT_GELU_NEW); break;               \
    case ACT_LNS: G8P_GO(TC, BNV, ACT_LNS); break;                                                       \
    case ACT_LNF: G8P_GO(TC, BNV, ACT_LNF); break;                                                       \
    case ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW: G8P_GO(TC, BNV, ACT_LNF + ACT_FWD + ICAP_ACT_GELU_NEW); break; \
    default: G8P_GO(TC, BNV, ACT_ANY); break;                                                            \
  }
  if (p.c_dtype == ICAP_BF16) {
    if (bn == 128) { G8P_ACT(bf16_t, 128) } else { G8P_ACT(bf16_t, 256) }
  } else {
    if (bn == 128) { G8P_ACT(float, 128) } else { G8P_ACT(float, 256) }
  }
#undef G8P_ACT
#undef G8P_GO
  return check_launch("icap_gemm(8-phase)");
}

}  // namespace icap

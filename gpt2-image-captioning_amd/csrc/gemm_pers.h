// The persistent split-role GEMM with an overlapped epilogue (round 6; variant 30, gemm_tile_pers.hip).
// C[M,N] = epi(alpha * A[M,K] . B[N,K]^T) for bf16 row-major operands, one K range per tile, every epilogue form of
// the tile kernels (gemm_tile.h), bitwise equal to them.
//
// The split-role ring of gemm_tile.h (ROLES) runs one tile per CU at a time, and its epilogue runs on the MFMA waves
// after their last k-step: for products of more than one round of tiles each CU pays prologue + main loop + epilogue
// per tile in series (3584 x 3072 x 768 on 96 x 128 tiles: 4 tiles per CU, 4 x (1.7 + 4.8 + 2-5) us). Here a block
// of 12 waves walks its tiles with three roles:
//   waves 0-3   MFMA: the 2 x 2 wave grid of 48 x 64 accumulators (96 x 128 tiles); after a tile's last k-step they
//               write the fp32 accumulators to an LDS C buffer and go straight on to the next tile, whose first
//               stages the loaders have already landed;
//   waves 4-7   loaders: LDS-DMA of the NST-stage ring, one continuous stream of k-steps across the block's tiles;
//   waves 8-11  epilogue: while the MFMA waves run tile j's k-steps, they apply tile j-1's epilogue from the C buffer
//               a slice of rows per k-step (bias / activation / aux / dact / residual / dropout / LayerNorm producer /
//               consumer: the tile kernels' arithmetic, epiw), prefetch tile j's residual / dact_src rows into
//               registers, and (LayerNorm consumer) build tile j's row-statistics table.
// Every wave passes the same barriers: B_0, then per tile one per k-step (B_g: the loaders' stage g landed, the MFMA
// waves' reads of stage g - 1 retired, the epilogue waves' slice before it done) and one after the C buffer is written
// (C_j). The epilogue of tile j-1 is done by the last k-step barrier of tile j, so the C buffer is free when the MFMA
// waves write tile j; the last tile's epilogue runs after C_{J-1}, once the other roles have left.
#pragma once
#include "gemm_tile.h"

// (diagnostic build, make stamps) per-block timestamps into icap_gemm_args.diag_stamps, 8 per block: [0] tiles of
// the block, [1] start, [2] the MFMA waves past B_0, [3..6] the MFMA waves past C_0 .. C_3, [7] the epilogue waves done
#ifdef ICAP_STAMPS
#define ICAP_PSTAMP(i, who, v)                                                                                   \
  do {                                                                                                         \
    if (p.diag_stamps && threadIdx.x == (who)) p.diag_stamps[(int64_t)blockIdx.x * 8 + (i)] = (uint64_t)(v);   \
  } while (0)
#else
#define ICAP_PSTAMP(i, who, v) do {} while (0)
#endif

namespace icap {

// LDS bytes of the persistent kernel: NST ring stages, the fp32 C buffer (rows padded by 4 floats), two LayerNorm row
// tables and two column tables (bias, LayerNorm wsum) — tile parity
__host__ __device__ constexpr int pers_lds_bytes(int nst, int bm, int bn) {
  return nst * (bm + bn) * GROWB + bm * (bn + 4) * 4 + 2 * 2 * bm * 4 + 2 * 2 * bn * 4;
}

template <typename TC, int NST, int TM, int TN, int ACT>
__global__ __launch_bounds__(768, 3) void gemm_pers_kernel(icap_gemm_args p, int tiles_n, int nk, uint32_t drop_thresh,
                                                           float inv_keep) {
  constexpr int WM = 2, WN = 2, NW = 4, NLW = 4;
  constexpr int BM = 16 * WM * TM, BN = 16 * WN * TN;
  constexpr int STB = (BM + BN) * GROWB;
  constexpr int CLD = BN + 4;             // fp32 row stride of the C buffer
  constexpr int AK = ACT & 0xFF;
  constexpr int LNX = ACT >> 8;
  constexpr int ES = 2, EPC = 8, BKE = 64;  // bf16: 16-byte chunks of 8, 64 K per stage
  constexpr int EW = 8;                     // epilogue columns per lane
  constexpr int LPR = BN / EW;              // lanes per row
  constexpr int RPI = 64 / LPR;             // rows per wave instruction
  constexpr int RG = BM / RPI;              // row groups of a tile
  constexpr int GQ = RG / 4;                // row groups per epilogue wave
  static_assert(64 % LPR == 0 && RG % 4 == 0, "pers: epilogue row groups");
  static_assert(pers_lds_bytes(NST, BM, BN) <= 160 * 1024, "pers: LDS");
  constexpr int P = (BM + BN) / (8 * NLW), PA = BM / (8 * NLW);
  static_assert((BM + BN) % (8 * NLW) == 0 && BM % (8 * NLW) == 0 && NST >= 3 && (NST - 2) * P < 64, "pers: ring");
  __shared__ __attribute__((aligned(16))) char smem[pers_lds_bytes(NST, BM, BN)];
  float* cbuf = reinterpret_cast<float*>(smem + NST * STB);
  float* lnr0 = cbuf + BM * CLD;  // two tables of (mean, rstd) per row: tile parity
  float* colt0 = lnr0 + 2 * 2 * BM;  // two tables of [bias; wsum] per column: tile parity

  int tid = threadIdx.x;
  asm volatile("" : "+v"(tid));
  const int lane = tid & 63, wave = tid >> 6;
  const int64_t M = p.M, N = p.N, K = p.K;
  const int64_t Mv = p.m_dev && (int64_t)*p.m_dev < M ? (int64_t)*p.m_dev : M;
  const int tiles_mv = (int)((Mv + BM - 1) / BM);
  const int nlive = tiles_mv * tiles_n;
  const int G = (int)gridDim.x;
  const int J = (int)blockIdx.x < nlive ? (nlive - 1 - (int)blockIdx.x) / G + 1 : 0;  // this block's tiles
  // tile j of this block -> (m0, n0): the gemm_body XCD remap over the live tiles (G is a multiple of 8, so every
  // tile of a block sits on the block's XCD: each XCD walks a contiguous range of tile ids), then tile ids in groups
  // of GM row tiles, column-major inside a group: the 32 tiles an XCD runs at once cover GM row panels x 32 / GM
  // column panels (3584 x 3072 x 768: 0.6 + 1.6 MB of operands) instead of one row panel x every column panel
  // (0.1 + 4.7 MB, more than the XCD's 4 MB L2)
  constexpr int GM = 4;
  auto tile_of = [&](int j, int64_t& m0, int64_t& n0) __attribute__((always_inline)) {
    const int bid = (int)blockIdx.x + j * G;
    const int xcd = bid & 7, q = nlive >> 3, r = nlive & 7;
    const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
    const int grp = wgid / (GM * tiles_n), in = wgid - grp * (GM * tiles_n);
    const int gr = tiles_mv - grp * GM < GM ? tiles_mv - grp * GM : GM;  // row tiles of this group
    const int tn = in / gr, tm = grp * GM + (in - tn * gr);
    m0 = (int64_t)tm * BM;
    n0 = (int64_t)tn * BN;
  };
  ICAP_PSTAMP(1, 0, ICAP_NOW());
  ICAP_PSTAMP(0, 0, J);
  const int lrow = lane >> 3;
  const int lchunk = ((lane & 7) ^ lrow) * EPC;
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>(smem);

  if (wave >= NW && wave < NW + NLW) {
    // ---------------- loaders ----------------
    const int lw = wave - NW;
    uint32_t voff[P];
#pragma unroll
    for (int i = 0; i < P; ++i) {
      const int qq = i * NLW + lw;
      const int row = (i < PA ? qq : qq - BM / 8) * 8 + lrow;
      voff[i] = (uint32_t)((int64_t)row * (i < PA ? p.lda : p.ldb) + lchunk) * ES;
    }
    int ji = 0, kti = 0;  // issue cursor: tile, k-step
    __amdgpu_buffer_rsrc_t ra, rb;
    auto set_tile = [&]() __attribute__((always_inline)) {
      int64_t m0 = 0, n0 = 0;
      if (ji < J) tile_of(ji, m0, n0);
      const int64_t mrows = Mv - m0 < BM ? Mv - m0 : BM, nrows = N - n0 < BN ? N - n0 : BN;
      ra = make_rsrc_u(reinterpret_cast<const char*>(p.A) + m0 * p.lda * ES,
                       ji < J ? (uint64_t)((mrows - 1) * p.lda + K) * ES : 0);
      rb = make_rsrc_u(reinterpret_cast<const char*>(p.B) + n0 * p.ldb * ES,
                       ji < J ? (uint64_t)((nrows - 1) * p.ldb + K) * ES : 0);
    };
    set_tile();
    auto issue = [&](int slot) __attribute__((always_inline)) {
      const bool live = ji < J;
      const int64_t k0 = live ? (int64_t)kti * BKE : 0;
      const uint32_t kb = (uint32_t)(k0 * ES);
      const bool kin = live && k0 + lchunk < K;
#pragma unroll
      for (int i = 0; i < P; ++i) {
        const uint32_t lds = __builtin_amdgcn_readfirstlane(sbase + (uint32_t)(slot * STB + (i * NLW + lw) * 1024));
        dma16a(i < PA ? ra : rb, lds, kin ? voff[i] + kb : OOB);
      }
      if (live && ++kti == nk) {
        kti = 0;
        ++ji;
        set_tile();
      }
    };
#pragma unroll
    for (int s = 0; s < NST - 1; ++s) issue(s);
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * P) : "memory");
    __builtin_amdgcn_s_barrier();  // B_0
    const int GS = J * nk;
    for (int g = 0; g < GS; ++g) {
      issue((g + NST - 1) % NST);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"((NST - 2) * P) : "memory");  // stage g + 1 landed
      __builtin_amdgcn_s_barrier();                                        // B_{g+1}
      if ((g + 1) % nk == 0) __builtin_amdgcn_s_barrier();                 // C_j
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the zero stages past the last tile, before the block ends
    return;
  }

  if (wave < NW) {
    // ---------------- MFMA waves ----------------
    const int wm = wave / WN, wn = wave - wm * WN;
    const int fr = lane & 15, fg = lane >> 4;
    uint32_t la[2], lb[2];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint32_t sw = (uint32_t)(((ks * 4 + fg) ^ (fr & 7)) << 4);
      la[ks] = (uint32_t)((wm * 16 * TM + fr) * GROWB) + sw;
      lb[ks] = (uint32_t)((wn * 16 * TN + fr) * GROWB) + sw;
    }
    typedef frag_u32x4_t u32x4_t;
    u32x4_t fa0[TM], fb0[TN], fa1[TM], fb1[TN];
    auto rd = [&](u32x4_t(&fa)[TM], u32x4_t(&fb)[TN], uint32_t a, uint32_t b) __attribute__((always_inline)) {
      lds_frags<0, TM, 0>::run(fa, a);
      lds_frags<0, TN, BM * GROWB>::run(fb, b);
    };
    auto retire = [&](u32x4_t(&fa)[TM], u32x4_t(&fb)[TN]) __attribute__((always_inline)) {
      __builtin_amdgcn_sched_barrier(0);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(fa[i]));
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(fb[j]));
      __builtin_amdgcn_sched_barrier(0);
    };
    f32x4_t acc[TM][TN];
    auto mm = [&](const u32x4_t(&fa)[TM], const u32x4_t(&fb)[TN]) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          mfma_chunk<bf16_t>(acc[i][j], __builtin_bit_cast(uint4, fa[i]), __builtin_bit_cast(uint4, fb[j]));
    };
    __builtin_amdgcn_s_barrier();  // B_0
    __builtin_amdgcn_sched_barrier(0);
    ICAP_PSTAMP(2, 0, ICAP_NOW());
    for (int jt = 0; jt < J; ++jt) {
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      const int g0 = jt * nk;
      {
        const uint32_t s0 = sbase + (uint32_t)((g0 % NST) * STB);
        rd(fa0, fb0, s0 + la[0], s0 + lb[0]);
      }
      for (int kt = 0; kt < nk; ++kt) {
        const int g = g0 + kt;
        const uint32_t sb = sbase + (uint32_t)((g % NST) * STB);
        retire(fa0, fb0);
        rd(fa1, fb1, sb + la[1], sb + lb[1]);
        mm(fa0, fb0);
        retire(fa1, fb1);
        __builtin_amdgcn_s_barrier();  // B_{g+1}
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 1 < nk) {
          const uint32_t sn = sbase + (uint32_t)(((g + 1) % NST) * STB);
          rd(fa0, fb0, sn + la[0], sn + lb[0]);
        }
        mm(fa1, fb1);
        __builtin_amdgcn_sched_barrier(0);
      }
      // the accumulators -> C buffer (free: the epilogue waves finished tile jt-1 before B_{g0+nk})
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int v = 0; v < 4; ++v)
            cbuf[(wm * 16 * TM + i * 16 + fg * 4 + v) * CLD + wn * 16 * TN + j * 16 + fr] = acc[i][j][v];
      __syncthreads();  // C_jt (also orders the LDS writes above before the epilogue waves' reads)
      if (jt < 4) ICAP_PSTAMP(3 + jt, 0, ICAP_NOW());
    }
    return;
  }

  // ---------------- epilogue waves ----------------
  const int ew = wave - NW - NLW;  // 0..3
  const int et = ew * 64 + lane;   // 0..255
  const int er = lane / LPR;
  const int ec = (lane - er * LPR) * EW;
  uint64_t seed = 0;
  if (drop_thresh != 0u) seed = eff_seed(p.seed, p.seed_ptr);
  typedef typename rawbf<EW>::T pre_t;
  const bf16_t* esrc = nullptr;
  int64_t eld = 0;
  bool want_pre = false;
  if constexpr (std::is_same<TC, bf16_t>::value) {
    if (AK >= ACT_BWD || (AK == ACT_ANY && p.dact != ICAP_ACT_NONE)) {
      esrc = reinterpret_cast<const bf16_t*>(p.dact_src);
      eld = p.ld_dact;
    } else if (p.resid) {
      esrc = reinterpret_cast<const bf16_t*>(p.resid);
      eld = p.ldr;
    }
    want_pre = esrc != nullptr && (eld % EW) == 0 && (reinterpret_cast<uintptr_t>(esrc) & 15) == 0 &&
               (p.ldc % EW) == 0 && (reinterpret_cast<uintptr_t>(p.C) & 15) == 0;
  }
  // (the LayerNorm consumer forms have no residual / dact_src operand in any product: no prefetch registers there, so
  // the row-statistics loads keep theirs)
  constexpr bool PRE = LNX != 2;
  if (!PRE) want_pre = false;
  pre_t preN[PRE ? GQ : 1], preC[PRE ? GQ : 1];  // this wave's prefetched rows of the tile being computed / stored
  // (row-group q of this wave = ew + 4 q: local rows (ew + 4 q) RPI + er)
  auto prefetch = [&](int64_t m0, int64_t n0) __attribute__((always_inline)) {
    const int64_t col = n0 + ec;
    if (PRE && want_pre && col + EW <= N) {
      static_for<0, PRE ? GQ : 0>([&](auto qc) {
        constexpr int q = decltype(qc)::value;
        const int64_t r0 = m0 + (ew + 4 * q) * RPI + er;
        const int64_t row = r0 < Mv ? r0 : Mv - 1;
        preN[q] = *reinterpret_cast<const pre_t*>(esrc + row * eld + col);
      });
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  // LayerNorm consumer: row statistics of tile j's A rows from the producer's (mean, M2) pairs, two threads per row
  // (the tile kernels' ln_prologue arithmetic), loads issued at the tile's first k-step, table written at its last
  constexpr int LNQ = 10;
  float4 lnv[LNX == 2 ? LNQ : 1];
  auto ln_load = [&](int64_t m0) __attribute__((always_inline)) {
    if constexpr (LNX == 2) {
      if (et < 2 * BM) {
        const int rr = et >> 1, hf = et & 1;
        const int64_t grow = m0 + rr < Mv ? m0 + rr : Mv - 1;
        const int Gp = (int)(K >> 5), nq = Gp >> 2;
        const float4* st = reinterpret_cast<const float4*>(p.ln_stats_in) + grow * (Gp >> 1) + hf * nq;
#pragma unroll
        for (int q = 0; q < LNQ; ++q)
          if (q < nq) lnv[q] = st[q];
      }
    }
  };
  auto ln_table = [&](int64_t m0, int64_t n0, float* lnr) __attribute__((always_inline)) {
    if constexpr (LNX == 2) {
      if (et < 2 * BM) {
        const int rr = et >> 1, hf = et & 1;
        const int Gp = (int)(K >> 5), nq = Gp >> 2;
        float sm = 0.f;
#pragma unroll
        for (int q = 0; q < LNQ; ++q)
          if (q < nq) sm += lnv[q].x + lnv[q].z;
        sm += __shfl_xor(sm, 1, 64);
        const float mean = sm / (float)Gp;
        float m2 = 0.f;
#pragma unroll
        for (int q = 0; q < LNQ; ++q)
          if (q < nq) {
            const float d0 = lnv[q].x - mean, d1 = lnv[q].z - mean;
            m2 += (lnv[q].y + 32.f * d0 * d0) + (lnv[q].w + 32.f * d1 * d1);
          }
        m2 += __shfl_xor(m2, 1, 64);
        const float rs = 1.f / sqrtf(m2 / (float)K + p.ln_eps);
        if (hf == 0) {
          lnr[2 * rr] = mean;
          lnr[2 * rr + 1] = rs;
          if (p.ln_mean_out && n0 == 0 && m0 + rr < Mv) {  // for the LayerNorm backward (one tile column)
            p.ln_mean_out[m0 + rr] = mean;
            p.ln_rstd_out[m0 + rr] = rs;
          }
        }
      }
    }
  };
  // row group q of this wave of the tile at (m0, n0), from the C buffer; pq: its prefetched residual / dact_src row
  auto store_group = [&](int64_t m0, int64_t n0, const float* lnr, const float* colt, int q, const pre_t* pq)
      __attribute__((always_inline)) {
    const int64_t col = n0 + ec;
    const bool fullw = col + EW <= N;
    float biasw[EW];
#pragma unroll
    for (int h = 0; h < EW / 4; ++h)
      *reinterpret_cast<float4*>(biasw + 4 * h) = *reinterpret_cast<const float4*>(colt + ec + 4 * h);
    const int lr = (ew + 4 * q) * RPI + er;  // 0..BM-1
    const int64_t row = m0 + lr;
    float x[EW];
#pragma unroll
    for (int h = 0; h < EW / 4; ++h)
      *reinterpret_cast<float4*>(x + 4 * h) = *reinterpret_cast<const float4*>(cbuf + lr * CLD + ec + 4 * h);
    const bool ok = row < Mv && col < N;
    if constexpr (LNX == 2) {
      const float mean = lnr[2 * lr], rs = lnr[2 * lr + 1];
      float wsumw[EW];
#pragma unroll
      for (int h = 0; h < EW / 4; ++h)
        *reinterpret_cast<float4*>(wsumw + 4 * h) = *reinterpret_cast<const float4*>(colt + BN + ec + 4 * h);
#pragma unroll
      for (int e = 0; e < EW; ++e) x[e] = rs * (x[e] - mean * wsumw[e]);
    }
    if (ok) epiw<TC, EW, AK>(p, row, col, x, biasw, fullw, seed, drop_thresh, inv_keep, (want_pre && fullw) ? pq : nullptr);
    if constexpr (LNX == 1) {
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
  // the column table of a tile: thread et loads one value at the tile's first k-step (bias for et < BN, the LayerNorm
  // consumer's wsum above), written to LDS at its last, so no chunk of the epilogue waits on a global load
  auto col_load = [&](int64_t n0) __attribute__((always_inline)) -> float {
    const int c = et < BN ? et : et - BN;
    const int64_t col = n0 + c;
    if (et < BN) return (p.bias && p.dact == ICAP_ACT_NONE && col < N) ? p.bias[col] : 0.f;
    if constexpr (LNX == 2) return (et < 2 * BN && col < N) ? p.ln_wsum[col] : 0.f;
    return 0.f;
  };
  // (the epilogue waves' barriers are compiler barriers too: no LDS or global access moves across them; they never
  // wait for their own stores)
  auto bar = [&]() __attribute__((always_inline)) {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };
  bar();  // B_0
  int64_t pm0 = 0, pn0 = 0;  // the tile whose accumulators the C buffer holds (tile jt - 1)
  int qn = 0;                // its next row group; preC[0] holds that group's prefetched row (a FIFO)
  float cv = 0.f;
  // jt = J: the last tile's remaining row groups, after the other roles have left (no barriers)
  for (int jt = 0; jt <= J; ++jt) {
    const bool cur = jt < J;
    int64_t m0 = 0, n0 = 0;
    if (cur) tile_of(jt, m0, n0);
    const int nch = cur ? nk : 1;
    for (int kt = 0; kt < nch; ++kt) {
      if (cur && kt == 0) {
        prefetch(m0, n0);
        ln_load(m0);
        cv = et < 2 * BN ? col_load(n0) : 0.f;
      }
#ifdef ICAP_PERS_NOEPI
      if (false) {  // (timing diagnostic only: the epilogue waves store nothing)
#else
      if (jt > 0) {
#endif
        const int q1 = cur ? (kt + 1) * GQ / nk : GQ;
        const int par = (jt - 1) & 1;
        for (; qn < q1; ++qn) {
          store_group(pm0, pn0, lnr0 + par * 2 * BM, colt0 + par * 2 * BN, qn, &preC[0]);
#pragma unroll
          for (int q = 0; q + 1 < (PRE ? GQ : 1); ++q) preC[q] = preC[q + 1];
        }
      }
      if (cur && kt == nk - 1) {
        ln_table(m0, n0, lnr0 + (jt & 1) * 2 * BM);
        if (et < 2 * BN) colt0[(jt & 1) * 2 * BN + et] = cv;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the tables, before the barrier (other waves read them)
      }
      if (cur) bar();  // B_{jt nk + kt + 1}
    }
    if (cur) {
      bar();  // C_jt: the C buffer holds tile jt
#pragma unroll
      for (int q = 0; q < (PRE ? GQ : 1); ++q) preC[q] = preN[q];
      pm0 = m0;
      pn0 = n0;
      qn = 0;
    }
  }
  ICAP_PSTAMP(7, 8 * 64, ICAP_NOW());
}

}  // namespace icap

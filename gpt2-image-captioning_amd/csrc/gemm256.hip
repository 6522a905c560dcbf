// 256x256-tile bf16 GEMM for gfx950: the 8-phase schedule (cdna_hip_programming.md §5 "The 256² 8-phase template",
// T2-T5) for the wide products of the train step (GPT-2 c_fc and its activation-gradient GEMM, QKV, CLIP fc1):
// C[M,N] = epi(alpha * A[M,K] . B[N,K]^T), both operands K-contiguous, C bf16 or f32.
//
// Geometry: 8 waves as 2 (M) x 4 (N); wave (wr, wc) owns rows wr*128 + [0,128) and columns wc*64 + [0,64) of the
// tile, as 8 x 4 MFMA 16x16x32 accumulators (128 VGPRs). K advances 64 per tile (BK).
//
// LDS: two K-tile buffers of 64 KiB. A K-tile is four 16 KiB half-tiles, each 128 LDS rows of 128 bytes (64 K):
//   h0 A-qm0: A rows {0..63} u {128..191}      (the first 64 rows of each wave-row's 128)
//   h1 B-qn0: B rows wc*64 + [0,32), wc = 0..3  (the first 32 columns of each wave-column's 64)
//   h2 B-qn1: B rows wc*64 + [32,64)
//   h3 A-qm1: A rows {64..127} u {192..255}
// with the 16-byte chunk index XOR-swizzled by (row & 7) (lds_off: conflict-free ds_read_b128 fragment reads);
// the LDS-DMA writes lane-linear 1 KiB pieces and the swizzle lives on the per-lane source address (rule 21).
//
// One K-tile = 4 phases, one output quadrant each (16 MFMAs per wave):
//   p0: read A(qm0) + B(qn0) fragments -> quadrant (qm0, qn0)
//   p1: read B(qn1)                     -> (qm0, qn1)
//   p2: read A(qm1)                     -> (qm1, qn1)
//   p3: no reads                        -> (qm1, qn0)
// and every phase is { ds_reads, one half-tile of LDS-DMA, [p3: counted vmcnt], s_barrier, lgkmcnt(0),
// setprio(1) 16 MFMA setprio(0), s_barrier }. Wave-row 1 runs one barrier behind wave-row 0 (one extra barrier
// after the prologue, balanced by row 0 after the loop), so on each SIMD one wave's MFMAs overlap the other's
// reads. Half-tile h of K-tile u is DMA'd at global phase 4u - 6 + h:
//   - RAW: phase 3 of tile u-1 waits with vmcnt(4) (the two half-tiles issued after tile u's last stay in
//     flight across the barrier) and tile u is read from the next phase on, after a barrier both rows passed
//     behind their waits;
//   - WAR: the half-tile it overwrites (tile u-2 in the same buffer) was last read at phase 4u-8 (h0, h1),
//     4u-7 (h2) or 4u-6 (h3): at least two phases earlier, which with the one-barrier stagger is what lets the
//     lagging row retire those reads (lgkmcnt(0)) before a barrier the issuing row has passed.
// Fragment reads are inline asm, so hipcc does not drain the DMA queue (vmcnt(0)) in front of them; every
// register an asm read writes is tied into the lgkmcnt wait that retires it.
//
// Epilogue: each wave stages its accumulators through LDS (two 64-row passes) and applies the shared epilogue
// (gemm_common.h epiw) on 8 consecutive columns per lane. Tiles are XCD-aware (the bijective remap of
// cdna_hip_programming.md §5: neighbouring tiles of one XCD share A row panels in its L2).
#include "gemm_common.h"

namespace icap {
namespace g256 {
constexpr int BM = 256, BN = 256;
constexpr int HT = 128 * GROWB;  // half-tile bytes
constexpr int TB = 4 * HT;       // one 64-deep K-tile
constexpr int ELD = 68;          // fp32 row stride of the epilogue staging (conflict-free ds_write_b32)
constexpr int EW = 64 * ELD * 4; // staging bytes per wave (64 rows x 64 columns)
constexpr int SMEM = (2 * TB > 8 * EW) ? 2 * TB : 8 * EW;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
}  // namespace g256

#define G256_RD(dst, addr, off) asm volatile("ds_read_b128 %0, %1 offset:" #off : "=v"(dst) : "v"(addr))

template <typename TC>
__global__ __launch_bounds__(512, 1) void gemm256_kernel(icap_gemm_args p, int tiles_n, uint32_t drop_thresh,
                                                        float inv_keep) {
  using namespace g256;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 2, wc = wave & 3;
  const int fr = lane & 15, fg = lane >> 4;
  const int G = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tm = wg / tiles_n, tn = wg - tm * tiles_n;
  const int64_t M = p.M, N = p.N, K = p.K;
  const int64_t m0 = (int64_t)tm * BM, n0 = (int64_t)tn * BN;
  const int64_t mr = M - m0 < BM ? M - m0 : BM, nr = N - n0 < BN ? N - n0 : BN;
  const int nk = (int)((K + 63) / 64);
  const bf16_t* Ag = reinterpret_cast<const bf16_t*>(p.A);
  const bf16_t* Bg = reinterpret_cast<const bf16_t*>(p.B);
  const __amdgpu_buffer_rsrc_t ra = make_rsrc_u(Ag + m0 * p.lda, (uint64_t)((mr - 1) * p.lda + K) * 2);
  const __amdgpu_buffer_rsrc_t rb = make_rsrc_u(Bg + n0 * p.ldb, (uint64_t)((nr - 1) * p.ldb + K) * 2);

  // ---- LDS-DMA: lane l of DMA piece (i, wave) fills LDS row lr = (8 i + wave) * 8 + l/8, slot l%8, which holds
  // source chunk c = slot ^ (lr & 7) = (l & 7) ^ (l >> 3) of tile row map_h(lr)
  const int c = (lane & 7) ^ (lane >> 3);
  uint32_t voff[4][2];
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int lr = (i * 8 + wave) * 8 + (lane >> 3);
      int trow;
      if (h == 0) trow = (lr & 63) + (lr >> 6) * 128;
      else if (h == 3) trow = (lr & 63) + (lr >> 6) * 128 + 64;
      else if (h == 1) trow = (lr >> 5) * 64 + (lr & 31);
      else trow = (lr >> 5) * 64 + 32 + (lr & 31);
      const int64_t ld = (h == 0 || h == 3) ? p.lda : p.ldb;
      voff[h][i] = (uint32_t)((trow * ld + c * 8) * 2);
    }
  auto issue = [&](auto hc, int u) __attribute__((always_inline)) {
    constexpr int H = decltype(hc)::value;
    if (u >= nk) return;  // block-uniform
    const int64_t k0 = (int64_t)u * 64;
    const bool kin = k0 + c * 8 < K;  // K % 8 == 0: a 16-byte chunk is wholly inside or outside
    char* dst = smem + (u & 1) * TB + H * HT;
    const uint32_t so = __builtin_amdgcn_readfirstlane((uint32_t)(k0 * 2));
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dma16s((H == 0 || H == 3) ? ra : rb, dst + (i * 8 + wave) * 1024, kin ? voff[H][i] : OOB, so);
  };

  // ---- fragment addressing: A rows wr*64 + mi*16 + fr of an A half, B rows wc*32 + nj*16 + fr of a B half
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>(smem);
  uint32_t la[2], lb[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const uint32_t sw = (uint32_t)(((ks * 4 + fg) ^ (fr & 7)) << 4);
    la[ks] = (uint32_t)((wr * 64 + fr) * GROWB) + sw;
    lb[ks] = (uint32_t)((wc * 32 + fr) * GROWB) + sw;
  }
  u32x4_t RA[2][4], RB0[2][2], RB1[2][2];
  f32x4_t acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto read_a = [&](uint32_t half_base) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint32_t a = half_base + la[ks];
      G256_RD(RA[ks][0], a, 0);
      G256_RD(RA[ks][1], a, 2048);
      G256_RD(RA[ks][2], a, 4096);
      G256_RD(RA[ks][3], a, 6144);
    }
  };
  auto read_b = [&](u32x4_t (&R)[2][2], uint32_t half_base) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const uint32_t a = half_base + lb[ks];
      G256_RD(R[ks][0], a, 0);
      G256_RD(R[ks][1], a, 2048);
    }
  };
  auto quad = [&](int am, int bn, u32x4_t (&RB)[2][2]) __attribute__((always_inline)) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 4; ++mi)
#pragma unroll
        for (int nj = 0; nj < 2; ++nj)
          mfma_chunk<bf16_t>(acc[am + mi][bn + nj], __builtin_bit_cast(uint4, RA[ks][mi]),
                             __builtin_bit_cast(uint4, RB[ks][nj]));
    __builtin_amdgcn_s_setprio(0);
  };
#define G256_WAIT_A_B(RB)                                                                                        \
  asm volatile("s_waitcnt lgkmcnt(0)"                                                                           \
               : "+v"(RA[0][0]), "+v"(RA[0][1]), "+v"(RA[0][2]), "+v"(RA[0][3]), "+v"(RA[1][0]), "+v"(RA[1][1]), \
                 "+v"(RA[1][2]), "+v"(RA[1][3]), "+v"(RB[0][0]), "+v"(RB[0][1]), "+v"(RB[1][0]), "+v"(RB[1][1]))
#define G256_WAIT_A()                                                                                            \
  asm volatile("s_waitcnt lgkmcnt(0)"                                                                           \
               : "+v"(RA[0][0]), "+v"(RA[0][1]), "+v"(RA[0][2]), "+v"(RA[0][3]), "+v"(RA[1][0]), "+v"(RA[1][1]), \
                 "+v"(RA[1][2]), "+v"(RA[1][3]))
#define G256_WAIT_B(RB) \
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(RB[0][0]), "+v"(RB[0][1]), "+v"(RB[1][0]), "+v"(RB[1][1]))
#define G256_FENCE() __builtin_amdgcn_sched_barrier(0)

  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;

  // prologue: tile 0 and the first two half-tiles of tile 1 in flight; wait for tile 0
  issue(I0{}, 0); issue(I1{}, 0); issue(I2{}, 0); issue(I3{}, 0);
  issue(I0{}, 1); issue(I1{}, 1);
  G256_FENCE();
  if (nk >= 2) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  // wave-row 1 runs one barrier behind wave-row 0: on every SIMD (one wave of each row) one wave's MFMAs overlap
  // the other's fragment reads and DMA issue
  if (wr == 1) __builtin_amdgcn_s_barrier();
  G256_FENCE();

  for (int t = 0; t < nk; ++t) {
    const uint32_t tb = sbase + (uint32_t)((t & 1) * TB);
    // p0: (qm0, qn0); DMA tile t+1 h2
    read_a(tb + 0 * HT);
    read_b(RB0, tb + 1 * HT);
    G256_FENCE();
    issue(I2{}, t + 1);
    G256_FENCE();
    __builtin_amdgcn_s_barrier();
    G256_WAIT_A_B(RB0);
    G256_FENCE();
    quad(0, 0, RB0);
    G256_FENCE();
    __builtin_amdgcn_s_barrier();
    G256_FENCE();
    // p1: (qm0, qn1); DMA tile t+1 h3
    read_b(RB1, tb + 2 * HT);
    G256_FENCE();
    issue(I3{}, t + 1);
    G256_FENCE();
    __builtin_amdgcn_s_barrier();
    G256_WAIT_B(RB1);
    G256_FENCE();
    quad(0, 2, RB1);
    G256_FENCE();
    __builtin_amdgcn_s_barrier();
    G256_FENCE();
    // p2: (qm1, qn1); DMA tile t+2 h0
    read_a(tb + 3 * HT);
    G256_FENCE();
    issue(I0{}, t + 2);
    G256_FENCE();
    __builtin_amdgcn_s_barrier();
    G256_WAIT_A();
    G256_FENCE();
    quad(4, 2, RB1);
    G256_FENCE();
    __builtin_amdgcn_s_barrier();
    G256_FENCE();
    // p3: (qm1, qn0); DMA tile t+2 h1; retire tile t+1 (tile t+2's two half-tiles stay in flight)
    issue(I1{}, t + 2);
    G256_FENCE();
    if (t + 2 < nk) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    G256_FENCE();
    quad(4, 0, RB0);
    G256_FENCE();
    __builtin_amdgcn_s_barrier();
    G256_FENCE();
  }
  if (wr == 0) __builtin_amdgcn_s_barrier();  // equal barrier counts: wave-row 0 waits for row 1's last phase
#undef G256_WAIT_A_B
#undef G256_WAIT_A
#undef G256_WAIT_B
#undef G256_FENCE

  // ---- epilogue: no DMA outstanding (the last wait was vmcnt(0)); every wave is past the last barrier ----------
  float* st = reinterpret_cast<float*>(smem + wave * EW);
  const int er = lane >> 3, ec = (lane & 7) * 8;
  const int64_t gcol = n0 + wc * 64 + ec;
  float bias8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (p.bias && p.dact == ICAP_ACT_NONE) {
#pragma unroll
    for (int e = 0; e < 8; ++e) bias8[e] = gcol + e < N ? p.bias[gcol + e] : 0.f;
  }
  const uint64_t seed = drop_thresh != 0u ? eff_seed(p.seed, p.seed_ptr) : 0ull;
#pragma unroll
  for (int qm = 0; qm < 2; ++qm) {
#pragma unroll
    for (int mi = 0; mi < 4; ++mi)
#pragma unroll
      for (int nj = 0; nj < 4; ++nj)
#pragma unroll
        for (int v = 0; v < 4; ++v) st[(mi * 16 + fg * 4 + v) * ELD + nj * 16 + fr] = acc[qm * 4 + mi][nj][v];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
      const int row = it * 8 + er;
      const int64_t grow = m0 + wr * 128 + qm * 64 + row;
      float x[8];
      const float4 v0 = *reinterpret_cast<const float4*>(st + row * ELD + ec);
      const float4 v1 = *reinterpret_cast<const float4*>(st + row * ELD + ec + 4);
      x[0] = v0.x; x[1] = v0.y; x[2] = v0.z; x[3] = v0.w;
      x[4] = v1.x; x[5] = v1.y; x[6] = v1.z; x[7] = v1.w;
      if (grow < M && gcol < N) epiw<TC, 8>(p, grow, gcol, x, bias8, gcol + 8 <= N, seed, drop_thresh, inv_keep);
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  }
}
#undef G256_RD

// host side (called from icap_gemm's plan in gemm.hip)
int gemm256_launch(const icap_gemm_args& p, uint32_t thr, float inv_keep, hipStream_t s) {
  const int tiles_m = (int)((p.M + 255) / 256), tiles_n = (int)((p.N + 255) / 256);
  const dim3 grid((unsigned)(tiles_m * tiles_n)), block(512);
  if (p.c_dtype == ICAP_BF16)
    hipLaunchKernelGGL((gemm256_kernel<bf16_t>), grid, block, 0, s, p, tiles_n, thr, inv_keep);
  else
    hipLaunchKernelGGL((gemm256_kernel<float>), grid, block, 0, s, p, tiles_n, thr, inv_keep);
  return check_launch("icap_gemm(256)");
}

}  // namespace icap

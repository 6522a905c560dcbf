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
#include "common.h"

namespace icap {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

constexpr int GBM = 128, GBN = 128, GROWB = 128, GNT = 256;
constexpr int STAGE_BYTES = (GBM + GBN) * GROWB;  // 32 KiB
constexpr int EPI_LD = 68;                         // fp32 row stride of the epilogue staging tile
constexpr uint32_t OOB = 0x80000000u;              // buffer offset beyond any num_records -> loads 0

__device__ __forceinline__ int lds_off(int row, int chunk) {
  return row * GROWB + ((chunk ^ (row & 7)) << 4);
}

template <typename TI>
__device__ __forceinline__ void mfma_chunk(f32x4_t& acc, const uint4& a, const uint4& b);

template <>
__device__ __forceinline__ void mfma_chunk<bf16_t>(f32x4_t& acc, const uint4& a, const uint4& b) {
  bf16x8_t av = __builtin_bit_cast(bf16x8_t, a);
  bf16x8_t bv = __builtin_bit_cast(bf16x8_t, b);
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(av, bv, acc, 0, 0, 0);
}
template <>
__device__ __forceinline__ void mfma_chunk<float>(f32x4_t& acc, const uint4& a, const uint4& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint64_t bytes) {
  const uint32_t n = bytes > 0x7fffffffull ? 0x7fffffffu : (uint32_t)bytes;
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)n, 0x00020000);
}

__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

template <typename T> struct vec4io;
template <> struct vec4io<float> {
  static __device__ __forceinline__ void ld(const float* p, float v[4]) { io<float>::ld4(p, v); }
  static __device__ __forceinline__ void st(float* p, const float v[4]) { io<float>::st4(p, v); }
};
template <> struct vec4io<bf16_t> {
  static __device__ __forceinline__ void ld(const bf16_t* p, float v[4]) { io<bf16_t>::ld4(p, v); }
  static __device__ __forceinline__ void st(bf16_t* p, const float v[4]) { io<bf16_t>::st4(p, v); }
};

template <typename TI, typename TC>
__global__ __launch_bounds__(GNT, 2) void gemm_kernel(icap_gemm_args p, int tiles_n, uint32_t drop_thresh,
                                                     float inv_keep) {
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE_BYTES];
  constexpr int ES = sizeof(TI);
  constexpr int EPC = 16 / ES;         // elements per 16-byte chunk
  constexpr int BKE = GROWB / ES;      // K elements per stage

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // bijective XCD-aware remap: blocks sharing an XCD get consecutive tiles
  // (consecutive tiles share the A row panel).
  const int bid = blockIdx.x, nwg = gridDim.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tm = wgid / tiles_n, tn = wgid - tm * tiles_n;
  const int64_t m0 = (int64_t)tm * GBM, n0 = (int64_t)tn * GBN;

  const int64_t M = p.M, N = p.N, K = p.K;
  // tile-relative buffer descriptors: rows past M / N fall beyond num_records and load zeros
  const char* Ab = reinterpret_cast<const char*>(p.A) + m0 * p.lda * ES;
  const char* Bb = reinterpret_cast<const char*>(p.B) + n0 * p.ldb * ES;
  const int64_t mrows = M - m0 < GBM ? M - m0 : GBM;
  const int64_t nrows = N - n0 < GBN ? N - n0 : GBN;
  const __amdgpu_buffer_rsrc_t ra_rsrc = make_rsrc(Ab, (uint64_t)((mrows - 1) * p.lda + K) * ES);
  const __amdgpu_buffer_rsrc_t rb_rsrc = make_rsrc(Bb, (uint64_t)((nrows - 1) * p.ldb + K) * ES);
  // LDS-DMA staging (buffer_load_dwordx4 ... lds): one wave-instruction writes 1 KiB = 8 LDS rows of
  // 128 B linearly (lane l -> row l>>3, physical chunk l&7). The XOR swizzle therefore goes on the SOURCE:
  // physical chunk pc of row r holds logical K-chunk pc ^ (r & 7) (cdna_hip_programming.md §5.4 rule 21).
  // Wave w stages rows [32w, 32w+32) of A and of B: 4 + 4 instructions per stage, no VGPR round trip.
  const int lrow = lane >> 3;
  const int lchunk = ((lane & 7) ^ lrow) * EPC;  // logical K offset (elements) of this lane's 16 B
  uint32_t a_off[4], b_off[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = wave * 32 + i * 8 + lrow;
    a_off[i] = (uint32_t)((row * p.lda + lchunk) * ES);
    b_off[i] = (uint32_t)((row * p.ldb + lchunk) * ES);
  }
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  auto load_stage = [&](int64_t k0, int s) {
    const uint32_t kb = (uint32_t)(k0 * ES);
    const bool kin = k0 + lchunk < K;
    char* As = smem + s * STAGE_BYTES;
    char* Bs = As + GBM * GROWB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r0 = wave * 32 + i * 8;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra_rsrc, (lds_ptr_t)(As + r0 * GROWB), 16, kin ? a_off[i] + kb : OOB,
                                               0, 0, 0);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rb_rsrc, (lds_ptr_t)(Bs + r0 * GROWB), 16, kin ? b_off[i] + kb : OOB,
                                               0, 0, 0);
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((K + BKE - 1) / BKE);
  load_stage(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const char* As = smem + cur * STAGE_BYTES;
    const char* Bs = As + GBM * GROWB;
    // all fragment reads of this stage first: hipcc waits vmcnt(0) before any LDS read that follows an
    // LDS-DMA issue, so the next stage's DMA is issued only after the reads (and overlaps the MFMAs)
    uint4 af[2][4], bfr[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fg;
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = *reinterpret_cast<const uint4*>(As + lds_off(wm * 64 + i * 16 + fr, ch));
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[ks][j] = *reinterpret_cast<const uint4*>(Bs + lds_off(wn * 64 + j * 16 + fr, ch));
    }
    // the other buffer was last read in iteration kt-1, which every wave finished before the barrier below
    if (kt + 1 < nk) load_stage((int64_t)(kt + 1) * BKE, cur ^ 1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) mfma_chunk<TI>(acc[i][j], af[ks][i], bfr[ks][j]);
    // keep the MFMAs above the wait: they are register-only, so without this fence hipcc sinks them below the
    // vmcnt/barrier and the DMA is waited for right after it is issued (cdna_hip_programming.md §5.4 rule 18)
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of stage kt+1 has landed
    __syncthreads();                                      // ... and every other wave's
  }

  // ---- epilogue (LDS-staged, 4 columns per lane) ----
  TC* C = reinterpret_cast<TC*>(p.C);
  TC* aux = reinterpret_cast<TC*>(p.aux);
  const TC* resid = reinterpret_cast<const TC*>(p.resid);
  const TC* dsrc = reinterpret_cast<const TC*>(p.dact_src);
  const bool use_drop = drop_thresh != 0u;
  const uint64_t seed = use_drop ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  float* cs = reinterpret_cast<float*>(smem) + wave * (32 * EPI_LD);
  const int er = lane >> 4;         // row within a 4-row group
  const int ec = (lane & 15) * 4;   // first of this lane's 4 columns in the 64-column wave tile
  const int64_t col = n0 + wn * 64 + ec;
  float bias4[4] = {0.f, 0.f, 0.f, 0.f};
  if (p.bias && p.dact == ICAP_ACT_NONE) {
#pragma unroll
    for (int e = 0; e < 4; ++e) bias4[e] = (col + e < N) ? p.bias[col + e] : 0.f;
  }
  const bool full4 = (col + 4 <= N) && ((p.ldc & 3) == 0);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // stage rows [32h, 32h+32) of this wave's 64x64 accumulator tile
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) cs[(ii * 16 + fg * 4 + v) * EPI_LD + j * 16 + fr] = acc[2 * h + ii][j][v];
    __syncthreads();
#pragma unroll 2
    for (int t = 0; t < 8; ++t) {
      const int lr = t * 4 + er;  // 0..31
      const int64_t row = m0 + wm * 64 + h * 32 + lr;
      float x[4];
      *reinterpret_cast<float4*>(x) = *reinterpret_cast<const float4*>(cs + lr * EPI_LD + ec);
      if (row < M) {
        const uint64_t didx = p.offset + (uint64_t)(row * N + col);
        float a4[4], r4[4], c4[4];
        if (p.dact != ICAP_ACT_NONE) {
          if (full4 && (p.ld_dact & 3) == 0) vec4io<TC>::ld(dsrc + row * p.ld_dact + col, a4);
          else for (int e = 0; e < 4; ++e) a4[e] = (col + e < N) ? io<TC>::ld(dsrc + row * p.ld_dact + col + e) : 0.f;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float y = p.alpha * x[e];
            if (use_drop) y *= drop_scale(seed, didx + e, drop_thresh, inv_keep);
            x[e] = y * act_bwd(p.dact, a4[e]);
          }
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) x[e] = p.alpha * x[e] + bias4[e];
          if (p.act != ICAP_ACT_NONE || aux) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const float y = act_fwd(p.act, x[e]);
              a4[e] = (p.act == ICAP_ACT_TANH) ? y : x[e];
              x[e] = y;
            }
            if (aux) {
              if (full4 && (p.ldaux & 3) == 0) vec4io<TC>::st(aux + row * p.ldaux + col, a4);
              else for (int e = 0; e < 4; ++e) if (col + e < N) io<TC>::st(aux + row * p.ldaux + col + e, a4[e]);
            }
          }
          if (use_drop) {
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] *= drop_scale(seed, didx + e, drop_thresh, inv_keep);
          }
          if (resid) {
            if (full4 && (p.ldr & 3) == 0) vec4io<TC>::ld(resid + row * p.ldr + col, r4);
            else for (int e = 0; e < 4; ++e) r4[e] = (col + e < N) ? io<TC>::ld(resid + row * p.ldr + col + e) : 0.f;
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] += r4[e];
          }
        }
        TC* cp = C + row * p.ldc + col;
        if (full4) {
          if (p.beta != 0.f) {
            vec4io<TC>::ld(cp, c4);
#pragma unroll
            for (int e = 0; e < 4; ++e) x[e] += p.beta * c4[e];
          }
          vec4io<TC>::st(cp, x);
        } else {
          for (int e = 0; e < 4; ++e)
            if (col + e < N) io<TC>::st(cp + e, p.beta != 0.f ? x[e] + p.beta * io<TC>::ld(cp + e) : x[e]);
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace icap

using namespace icap;

extern "C" int icap_gemm(const icap_gemm_args* a, void* stream) {
  ICAP_REQUIRE(a != nullptr, "icap_gemm: null args");
  const icap_gemm_args& p = *a;
  ICAP_REQUIRE(p.M >= 0 && p.N >= 0 && p.K >= 0, "icap_gemm: negative size");
  if (p.M == 0 || p.N == 0) return ICAP_OK;
  ICAP_REQUIRE(p.A && p.B && p.C, "icap_gemm: null operand");
  ICAP_REQUIRE(p.in_dtype == ICAP_F32 || p.in_dtype == ICAP_BF16, "icap_gemm: bad in_dtype");
  ICAP_REQUIRE(p.c_dtype == ICAP_F32 || p.c_dtype == ICAP_BF16, "icap_gemm: bad c_dtype");
  const int epc = p.in_dtype == ICAP_BF16 ? 8 : 4;
  ICAP_REQUIRE(p.K % epc == 0, "icap_gemm: K must be a multiple of 8 (bf16) / 4 (f32)");
  ICAP_REQUIRE(p.lda % epc == 0 && p.ldb % epc == 0, "icap_gemm: lda/ldb must be multiples of 8 (bf16) / 4 (f32)");
  ICAP_REQUIRE(p.lda >= p.K && p.ldb >= p.K && p.ldc >= p.N, "icap_gemm: leading dimension too small");
  ICAP_REQUIRE((reinterpret_cast<uintptr_t>(p.A) & 15) == 0 && (reinterpret_cast<uintptr_t>(p.B) & 15) == 0,
               "icap_gemm: A and B must be 16-byte aligned");
  const int es = p.in_dtype == ICAP_BF16 ? 2 : 4;
  ICAP_REQUIRE((int64_t)GBM * p.lda * es < 0x7fffffffll && (int64_t)GBN * p.ldb * es < 0x7fffffffll,
               "icap_gemm: a 128-row operand panel must stay below 2 GiB");
  ICAP_REQUIRE(p.beta == 0.f || p.c_dtype == ICAP_F32, "icap_gemm: beta != 0 requires f32 C");
  ICAP_REQUIRE(p.dact == ICAP_ACT_NONE || p.dact_src != nullptr, "icap_gemm: dact requires dact_src");
  ICAP_REQUIRE(p.drop_p >= 0.f && p.drop_p < 1.f, "icap_gemm: drop_p out of range");
  const int64_t tiles_m = (p.M + GBM - 1) / GBM, tiles_n = (p.N + GBN - 1) / GBN;
  ICAP_REQUIRE(tiles_m * tiles_n < (1ll << 31), "icap_gemm: too many tiles");
  const uint32_t thr = p.drop_p > 0.f ? drop_threshold(p.drop_p) : 0u;
  const float inv_keep = p.drop_p > 0.f ? 1.f / (1.f - p.drop_p) : 1.f;
  dim3 grid((unsigned)(tiles_m * tiles_n)), block(GNT);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (p.in_dtype == ICAP_BF16) {
    if (p.c_dtype == ICAP_BF16)
      hipLaunchKernelGGL((gemm_kernel<bf16_t, bf16_t>), grid, block, 0, s, p, (int)tiles_n, thr, inv_keep);
    else
      hipLaunchKernelGGL((gemm_kernel<bf16_t, float>), grid, block, 0, s, p, (int)tiles_n, thr, inv_keep);
  } else {
    if (p.c_dtype == ICAP_BF16)
      hipLaunchKernelGGL((gemm_kernel<float, bf16_t>), grid, block, 0, s, p, (int)tiles_n, thr, inv_keep);
    else
      hipLaunchKernelGGL((gemm_kernel<float, float>), grid, block, 0, s, p, (int)tiles_n, thr, inv_keep);
  }
  return check_launch("icap_gemm");
}

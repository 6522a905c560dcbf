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
// (loads for stage k+1 are issued before the MFMAs of stage k: T14).
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
  const char* Ag = reinterpret_cast<const char*>(p.A);
  const char* Bg = reinterpret_cast<const char*>(p.B);

  // staging: each thread moves 4 chunks of A and 4 of B per stage
  uint4 ra[4], rb[4];
  auto load_stage = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + i * GNT;
      const int row = c >> 3, kc = c & 7;
      const int64_t gk = k0 + kc * EPC;
      const int64_t gm = m0 + row, gn = n0 + row;
      uint4 za = make_uint4(0, 0, 0, 0), zb = za;
      if (gm < M && gk < K) za = *reinterpret_cast<const uint4*>(Ag + (gm * p.lda + gk) * ES);
      if (gn < N && gk < K) zb = *reinterpret_cast<const uint4*>(Bg + (gn * p.ldb + gk) * ES);
      ra[i] = za; rb[i] = zb;
    }
  };
  auto store_stage = [&](int s) {
    char* As = smem + s * STAGE_BYTES;
    char* Bs = As + GBM * GROWB;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = tid + i * GNT;
      const int row = c >> 3, kc = c & 7;
      *reinterpret_cast<uint4*>(As + lds_off(row, kc)) = ra[i];
      *reinterpret_cast<uint4*>(Bs + lds_off(row, kc)) = rb[i];
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  const int nk = (int)((K + BKE - 1) / BKE);
  load_stage(0);
  store_stage(0);
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_stage((int64_t)(kt + 1) * BKE);
    const char* As = smem + cur * STAGE_BYTES;
    const char* Bs = As + GBM * GROWB;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fg;
      uint4 af[4], bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wm * 64 + i * 16 + fr;
        af[i] = *reinterpret_cast<const uint4*>(As + lds_off(row, ch));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wn * 64 + j * 16 + fr;
        bfr[j] = *reinterpret_cast<const uint4*>(Bs + lds_off(row, ch));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) mfma_chunk<TI>(acc[i][j], af[i], bfr[j]);
    }
    if (kt + 1 < nk) store_stage(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue ----
  TC* C = reinterpret_cast<TC*>(p.C);
  TC* aux = reinterpret_cast<TC*>(p.aux);
  const TC* resid = reinterpret_cast<const TC*>(p.resid);
  const TC* dsrc = reinterpret_cast<const TC*>(p.dact_src);
  const bool use_drop = drop_thresh != 0u;
  const uint64_t seed = use_drop ? eff_seed(p.seed, p.seed_ptr) : 0ull;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t col = n0 + wn * 64 + j * 16 + fr;
    if (col >= N) continue;
    const float bcol = p.bias ? p.bias[col] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int64_t row = m0 + wm * 64 + i * 16 + fg * 4 + v;
        if (row >= M) continue;
        float x = p.alpha * acc[i][j][v];
        if (p.dact != ICAP_ACT_NONE) {
          if (use_drop) x *= drop_scale(seed, p.offset + (uint64_t)(row * N + col), drop_thresh, inv_keep);
          x *= act_bwd(p.dact, io<TC>::ld(dsrc + row * p.ld_dact + col));
        } else {
          x += bcol;
          if (p.act != ICAP_ACT_NONE) {
            const float y = act_fwd(p.act, x);
            if (aux) io<TC>::st(aux + row * p.ldaux + col, p.act == ICAP_ACT_TANH ? y : x);
            x = y;
          } else if (aux) {
            io<TC>::st(aux + row * p.ldaux + col, x);
          }
          if (use_drop) x *= drop_scale(seed, p.offset + (uint64_t)(row * N + col), drop_thresh, inv_keep);
          if (resid) x += io<TC>::ld(resid + row * p.ldr + col);
        }
        TC* cp = C + row * p.ldc + col;
        if (p.beta != 0.f) x += p.beta * io<TC>::ld(cp);
        io<TC>::st(cp, x);
      }
    }
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

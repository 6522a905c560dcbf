// Shared pieces of the GEMM kernels (gemm.hip: tile / skinny kernels; gemm256.hip: the 256x256 8-phase
// kernel): MFMA chunk wrappers, buffer descriptors, LDS-DMA and buffer-load helpers, the XOR-swizzled LDS row
// layout, and the epilogue arithmetic every kernel applies (one formula, fixed contraction: bitwise-equal
// outputs across kernels that accumulate in the same order).
#pragma once

#include "common.h"

#include <type_traits>

namespace icap {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));
typedef int i32x8_t __attribute__((ext_vector_type(8)));

// OCP e4m3fn storage element of the MX block-scaled path (ICAP_FP8_MX): one byte, per-32-element E8M0 scales kept
// beside the data (icap_gemm_args.a_scale / b_scale)
struct fp8_t {
  uint8_t v;
};

// One block-scaled MFMA 16x16x128 (v_mfma_scale_f32_16x16x128_f8f6f4, e4m3 A and B). Lane map, measured
// (tools/microbench/mx_probe.hip + tools/mx_probe_check.py, profiles/r03_mx_probe_check.txt): lane l = (g = l >> 4,
// r = l & 15) supplies row r's bytes k = 16 g .. 16 g + 15 (operand bytes 0-15) and k = 64 + 16 g .. (bytes 16-31) —
// the bf16 16x16x32 kernel's chunk pattern {g, 4 + g} of a 128-byte row — and, in byte op_sel of its scale VGPR,
// the E8M0 scale of row r's 32-element block g (k = 32 g .. 32 g + 31), whichever lane holds that block's data.
__device__ __forceinline__ void mfma_mx(f32x4_t& acc, const i32x8_t& a, const i32x8_t& b, uint32_t sa, uint32_t sb) {
  acc = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, acc, 0, 0, 0, (int)sa, 0, (int)sb);
}
// the 32-byte MX operand of one lane from two 16-byte LDS chunks (written straight into the tuple's halves so the
// 8 registers are allocated adjacent: no copies before the MFMA)
__device__ __forceinline__ i32x8_t ld_mx_frag(const char* lo, const char* hi) {
  typedef int i32x4_t __attribute__((ext_vector_type(4)));
  i32x8_t v;
  v.lo = *reinterpret_cast<const i32x4_t*>(lo);
  v.hi = *reinterpret_cast<const i32x4_t*>(hi);
  return v;
}

// MX scale layout of an operand with R rows and K columns (K % 128 == 0): for 128-element K stage s and 64-row group
// g = row / 64, 256 bytes at ((s * ceil(R / 64) + g) * 16 + row % 16) * 16: 16 bytes per row % 16, holding for
// q = (row / 16) % 4 the 4 scale bytes of the stage's 32-element blocks (byte q * 4 + kb). One 16-byte load gives
// a lane the scales of the 4 rows i * 16 + r16 (i = 0..3) of a 64-row wave tile.
__host__ __device__ __forceinline__ int64_t mx_scale_off(int64_t R, int64_t row, int64_t kblock) {
  const int64_t rg = (R + 63) / 64, s = kblock >> 2;
  return ((s * rg + (row >> 6)) * 16 + (row & 15)) * 16 + ((row >> 4) & 3) * 4 + (kblock & 3);
}

constexpr int GBM = 128, GBN = 128, GROWB = 128, GNT = 256;  // default 128x128 tile, 128-byte LDS rows
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

// same, with the inputs forced into SGPRs (readfirstlane) so hipcc can prove the descriptor wave-uniform and
// emits no waterfall loop around the buffer ops (cdna_hip_programming.md T20)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc_u(const void* base, uint64_t bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes > 0x7fffffffull ? 0x7fffffffu : (uint32_t)bytes);
  void* pb = reinterpret_cast<void*>(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(pb, (short)0, (int)n, 0x00020000);
}

// 16-byte LDS-DMA of one wave: lane l's 16 bytes land at lds + 16 l
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t off) {
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(lds), 16, off, 0, 0, 0);
}

// same with the LDS destination as an integer byte address that the caller made wave-uniform (readfirstlane), so M0
// is written from an SGPR with no waterfall loop. (Not through a generic pointer built from that integer: a value of
// 0 — the first byte of LDS — would be cast to the LDS null, 0xffffffff.)
__device__ __forceinline__ void dma16a(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t off) {
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(uintptr_t)lds, 16, off, 0, 0, 0);
}

// same with a wave-uniform soffset (row / k offsets in SGPRs, one per-lane VGPR offset)
__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff, uint32_t soff) {
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(lds), 16, voff, soff, 0, 0);
}

__device__ __forceinline__ uint4 bload(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [I0, N)
template <int I, int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

// W consecutive elements (W = 4 or 8) as fp32, through one 8- or 16-byte access (bf16) or one / two float4 (f32)
template <typename T, int W> struct vecio;
template <int W> struct vecio<float, W> {
  static __device__ __forceinline__ void ld(const float* p, float v[W]) {
#pragma unroll
    for (int q = 0; q < W / 4; ++q) io<float>::ld4(p + 4 * q, v + 4 * q);
  }
  static __device__ __forceinline__ void st(float* p, const float v[W]) {
#pragma unroll
    for (int q = 0; q < W / 4; ++q) io<float>::st4(p + 4 * q, v + 4 * q);
  }
};
template <> struct vecio<bf16_t, 4> {
  static __device__ __forceinline__ void ld(const bf16_t* p, float v[4]) { io<bf16_t>::ld4(p, v); }
  static __device__ __forceinline__ void st(bf16_t* p, const float v[4]) { io<bf16_t>::st4(p, v); }
};
template <> struct vecio<bf16_t, 8> {
  static __device__ __forceinline__ void ld(const bf16_t* p, float v[8]) {
    const uint4 t = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q] = __uint_as_float(w[q] << 16);
      v[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void st(bf16_t* p, const float v[8]) {
    *reinterpret_cast<uint4*>(p) = make_uint4(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]), f2bf2(v[4], v[5]), f2bf2(v[6], v[7]));
  }
};
// raw bf16 vector of W elements (prefetched epilogue operands)
template <int W> struct rawbf;
template <> struct rawbf<4> { typedef uint2 T; };
template <> struct rawbf<8> { typedef uint4 T; };
__device__ __forceinline__ void unpack_bf16(const uint2 w, float v[4]) {
  v[0] = __uint_as_float(w.x << 16);
  v[1] = __uint_as_float(w.x & 0xffff0000u);
  v[2] = __uint_as_float(w.y << 16);
  v[3] = __uint_as_float(w.y & 0xffff0000u);
}
__device__ __forceinline__ void unpack_bf16(const uint4 w, float v[8]) {
  unpack_bf16(make_uint2(w.x, w.y), v);
  unpack_bf16(make_uint2(w.z, w.w), v + 4);
}

// The epilogue arithmetic, shared by every GEMM kernel (tile, split-K reduce, skinny, 256 x 256): one formula with a
// fixed contraction (explicit fma for alpha*acc + bias, no other fusing), so two kernels that accumulate a product
// in the same order store bitwise-identical outputs (tests/test_gemm256_gpu.py).
// The activation is a runtime argument: it is dispatched ONCE per W-element call, each case a straight run over the
// W elements. (A switch inside the element loop put every activation's code — libm tanhf / erff included — W times
// into every unrolled epilogue call site; any activated launch then executed through that code and paid for it in
// instruction fetch: 8320 x 3072 x 768 with relu 97 us vs 61 plain, tools/act_epilogue_probe.py.) The arithmetic
// per element is unchanged (act_fwd / act_bwd), so outputs are bitwise the same.
// backward form: x = alpha * acc * dropmask * act'(a)
// Activation kinds of an epilogue instantiation (template int ACT): ACT_OFF none (the host guarantees act == dact ==
// NONE), ACT_ANY the runtime dispatch below, ACT_FWD + a forward activation a only, ACT_BWD + a backward dact a only:
// the specialised forms compile a single straight run (no dispatch, none of the other activations' code, fewer live
// registers in the epilogue); the arithmetic per element is act_fwd / act_bwd in every form (bitwise the same).
constexpr int ACT_OFF = 0, ACT_ANY = 1, ACT_FWD = 16, ACT_BWD = 32;
// LayerNorm statistics hand-off of the tile kernels (icap_gemm_args.ln_stats_out / ln_stats_in), or-ed into the
// kernel's ACT template int above its activation kind: ACT_LNS = the producer writes (mean, M2) per row and 32-column
// group of C; ACT_LNF = the consumer folds the LayerNorm of its A operand into its epilogue.
constexpr int ACT_LNS = 256, ACT_LNF = 512;
template <int W, int ACT = ACT_ANY>
__device__ __forceinline__ void epi_bwd_math(const icap_gemm_args& p, float x[W], const float a[W], uint64_t seed,
                                             uint64_t didx, uint32_t drop_thresh, float inv_keep) {
#pragma clang fp contract(off)
  float y[W];
#pragma unroll
  for (int e = 0; e < W; ++e) {
    y[e] = p.alpha * x[e];
    if (drop_thresh != 0u) y[e] = y[e] * drop_scale(seed, didx + e, drop_thresh, inv_keep);
  }
  if constexpr (ACT >= ACT_BWD) {
#pragma unroll
    for (int e = 0; e < W; ++e) x[e] = y[e] * act_bwd(ACT - ACT_BWD, a[e]);
    return;
  }
  switch (p.dact) {
#define ICAP_DACT_CASE(A)                                              \
  case A:                                                              \
    _Pragma("unroll") for (int e = 0; e < W; ++e) x[e] = y[e] * act_bwd(A, a[e]); \
    break;
    ICAP_DACT_CASE(ICAP_ACT_GELU_NEW)
    ICAP_DACT_CASE(ICAP_ACT_RELU)
    ICAP_DACT_CASE(ICAP_ACT_QUICK_GELU)
    ICAP_DACT_CASE(ICAP_ACT_TANH)
    ICAP_DACT_CASE(ICAP_ACT_GELU_ERF)
#undef ICAP_DACT_CASE
    default:
#pragma unroll
      for (int e = 0; e < W; ++e) x[e] = y[e] * act_bwd(ICAP_ACT_NONE, a[e]);
  }
}
// forward form, first half: x = act(alpha * acc + bias); a = the aux value (pre-activation, or tanh output).
// ACT = false: an instantiation for launches without an activation (the host guarantees act == dact == NONE), so
// none of the activation code is compiled into that kernel (see gemm_kernel's ACT parameter).
template <int W, int ACT = ACT_ANY>
__device__ __forceinline__ void epi_fwd_act(const icap_gemm_args& p, float x[W], const float biasw[W], float a[W]) {
#pragma clang fp contract(off)
#pragma unroll
  for (int e = 0; e < W; ++e) x[e] = __builtin_fmaf(p.alpha, x[e], biasw[e]);
  if constexpr (ACT >= ACT_FWD && ACT < ACT_BWD) {
    constexpr int A = ACT - ACT_FWD;
#pragma unroll
    for (int e = 0; e < W; ++e) {
      const float y = act_fwd(A, x[e]);
      a[e] = (A == ICAP_ACT_TANH) ? y : x[e];
      x[e] = y;
    }
    return;
  }
  if (ACT == ACT_OFF || ACT >= ACT_BWD || __builtin_expect(p.act == ICAP_ACT_NONE, 1)) {  // no activation: short, first
    if (p.aux) {
#pragma unroll
      for (int e = 0; e < W; ++e) a[e] = x[e];
    }
    return;
  }
  switch (p.act) {
#define ICAP_ACT_CASE(A)                                              \
  case A:                                                             \
    _Pragma("unroll") for (int e = 0; e < W; ++e) {                   \
      const float y = act_fwd(A, x[e]);                               \
      a[e] = (A == ICAP_ACT_TANH) ? y : x[e];                         \
      x[e] = y;                                                       \
    }                                                                 \
    break;
    ICAP_ACT_CASE(ICAP_ACT_GELU_NEW)
    ICAP_ACT_CASE(ICAP_ACT_RELU)
    ICAP_ACT_CASE(ICAP_ACT_QUICK_GELU)
    ICAP_ACT_CASE(ICAP_ACT_TANH)
    ICAP_ACT_CASE(ICAP_ACT_GELU_ERF)
#undef ICAP_ACT_CASE
    default:
      break;
  }
}
// forward form, second half: x = x * dropmask (+ r)
template <int W>
__device__ __forceinline__ void epi_fwd_tail(float x[W], const float r[W], bool add_r, uint64_t seed, uint64_t didx,
                                             uint32_t drop_thresh, float inv_keep) {
#pragma clang fp contract(off)
  if (drop_thresh != 0u) {
#pragma unroll
    for (int e = 0; e < W; ++e) x[e] = x[e] * drop_scale(seed, didx + e, drop_thresh, inv_keep);
  }
  if (add_r) {
#pragma unroll
    for (int e = 0; e < W; ++e) x[e] = x[e] + r[e];
  }
}

// Epilogue of W consecutive columns [col, col+W) of row `row` (the order is the one include/icap.h documents).
// x: alpha-unscaled fp32 accumulators; biasw: bias[col..col+W-1] (0 past N); fullw: all W columns in range;
// W-wide vector access is used per operand where its leading dimension and base pointer are W-aligned.
// pre: optional prefetched raw bf16 vector of the epilogue's input operand at (row, col..) — dact_src in the
// backward form, resid in the forward form — loaded by the caller ahead of the LDS staging (fullw rows only).
template <typename TC, int W, int ACT = ACT_ANY>
__device__ __forceinline__ void epiw(const icap_gemm_args& p, int64_t row, int64_t col, float x[W],
                                     const float biasw[W], bool fullw, uint64_t seed, uint32_t drop_thresh,
                                     float inv_keep, const typename rawbf<W>::T* pre = nullptr) {
  const int64_t N = p.N;
  TC* C = reinterpret_cast<TC*>(p.C);
  TC* aux = reinterpret_cast<TC*>(p.aux);
  const TC* resid = reinterpret_cast<const TC*>(p.resid);
  const TC* dsrc = reinterpret_cast<const TC*>(p.dact_src);
  const uint64_t didx = p.offset + (uint64_t)(row * N + col);
  float a[W], r[W], c[W];
  // W-wide vector access needs the leading dimension AND the base pointer aligned to W elements (16 B suffices
  // for 8 f32: two float4)
  constexpr uintptr_t VA = (W * sizeof(TC) > 16 ? 16 : W * sizeof(TC)) - 1;
  auto vok = [&](int64_t ld, const void* ptr) { return (ld % W) == 0 && (reinterpret_cast<uintptr_t>(ptr) & VA) == 0; };
  fullw = fullw && vok(p.ldc, C);
  if (ACT >= ACT_BWD || (ACT == ACT_ANY && p.dact != ICAP_ACT_NONE)) {
    if (pre) unpack_bf16(*pre, a);
    else if (fullw && vok(p.ld_dact, dsrc)) vecio<TC, W>::ld(dsrc + row * p.ld_dact + col, a);
    else for (int e = 0; e < W; ++e) a[e] = (col + e < N) ? io<TC>::ld(dsrc + row * p.ld_dact + col + e) : 0.f;
    epi_bwd_math<W, ACT>(p, x, a, seed, didx, drop_thresh, inv_keep);
  } else {
    epi_fwd_act<W, ACT>(p, x, biasw, a);
    if (aux) {
      if (fullw && vok(p.ldaux, aux)) vecio<TC, W>::st(aux + row * p.ldaux + col, a);
      else for (int e = 0; e < W; ++e) if (col + e < N) io<TC>::st(aux + row * p.ldaux + col + e, a[e]);
    }
    if (resid) {
      if (pre) unpack_bf16(*pre, r);
      else if (fullw && vok(p.ldr, resid)) vecio<TC, W>::ld(resid + row * p.ldr + col, r);
      else for (int e = 0; e < W; ++e) r[e] = (col + e < N) ? io<TC>::ld(resid + row * p.ldr + col + e) : 0.f;
    }
    epi_fwd_tail<W>(x, r, resid != nullptr, seed, didx, drop_thresh, inv_keep);
  }
  TC* cp = C + row * p.ldc + col;
  if (fullw) {
    if (p.beta != 0.f) {
      vecio<TC, W>::ld(cp, c);
#pragma unroll
      for (int e = 0; e < W; ++e) x[e] += p.beta * c[e];
    }
    vecio<TC, W>::st(cp, x);
  } else {
    for (int e = 0; e < W; ++e)
      if (col + e < N) io<TC>::st(cp + e, p.beta != 0.f ? x[e] + p.beta * io<TC>::ld(cp + e) : x[e]);
  }
}

template <typename TC>
__device__ __forceinline__ void epi4(const icap_gemm_args& p, int64_t row, int64_t col, float x[4],
                                     const float bias4[4], bool full4, uint64_t seed, uint32_t drop_thresh,
                                     float inv_keep) {
  epiw<TC, 4>(p, row, col, x, bias4, full4, seed, drop_thresh, inv_keep);
}


}  // namespace icap

// Shared device helpers for the icap HIP library (gfx950 / CDNA4 only).
//
// Storage types: activations/weights are either fp32 or bf16 (raw 16-bit words);
// every kernel computes in fp32. Wave size is 64 (hard-coded, see
// /opt/skills/guides/cdna_hip_programming.md §1).
#pragma once

#include <hip/hip_runtime.h>

// Diagnostic build only (make stamps: -DICAP_STAMPS): A/B overrides of the kernel choice read from the process
// environment (tools/ab). The product library reads no environment variable: in it every choice is a function of
// the call's arguments and diag_env returns its default at compile time.
#ifdef ICAP_STAMPS
#include <cstdlib>
static inline int diag_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}
#else
static constexpr int diag_env(const char*, int dflt) { return dflt; }
#endif
#include <stdint.h>
#include <string>

#include "icap.h"

namespace icap {

typedef uint16_t bf16_t;

// ---- error reporting (thread-local, C-ABI icap_last_error) -------------------
void set_error(const std::string& msg);
int check_launch(const char* what);

#define ICAP_REQUIRE(cond, msg)                 \
  do {                                          \
    if (!(cond)) {                              \
      ::icap::set_error(std::string(msg));      \
      return ICAP_ERR_ARG;                      \
    }                                           \
  } while (0)

// ---- bf16 <-> f32 ------------------------------------------------------------
__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}
// round-to-nearest-even (gfx950 v_cvt_pk_bf16_f32); NaN stays NaN
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
// two floats -> packed bf16 pair (lo = a) in one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t f2bf2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){a, b}, bf16x2_t));
}

template <typename T> struct io;
template <> struct io<float> {
  static __device__ __forceinline__ float ld(const float* p) { return *p; }
  static __device__ __forceinline__ void st(float* p, float v) { *p = v; }
  // 4 consecutive elements
  static __device__ __forceinline__ void ld4(const float* p, float v[4]) {
    float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  }
  static __device__ __forceinline__ void st4(float* p, const float v[4]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  }
  // 8 consecutive elements (16-byte aligned)
  static __device__ __forceinline__ void ld8(const float* p, float v[8]) { ld4(p, v); ld4(p + 4, v + 4); }
  static __device__ __forceinline__ void st8(float* p, const float v[8]) { st4(p, v); st4(p + 4, v + 4); }
};
template <> struct io<bf16_t> {
  static __device__ __forceinline__ float ld(const bf16_t* p) { return bf2f(*p); }
  static __device__ __forceinline__ void st(bf16_t* p, float v) { *p = f2bf(v); }
  static __device__ __forceinline__ void ld4(const bf16_t* p, float v[4]) {
    uint2 t = *reinterpret_cast<const uint2*>(p);
    v[0] = __uint_as_float(t.x << 16); v[1] = __uint_as_float(t.x & 0xffff0000u);
    v[2] = __uint_as_float(t.y << 16); v[3] = __uint_as_float(t.y & 0xffff0000u);
  }
  static __device__ __forceinline__ void st4(bf16_t* p, const float v[4]) {
    *reinterpret_cast<uint2*>(p) = make_uint2(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]));
  }
  // 8 consecutive elements in one 16-byte access (16-byte aligned)
  static __device__ __forceinline__ void ld8(const bf16_t* p, float v[8]) {
    const uint4 t = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      v[2 * q] = __uint_as_float(w[q] << 16);
      v[2 * q + 1] = __uint_as_float(w[q] & 0xffff0000u);
    }
  }
  static __device__ __forceinline__ void st8(bf16_t* p, const float v[8]) {
    *reinterpret_cast<uint4*>(p) = make_uint4(f2bf2(v[0], v[1]), f2bf2(v[2], v[3]), f2bf2(v[4], v[5]), f2bf2(v[6], v[7]));
  }
};

// ---- wave reductions (64 lanes) ---------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// ---- counter-based dropout RNG -----------------------------------------------
// keep(idx) is a pure function of (seed, idx): forward and backward regenerate
// the same mask without storing it. 32-bit arithmetic only: (lo ^ s0) * golden
// + hi, xor s1, then the lowbias32 finaliser (Wellons) — three v_mul_lo_u32
// (quarter rate) per element instead of the twelve a 64-bit splitmix64 chain
// costs; dropout runs on every GPT-2 / mapper activation and attention prob of
// a train step (~0.7 G draws), where the 64-bit chain was ~1 ms of VALU a step.
// For a fixed seed the map idx -> hash is a bijection on idx < 2^32 (odd
// multiply, xor and the finaliser are all invertible), so no two elements of
// one tensor share a draw. tests/test_dropout_hash.py restates it in numpy.
__device__ __forceinline__ uint32_t hash32(uint64_t seed, uint64_t idx) {
  uint32_t x = (((uint32_t)idx ^ (uint32_t)seed) * 0x9E3779B9u + (uint32_t)(idx >> 32)) ^ (uint32_t)(seed >> 32);
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}
__device__ __forceinline__ uint64_t eff_seed(uint64_t seed, const uint64_t* ptr) {
  return ptr ? seed + (*ptr) * 0x9E3779B97F4A7C15ull : seed;
}
// returns 0 or 1/(1-p)
__device__ __forceinline__ float drop_scale(uint64_t seed, uint64_t idx, uint32_t thresh, float inv_keep) {
  return hash32(seed, idx) >= thresh ? inv_keep : 0.f;
}
inline uint32_t drop_threshold(float p) {
  double t = (double)p * 4294967296.0;
  if (t >= 4294967295.0) t = 4294967295.0;
  if (t < 0) t = 0;
  return (uint32_t)t;
}

// ---- activations -------------------------------------------------------------
__device__ __forceinline__ float act_fwd(int act, float x) {
  switch (act) {
    case ICAP_ACT_GELU_NEW: {
      // HF activations.py NewGELUActivation: 0.5x(1+tanh(sqrt(2/pi)(x+0.044715x^3)))
      // 0.5(1+tanh(u)) == sigmoid(2u): one v_exp + one v_rcp instead of a libm tanhf
      const float c2 = 2.f * 0.7978845608028654f;
      return x * __builtin_amdgcn_rcpf(1.f + __expf(-c2 * (x + 0.044715f * x * x * x)));
    }
    case ICAP_ACT_RELU: return x > 0.f ? x : 0.f;
    case ICAP_ACT_QUICK_GELU: return x * __builtin_amdgcn_rcpf(1.f + __expf(-1.702f * x));  // (v_rcp, not a full division)
    case ICAP_ACT_TANH: return tanhf(x);
    case ICAP_ACT_GELU_ERF: return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));  // HF ACT2FN["gelu"]
    default: return x;
  }
}
// derivative; `a` is the value stored by the forward as aux:
//   gelu_new / quick_gelu: pre-activation z;  relu: z or relu(z);  tanh: tanh(z)
__device__ __forceinline__ float act_bwd(int act, float a) {
  switch (act) {
    case ICAP_ACT_GELU_NEW: {
      // s = sigmoid(2u) = 0.5(1+tanh u);  d/da = s + a * 2s(1-s) * du/da
      const float c = 0.7978845608028654f;
      const float x2 = a * a;
      const float s = __builtin_amdgcn_rcpf(1.f + __expf(-2.f * c * (a + 0.044715f * x2 * a)));
      const float du = c * (1.f + 3.f * 0.044715f * x2);
      return s + 2.f * a * s * (1.f - s) * du;
    }
    case ICAP_ACT_RELU: return a > 0.f ? 1.f : 0.f;
    case ICAP_ACT_QUICK_GELU: {
      float s = 1.f / (1.f + __expf(-1.702f * a));
      return s + a * 1.702f * s * (1.f - s);
    }
    case ICAP_ACT_TANH: return 1.f - a * a;
    case ICAP_ACT_GELU_ERF:  // Phi(a) + a phi(a)
      return 0.5f * (1.f + erff(a * 0.70710678118654752f)) + a * 0.3989422804014327f * __expf(-0.5f * a * a);
    default: return 1.f;
  }
}

inline int dsize(int dtype) { return dtype == ICAP_BF16 ? 2 : 4; }

}  // namespace icap

// MX block quantisation for the fp8 GEMM path (ICAP_FP8_MX): rows of an f32 / bf16 matrix -> OCP e4m3fn bytes with
// one E8M0 scale per 32-element K block (the OCP Microscaling block: shared power-of-two scale, 8-bit elements).
//
// Scale choice: X = the smallest integer with amax <= 448 * 2^X (448 = e4m3's largest finite value), so no element
// of the block saturates; the stored code is X + 127. Elements: v * 2^-X (exact) -> e4m3 by round-to-nearest-even
// (v_cvt_pk_fp8_f32; pinned against oracle.mx_quantize bit for bit in tests). An all-zero block gets X = 0.
// rows_dev (optional device int32 <= R): rows from it on are neither read nor written (their scale bytes are
// still written, as 1.0): a GEMM bounded by the same device row count (m_dev) never uses them.
// The scales go out in the layout the MX GEMM reads (gemm_common.h mx_scale_off); rows from R up to the next
// multiple of 64 get scale 1.0 (code 127), so the GEMM never meets an E8M0 NaN code in its padded row groups.
//
// One thread per (row, 32-element block): 64 bytes (bf16) or 128 bytes (f32) in, 32 bytes + 1 scale out, with
// consecutive threads on consecutive blocks of a row (coalesced); the 4 scale bytes of a 128-element stage are
// gathered by shuffles and stored as one dword. HBM-bound: (in + 1.03 B) per element.
#include "gemm_common.h"

namespace icap {

__device__ __forceinline__ int mx_exponent(float amax) {
  if (!(amax > 0.f) || !isfinite(amax)) return 0;
  const int e = ilogbf(amax);  // amax in [2^e, 2^(e+1))
  int x = e - 8;               // 448 * 2^(e-8) = 1.75 * 2^e
  if (amax > ldexpf(448.f, x)) x += 1;
  return x < -127 ? -127 : (x > 127 ? 127 : x);
}

template <typename T>
__global__ __launch_bounds__(256) void quantize_mx_kernel(int64_t R, int64_t K, const T* __restrict__ x, int64_t ldx,
                                                          uint8_t* __restrict__ q, int64_t ldq,
                                                          uint8_t* __restrict__ sc, const int32_t* rows_dev) {
  const int64_t nkb = K / 32;
  const int64_t Rv = rows_dev && (int64_t)*rows_dev < R ? (int64_t)*rows_dev : R;  // rows past it: not read
  const int64_t Rs = (R + 63) / 64 * 64;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = t < Rs * nkb;
  const int64_t row = live ? t / nkb : 0, kb = live ? t - row * nkb : 0;
  int code = 127;
  if (live && row < Rv) {
    float v[32];
    const T* src = x + row * ldx + kb * 32;
#pragma unroll
    for (int c = 0; c < 32; c += 8) vecio<T, 8>::ld(src + c, v + c);
    float amax = 0.f;
#pragma unroll
    for (int e = 0; e < 32; ++e) amax = fmaxf(amax, fabsf(v[e]));
    const int X = mx_exponent(amax);
    code = X + 127;
    const float inv = ldexpf(1.f, -X);
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i] * inv, v[4 * i + 1] * inv, 0, false);
      w[i] = (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i + 2] * inv, v[4 * i + 3] * inv, lo, true);
    }
    uint4* dst = reinterpret_cast<uint4*>(q + row * ldq + kb * 32);
    dst[0] = make_uint4(w[0], w[1], w[2], w[3]);
    dst[1] = make_uint4(w[4], w[5], w[6], w[7]);
  }
  // the stage's 4 block codes -> one dword (threads 4s..4s+3 of a row share row and stage: nkb % 4 == 0)
  uint32_t word = (uint32_t)code << (8 * (kb & 3));
  word |= __shfl_xor(word, 1, 64);
  word |= __shfl_xor(word, 2, 64);
  if (live && (kb & 3) == 0) *reinterpret_cast<uint32_t*>(sc + mx_scale_off(R, row, kb)) = word;
}

}  // namespace icap

using namespace icap;

extern "C" size_t icap_mx_scale_bytes(int64_t R, int64_t K) {
  if (R < 0 || K < 0 || K % 128) return 0;
  return (size_t)((K / 32) * ((R + 63) / 64) * 64);
}

extern "C" int icap_quantize_mx(int32_t dtype, int64_t R, int64_t K, const void* x, int64_t ldx, void* q, int64_t ldq,
                                void* scales, const int32_t* rows_dev, void* stream) {
  ICAP_REQUIRE(dtype == ICAP_F32 || dtype == ICAP_BF16, "icap_quantize_mx: dtype must be f32 or bf16");
  ICAP_REQUIRE(R >= 0 && K >= 0 && K % 128 == 0, "icap_quantize_mx: K must be a multiple of 128");
  ICAP_REQUIRE(ldx >= K && ldq >= K && ldq % 16 == 0, "icap_quantize_mx: ldx >= K, ldq >= K and ldq % 16 == 0");
  ICAP_REQUIRE(x && q && scales, "icap_quantize_mx: null pointer");
  const int64_t es = dtype == ICAP_BF16 ? 2 : 4;
  ICAP_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0 && (ldx * es) % 16 == 0 &&
                   (reinterpret_cast<uintptr_t>(q) & 15) == 0 && (reinterpret_cast<uintptr_t>(scales) & 15) == 0,
               "icap_quantize_mx: x / q / scales must be 16-byte aligned (rows too)");
  if (R == 0 || K == 0) return ICAP_OK;
  const int64_t n = (R + 63) / 64 * 64 * (K / 32);
  const dim3 grid((unsigned)((n + 255) / 256));
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (dtype == ICAP_BF16)
    hipLaunchKernelGGL(quantize_mx_kernel<bf16_t>, grid, dim3(256), 0, s, R, K, (const bf16_t*)x, ldx, (uint8_t*)q, ldq,
                       (uint8_t*)scales, rows_dev);
  else
    hipLaunchKernelGGL(quantize_mx_kernel<float>, grid, dim3(256), 0, s, R, K, (const float*)x, ldx, (uint8_t*)q, ldq,
                       (uint8_t*)scales, rows_dev);
  return check_launch("icap_quantize_mx");
}

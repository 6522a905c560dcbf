// CLIP image preprocessing on the device: the reference's
// CLIPImageProcessor (src/embeddings/clip.py:129 -> HF image_processing_clip: convert RGB, shortest-edge
// resize to 224 with PIL BICUBIC, centre crop 224, x 1/255, (x - mean) / std) for a batch of decoded RGB
// images of any sizes, producing the fp32 [n, 3, crop, crop] pixel_values the vision tower consumes.
//
// The resize is Pillow's two-pass fixed-point resampler (libImaging/Resample.c, Pillow 4-12): per axis,
// coefficients from the bicubic kernel (a = -0.5) widened by the downscale factor, normalised in double,
// then rounded to 22-bit fixed point; the horizontal pass writes uint8 rows (round-half-up via the
// 1 << 21 bias, then clip), the vertical pass reads them. An axis whose size does not change is not
// resampled at all (Pillow skips that pass). Only the pixels inside the centre crop are produced: the
// horizontal pass covers the crop's columns for the source rows the crop's vertical windows touch.
// Coefficient arithmetic is IEEE double with contraction off, so the fixed-point weights are Pillow's.
//
// geo (device, int64 [n][GEO]): src_off, in_h, in_w, new_h, new_w, top, left, tmp_off, y_first, tmp_rows
// (tools-side rules in icap/ops.py clip_preprocess). tmp: uint8 [sum tmp_rows][crop][3].
#include "common.h"

namespace icap {

constexpr int GEO = 10;
constexpr int RS_BITS = 22;  // Pillow PRECISION_BITS for 8-bit images

#pragma clang fp contract(off)
__device__ __forceinline__ double bicubic_w(double x) {
  const double a = -0.5;
  if (x < 0.0) x = -x;
  if (x < 1.0) return ((a + 2.0) * x - (a + 3.0)) * x * x + 1;
  if (x < 2.0) return (((x - 5) * x + 8) * x - 4) * a;
  return 0.0;
}

// Pillow precompute_coeffs + normalize_coeffs_8bpc for output index xx (in -> out along one axis), without
// a coefficient array: the window and the weight sum first, then each tap's fixed-point weight on demand
// (the same double expressions, so the same values)
struct ResWin {
  double center, ss, ww;
  int xmin, taps;
};
__device__ ResWin resample_window(int in_size, int out_size, int xx) {
  ResWin r;
  const double scale = (double)in_size / (double)out_size;
  const double filterscale = scale < 1.0 ? 1.0 : scale;
  const double support = 2.0 * filterscale;
  r.center = (xx + 0.5) * scale;
  r.ss = 1.0 / filterscale;
  int xmin = (int)(r.center - support + 0.5);
  if (xmin < 0) xmin = 0;
  int xmax = (int)(r.center + support + 0.5);
  if (xmax > in_size) xmax = in_size;
  r.xmin = xmin;
  r.taps = xmax - xmin;
  double ww = 0.0;
  for (int x = 0; x < r.taps; ++x) ww += bicubic_w((x + xmin - r.center + 0.5) * r.ss);
  r.ww = ww;
  return r;
}
__device__ __forceinline__ int resample_tap(const ResWin& r, int x) {
  double v = bicubic_w((x + r.xmin - r.center + 0.5) * r.ss);
  if (r.ww != 0.0) v /= r.ww;
  return v < 0 ? (int)(-0.5 + v * (1 << RS_BITS)) : (int)(0.5 + v * (1 << RS_BITS));
}
#pragma clang fp contract(on)

__device__ __forceinline__ int clip8(int v) {
  v >>= RS_BITS;
  return v < 0 ? 0 : (v > 255 ? 255 : v);
}

// horizontal pass: one thread per (image, tmp row, crop column); 3 channels
__global__ __launch_bounds__(256) void resize_h_kernel(int n, int crop, const uint8_t* __restrict__ px,
                                                       const int64_t* __restrict__ geo, uint8_t* __restrict__ tmp,
                                                       int max_rows) {
  const int img = blockIdx.z;
  const int64_t* g = geo + (int64_t)img * GEO;
  const int in_w = (int)g[2], new_w = (int)g[4], left = (int)g[6], y_first = (int)g[8], rows = (int)g[9];
  const int r = blockIdx.y;
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (img >= n || r >= rows || r >= max_rows || x >= crop) return;
  const uint8_t* src = px + g[0] + (int64_t)(y_first + r) * in_w * 3;
  uint8_t* dst = tmp + g[7] + ((int64_t)r * crop + x) * 3;
  const int ox = left + x;
  if (new_w == in_w) {  // Pillow skips the pass
    dst[0] = src[ox * 3 + 0];
    dst[1] = src[ox * 3 + 1];
    dst[2] = src[ox * 3 + 2];
    return;
  }
  const ResWin w = resample_window(in_w, new_w, ox);
  int s0 = 1 << (RS_BITS - 1), s1 = s0, s2 = s0;
  for (int t = 0; t < w.taps; ++t) {
    const int k = resample_tap(w, t);
    const uint8_t* p = src + (w.xmin + t) * 3;
    s0 += p[0] * k;
    s1 += p[1] * k;
    s2 += p[2] * k;
  }
  dst[0] = (uint8_t)clip8(s0);
  dst[1] = (uint8_t)clip8(s1);
  dst[2] = (uint8_t)clip8(s2);
}

// vertical pass + crop + rescale + normalise: one thread per (image, crop row, crop column)
__global__ __launch_bounds__(256) void resize_v_kernel(int n, int crop, const int64_t* __restrict__ geo,
                                                       const uint8_t* __restrict__ tmp, const float* __restrict__ mean,
                                                       const float* __restrict__ stdv, float* __restrict__ out) {
  const int img = blockIdx.z;
  const int64_t* g = geo + (int64_t)img * GEO;
  const int in_h = (int)g[1], new_h = (int)g[3], top = (int)g[5], y_first = (int)g[8];
  const int y = blockIdx.y;
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (img >= n || y >= crop || x >= crop) return;
  const uint8_t* t0 = tmp + g[7];
  int v[3];
  if (new_h == in_h) {  // Pillow skips the pass: tmp row r = source row y_first + r = top + y
    const uint8_t* p = t0 + ((int64_t)(top + y - y_first) * crop + x) * 3;
    v[0] = p[0];
    v[1] = p[1];
    v[2] = p[2];
  } else {
    const ResWin w = resample_window(in_h, new_h, top + y);
    int s0 = 1 << (RS_BITS - 1), s1 = s0, s2 = s0;
    for (int t = 0; t < w.taps; ++t) {
      const int k = resample_tap(w, t);
      const uint8_t* p = t0 + ((int64_t)(w.xmin + t - y_first) * crop + x) * 3;
      s0 += p[0] * k;
      s1 += p[1] * k;
      s2 += p[2] * k;
    }
    v[0] = clip8(s0);
    v[1] = clip8(s1);
    v[2] = clip8(s2);
  }
  const int64_t plane = (int64_t)crop * crop;
  float* o = out + (int64_t)img * 3 * plane + (int64_t)y * crop + x;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    // HF rescale: float64 multiply by 1/255 then float32; normalize: (x - mean) / std in float32
    const float xs = (float)((double)v[c] * (1.0 / 255.0));
    o[c * plane] = (xs - mean[c]) / stdv[c];
  }
}

}  // namespace icap

using namespace icap;

extern "C" int icap_clip_preprocess(int32_t n, const uint8_t* pixels, const int64_t* geo, int32_t crop,
                                    int32_t max_tmp_rows, uint8_t* tmp, const float* mean, const float* stdv,
                                    float* out, void* stream) {
  ICAP_REQUIRE(n >= 0 && crop > 0 && max_tmp_rows > 0, "icap_clip_preprocess: bad sizes");
  ICAP_REQUIRE(pixels && geo && tmp && mean && stdv && out, "icap_clip_preprocess: null pointer");
  if (n == 0) return ICAP_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 blk(256);
  const dim3 gh((unsigned)((crop + 255) / 256), (unsigned)max_tmp_rows, (unsigned)n);
  hipLaunchKernelGGL(resize_h_kernel, gh, blk, 0, s, n, crop, pixels, geo, tmp, max_tmp_rows);
  const int rc = check_launch("icap_clip_preprocess(h)");
  if (rc != ICAP_OK) return rc;
  const dim3 gv((unsigned)((crop + 255) / 256), (unsigned)crop, (unsigned)n);
  hipLaunchKernelGGL(resize_v_kernel, gv, blk, 0, s, n, crop, geo, tmp, mean, stdv, out);
  return check_launch("icap_clip_preprocess(v)");
}

// LayerNorm forward/backward (HBM-bound): one wave per row, 4 waves per block,
// grid-stride over rows; each lane owns D/256 float4 groups (D <= 1024).
// Stats in fp32 with a two-pass variance held in registers.
#include "common.h"

namespace icap {

constexpr int LN_MAXV = 4;       // float4 groups per lane -> D <= 1024
constexpr int LN_BWD_BLOCKS = 256;

template <typename T>
__global__ __launch_bounds__(256) void ln_fwd_kernel(int64_t rows, int D, const T* __restrict__ x, int64_t ldx,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, float eps,
                                                    T* __restrict__ y, int64_t ldy, float* mean_out,
                                                    float* rstd_out, const int32_t* __restrict__ y_rowmap,
                                                    const int32_t* __restrict__ rows_dev) {
  if (rows_dev && (int64_t)*rows_dev < rows) rows = *rows_dev;
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int D4 = D >> 2;
  const float invD = 1.f / (float)D;
  for (int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < rows; r += nw) {
    float v[LN_MAXV][4];
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
      const int g = lane + 64 * t;
      if (g < D4) {
        io<T>::ld4(x + r * ldx + 4 * g, v[t]);
        s += (v[t][0] + v[t][1]) + (v[t][2] + v[t][3]);
      }
    }
    const float mean = wave_sum(s) * invD;
    float s2 = 0.f;
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
      const int g = lane + 64 * t;
      if (g < D4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float d = v[t][e] - mean;
          s2 += d * d;
        }
      }
    }
    const float var = wave_sum(s2) * invD;
    const float rs = 1.f / sqrtf(var + eps);
    const int64_t yr = y_rowmap ? (int64_t)y_rowmap[r] : r;
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
      const int g = lane + 64 * t;
      if (g < D4 && yr >= 0) {
        const float4 gm = *reinterpret_cast<const float4*>(gamma + 4 * g);
        const float4 bt = *reinterpret_cast<const float4*>(beta + 4 * g);
        float o[4];
        o[0] = (v[t][0] - mean) * rs * gm.x + bt.x;
        o[1] = (v[t][1] - mean) * rs * gm.y + bt.y;
        o[2] = (v[t][2] - mean) * rs * gm.z + bt.z;
        o[3] = (v[t][3] - mean) * rs * gm.w + bt.w;
        io<T>::st4(y + yr * ldy + 4 * g, o);
      }
    }
    if (lane == 0) {
      if (mean_out) mean_out[r] = mean;
      if (rstd_out) rstd_out[r] = rs;
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void ln_bwd_kernel(int64_t rows, int D, const T* __restrict__ x, int64_t ldx,
                                                    const float* __restrict__ gamma,
                                                    const float* __restrict__ mean_in,
                                                    const float* __restrict__ rstd_in,
                                                    const T* __restrict__ dy, int64_t lddy,
                                                    const T* __restrict__ dres, int64_t lddres,
                                                    T* __restrict__ dx, int64_t lddx, T* __restrict__ dx_drop,
                                                    uint32_t thr, float inv_keep, uint64_t seed0,
                                                    const uint64_t* seed_ptr, uint64_t offset,
                                                    float* __restrict__ partial,
                                                    const int32_t* __restrict__ dy_rowmap,
                                                    const int32_t* __restrict__ rows_dev) {
  if (rows_dev && (int64_t)*rows_dev < rows) rows = *rows_dev;
  __shared__ float red[4][2][LN_MAXV * 256];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int D4 = D >> 2;
  const float invD = 1.f / (float)D;
  const uint64_t seed = thr ? eff_seed(seed0, seed_ptr) : 0ull;
  float dg[LN_MAXV][4], db[LN_MAXV][4];
#pragma unroll
  for (int t = 0; t < LN_MAXV; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) dg[t][e] = db[t][e] = 0.f;

  // rows are processed with the NEXT row's x / dy / dres already in flight (each wave owns ~rows/nw rows,
  // so without the prefetch every row pays a full memory latency before its two reductions)
  float xv[LN_MAXV][4], dv[LN_MAXV][4], rv[LN_MAXV][4];
  auto load_row = [&](int64_t r) {
    const int64_t dyr = dy_rowmap ? (int64_t)dy_rowmap[r] : r;
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
      const int g = lane + 64 * t;
      if (g < D4) {
        io<T>::ld4(x + r * ldx + 4 * g, xv[t]);
        if (dyr >= 0) io<T>::ld4(dy + dyr * lddy + 4 * g, dv[t]);
        else dv[t][0] = dv[t][1] = dv[t][2] = dv[t][3] = 0.f;
        if (dres) io<T>::ld4(dres + r * lddres + 4 * g, rv[t]);
      }
    }
  };
  int64_t r = (int64_t)blockIdx.x * 4 + wv;
  if (r < rows) load_row(r);
  for (; r < rows; r += nw) {
    const float mean = mean_in[r], rs = rstd_in[r];
    float xh[LN_MAXV][4], gy[LN_MAXV][4], dres4[LN_MAXV][4];
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
      const int g = lane + 64 * t;
      if (g < D4) {
        const float4 gm = *reinterpret_cast<const float4*>(gamma + 4 * g);
        const float gmv[4] = {gm.x, gm.y, gm.z, gm.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          xh[t][e] = (xv[t][e] - mean) * rs;
          gy[t][e] = dv[t][e] * gmv[e];
          s1 += gy[t][e];
          s2 += gy[t][e] * xh[t][e];
          dg[t][e] += dv[t][e] * xh[t][e];
          db[t][e] += dv[t][e];
          dres4[t][e] = dres ? rv[t][e] : 0.f;
        }
      }
    }
    if (r + nw < rows) load_row(r + nw);
    const float m1 = wave_sum(s1) * invD;
    const float m2 = wave_sum(s2) * invD;
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
      const int g = lane + 64 * t;
      if (g < D4) {
        float o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) o[e] = rs * (gy[t][e] - m1 - xh[t][e] * m2) + dres4[t][e];
        io<T>::st4(dx + r * lddx + 4 * g, o);
        if (dx_drop) {
          const uint64_t base = offset + (uint64_t)(r * D + 4 * g);
#pragma unroll
          for (int e = 0; e < 4; ++e) o[e] *= drop_scale(seed, base + e, thr, inv_keep);
          io<T>::st4(dx_drop + r * lddx + 4 * g, o);
        }
      }
    }
  }
  if (partial) {
#pragma unroll
    for (int t = 0; t < LN_MAXV; ++t) {
      const int g = lane + 64 * t;
      if (g < D4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          red[wv][0][4 * g + e] = dg[t][e];
          red[wv][1][4 * g + e] = db[t][e];
        }
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 256) {
      float a = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
      float b = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
      partial[(int64_t)blockIdx.x * 2 * D + c] = a;
      partial[(int64_t)blockIdx.x * 2 * D + D + c] = b;
    }
  }
}

// grid (ceil(D/64), 2): blockIdx.y selects dgamma / dbeta; 16 waves split the partial rows (fixed order, so the
// result is deterministic), 64 lanes = 64 columns
__global__ __launch_bounds__(1024) void ln_param_reduce(int nblk, int D, const float* __restrict__ partial,
                                                       float* dgamma, float* dbeta, int acc) {
  __shared__ float red[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int which = blockIdx.y;
  float a = 0.f;
  if (c < D) {
    // the 16 row loads of a thread (nblk <= 256: LN_BWD_BLOCKS) issued together, then added in row order
#pragma unroll 16
    for (int i = ty; i < nblk; i += 16) a += partial[(int64_t)i * 2 * D + which * D + c];
  }
  red[ty][tx] = a;
  __syncthreads();
  if (ty == 0 && c < D) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][tx];
    float* dst = which ? dbeta : dgamma;
    if (dst) dst[c] = acc ? dst[c] + s : s;
  }
}

// ---- 16-byte variants (D % 8 == 0, 8-aligned strides, 16-byte aligned bases: every GPT-2 / mapper / CLIP LN) --
// Half a wave per row: 32 lanes x LN8_MAXC chunks of 8 elements, each one 16-byte access (the 4-wide form moves
// 8 bytes per lane and access; these kernels are access-issue bound, like the GEMM store tail). 8 rows per
// 256-thread block; the row reductions stay inside the half-wave (xor shuffles 16..1).
// LN8_MAXC (template): chunks per lane, 3 for D <= 768, 4 for D <= 1024, 5 for D <= 1280 (GPT-2 large), 6 for
// D <= 1536
constexpr int LN8_DMAX = 6 * 32 * 8;

// Sum over a 32-lane half-wave, in every lane of it, on the VALU's cross-lane paths (round 5): DPP quad_perm for
// lane ^ 1 and ^ 2, row_half_mirror (i <-> 7 - i: the other quad of each 8), row_ror:8 (lane ^ 8 within a 16-lane
// row) and v_permlane16_swap for the other row of the half (the __shfl_xor butterfly it replaces lowered to
// ds_bpermute_b32: 5 LDS round trips). The operation order is fixed and lane-independent, so every lane of the half
// holds the same bits. Both halves of a wave must be active or inactive together (the row loops are uniform per
// half). (The side-stream nondeterminism first blamed on the bpermute form was the packed-FP32 instructions of the
// row arithmetic, not this sum: the readlane, bpermute and DPP forms all failed the same way with them and none
// does without them — Makefile, DESIGN.md "Concurrency: the packed-FP32 race".)
__device__ __forceinline__ float half_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));   // ^1
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));   // ^2
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false));  // 7-i
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x128, 0xF, 0xF, false));  // ror 8
  const auto sw = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                   false, false);
  return __builtin_bit_cast(float, (unsigned)sw[0]) + __builtin_bit_cast(float, (unsigned)sw[1]);
}

template <typename T, int LN8_MAXC>
__global__ __launch_bounds__(256) void ln_fwd8_kernel(int64_t rows, int D, const T* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, float eps,
                                                     T* __restrict__ y, int64_t ldy, float* mean_out,
                                                     float* rstd_out, const int32_t* __restrict__ y_rowmap,
                                                    const int32_t* __restrict__ rows_dev) {
  if (rows_dev && (int64_t)*rows_dev < rows) rows = *rows_dev;
  const int hl = threadIdx.x & 31;
  const int64_t nr = (int64_t)gridDim.x * 8;
  const int D8 = D >> 3;
  const float invD = 1.f / (float)D;
  for (int64_t r = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5); r < rows; r += nr) {
    float v[LN8_MAXC][8];
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < LN8_MAXC; ++t) {
      const int g = hl + 32 * t;
      if (g < D8) {
        io<T>::ld8(x + r * ldx + 8 * g, v[t]);
#pragma unroll
        for (int e = 0; e < 8; e += 2) s += v[t][e] + v[t][e + 1];
      }
    }
    const float mean = half_sum(s) * invD;
    float s2 = 0.f;
#pragma unroll
    for (int t = 0; t < LN8_MAXC; ++t) {
      const int g = hl + 32 * t;
      if (g < D8) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = v[t][e] - mean;
          s2 += d * d;
        }
      }
    }
    const float rs = 1.f / sqrtf(half_sum(s2) * invD + eps);
    const int64_t yr = y_rowmap ? (int64_t)y_rowmap[r] : r;
#pragma unroll
    for (int t = 0; t < LN8_MAXC; ++t) {
      const int g = hl + 32 * t;
      if (g < D8 && yr >= 0) {
        float gm[8], bt[8], o[8];
        io<float>::ld8(gamma + 8 * g, gm);
        io<float>::ld8(beta + 8 * g, bt);
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = (v[t][e] - mean) * rs * gm[e] + bt[e];
        io<T>::st8(y + yr * ldy + 8 * g, o);
      }
    }
    if (hl == 0) {
      if (mean_out) mean_out[r] = mean;
      if (rstd_out) rstd_out[r] = rs;
    }
  }
}

// v + the same register of lane ^ 32 (v_permlane32_swap; the bits equal v + __shfl_xor(v, 32) in every lane)
__device__ __forceinline__ float lane_pair_sum(float v) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                   false, false);
  return __builtin_bit_cast(float, (unsigned)sw[0]) + __builtin_bit_cast(float, (unsigned)sw[1]);
}

// PARAMS: accumulate dgamma / dbeta partials (per block, combined by ln_param_reduce); GPT-2's LNs are frozen
template <typename T, bool PARAMS, int LN8_MAXC>
__global__ __launch_bounds__(256) void ln_bwd8_kernel(int64_t rows, int D, const T* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ gamma,
                                                     const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in,
                                                     const T* __restrict__ dy, int64_t lddy,
                                                     const T* __restrict__ dres, int64_t lddres,
                                                     T* __restrict__ dx, int64_t lddx, T* __restrict__ dx_drop,
                                                     uint32_t thr, float inv_keep, uint64_t seed0,
                                                     const uint64_t* seed_ptr, uint64_t offset,
                                                     float* __restrict__ partial,
                                                     const int32_t* __restrict__ dy_rowmap,
                                                    const int32_t* __restrict__ rows_dev) {
  if (rows_dev && (int64_t)*rows_dev < rows) rows = *rows_dev;
  __shared__ float red[PARAMS ? 4 : 1][2][PARAMS ? LN8_MAXC * 256 : 1];  // [wave][dgamma|dbeta][column]
  const int hl = threadIdx.x & 31;
  const int wv = threadIdx.x >> 6;
  const int64_t nr = (int64_t)gridDim.x * 8;
  const int D8 = D >> 3;
  const float invD = 1.f / (float)D;
  const uint64_t seed = thr ? eff_seed(seed0, seed_ptr) : 0ull;
  float gm[LN8_MAXC][8];
#pragma unroll
  for (int t = 0; t < LN8_MAXC; ++t)
    if (hl + 32 * t < D8) io<float>::ld8(gamma + 8 * (hl + 32 * t), gm[t]);
  float dg[PARAMS ? LN8_MAXC : 1][8], db[PARAMS ? LN8_MAXC : 1][8];
  if constexpr (PARAMS) {
#pragma unroll
    for (int t = 0; t < LN8_MAXC; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) dg[t][e] = db[t][e] = 0.f;
  }
  for (int64_t r = (int64_t)blockIdx.x * 8 + (threadIdx.x >> 5); r < rows; r += nr) {
    // every load of the row is issued unconditionally, from a valid row (a gathered row < 0 reads row 0, a missing
    // dres re-reads x), and the values are selected afterwards: the data-dependent branches around each load made
    // hipcc wait for every load before issuing the next (a serial chain of 9 round trips per row)
    const int64_t dyr0 = dy_rowmap ? (int64_t)dy_rowmap[r] : r;
    const bool dy_ok = dyr0 >= 0, has_res = dres != nullptr;
    const T* xp = x + r * ldx;
    const T* dp = dy + (dy_ok ? dyr0 : 0) * lddy;
    const T* rp = has_res ? dres + r * lddres : xp;
    float xv[LN8_MAXC][8], dv[LN8_MAXC][8], rv[LN8_MAXC][8];
#pragma unroll
    for (int t = 0; t < LN8_MAXC; ++t) {
      const int g = hl + 32 * t, gc = g < D8 ? g : D8 - 1;  // (chunks past D re-read the last one; zeroed below)
      io<T>::ld8(xp + 8 * gc, xv[t]);
      io<T>::ld8(dp + 8 * gc, dv[t]);
      io<T>::ld8(rp + 8 * gc, rv[t]);
    }
    const float mean = mean_in[r], rs = rstd_in[r];
#pragma unroll
    for (int t = 0; t < LN8_MAXC; ++t) {
      const bool in = hl + 32 * t < D8;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        xv[t][e] = in ? xv[t][e] : 0.f;
        dv[t][e] = (in && dy_ok) ? dv[t][e] : 0.f;
        rv[t][e] = (in && has_res) ? rv[t][e] : 0.f;
      }
    }
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int t = 0; t < LN8_MAXC; ++t) {
      if (hl + 32 * t < D8) {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xh = (xv[t][e] - mean) * rs;
          if constexpr (PARAMS) {
            dg[t][e] += dv[t][e] * xh;
            db[t][e] += dv[t][e];
          }
          const float gy = dv[t][e] * gm[t][e];
          s1 += gy;
          s2 += gy * xh;
          xv[t][e] = xh;
          dv[t][e] = gy;
        }
      }
    }
    const float m1 = half_sum(s1) * invD;
    const float m2 = half_sum(s2) * invD;
#pragma unroll
    for (int t = 0; t < LN8_MAXC; ++t) {
      const int g = hl + 32 * t;
      if (g < D8) {
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = rs * (dv[t][e] - m1 - xv[t][e] * m2) + rv[t][e];
        io<T>::st8(dx + r * lddx + 8 * g, o);
        if (dx_drop) {
          const uint64_t base = offset + (uint64_t)(r * D + 8 * g);
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] *= drop_scale(seed, base + e, thr, inv_keep);
          io<T>::st8(dx_drop + r * lddx + 8 * g, o);
        }
      }
    }
  }
  if constexpr (PARAMS) {
    // the two half-waves of a wave hold the same columns: fold them, then one wave's partial per LDS slot
#pragma unroll
    for (int t = 0; t < LN8_MAXC; ++t)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        dg[t][e] = lane_pair_sum(dg[t][e]);
        db[t][e] = lane_pair_sum(db[t][e]);
      }
    if ((threadIdx.x & 63) < 32) {
#pragma unroll
      for (int t = 0; t < LN8_MAXC; ++t) {
        const int g = hl + 32 * t;
        if (g < D8) {
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            red[wv][0][8 * g + e] = dg[t][e];
            red[wv][1][8 * g + e] = db[t][e];
          }
        }
      }
    }
    __syncthreads();
    for (int c = threadIdx.x; c < D; c += 256) {
      partial[(int64_t)blockIdx.x * 2 * D + c] = red[0][0][c] + red[1][0][c] + red[2][0][c] + red[3][0][c];
      partial[(int64_t)blockIdx.x * 2 * D + D + c] = red[0][1][c] + red[1][1][c] + red[2][1][c] + red[3][1][c];
    }
  }
}

}  // namespace icap

using namespace icap;

// the 16-byte kernels need D % 8 == 0, an 8-element stride and a 16-byte aligned base
static bool ln8_ok(int32_t dtype, int64_t D, const void* p, int64_t ld) {
  const int es = dtype == ICAP_BF16 ? 2 : 4;
  return D % 8 == 0 && ld % 8 == 0 && (reinterpret_cast<uintptr_t>(p) & 15) == 0 && (D * es) % 16 == 0;
}

static int ln_blocks8(int64_t rows, int cap) {
  int64_t b = (rows + 7) / 8;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

static int ln_blocks(int64_t rows, int cap) {
  int64_t b = (rows + 3) / 4;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

extern "C" int icap_layernorm_fwd(int32_t dtype, int64_t rows, int64_t D, const void* x, int64_t ldx,
                                  const float* gamma, const float* beta, float eps, void* y, int64_t ldy,
                                  float* mean, float* rstd, const int32_t* y_rowmap, const int32_t* rows_dev,
                                  void* stream) {
  ICAP_REQUIRE(x && y && gamma && beta, "icap_layernorm_fwd: null pointer");
  ICAP_REQUIRE(D > 0 && D % 4 == 0 && (D <= 4 * 64 * LN_MAXV || (D <= LN8_DMAX && ln8_ok(dtype, D, x, ldx) &&
                                                               ln8_ok(dtype, D, y, ldy))),
               "icap_layernorm_fwd: D must be a multiple of 4, <= 1024 (<= 1536 with 16-byte rows)");
  ICAP_REQUIRE(ldx % 4 == 0 && ldy % 4 == 0, "icap_layernorm_fwd: strides must be multiples of 4");
  if (rows == 0) return ICAP_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (ln8_ok(dtype, D, x, ldx) && ln8_ok(dtype, D, y, ldy)) {
    const int nb8 = ln_blocks8(rows, 4096);
#define ICAP_LN_FWD8(T, NC)                                                                                    \
  hipLaunchKernelGGL((ln_fwd8_kernel<T, NC>), dim3(nb8), dim3(256), 0, s, rows, (int)D, (const T*)x, ldx, gamma, \
                     beta, eps, (T*)y, ldy, mean, rstd, y_rowmap, rows_dev)
    if (dtype == ICAP_BF16) {
      if (D <= 768) ICAP_LN_FWD8(bf16_t, 3); else if (D <= 1024) ICAP_LN_FWD8(bf16_t, 4);
      else if (D <= 1280) ICAP_LN_FWD8(bf16_t, 5); else ICAP_LN_FWD8(bf16_t, 6);
    } else {
      if (D <= 768) ICAP_LN_FWD8(float, 3); else if (D <= 1024) ICAP_LN_FWD8(float, 4);
      else if (D <= 1280) ICAP_LN_FWD8(float, 5); else ICAP_LN_FWD8(float, 6);
    }
#undef ICAP_LN_FWD8
    return check_launch("icap_layernorm_fwd");
  }
  const int nb = ln_blocks(rows, 4096);
  if (dtype == ICAP_BF16)
    hipLaunchKernelGGL(ln_fwd_kernel<bf16_t>, dim3(nb), dim3(256), 0, s, rows, (int)D,
                       (const bf16_t*)x, ldx, gamma, beta, eps, (bf16_t*)y, ldy, mean, rstd, y_rowmap, rows_dev);
  else
    hipLaunchKernelGGL(ln_fwd_kernel<float>, dim3(nb), dim3(256), 0, s, rows, (int)D, (const float*)x,
                       ldx, gamma, beta, eps, (float*)y, ldy, mean, rstd, y_rowmap, rows_dev);
  return check_launch("icap_layernorm_fwd");
}

extern "C" size_t icap_layernorm_bwd_workspace_bytes(int64_t rows, int64_t D) {
  return (size_t)ln_blocks(rows, LN_BWD_BLOCKS) * 2 * (size_t)D * sizeof(float);
}

extern "C" int icap_layernorm_bwd(int32_t dtype, int64_t rows, int64_t D, const void* x, int64_t ldx,
                                  const float* gamma, const float* mean, const float* rstd,
                                  const void* dy, int64_t lddy, const void* dres, int64_t lddres,
                                  void* dx, int64_t lddx, void* dx_drop, float drop_p, uint64_t seed,
                                  uint64_t offset, const uint64_t* seed_ptr, float* dgamma, float* dbeta,
                                  void* workspace, const int32_t* dy_rowmap, const int32_t* rows_dev,
                                  int32_t param_overwrite, void* stream) {
  ICAP_REQUIRE(x && gamma && mean && rstd && dy && dx, "icap_layernorm_bwd: null pointer");
  const bool wide8 = ln8_ok(dtype, D, x, ldx) && ln8_ok(dtype, D, dy, lddy) && ln8_ok(dtype, D, dx, lddx) &&
                     (dres == nullptr || ln8_ok(dtype, D, dres, lddres)) &&
                     (dx_drop == nullptr || ln8_ok(dtype, D, dx_drop, lddx));
  ICAP_REQUIRE(D > 0 && D % 4 == 0 && (D <= 4 * 64 * LN_MAXV || (D <= LN8_DMAX && wide8)),
               "icap_layernorm_bwd: D must be a multiple of 4, <= 1024 (<= 1536 with 16-byte rows)");
  ICAP_REQUIRE((dgamma == nullptr && dbeta == nullptr) || workspace != nullptr,
               "icap_layernorm_bwd: dgamma/dbeta need a workspace");
  ICAP_REQUIRE(drop_p >= 0.f && drop_p < 1.f, "icap_layernorm_bwd: drop_p out of range");
  if (rows == 0) return ICAP_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const bool want_params = dgamma || dbeta;
  const int nb = ln_blocks(rows, want_params ? LN_BWD_BLOCKS : 4096);
  const uint32_t thr = drop_p > 0.f ? drop_threshold(drop_p) : 0u;
  const float inv_keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  float* partial = want_params ? reinterpret_cast<float*>(workspace) : nullptr;
  if (wide8) {
    // same block count as the partial workspace is sized for (8 rows per block here, 4 in the 4-wide form)
    const int nb8 = want_params ? nb : ln_blocks8(rows, 4096);
#define ICAP_LN_BWD8(T, P)                                                                                      \
  if (D <= 768) ICAP_LN_BWD8N(T, P, 3); else if (D <= 1024) ICAP_LN_BWD8N(T, P, 4);              \
  else if (D <= 1280) ICAP_LN_BWD8N(T, P, 5); else ICAP_LN_BWD8N(T, P, 6)
#define ICAP_LN_BWD8N(T, P, NC)                                                                                 \
  hipLaunchKernelGGL((ln_bwd8_kernel<T, P, NC>), dim3(nb8), dim3(256), 0, s, rows, (int)D, (const T*)x, ldx, gamma, \
                     mean, rstd, (const T*)dy, lddy, (const T*)dres, lddres, (T*)dx, lddx, (T*)dx_drop, thr,     \
                     inv_keep, seed, seed_ptr, offset, partial, dy_rowmap, rows_dev)
    if (dtype == ICAP_BF16) {
      if (want_params) ICAP_LN_BWD8(bf16_t, true); else ICAP_LN_BWD8(bf16_t, false);
    } else {
      if (want_params) ICAP_LN_BWD8(float, true); else ICAP_LN_BWD8(float, false);
    }
#undef ICAP_LN_BWD8
#undef ICAP_LN_BWD8N
  } else if (dtype == ICAP_BF16)
    hipLaunchKernelGGL(ln_bwd_kernel<bf16_t>, dim3(nb), dim3(256), 0, s, rows, (int)D, (const bf16_t*)x, ldx,
                       gamma, mean, rstd, (const bf16_t*)dy, lddy, (const bf16_t*)dres, lddres, (bf16_t*)dx,
                       lddx, (bf16_t*)dx_drop, thr, inv_keep, seed, seed_ptr, offset, partial, dy_rowmap, rows_dev);
  else
    hipLaunchKernelGGL(ln_bwd_kernel<float>, dim3(nb), dim3(256), 0, s, rows, (int)D, (const float*)x, ldx,
                       gamma, mean, rstd, (const float*)dy, lddy, (const float*)dres, lddres, (float*)dx,
                       lddx, (float*)dx_drop, thr, inv_keep, seed, seed_ptr, offset, partial, dy_rowmap, rows_dev);
  int rc = check_launch("icap_layernorm_bwd");
  if (rc != ICAP_OK || !want_params || (param_overwrite & 2)) return rc;  // (bit 1: the caller batches the reduce)
  hipLaunchKernelGGL(ln_param_reduce, dim3((unsigned)((D + 63) / 64), 2), dim3(1024), 0, s, nb, (int)D, partial,
                     dgamma, dbeta, (param_overwrite & 1) ? 0 : 1);
  return check_launch("icap_layernorm_bwd(reduce)");
}

// The deferred parameter reduces of several LayerNorm backwards in one launch: blockIdx.z = item, the same
// per-block sums as ln_param_reduce (so the stored dgamma / dbeta are bitwise the unbatched ones).
struct LnParamBatch {
  icap_ln_param_item it[ICAP_LN_PARAM_BATCH_MAX];
  int nblk[ICAP_LN_PARAM_BATCH_MAX];
};
__global__ __launch_bounds__(1024) void ln_param_reduce_batch(LnParamBatch b) {
  const icap_ln_param_item& it = b.it[blockIdx.z];
  const int D = (int)it.D;
  if ((int)blockIdx.x * 64 >= D) return;  // (items narrower than the widest)
  __shared__ float red[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + tx;
  const int which = blockIdx.y;
  const float* partial = reinterpret_cast<const float*>(it.workspace);
  float a = 0.f;
  if (c < D) {
#pragma unroll 16
    for (int i = ty; i < b.nblk[blockIdx.z]; i += 16) a += partial[(int64_t)i * 2 * D + which * D + c];
  }
  red[ty][tx] = a;
  __syncthreads();
  if (ty == 0 && c < D) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][tx];
    float* dst = which ? it.dbeta : it.dgamma;
    if (dst) dst[c] = it.overwrite ? s : dst[c] + s;
  }
}

extern "C" int icap_ln_param_reduce_batch(int32_t n, const icap_ln_param_item* items, void* stream) {
  ICAP_REQUIRE(n >= 0 && n <= ICAP_LN_PARAM_BATCH_MAX && (n == 0 || items),
               "icap_ln_param_reduce_batch: 0 ... ICAP_LN_PARAM_BATCH_MAX items");
  if (n == 0) return ICAP_OK;
  LnParamBatch b{};
  int64_t dmax = 0;
  for (int i = 0; i < n; ++i) {
    const icap_ln_param_item& it = items[i];
    ICAP_REQUIRE(it.workspace && it.rows > 0 && it.D > 0 && it.D % 4 == 0 && it.D <= LN8_DMAX,
                 "icap_ln_param_reduce_batch: workspace, rows > 0 and D (a multiple of 4, <= 1536) per item");
    b.it[i] = it;
    b.nblk[i] = ln_blocks(it.rows, LN_BWD_BLOCKS);
    if (it.D > dmax) dmax = it.D;
  }
  hipLaunchKernelGGL(ln_param_reduce_batch, dim3((unsigned)((dmax + 63) / 64), 2, (unsigned)n), dim3(1024), 0,
                     reinterpret_cast<hipStream_t>(stream), b);
  return check_launch("icap_ln_param_reduce_batch");
}

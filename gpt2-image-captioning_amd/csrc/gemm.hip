#include "gemm_tile.h"
#include "gemm_plan.h"

namespace icap {

// Skinny-M GEMM (M <= 128: greedy-decode steps over the batch, CLIP projection, mapper input Linear).
// A weight-streaming, latency-bound problem: block = 8 waves over a 16*NT-column slab of B (= W rows) and a
// 16*MT-row slab of A (grid.y walks M, so no block streams all of A through its CU: per-CU L2 bandwidth, not
// HBM, bounded the all-rows form); the waves split the K steps round-robin and keep SK_U steps of MFMA
// fragments in flight each (range-checked buffer loads straight from HBM/L2). The fp32 partial tiles are reduced
// through LDS in two rounds before the shared epilogue. One launch, no slabs.
// Accumulators use the C layout (lane = column, 4 consecutive rows per lane).
// one 16-byte A chunk -> LayerNorm-ed chunk in the input dtype
template <typename TI>
__device__ __forceinline__ uint4 ln_chunk(const uint4 a, float mean, float rs, const float* g, const float* bt);
template <>
__device__ __forceinline__ uint4 ln_chunk<bf16_t>(const uint4 a, float mean, float rs, const float* g, const float* bt) {
  const uint32_t w[4] = {a.x, a.y, a.z, a.w};
  uint32_t o[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float v0 = (__uint_as_float(w[q] << 16) - mean) * rs * g[2 * q] + bt[2 * q];
    const float v1 = (__uint_as_float(w[q] & 0xffff0000u) - mean) * rs * g[2 * q + 1] + bt[2 * q + 1];
    o[q] = f2bf2(v0, v1);
  }
  return make_uint4(o[0], o[1], o[2], o[3]);
}
template <>
__device__ __forceinline__ uint4 ln_chunk<float>(const uint4 a, float mean, float rs, const float* g, const float* bt) {
  return make_uint4(__float_as_uint((__uint_as_float(a.x) - mean) * rs * g[0] + bt[0]),
                    __float_as_uint((__uint_as_float(a.y) - mean) * rs * g[1] + bt[1]),
                    __float_as_uint((__uint_as_float(a.z) - mean) * rs * g[2] + bt[2]),
                    __float_as_uint((__uint_as_float(a.w) - mean) * rs * g[3] + bt[3]));
}

// v + the same register of lane ^ 16 / lane ^ 32 on the VALU's cross-lane paths (v_permlane16_swap /
// v_permlane32_swap; the bits equal v + __shfl_xor(v, 16 / 32), whose ds_bpermute is an LDS round trip each)
__device__ __forceinline__ float xor16_sum(float v) {
  const auto sw = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                   false, false);
  return __builtin_bit_cast(float, (unsigned)sw[0]) + __builtin_bit_cast(float, (unsigned)sw[1]);
}
__device__ __forceinline__ float xor32_sum(float v) {
  const auto sw = __builtin_amdgcn_permlane32_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                   false, false);
  return __builtin_bit_cast(float, (unsigned)sw[0]) + __builtin_bit_cast(float, (unsigned)sw[1]);
}

constexpr int SK_WAVES = 8;
constexpr int SK_LNK = 1280;  // LN-fused launches up to this K stage gamma / beta in LDS
// NT: 16-column slabs per block (the host picks the fewest that fit the grid in one pass over the CUs);
// SKU: k-steps in flight per wave (the host picks enough for one memory round trip over all of K where the
// registers allow). Neither changes the arithmetic: every wave accumulates its steps in step order and the waves
// are summed in a fixed order, so all (NT, SKU) instantiations store bitwise-identical outputs.
template <typename TI, typename TC, int NT, int MT, int SKU>
__global__ __launch_bounds__(64 * SK_WAVES) void gemm_skinny_kernel(icap_gemm_args p, uint32_t drop_thresh,
                                                                  float inv_keep) {
  constexpr int ES = sizeof(TI);
  constexpr int EPC = 16 / ES;        // K elements per lane chunk
  constexpr int KSTEP = 4 * EPC;      // K elements per MFMA chunk step (4 lane groups)
  constexpr int BN = 16 * NT;
  constexpr int RLD = BN + 4;         // fp32 stride of the LDS partial tiles
  constexpr int HALF = SK_WAVES / 2;
  constexpr int BM = 16 * MT;
  constexpr int QPR = BN / 4;         // 4-column epilogue quads per row
  static_assert(BM * QPR <= 64 * SK_WAVES, "one epilogue quad per thread");
  __shared__ __attribute__((aligned(16))) float red[HALF][BM * RLD];
  __shared__ __attribute__((aligned(16))) float lngb[2 * SK_LNK];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t N = p.N, K = p.K;
  const int64_t n0 = (int64_t)blockIdx.x * BN, m0 = (int64_t)blockIdx.y * BM;
  const int64_t M = p.m_dev && (int64_t)*p.m_dev < p.M ? (int64_t)*p.m_dev : p.M;  // device row count
  if (m0 >= M) return;
  const int64_t nrows = N - n0 < BN ? N - n0 : BN;
  const int64_t mrows = M - m0 < BM ? M - m0 : BM;
  const __amdgpu_buffer_rsrc_t ra =
      make_rsrc(reinterpret_cast<const char*>(p.A) + m0 * p.lda * ES, (uint64_t)((mrows - 1) * p.lda + K) * ES);
  const __amdgpu_buffer_rsrc_t rb =
      make_rsrc(reinterpret_cast<const char*>(p.B) + n0 * p.ldb * ES, (uint64_t)((nrows - 1) * p.ldb + K) * ES);
  f32x4_t acc[MT][NT];
#pragma unroll
  for (int i = 0; i < MT; ++i)
#pragma unroll
    for (int j = 0; j < NT; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  // rows past M / N lie beyond the descriptor range (zero-filled); K-tail chunks and steps past the end are
  // redirected out of range (zero fragments: the MFMAs on them add nothing)
  uint32_t aoff[MT], boff[NT];
#pragma unroll
  for (int i = 0; i < MT; ++i) aoff[i] = (uint32_t)(((i * 16 + fr) * p.lda + fg * EPC) * ES);
#pragma unroll
  for (int j = 0; j < NT; ++j) boff[j] = (uint32_t)(((j * 16 + fr) * p.ldb + fg * EPC) * ES);
  const int64_t nks = (K + KSTEP - 1) / KSTEP;
  uint4 af[SKU][MT], bfr[SKU][NT];
  auto load_steps = [&](int64_t base) {  // steps past the end load zero fragments (the MFMAs add nothing)
#pragma unroll
    for (int u = 0; u < SKU; ++u) {
      const int64_t k0 = (base + (int64_t)u * SK_WAVES) * KSTEP;
      const bool kin = k0 + fg * EPC < K;
      const uint32_t kb = (uint32_t)(k0 * ES);
#pragma unroll
      for (int j = 0; j < NT; ++j) bfr[u][j] = bload(rb, kin ? boff[j] + kb : OOB);
#pragma unroll
      for (int i = 0; i < MT; ++i) af[u][i] = bload(ra, kin ? aoff[i] + kb : OOB);
    }
  };
  // LN gamma / beta (K <= SK_LNK) are loaded first, so storing them to LDS waits for these loads only, not for
  // the fragment loads behind them
  const bool fuse_ln = p.ln_gamma != nullptr;
  const bool ln_lds = fuse_ln && K <= SK_LNK;
  constexpr int LNS = (SK_LNK + 64 * SK_WAVES - 1) / (64 * SK_WAVES);  // gamma (and beta) values per thread
  float lg[LNS], lb[LNS];
  if (ln_lds) {
#pragma unroll
    for (int q = 0; q < LNS; ++q) {
      const int k = threadIdx.x + q * 64 * SK_WAVES;
      lg[q] = k < K ? p.ln_gamma[k] : 0.f;
      lb[q] = k < K ? p.ln_beta[k] : 0.f;
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  // every wave runs at least one (possibly all-zero) pass, so the LN-stats barrier below is block-uniform
  load_steps(wave);
  // LayerNorm statistics from the fragments (below): each row's first element, issued with the fragment loads
  // (instantiations with few fragment registers only: the others would spill; LN-fused launches have K = D)
  constexpr bool LN_FRAG = ES == 2 && SKU * (MT + NT) <= 24;
  const bool fold = p.ln_wsum != nullptr;
  const bool ln_frag = LN_FRAG && (fuse_ln || fold) && nks <= (int64_t)SK_WAVES * SKU;
  uint4 x0raw[MT];
  if (LN_FRAG && ln_frag) {
#pragma unroll
    for (int i = 0; i < MT; ++i) x0raw[i] = bload(ra, (uint32_t)((i * 16 + fr) * p.lda * ES));  // rows past M: zero
  }
  __builtin_amdgcn_sched_barrier(0);
  if (ln_lds) {
#pragma unroll
    for (int q = 0; q < LNS; ++q) {
      const int k = threadIdx.x + q * 64 * SK_WAVES;
      if (k < K) {
        lngb[k] = lg[q];
        lngb[SK_LNK + k] = lb[q];
      }
    }
  }

  // Epilogue operands, fetched now so their latency hides under the main loop's: one 4-column quad per thread
  // (bias; the bf16 residual, or dact_src in the backward form, for full quads).
  const int er = threadIdx.x / QPR, ec = (threadIdx.x - er * QPR) * 4;
  const int64_t erow = m0 + er, ecol = n0 + ec;
  const bool eact = threadIdx.x < BM * QPR && erow < M && ecol < N;
  float bias4[4] = {0.f, 0.f, 0.f, 0.f};
  float wsum4[4] = {0.f, 0.f, 0.f, 0.f};  // (folded LayerNorm: W row sums, fetched here, not after the reduction)
  uint2 pre = make_uint2(0u, 0u);
  bool use_pre = false;
  if (eact) {
    // one 16-byte load per operand for a full, aligned quad (the bias / wsum vectors of the decode launches)
    auto quad = [&](const float* v, float* dst) {
      if (ecol + 4 <= N && (reinterpret_cast<uintptr_t>(v + ecol) & 15) == 0) {
        const float4 q = *reinterpret_cast<const float4*>(v + ecol);
        dst[0] = q.x; dst[1] = q.y; dst[2] = q.z; dst[3] = q.w;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) dst[e] = (ecol + e < N) ? v[ecol + e] : 0.f;
      }
    };
    if (p.bias && p.dact == ICAP_ACT_NONE) quad(p.bias, bias4);
    if (p.ln_wsum) quad(p.ln_wsum, wsum4);
    if constexpr (sizeof(TC) == 2) {
      const bf16_t* src = reinterpret_cast<const bf16_t*>(p.dact != ICAP_ACT_NONE ? p.dact_src : p.resid);
      const int64_t lds_ = p.dact != ICAP_ACT_NONE ? p.ld_dact : p.ldr;
      if (src && ecol + 4 <= N && (lds_ & 3) == 0 && (reinterpret_cast<uintptr_t>(src) & 7) == 0) {
        pre = *reinterpret_cast<const uint2*>(src + erow * lds_ + ecol);
        use_pre = true;
      }
    }
  }

  // LayerNorm-fused A (icap_gemm_args.ln_gamma): mean / rstd of the block's rows over all K (two passes: mean,
  // then the centred sum of squares), then (x - mean) * rstd * gamma + beta -> input dtype per fragment.
  // bf16 with every k-step in registers (nks <= 8 SKU, the decode launches): the statistics come from the
  // fragments themselves (lane sums -> the 4 lane groups -> the 8 waves through LDS, fixed order), so LN costs no
  // extra global reads; otherwise the loop form (16 threads per row, the order and rounding of ln_fwd8_kernel).
  // gamma / beta are staged in LDS when K <= SK_LNK (above); the barriers below publish them.
  __shared__ float ln_mr[BM][2];
  __shared__ float lnp[SK_WAVES][BM];
  __shared__ float lnp2[SK_WAVES][BM];
  // folded LayerNorm (icap_gemm_args.ln_wsum): the same row statistics, but only the epilogue needs them
  // (C = rstd (A.B^T - mean wsum) + bias), so the MFMAs run on the raw fragments without waiting for them: the
  // wave partials are computed after the MFMAs are issued (the VALU pass overlaps the matrix cores), go to LDS and
  // are summed by the epilogue threads after the partial-tile reduction barrier
  float ln_mean[MT], ln_rs[MT];
  // one pass over the fragments: per-row sums of (x - x0) and (x - x0)^2 with x0 the row's first element (the
  // shifted-data form: no cancellation between E[x^2] and mean^2 when |mean| >> std), reduced together (lane
  // groups by shuffles, the 8 waves through LDS in a fixed order); mean = x0 + E[d], var = E[d^2] - E[d]^2
  auto frag_stats = [&]() {
    auto chunk_in = [&](int u) { return (int64_t)(wave + u * SK_WAVES) * KSTEP + fg * EPC < K; };
    float part[MT], part2[MT], x0[MT];
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      float v0[8];
      unpack_bf16(x0raw[i], v0);
      x0[i] = v0[0];
      part[i] = 0.f;
      part2[i] = 0.f;
#pragma unroll
      for (int u = 0; u < SKU; ++u) {
        if (chunk_in(u)) {
          const int64_t kc = (int64_t)(wave + u * SK_WAVES) * KSTEP + fg * EPC;
          float v[8];
          unpack_bf16(af[u][i], v);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = kc + e < K ? v[e] - x0[i] : 0.f;
            part[i] += d;
            part2[i] += d * d;
          }
        }
      }
      part[i] = xor32_sum(xor16_sum(part[i]));
      part2[i] = xor32_sum(xor16_sum(part2[i]));
      if (fg == 0) {
        lnp[wave][i * 16 + fr] = part[i];
        lnp2[wave][i * 16 + fr] = part2[i];
        if (fold && wave == 0) ln_mr[i * 16 + fr][0] = x0[i];
      }
    }
  };
  if (LN_FRAG && ln_frag && fuse_ln) {
    frag_stats();
    {
      __syncthreads();
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        float t = 0.f, t2 = 0.f;
#pragma unroll
        for (int w = 0; w < SK_WAVES; ++w) {
          t += lnp[w][i * 16 + fr];
          t2 += lnp2[w][i * 16 + fr];
        }
        const float dm = t / (float)K;
        float v0[8];
        unpack_bf16(x0raw[i], v0);
        ln_mean[i] = v0[0] + dm;
        const float var = t2 / (float)K - dm * dm;
        ln_rs[i] = 1.f / sqrtf((var > 0.f ? var : 0.f) + p.ln_eps);
      }
    }
  } else if ((fuse_ln || fold) && !(LN_FRAG && ln_frag)) {
    const int t = threadIdx.x & 15;
    for (int rr = threadIdx.x >> 4; rr < BM; rr += 64 * SK_WAVES / 16) {
      const int64_t row = m0 + rr < M ? m0 + rr : M - 1;
      const TI* xr = reinterpret_cast<const TI*>(p.A) + row * p.lda;
      float s = 0.f;
      for (int64_t k = (int64_t)t * EPC; k < K; k += 16 * EPC) {
        float v[EPC];
        if constexpr (EPC == 8) io<TI>::ld8(xr + k, v); else io<TI>::ld4(xr + k, v);
#pragma unroll
        for (int e = 0; e < EPC; ++e) s += v[e];
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
      const float mean = s / (float)K;
      float s2 = 0.f;
      for (int64_t k = (int64_t)t * EPC; k < K; k += 16 * EPC) {
        float v[EPC];
        if constexpr (EPC == 8) io<TI>::ld8(xr + k, v); else io<TI>::ld4(xr + k, v);
#pragma unroll
        for (int e = 0; e < EPC; ++e) s2 += (v[e] - mean) * (v[e] - mean);
      }
#pragma unroll
      for (int o = 8; o > 0; o >>= 1) s2 += __shfl_xor(s2, o, 64);
      if (t == 0) {
        ln_mr[rr][0] = mean;
        ln_mr[rr][1] = 1.f / sqrtf(s2 / (float)K + p.ln_eps);
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      ln_mean[i] = ln_mr[i * 16 + fr][0];
      ln_rs[i] = ln_mr[i * 16 + fr][1];
    }
  }
  for (int64_t base = wave;;) {
    // all SKU steps' loads are issued before the first MFMA waits (without this fence hipcc sinks each load
    // to its use and every MFMA waits out a full memory latency)
    __builtin_amdgcn_sched_barrier(0);
    if (fuse_ln) {
#pragma unroll
      for (int u = 0; u < SKU; ++u) {
        const int64_t k0 = (base + (int64_t)u * SK_WAVES) * KSTEP + fg * EPC;
        if (k0 < K) {  // K-tail / past-the-end chunks stay zero
          float g[EPC], bt[EPC];
          if (ln_lds) {
#pragma unroll
            for (int e = 0; e < EPC; e += 4) {
              const float4 gv = *reinterpret_cast<const float4*>(&lngb[k0 + e]);
              const float4 bv = *reinterpret_cast<const float4*>(&lngb[SK_LNK + k0 + e]);
              g[e] = gv.x; g[e + 1] = gv.y; g[e + 2] = gv.z; g[e + 3] = gv.w;
              bt[e] = bv.x; bt[e + 1] = bv.y; bt[e + 2] = bv.z; bt[e + 3] = bv.w;
            }
          } else if constexpr (EPC == 8) {
            io<float>::ld8(p.ln_gamma + k0, g); io<float>::ld8(p.ln_beta + k0, bt);
          } else {
            io<float>::ld4(p.ln_gamma + k0, g); io<float>::ld4(p.ln_beta + k0, bt);
          }
#pragma unroll
          for (int i = 0; i < MT; ++i) af[u][i] = ln_chunk<TI>(af[u][i], ln_mean[i], ln_rs[i], g, bt);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < SKU; ++u)
#pragma unroll
      for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) mfma_chunk<TI>(acc[i][j], af[u][i], bfr[u][j]);
    base += SK_WAVES * SKU;
    if (base >= nks) break;
    load_steps(base);
  }
  if (LN_FRAG && ln_frag && !fuse_ln) frag_stats();  // folded: one pass, after the MFMAs are issued
  // round 1: waves [HALF, 2 HALF) park their partials, waves [0, HALF) add them; round 2: the HALF sums -> LDS
  auto park = [&](float* dst) {
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) dst[(i * 16 + fg * 4 + v) * RLD + j * 16 + fr] = acc[i][j][v];
  };
  if (wave >= HALF) park(red[wave - HALF]);
  __syncthreads();
  if (wave < HALF) {
    const float* src = red[wave];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) acc[i][j][v] += src[(i * 16 + fg * 4 + v) * RLD + j * 16 + fr];
    park(red[wave]);  // same addresses this lane just read: no cross-lane hazard
  }
  __syncthreads();
  if (!eact) return;
  const uint64_t seed = drop_thresh != 0u ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  float x[4];
  *reinterpret_cast<float4*>(x) = *reinterpret_cast<const float4*>(&red[0][er * RLD + ec]);
#pragma unroll
  for (int w = 1; w < HALF; ++w) {
    const float4 v = *reinterpret_cast<const float4*>(&red[w][er * RLD + ec]);
    x[0] += v.x; x[1] += v.y; x[2] += v.z; x[3] += v.w;
  }
  if (fold) {  // rstd (acc - mean wsum); the host passed bias = b + W . beta
    float mean, rs;
    if (ln_frag) {  // the wave partials in wave order (the order of the LN-fused form above)
      float t = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < SK_WAVES; ++w) {
        t += lnp[w][er];
        t2 += lnp2[w][er];
      }
      const float dm = t / (float)K;
      mean = ln_mr[er][0] + dm;
      const float var = t2 / (float)K - dm * dm;
      rs = 1.f / sqrtf((var > 0.f ? var : 0.f) + p.ln_eps);
    } else {
      mean = ln_mr[er][0];
      rs = ln_mr[er][1];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) x[e] = ecol + e < N ? rs * (x[e] - mean * wsum4[e]) : x[e];
  }
  // two call sites rather than a selected pointer (a pointer select on a local puts it in scratch)
  if (use_pre) epiw<TC, 4>(p, erow, ecol, x, bias4, ecol + 4 <= N, seed, drop_thresh, inv_keep, &pre);
  else epiw<TC, 4>(p, erow, ecol, x, bias4, ecol + 4 <= N, seed, drop_thresh, inv_keep);
}

// Split-K reduction: sum the fp32 partial slabs of `splits` K-ranges in a fixed order (deterministic) and
// apply the full epilogue. One thread per 4 consecutive columns.
template <typename TC>
__global__ __launch_bounds__(256) void gemm_splitk_reduce(icap_gemm_args p, int splits, uint32_t drop_thresh,
                                                         float inv_keep) {
  const int64_t M = p.M, N = p.N;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n4 = N >> 2;
  if (q >= M * n4) return;
  const int64_t row = q / n4, col = (q - row * n4) * 4;
  if (p.m_dev && row >= (int64_t)*p.m_dev) return;
  const float* ws = reinterpret_cast<const float*>(p.workspace) + row * N + col;
  float x[4];
  *reinterpret_cast<float4*>(x) = *reinterpret_cast<const float4*>(ws);
  for (int s = 1; s < splits; ++s) {
    const float4 v = *reinterpret_cast<const float4*>(ws + (int64_t)s * M * N);
    x[0] += v.x; x[1] += v.y; x[2] += v.z; x[3] += v.w;
  }
  float bias4[4] = {0.f, 0.f, 0.f, 0.f};
  if (p.bias && p.dact == ICAP_ACT_NONE) {
#pragma unroll
    for (int e = 0; e < 4; ++e) bias4[e] = p.bias[col + e];  // flat-parameter views: only 4-byte aligned
  }
  const uint64_t seed = drop_thresh != 0u ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  epi4<TC>(p, row, col, x, bias4, true, seed, drop_thresh, inv_keep);
}


// ---------------------------------------------------------------------------------------------------------------
}  // namespace icap

using namespace icap;

// Tile-kernel variant. Measured on MI355X (tools/gemm_bench.py, profiles/r01_gemm_variants.txt): short K (<= 16 stages) is
// bound by the per-block prologue/epilogue, which co-resident blocks hide -> single LDS buffer, 3-4 blocks/CU (4
// when the epilogue moves a second M x N tensor: dact_src read / aux store); long K favours the double-buffered
// main loop at 2 blocks/CU.
static int gemm_variant(const icap_gemm_args& p, int64_t nk_per_block) {
  if (nk_per_block > 16) return 0;
  const bool heavy = p.dact != ICAP_ACT_NONE || p.aux;
  const bool act = p.act != ICAP_ACT_NONE || p.dact != ICAP_ACT_NONE;
  // (A/B) ICAP_VAR_HEAVY / ICAP_VAR_ACT / ICAP_VAR_LIGHT: variant for short-K launches with dact / aux, with an
  // activation only, and with neither. Round 4: dact / aux launches at 3 blocks / CU too — the 4-block form (128
  // VGPRs) spills with those epilogues (profiles/r04_gemm_tiles_ab.txt: GPT-2 c_fc gelu + aux 42.2 vs 46.2 us,
  // mlp c_proj dgelu 43.4 vs 43.5)
  static const int vh = diag_env("ICAP_VAR_HEAVY", 4), va = diag_env("ICAP_VAR_ACT", 4), vl = diag_env("ICAP_VAR_LIGHT", 4);
  return heavy ? vh : act ? va : vl;
}

// compute units of the current device (the skinny-GEMM grid rule, the 256 x 256 kernel's pick)
static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cus[dev] = n;
  }
  return cus[dev];
}

namespace icap {
int gemm256_launch(const icap_gemm_args& p, uint32_t thr, float inv_keep, hipStream_t s);
int gemm8p_launch(const icap_gemm_args& p, int bn, int actk, uint32_t thr, float inv_keep, hipStream_t s);
}

// The 256-row 8-phase kernel (gemm8p.hip): bf16 row-major operands, one K range (no split), the epilogue forms it
// instantiates (none / gelu_new fwd or bwd / any, the LayerNorm producer without an activation, the consumer without
// one or with gelu_new). Returns its epilogue kind (ACT_* | ACT_LNS / ACT_LNF), or -1 when the launch is not one
// of them. (diagnostic build) ICAP_GEMM8P = 0 never, 128 / 256 forced where eligible, default the shape rule.
static int g8p_actk(const icap_gemm_args& p) {
  if (p.in_dtype != ICAP_BF16 || p.trans_ab || p.ln_gamma || (p.ln_wsum && !p.ln_stats_in) || p.split_k > 1) return -1;
  if (p.M < 256 || p.K < 64 || p.path == 1 || p.path == 3 || p.path >= 6) return -1;  // (6 ... 10: other forced forms)
  if (p.M * p.lda >= (1ll << 30) || p.N * p.ldb >= (1ll << 30)) return -1;  // 32-bit DMA byte offsets per tile
  const int fa = p.dact == ICAP_ACT_NONE ? p.act : -1, ba = p.act == ICAP_ACT_NONE ? p.dact : -1;
  int a;
  if (p.act == ICAP_ACT_NONE && p.dact == ICAP_ACT_NONE) a = ACT_OFF;
  else if (fa == ICAP_ACT_GELU_NEW) a = ACT_FWD + ICAP_ACT_GELU_NEW;
  else if (ba == ICAP_ACT_GELU_NEW) a = ACT_BWD + ICAP_ACT_GELU_NEW;
  else a = ACT_ANY;
  if (p.ln_stats_out) return a == ACT_OFF ? ACT_LNS : -1;
  if (p.ln_stats_in) return (a == ACT_OFF || a == ACT_FWD + ICAP_ACT_GELU_NEW) ? ACT_LNF + a : -1;
  return a;
}
static int g8p_mode() { return diag_env("ICAP_GEMM8P", 1); }

// Variant 22 (gemm_tile_r256.hip: 256 x 128 tiles, 8 waves, 3-stage ring, one block per CU): its epilogue kind for
// an unsplit bf16 row-major launch, or -1 (the forms it instantiates: none, gelu_new fwd / bwd, quick_gelu fwd, any;
// the LayerNorm producer without an activation, the consumer without one or with gelu_new / quick_gelu).
static int r256_actk(const icap_gemm_args& p) {
  if (p.in_dtype != ICAP_BF16 || p.trans_ab || p.ln_gamma || (p.ln_wsum && !p.ln_stats_in)) return -1;
  const int fa = p.dact == ICAP_ACT_NONE ? p.act : -1, ba = p.act == ICAP_ACT_NONE ? p.dact : -1;
  int a;
  if (p.act == ICAP_ACT_NONE && p.dact == ICAP_ACT_NONE) a = ACT_OFF;
  else if (fa == ICAP_ACT_GELU_NEW) a = ACT_FWD + ICAP_ACT_GELU_NEW;
  else if (ba == ICAP_ACT_GELU_NEW) a = ACT_BWD + ICAP_ACT_GELU_NEW;
  else if (fa == ICAP_ACT_QUICK_GELU) a = ACT_FWD + ICAP_ACT_QUICK_GELU;
  else a = ACT_ANY;
  if (p.c_dtype != ICAP_BF16) return (p.ln_stats_out || p.ln_stats_in) ? -1 : (a == ACT_OFF ? ACT_OFF : ACT_ANY);
  if (p.ln_stats_out) return a == ACT_OFF ? ACT_LNS : -1;
  if (p.ln_stats_in) return (a == ACT_OFF || a == ACT_FWD + ICAP_ACT_GELU_NEW || a == ACT_FWD + ICAP_ACT_QUICK_GELU) ? ACT_LNF + a : -1;
  return a;
}
// epilogue kind of variant 24 (192 x 64 tiles), -1 where it has no form: bf16 row-major operands, no LayerNorm fold /
// consumer; the statistics producer and activation-free launches get their own kinds, the rest the dispatching one
static int w192_actk(const icap_gemm_args& p) {
  if (p.in_dtype != ICAP_BF16 || p.trans_ab || p.ln_gamma || p.ln_wsum || p.ln_stats_in) return -1;
  const bool plain = p.act == ICAP_ACT_NONE && p.dact == ICAP_ACT_NONE;
  if (p.ln_stats_out) return (plain && p.c_dtype == ICAP_BF16) ? ACT_LNS : -1;
  return plain ? ACT_OFF : ACT_ANY;
}
// epilogue kind of the split-role ring variants (26: 128 x 256, 27: 96 x 128), -1 where it has no form: bf16 row-major
// operands, no ln_gamma / decode fold; 27 has no LayerNorm consumer (its 96-row tiles do not pair two threads per row)
static int roles_actk(const icap_gemm_args& p, int v) {
  if (p.in_dtype != ICAP_BF16 || p.trans_ab || p.ln_gamma || (p.ln_wsum && !p.ln_stats_in)) return -1;
  const int fa = p.dact == ICAP_ACT_NONE ? p.act : -1, ba = p.act == ICAP_ACT_NONE ? p.dact : -1;
  int a;
  if (p.act == ICAP_ACT_NONE && p.dact == ICAP_ACT_NONE) a = ACT_OFF;
  else if (v == 27 || v == 32) a = ACT_ANY;
  else if (fa == ICAP_ACT_GELU_NEW) a = ACT_FWD + ICAP_ACT_GELU_NEW;
  else if (ba == ICAP_ACT_GELU_NEW) a = ACT_BWD + ICAP_ACT_GELU_NEW;
  else if (fa == ICAP_ACT_QUICK_GELU) a = ACT_FWD + ICAP_ACT_QUICK_GELU;
  else if (v == 28 && fa == ICAP_ACT_RELU) a = ACT_FWD + ICAP_ACT_RELU;
  else if (v == 28 && ba == ICAP_ACT_RELU) a = ACT_BWD + ICAP_ACT_RELU;
  else a = ACT_ANY;
  if (p.c_dtype != ICAP_BF16) return (p.ln_stats_out || p.ln_stats_in) ? -1 : (a == ACT_OFF ? ACT_OFF : ACT_ANY);
  if (p.ln_stats_out) return a == ACT_OFF ? ACT_LNS : -1;
  if (p.ln_stats_in) {
    if (v == 27 || v == 32) return -1;
    return (a == ACT_OFF || a == ACT_FWD + ICAP_ACT_GELU_NEW || a == ACT_FWD + ICAP_ACT_QUICK_GELU) ? ACT_LNF + a : -1;
  }
  return a;
}
// (diagnostic build) ICAP_ROLES = 0: never take variants 26 / 27 automatically
static int roles_mode() { return diag_env("ICAP_ROLES", 1); }

// (diagnostic build) ICAP_W192 = 1: take variant 24 / 25 for every eligible launch of path 0; 2: never automatically
static int w192_mode() { return diag_env("ICAP_W192", 0); }
// (diagnostic build) ICAP_R256 = 1: take variant 22 for every eligible unsplit launch of path 0
static int r256_mode() { return diag_env("ICAP_R256", 0); }

// (diagnostic build) ICAP_GEMM256: 0 = never, 2 = wherever eligible, default = the shape rule below
static int g256_mode() {
  static const int m = [] {
    const int v = diag_env("ICAP_GEMM256", 1);
    return v == 0 || v == 2 ? v : 1;
  }();
  return m;
}

// The 256 x 256 kernel's preconditions, and when it is the automatic choice. It runs one block per CU, so a
// tile's prologue (first DMA round trip) and epilogue do not overlap other tiles' MFMAs: it beats the 128-row
// tile kernels (2-3 blocks per CU) on long K (4096^3: 1.09-1.22 vs 0.95 PF) and on many full tile rounds (LM
// head 8320 x 50304 x 768: 758 vs 835 us), not on the train step's 2-round K = 768 products (8320 x 3072 x 768:
// 84 vs 80 us) (profiles/r02_gemm256_bench.txt). path 3 forces it where eligible.
static bool g256_pick(const icap_gemm_args& p) {
  if (p.path == 1 || (p.path >= 4 && p.path <= 12)) return false;
  if (p.in_dtype != ICAP_BF16 || p.trans_ab || p.ln_gamma || p.beta != 0.f || p.m_dev || p.split_k > 1) return false;
  if (p.ln_stats_out || p.ln_stats_in) return false;
  if (p.M < 256 || p.N < 256 || p.K < 64) return false;
  if (p.path == 3 || g256_mode() == 2) return true;
  if (g256_mode() == 0) return false;
  const int64_t tiles = ((p.M + 255) / 256) * ((p.N + 255) / 256);
  const int64_t cus = device_cus();
  const int64_t rounds = (tiles + cus - 1) / cus;
  const bool full = tiles * 10 >= rounds * cus * 7;  // rounds at least 70 % occupied
  return (p.K >= 2048 && tiles * 4 >= cus * 3 && full) || (rounds >= 4 && tiles * 10 >= rounds * cus * 8);
}

static bool al16(const void* ptr) { return (reinterpret_cast<uintptr_t>(ptr) & 15) == 0; }

// A/B switches for the in-launch split-K: ICAP_FUSED_S = forced split count (read once), ICAP_FUSED_NST = 1 gives
// its K ranges the variant rule, 4 the 4-stage ring (default: the double-buffered kernel)
static int fused_s_override() {
  static const int v = diag_env("ICAP_FUSED_S", 0);
  return v;
}
// K-skew: tile (tm, tn) walks its K range starting at step ((7 tm + tn) * skew) mod nk and wraps, so the tiles of
// one XCD that share an A row panel (consecutive tn) or a B panel do not request the same lines in lockstep (a
// line they all miss on is fetched once and waited for by every one of them). Measured over the packed train step
// (eager per-shape table, profiles/r03_kskew_ab.txt): skew 1 took the N = 768 products 5-15 % shorter and the step
// 11.3 -> 10.9 ms; skew 2-4 less; launches over more than 64 k-steps per split (the LM-head dX, K = 50304) ran
// longer, so they keep the natural order. ICAP_KSKEW overrides the skew (0 = off; A/B only); path 1 (tile_only)
// keeps the natural order (the path-equality tests compare it bitwise with the 256 x 256 kernel).
static int kskew_for(const icap_gemm_args& p, int64_t nk_split) {
  static const int v = diag_env("ICAP_KSKEW", 1);
  if (p.path == 1 || p.path >= 6 || p.in_dtype == ICAP_FP8_MX || nk_split > 64) return 0;
  return v > 0 && v < 256 ? v : 0;
}
// ICAP_GEMM_DIAG = 1 / 2 / 3: drop the A / B / both operands' staging loads of the tile kernels (zero-record
// descriptors) — a timing diagnostic for what the operand traffic costs; the outputs are wrong. Never in a real run.
// ICAP_FUSED_ACQUIRE=1: the in-launch split-K's last arriver runs an agent-scope acquire after its ticket poll
static int gemm_acquire() { return diag_env("ICAP_FUSED_ACQUIRE", 0) == 1 ? 1 : 0; }
// (diagnostic build) ICAP_KOUT_FUSED=1: K-outer weight-gradient splits combine in the launch
static bool kout_fused_on() { return diag_env("ICAP_KOUT_FUSED", 0) == 1; }
// (diagnostic build, read per launch: an A/B driver toggles it in one process)
static int gemm_diag() { return diag_env("ICAP_GEMM_DIAG", 0) & 3; }
// (diagnostic build) ICAP_SPEC_ACT=0: the runtime-dispatch epilogue everywhere
static bool spec_act_on() { return diag_env("ICAP_SPEC_ACT", 1) != 0; }
// (diagnostic build, read per call) ICAP_FUSED_MINK: fewest K stages for the in-launch split
static int fused_min_nk() {
  const int v = diag_env("ICAP_FUSED_MINK", 0);
  return v >= 2 ? v : 24;
}
// (diagnostic build, read per call: tools/gemm_tiles_ab.py toggles it in one process)
static int fused_nst_override() { return diag_env("ICAP_FUSED_NST", 0); }


// The automatic choice of the split-role variants (0 = neither), one round of tiles at one block per CU (the kernel
// walks the tiles, but a second round pays a whole prologue / main loop / epilogue with nothing beside it). Measured
// against the automatic plan of round 5 (profiles/r06_roles_ab.txt, graph replay, packed rows): N <= 1024 on 96 x 128
// tiles — GPT-2 c_attn dX 3584 x 768 x 2304 30.5 -> 20.3 us, c_fc dX x 3072 33.9 -> 24.4, mlp c_proj fwd (+ LayerNorm
// statistics) 38.5 -> 28.1, attn c_proj 17.0 -> 14.4 / 12.4 -> 11.0, mapper 3200 x 768 x 3072 33.1 -> 25.3, CLIP fc2
// 6400 x 768 x 3072 (1.6 rounds, long K) 53.2 -> 48.2; CLIP's 6400 x 768 x 768 (1.6 rounds, short K) 20.4 -> 23.0: not
// taken. N > 1024 on 128 x 256 tiles where they fill one round: c_attn (LayerNorm consumer) 26.4 -> 24.5, mapper qkv
// 22.5 -> 19.9; the N = 3072 products (336 tiles: two rounds) 36.9 -> 45.1: not taken. Long K over fewer tiles
// (the LM-head dX, K = 50304 over 1792 rows) keeps the split-K kernels.
static int roles_pick(const icap_gemm_args& p, int64_t m_plan, int64_t nk, int64_t cus) {
  if (p.in_dtype != ICAP_BF16 || p.trans_ab || p.split_k > 1) return 0;
  if (p.N <= 1024) {
    const int64_t t = ((m_plan + 95) / 96) * ((p.N + 127) / 128);
    // more than one round of 96 x 128 tiles, one of 160 x 128 at least 80 % full: 160 x 128 (CLIP-B/32's 6400 x 768
    // out_proj / fc2 with the LayerNorm statistics: 240 tiles against 402, profiles/r06_roles160_ab.txt)
    const int64_t t160 = ((m_plan + 159) / 160) * ((p.N + 127) / 128);
    if (nk <= 96 && t > cus && t160 <= cus && t160 * 10 >= cus * 8) return 32;
    if (nk > 96 || t * 5 < cus * 3) return 0;
    return (t <= cus || (nk >= 32 && 2 * t >= 3 * cus && t <= 2 * cus)) ? 27 : 0;
  }
  // (one row tile — the greedy decode's LM head, 128 x 50304 — stays on the double-buffered tile loop below: 20.4
  // vs 21.9 us, profiles/r06_lmhead_dx_ab.txt)
  const int64_t t = ((m_plan + 127) / 128) * ((p.N + 255) / 256);
  return (m_plan > 128 && t <= cus && t * 5 >= cus * 3) ? 26 : 0;
}

static int gemm_plan(const icap_gemm_args& p, GemmPlan& pl) {
  ICAP_REQUIRE(p.M >= 0 && p.N >= 0 && p.K >= 0, "icap_gemm: negative size");
  ICAP_REQUIRE(p.path == 0 || p.path == 1 || (p.path >= 3 && p.path <= 12), "icap_gemm: path must be 0, 1 or 3 ... 12");
  ICAP_REQUIRE(p.A && p.B && p.C, "icap_gemm: null operand");
  ICAP_REQUIRE(p.in_dtype == ICAP_F32 || p.in_dtype == ICAP_BF16 || p.in_dtype == ICAP_FP8_MX,
               "icap_gemm: bad in_dtype");
  ICAP_REQUIRE(p.c_dtype == ICAP_F32 || p.c_dtype == ICAP_BF16, "icap_gemm: bad c_dtype");
  const bool mx = p.in_dtype == ICAP_FP8_MX;
  if (mx) {
    ICAP_REQUIRE(p.K % 128 == 0 && p.lda % 16 == 0 && p.ldb % 16 == 0,
                 "icap_gemm: FP8_MX needs K % 128 == 0 and lda, ldb multiples of 16");
    ICAP_REQUIRE(p.a_scale && p.b_scale && al16(p.a_scale) && al16(p.b_scale),
                 "icap_gemm: FP8_MX needs 16-byte aligned a_scale / b_scale");
    ICAP_REQUIRE(!p.trans_ab && !p.ln_gamma && p.path != 3, "icap_gemm: FP8_MX takes no trans_ab / ln / path 3");
    ICAP_REQUIRE((p.K / 32) * ((p.M + 63) / 64) * 64 < 0x7fffffffll && (p.K / 32) * ((p.N + 63) / 64) * 64 < 0x7fffffffll,
                 "icap_gemm: FP8_MX scale arrays must stay below 2 GiB");
  }
  const int epc = p.in_dtype == ICAP_BF16 ? 8 : mx ? 16 : 4;
  ICAP_REQUIRE(p.trans_ab || p.K % epc == 0, "icap_gemm: K must be a multiple of 8 (bf16) / 4 (f32)");
  ICAP_REQUIRE(p.lda % epc == 0 && p.ldb % epc == 0, "icap_gemm: lda/ldb must be multiples of 8 (bf16) / 4 (f32)");
  ICAP_REQUIRE((p.trans_ab || (p.lda >= p.K && p.ldb >= p.K)) && p.ldc >= p.N, "icap_gemm: leading dimension too small");
  ICAP_REQUIRE((reinterpret_cast<uintptr_t>(p.A) & 15) == 0 && (reinterpret_cast<uintptr_t>(p.B) & 15) == 0,
               "icap_gemm: A and B must be 16-byte aligned");
  const int es = p.in_dtype == ICAP_BF16 ? 2 : mx ? 1 : 4;
  ICAP_REQUIRE((int64_t)256 * p.lda * es < 0x7fffffffll && (int64_t)256 * p.ldb * es < 0x7fffffffll,
               "icap_gemm: a 256-row operand panel must stay below 2 GiB");
  ICAP_REQUIRE(p.beta == 0.f || p.c_dtype == ICAP_F32, "icap_gemm: beta != 0 requires f32 C");
  ICAP_REQUIRE(p.dact == ICAP_ACT_NONE || p.dact_src != nullptr, "icap_gemm: dact requires dact_src");
  ICAP_REQUIRE(p.act >= ICAP_ACT_NONE && p.act <= ICAP_ACT_GELU_ERF && p.dact >= ICAP_ACT_NONE &&
                   p.dact <= ICAP_ACT_GELU_ERF, "icap_gemm: unknown activation");
  ICAP_REQUIRE(p.drop_p >= 0.f && p.drop_p < 1.f, "icap_gemm: drop_p out of range");
  if (p.trans_ab) {
    ICAP_REQUIRE(p.in_dtype == ICAP_BF16, "icap_gemm: trans_ab needs bf16 inputs");
    ICAP_REQUIRE(p.lda >= p.M && p.ldb >= p.N, "icap_gemm: trans_ab needs lda >= M, ldb >= N");
    ICAP_REQUIRE(p.m_dev == nullptr, "icap_gemm: trans_ab does not take m_dev");
    ICAP_REQUIRE((int64_t)(p.K + 64) * p.lda * 2 < 0x7fffffffll && (int64_t)(p.K + 64) * p.ldb * 2 < 0x7fffffffll,
                 "icap_gemm: trans_ab operands must stay below 2 GiB");
  }
  const int64_t tiles_m = (p.M + GBM - 1) / GBM;
  int64_t tiles_n = (p.N + GBN - 1) / GBN;
  int64_t tiles = tiles_m * tiles_n;
  ICAP_REQUIRE(tiles < (1ll << 26), "icap_gemm: too many tiles");
  ICAP_REQUIRE(p.split_k >= 0, "icap_gemm: split_k must be >= 0");
  pl.thr = p.drop_p > 0.f ? drop_threshold(p.drop_p) : 0u;
  pl.inv_keep = p.drop_p > 0.f ? 1.f / (1.f - p.drop_p) : 1.f;
  const bool fuse_ln = p.ln_gamma != nullptr;
  ICAP_REQUIRE(!fuse_ln || (p.ln_beta && p.M <= 128 && p.split_k == 0 && !p.trans_ab && p.K <= 4096),
               "icap_gemm: ln_gamma needs ln_beta, M <= 128, K <= 4096, no split_k / trans_ab");
  const bool lnx = p.ln_stats_out || p.ln_stats_in;  // the tile kernels' LayerNorm statistics hand-off
  if (lnx) {
    ICAP_REQUIRE(p.in_dtype == ICAP_BF16 && p.c_dtype == ICAP_BF16 && !p.trans_ab && !fuse_ln && p.path != 3 &&
                     !(p.ln_stats_out && p.ln_stats_in) && p.beta == 0.f,
                 "icap_gemm: ln_stats_out / ln_stats_in: bf16 A/B/C, no trans_ab / ln_gamma / path 3 / beta, not both");
    ICAP_REQUIRE(!p.ln_stats_out || (p.N % 32 == 0 && p.act == ICAP_ACT_NONE && p.dact == ICAP_ACT_NONE),
                 "icap_gemm: ln_stats_out needs N % 32 == 0 and no activation");
    ICAP_REQUIRE(!p.ln_stats_in || (p.ln_wsum && p.K % 128 == 0 && p.K <= 1280 && p.dact == ICAP_ACT_NONE &&
                                    al16(p.ln_stats_in) && (p.ln_mean_out == nullptr) == (p.ln_rstd_out == nullptr)),
                 "icap_gemm: ln_stats_in needs ln_wsum, K % 128 == 0, K <= 1280, 16-byte aligned statistics, no dact, "
                 "ln_mean_out with ln_rstd_out");
  }
  const bool fold_ln = p.ln_wsum != nullptr && !p.ln_stats_in;  // (the skinny decode form: stats from A fragments)
  ICAP_REQUIRE(!fold_ln || (!fuse_ln && p.M <= 128 && p.split_k == 0 && !p.trans_ab && !mx && p.K <= 4096),
               "icap_gemm: ln_wsum needs M <= 128, no ln_gamma / split_k / trans_ab / FP8_MX, K <= 4096");
  if (p.M <= 128 && p.split_k == 0 && (tiles <= 128 || fuse_ln || fold_ln) && !p.trans_ab && !mx && !lnx) {
    pl.skinny = true;
    // the fewest 16-column slabs per block that keep the grid within one pass over the CUs (every CU streams one
    // block's A rows + W slab; a second block on a CU doubles its bytes), then enough k-steps in flight per wave
    // to cover K in one round trip where the fragment registers allow (SKU in {3, 4, 6}; 12 for one-slab blocks)
    const int64_t gy = (p.M + 31) / 32;
    const int cus = device_cus();
    pl.nt = 4;
    for (int nt = 1; nt <= 4; ++nt)
      if ((p.N + 16 * nt - 1) / (16 * nt) * gy <= cus) { pl.nt = nt; break; }
    if (p.in_dtype == ICAP_BF16) {
      const int64_t need = ((p.K + 31) / 32 + SK_WAVES - 1) / SK_WAVES;
      pl.sku = need <= 3 ? 3 : need <= 4 ? 4 : (need <= 6 || pl.nt > 1) ? 6 : 12;
    } else {
      pl.sku = 6;
    }
    pl.grid = dim3((unsigned)((p.N + 16 * pl.nt - 1) / (16 * pl.nt)), (unsigned)gy);
    pl.block = dim3(64 * SK_WAVES);
    return ICAP_OK;
  }
  // 256 x 256 8-phase kernel (gemm256.hip) for wide products whose 256-tiles fill the chip in few, full rounds
  if (g256_pick(p)) {
    pl.g256 = true;
    return ICAP_OK;
  }
  // the 256-row 8-phase kernel (gemm8p.hip) where its tiles fill the chip in one round
  if (const int a8 = g8p_actk(p); a8 >= 0) {
    const int mode = p.path == 4 ? 128 : p.path == 5 ? 256 : g8p_mode();
    int bn = 0;
    if (mode == 128 || mode == 256) {
      bn = mode;
    } else if (mode == 1) {
      // one round of 256 x 256 tiles at least 80 % full, K <= 1536: there it beat every 128-row form (CLIP-B/32's
      // 6400 x 2304 x 768 QKV: 30.6 vs 38.6 us; x 1536: 47.6 vs 68.5); 256 x 128 tiles and other shapes did not
      // (the 3584-row products: within 3 %; N = 768: 30-60 % slower) — profiles/r05_g8p_ab.txt
      const int64_t m_pl = (p.m_dev && p.m_hint > 0 && p.m_hint < p.M) ? p.m_hint : p.M;
      const int64_t t256 = ((m_pl + 255) / 256) * ((p.N + 255) / 256);
      const int64_t cus = device_cus();
      // and (round 6) many rounds of them: the compact LM head, 1664 live rows x 50304 x 768 = 1379 tiles: 157 vs
      // 180 us on the 3-block 128 x 128 tiles (hipBLASLt 146; profiles/r06_lmhead_ab.txt)
      if (p.K <= 1536 && ((t256 * 10 >= cus * 8 && t256 <= cus) || t256 >= 4 * cus)) bn = 256;
    }
    if (bn) {
      pl.g8p = bn;
      pl.actk = a8;
      pl.thr = p.drop_p > 0.f ? drop_threshold(p.drop_p) : 0u;
      pl.inv_keep = p.drop_p > 0.f ? 1.f / (1.f - p.drop_p) : 1.f;
      return ICAP_OK;
    }
  }
  // variant 31 (round 6): the K-outer weight-gradient products on the split-role ring (4 MFMA + 4 LDS-DMA waves,
  // 128 x 128 tiles, 4 stages, one block per CU), K split so tiles x splits fill about one round of CUs, the splits
  // combined by the slab + reduce pass. path 11 forces it for bf16 K-outer launches.
  if (p.trans_ab && p.in_dtype == ICAP_BF16 && p.path == 11) {
    const int64_t nk31 = (p.K + 63) / 64;
    const int64_t cus = device_cus();
    int64_t s31 = p.split_k >= 1 ? p.split_k : cus / tiles;
    if (s31 > 8) s31 = 8;
    while (s31 > 1 && nk31 / s31 < 4) --s31;
    if (s31 < 1) s31 = 1;
    const int64_t nks31 = (nk31 + s31 - 1) / s31;
    s31 = (nk31 + nks31 - 1) / nks31;  // every split gets >= 1 stage
    if (s31 > 1) {
      ICAP_REQUIRE((p.N & 3) == 0, "icap_gemm: split-K requires N % 4 == 0");
      ICAP_REQUIRE(p.workspace && (reinterpret_cast<uintptr_t>(p.workspace) & 15) == 0 &&
                       p.workspace_bytes >= s31 * p.M * p.N * (int64_t)sizeof(float),
                   "icap_gemm: split-K workspace missing, misaligned or too small");
    }
    pl.variant = 31;
    pl.splits = (int)s31;
    pl.fused = false;
    pl.nk_split = (int)nks31;
    pl.tiles_n = (int)tiles_n;
    pl.actk = (p.act == ICAP_ACT_NONE && p.dact == ICAP_ACT_NONE) ? ACT_OFF : ACT_ANY;
    pl.block = dim3(2 * GNT);
    pl.grid = dim3((unsigned)(tiles * s31 < cus ? tiles * s31 : cus));  // the kernel walks tiles x splits
    return ICAP_OK;
  }
  // split-K over K stages for launches that cannot fill the chip (decode-time M = batch, small projections):
  // fp32 partial slabs in the caller's workspace + one deterministic reduce/epilogue pass — or, with tickets, the
  // in-launch combine (long K over fewer tiles than CUs: the packed step's N = 768 products, the mapper's M = 3200
  // products and weight gradients): S = 2 * CUs / tiles rounded, 2..4, so the tile x split blocks fill the chip
  // about twice, and no slab round trip or extra launch.
  const int64_t bke = 128 / es;
  const int64_t nk = (p.K + bke - 1) / bke;
  const int64_t slab = p.M * p.N * (int64_t)sizeof(float);
  const int64_t cus = device_cus();
  // with a device row count the kernel choice follows the expected count (m_hint)
  const int64_t m_plan = (p.m_dev && p.m_hint > 0 && p.m_hint < p.M) ? p.m_hint : p.M;
  const int64_t tiles_plan = ((m_plan + GBM - 1) / GBM) * tiles_n;
  // The split count is a function of the shape (M, N, K, dtype, trans_ab; with a device row count, the caller's
  // expected count m_hint) alone — never of the workspace size or of whether tickets are attached — so the partial
  // sums are always added in the same order. Tickets only choose HOW the splits combine (inside the launch or in a
  // reduce pass over slabs); both add the partials in split order starting from split 0 and apply the same epilogue
  // formula, so the two mechanisms store bitwise-identical outputs (tests/test_fused_splitk_gpu.py). A NULL workspace
  // turns the automatic split off (documented: include/icap.h); a given one too small for the shape's split is an error.
  int64_t splits = 1;
  pl.fused = false;
  bool fusable = false;  // the long-K / few-tiles rule below (the splits may combine inside the launch)
  // (not for the K-outer weight-gradient products: measured, their in-launch combine ran 6-7 µs slower than the
  // slab + reduce pass — 768x3072x3200 53 vs 47 µs, profiles/r03_gemm_detail_fused.txt — since the last arriver of
  // a 3-block-per-CU tile reads its partials one accumulator row at a time)
  if (p.split_k == 0 && p.workspace && !p.trans_ab && (p.N & 3) == 0 && nk >= fused_min_nk() && tiles_plan < cus) {
    int64_t sf = (2 * cus + tiles_plan / 2) / tiles_plan;
    if (sf > 4) sf = 4;
    while (sf > 2 && nk / sf < 8) --sf;
    // A/B measurements only (ICAP_FUSED_S): the in-launch combine reads at most 3 other partials (4 splits)
    if (fused_s_override() > 1) sf = fused_s_override() < 4 ? fused_s_override() : 4;
    if (sf >= 2) {
      splits = sf;
      fusable = true;
    }
  }
  if (fusable) {
    const int64_t pbytes = (int64_t)GBM * GBN * (int64_t)sizeof(float);
    const int64_t sfin = splits;
    const int64_t nks_ = (nk + sfin - 1) / sfin;
    const int64_t sreal = (nk + nks_ - 1) / nks_;  // the split count after every split got >= 1 stage (below)
    // with a device row count the grid still covers every row tile of M, so tickets / partials for all of them
    pl.fused = p.tickets && p.tickets_len >= 2 * tiles && p.workspace_bytes >= tiles * sreal * pbytes;
  } else if (p.split_k > 1) {
    splits = p.split_k;
  } else if (p.split_k == 0 && p.workspace && p.trans_ab && (p.N & 3) == 0 && nk >= 16 && tiles < 320) {
    // K-outer weight gradients over the token rows (the mapper's 3200-row products): about 320 blocks, at most 6
    // splits — measured 31.8 / 23.3 / 35.4 / 35.8 us for 2304x768 / 768x768 / 3072x768 / 768x3072 over 3200 rows
    // against 33.9 / 24.7 / 40.3 / 40.2 with the 512-block rule below (profiles/r03_dw_bench.txt)
    splits = (320 + tiles - 1) / tiles;
    if (splits > 6) splits = 6;
    if (kout_fused_on() && splits >= 2) {  // A/B only (ICAP_KOUT_FUSED=1): in-launch combine, at most 4 splits
      if (splits > 4) splits = 4;
      const int64_t pbytes = (int64_t)GBM * GBN * (int64_t)sizeof(float);
      const int64_t nks_ = (nk + splits - 1) / splits;
      const int64_t sreal = (nk + nks_ - 1) / nks_;
      pl.fused = p.tickets && p.tickets_len >= 2 * tiles && p.workspace_bytes >= tiles * sreal * pbytes;
    }
  } else if (p.split_k == 0 && p.workspace && (p.N & 3) == 0 && nk >= 2 && (tiles <= 64 || (tiles < 256 && nk >= 16))) {
    // the count depends on the shape alone — never on the workspace a caller passes — so a product computed on
    // another stream with its own scratch sums its K ranges in the same order and rounds identically (a
    // workspace too small for the shape's split is an error below, not a silent change of the summation order)
    splits = (512 + tiles - 1) / tiles;
    if (tiles > 64 && splits > nk / 4) splits = nk / 4;
    if (splits > 32) splits = 32;
  }
  // the LayerNorm statistics hand-off needs the full epilogue in the tile kernel: a split that could only combine
  // through the reduce pass is not taken (a rule of the call's arguments, so still one summation order per call)
  if (lnx && !fusable && p.split_k != 1) splits = 1;
  if (splits > nk) splits = nk;
  if (splits < 1) splits = 1;
  const int64_t nk_split = nk > 0 ? (nk + splits - 1) / splits : 0;
  if (nk_split > 0) splits = (nk + nk_split - 1) / nk_split;  // every split gets >= 1 stage
  if (splits > 1 && !pl.fused) {
    ICAP_REQUIRE((p.N & 3) == 0, "icap_gemm: split-K requires N % 4 == 0");
    ICAP_REQUIRE(p.workspace && (reinterpret_cast<uintptr_t>(p.workspace) & 15) == 0 &&
                     p.workspace_bytes >= splits * slab,
                 "icap_gemm: split-K workspace missing, misaligned or too small");
  }
  if (pl.fused)
    ICAP_REQUIRE((reinterpret_cast<uintptr_t>(p.workspace) & 15) == 0 && (reinterpret_cast<uintptr_t>(p.tickets) & 7) == 0,
                 "icap_gemm: split-K workspace / tickets misaligned");
  // Short-K launches (<= 16 stages) of fewer than 4 tiles of 128 x 128 per CU (the N = 768 products, the mapper's
  // M = 3200 and CLIP's M = 6400 ones) run faster on 128 x 64 tiles: twice the blocks, so a CU holds more of them
  // to hide each one's prologue / epilogue; longer K keeps 128 x 128 (profiles/r01_gemm_narrow.txt).
  const bool narrow = p.in_dtype == ICAP_BF16 && p.M > 128 && !p.trans_ab && tiles < 1024 && nk <= 16 && splits == 1;
  pl.splits = (int)splits;
  pl.nk_split = (int)nk_split;
  pl.variant = gemm_variant(p, nk_split);
  // one row tile over many column tiles (the greedy decode's LM head, 128 x 50304 x 768): the double-buffered loop
  // (20.8 vs 22.8 µs, profiles/r05_lmhead_probe.txt)
  if (tiles_m == 1 && tiles_n > 256 && splits == 1 && pl.variant == 4) pl.variant = 0;
  // in-launch split-K: the double-buffered main loop at 2 blocks per CU for every split's K range (measured on the
  // packed 3584 x 768 x 3072 / x 2304 products: 36.6 / 30.4 vs 40.1 / 32.4 µs with the single-stage form the
  // per-split K of 16 stages would pick; profiles/r03_fused_ab.txt); ICAP_FUSED_NST=1 restores the variant rule
  if (pl.fused && fused_nst_override() != 1) pl.variant = 0;
  // (A/B only) ICAP_FUSED_NST=4: the in-launch split-K on the 4-stage ring at one block per CU (three stages in
  // flight per CU instead of the double-buffered pair's two)
  if (pl.fused && fused_nst_override() == 4 && p.in_dtype == ICAP_BF16 && !p.trans_ab && !lnx) pl.variant = 16;
  // Long K over at most one 128 x 128 tile per CU and no split (no tickets given): the 4-stage ring at one block per
  // CU (the double-buffered loop at 2 blocks per CU only pays when a CU holds two tiles). Not for the LayerNorm
  // statistics hand-off (the ring has no such epilogue: GPT-2 large's 1280 x 1280 products at small batch).
  if (p.in_dtype == ICAP_BF16 && !p.trans_ab && splits == 1 && nk_split > 16 && tiles_plan <= cus && !lnx)
    pl.variant = 16;
  if (mx && pl.variant == 5) pl.variant = 4;  // MX at 4 blocks / CU (128 VGPRs) spills: 3 blocks / CU
  if (narrow) {
    tiles_n = (p.N + 63) / 64;
    tiles = tiles_m * tiles_n;
    pl.variant = tiles < 256 ? 12 : 13;
  }
  if (p.trans_ab) pl.variant = nk_split > 16 ? 14 : 15;  // K-outer forms of variants 0 / 4
  // (diagnostic build) ICAP_FORCE_TILE = 0 / 4 / 5 / 12 / 13 / 16: that tile variant for unsplit bf16 row-major
  // launches (read per call so one process can interleave the forms). (Round 5 also tried 256 x 128 tiles of 8
  // waves on this template, double-buffered and single-buffered: no faster on any of the step's shapes,
  // profiles/r05_tile_graph_ab.txt; removed.)
  if (const int v = diag_env("ICAP_FORCE_TILE", -1); v >= 0) {
    if (p.in_dtype == ICAP_BF16 && !p.trans_ab && splits == 1 &&
        (v == 0 || v == 4 || v == 5 || v == 12 || v == 13 || (v == 16 && !lnx))) {
      pl.variant = v;
      tiles_n = (v == 12 || v == 13) ? (p.N + 63) / 64 : (p.N + GBN - 1) / GBN;
      tiles = tiles_m * tiles_n;
    }
  }
  // (diagnostic build, read per call) ICAP_LN_VAR = 0 / 4 / 5: that 128 x 128 variant for the LayerNorm hand-off
  if (lnx && (pl.variant == 0 || pl.variant == 4 || pl.variant == 5)) {
    const int lv = diag_env("ICAP_LN_VAR", -1);
    if (lv == 0 || lv == 4 || lv == 5) pl.variant = lv;
  }
  // the LayerNorm-folded quick_gelu consumer (CLIP c_fc) exists at 3 blocks / CU only (gemm_tile_ln.hip)
  if (lnx && pl.variant == 0 && p.act == ICAP_ACT_QUICK_GELU) pl.variant = 4;
  // variants 26 / 27: the split-role ring (gemm_tile.h ROLES) on 128 x 256 / 96 x 128 tiles, one K range per tile
  // (path 8 / 9 force them where eligible; the automatic rule: roles_pick)
  {
    const int rv = p.path == 8 ? 26 : p.path == 9 ? 27 : p.path == 10 ? 28 : p.path == 12 ? 32
                   : (p.path == 0 && roles_mode() != 0) ? roles_pick(p, m_plan, nk, cus) : 0;
    const int bm = rv == 26 ? 128 : rv == 27 ? 96 : rv == 32 ? 160 : 192, bn = (rv == 27 || rv == 32) ? 128 : 256;
    // a caller's split_k > 1 (the long-K LM head dX): K ranges over fp32 slabs + the reduce pass, as the tile path
    // (no LayerNorm hand-off: it needs the whole epilogue in the kernel)
    const bool rsplit = p.split_k > 1 && !lnx && rv != 28;
    if (rv && p.M >= bm && (p.split_k <= 1 || rsplit)) {
      if (const int ar = roles_actk(p, rv); ar >= 0) {
        int64_t rs = 1;
        if (rsplit) {
          rs = p.split_k < nk ? p.split_k : nk;
          rs = (nk + (nk + rs - 1) / rs - 1) / ((nk + rs - 1) / rs);  // every split gets >= 1 stage
        }
        if (rs > 1) {
          ICAP_REQUIRE((p.N & 3) == 0, "icap_gemm: split-K requires N % 4 == 0");
          ICAP_REQUIRE(p.workspace && (reinterpret_cast<uintptr_t>(p.workspace) & 15) == 0 &&
                           p.workspace_bytes >= rs * p.M * p.N * (int64_t)sizeof(float),
                       "icap_gemm: split-K workspace missing, misaligned or too small");
        }
        pl.variant = rv;
        pl.splits = (int)rs;
        pl.fused = false;
        pl.nk_split = (int)((nk + rs - 1) / rs);
        tiles_n = (p.N + bn - 1) / bn;
        tiles = ((p.M + bm - 1) / bm) * tiles_n;
        pl.tiles_n = (int)tiles_n;
        pl.actk = ar;
        pl.block = dim3(rv == 28 ? 3 * GNT : 2 * GNT);  // 12 / 8 waves
        pl.grid = dim3((unsigned)(tiles * rs < cus ? tiles * rs : cus));  // the kernel walks the live tiles
        return ICAP_OK;
      }
    }
  }
  // variant 22: 256 x 128 tiles on the 3-stage ring (path 6 forces it where eligible)
  if (splits == 1 && p.M >= 256 && (p.path == 6 || (p.path == 0 && r256_mode() == 1))) {
    if (const int a22 = r256_actk(p); a22 >= 0) {
      pl.variant = 22;
      tiles_n = (p.N + 127) / 128;
      tiles = ((p.M + 255) / 256) * tiles_n;
      pl.tiles_n = (int)tiles_n;
      pl.actk = a22;
      pl.block = dim3(2 * GNT);
      pl.grid = dim3((unsigned)tiles);
      return ICAP_OK;
    }
  }
  // variant 24: 192 x 64 tiles, unsplit (path 7 forces it where eligible). The automatic plan takes it for the
  // products with N <= 1024 that run unsplit on 128 x 64 tiles (K <= 16 stages: 3584 / 3200 / 6400 x 768 x 768 —
  // one round of 228 / 204 tiles instead of 1.3-2.6 rounds) or on 128 x 128 tiles filling one to two rounds
  // (CLIP's 6400 x 768 x 3072), measured 0.7-1.6 and 5 us faster per launch (profiles/r05_w192_ab.txt); the
  // long-K products that split K inside the launch stay there (33.9 vs 43.9 us on the mapper's 3200 x 768 x 3072).
  // A LayerNorm statistics producer takes the kernel its plain product takes (equal C, tests/test_lnfold_gpu.py;
  // 17.0 vs 17.1 us for GPT-2's attn c_proj)
  bool w24 = p.path == 7 || (p.path == 0 && w192_mode() == 1);
  if (p.path == 0 && w192_mode() != 2 && !p.ln_stats_in && p.N <= 1024 && p.in_dtype == ICAP_BF16 && !p.trans_ab) {
    const int64_t t192 = ((m_plan + 191) / 192) * ((p.N + 63) / 64);
    if (splits == 1 && !pl.fused) {
      if (narrow) w24 = true;
      else if (nk_split > 16 && !p.m_dev && tiles_plan >= cus && tiles_plan <= 2 * cus && t192 <= 2 * cus) w24 = true;
    }
    // (Not for the launches that split K inside the launch: GPT-2's c_attn dX 3584 x 768 x 2304 runs 27.7-28.5 µs
    // unsplit on the 192 x 64 ring against 29.4-30.1 split in isolation, but the step with that rule measured 0.5 %
    // slower — 12833 / 12811 vs 12876 / 12895 images/s, profiles/r05_w192_ab.txt — so the split stays.)
  }
  if (p.M >= 192 && w24) {
    if (const int a24 = w192_actk(p); a24 >= 0) {
      // K > 16 stages over one round of tiles: the 4-stage ring at one block per CU (ICAP_W192R = 2 in the
      // diagnostic build: never). Measured (profiles/r05_w192_ab.txt): GPT-2 c_attn dX 3584 x 768 x
      // 2304 28.1 µs on the ring, 33.0 double-buffered (29.4 with the automatic in-launch split-K); past one round
      // the double-buffered loop at 2 blocks per CU wins by far (CLIP fc2, 408 tiles: 48.2 vs 64.8 µs)
      const int wr = diag_env("ICAP_W192R", 4);
      const int64_t t192 = ((m_plan + 191) / 192) * ((p.N + 63) / 64);
      pl.variant = nk > 16 && wr != 2 && t192 <= cus ? 25 : 24;
      pl.splits = 1;
      pl.fused = false;
      pl.nk_split = (int)nk;
      tiles_n = (p.N + 63) / 64;
      tiles = ((p.M + 191) / 192) * tiles_n;
      pl.tiles_n = (int)tiles_n;
      pl.actk = a24;
      pl.block = dim3(GNT);
      pl.grid = dim3((unsigned)tiles);
      return ICAP_OK;
    }
  }
  pl.tiles_n = (int)tiles_n;
  const bool any_act = (splits == 1 || pl.fused) && (p.act != ICAP_ACT_NONE || p.dact != ICAP_ACT_NONE);
  pl.actk = any_act ? ACT_ANY : ACT_OFF;
  // the step's activated products get an epilogue compiled for their one activation (gemm_common.h ACT_FWD /
  // ACT_BWD): GPT-2 c_fc gelu_new (+ aux) and its dgelu, CLIP c_fc quick_gelu, ViT / DINOv3 c_fc erf gelu, the
  // mapper's relu / drelu (128 x 64 tiles). Measured over the packed step (tools/specact_ab.sh, profiles/
  // r03_specact_ab.txt): 10.98 -> 10.61 ms; the mapper's 3200x3072x768 relu 36.4 -> 29.1 µs, CLIP's quick_gelu
  // 68.6 -> 64.0, gelu + aux 64.5 -> 57.6 — the runtime dispatch over five activations (libm erff / tanhf / expf
  // inlined per case) cost registers and scratch in the epilogue of every activated launch.
  if (any_act && p.in_dtype == ICAP_BF16 && p.c_dtype == ICAP_BF16 && !p.trans_ab && spec_act_on()) {
    const int fa = p.dact == ICAP_ACT_NONE ? p.act : -1, ba = p.act == ICAP_ACT_NONE ? p.dact : -1;
    const bool v045 = pl.variant == 0 || pl.variant == 4 || pl.variant == 5;
    if (v045 && fa == ICAP_ACT_GELU_NEW) pl.actk = ACT_FWD + ICAP_ACT_GELU_NEW;
    else if (v045 && ba == ICAP_ACT_GELU_NEW) pl.actk = ACT_BWD + ICAP_ACT_GELU_NEW;
    else if (pl.variant == 4 && fa == ICAP_ACT_QUICK_GELU) pl.actk = ACT_FWD + ICAP_ACT_QUICK_GELU;
    else if (pl.variant == 4 && fa == ICAP_ACT_GELU_ERF) pl.actk = ACT_FWD + ICAP_ACT_GELU_ERF;
    else if (pl.variant == 13 && fa == ICAP_ACT_RELU) pl.actk = ACT_FWD + ICAP_ACT_RELU;
    else if (pl.variant == 13 && ba == ICAP_ACT_RELU) pl.actk = ACT_BWD + ICAP_ACT_RELU;
  }
  if (lnx) {
    ICAP_REQUIRE(splits == 1 || pl.fused,
                 "icap_gemm: ln_stats_* launches combine split-K inside the launch only (give the workspace tickets)");
    const int v = pl.variant, a = pl.actk;
    const bool ok = p.ln_stats_out
                        ? ((v == 0 || v == 4 || v == 5 || v == 12 || v == 13) && a == ACT_OFF)
                        : ((v == 0 || v == 4 || v == 5 || v == 12 || v == 13) && a == ACT_OFF) ||
                              ((v == 0 || v == 4 || v == 5) && a == ACT_FWD + ICAP_ACT_GELU_NEW) ||
                              (v == 4 && a == ACT_FWD + ICAP_ACT_QUICK_GELU) || ((v == 12 || v == 13) && a == ACT_ANY);
    ICAP_REQUIRE(ok, "icap_gemm: no LayerNorm-statistics form of the tile kernel this launch plans");
    pl.actk |= p.ln_stats_out ? ACT_LNS : ACT_LNF;
  }
  pl.block = dim3(GNT);
  pl.grid = dim3((unsigned)(tiles * splits));
  return ICAP_OK;
}

// "TI, TC, template ints" of each tile variant (keep in sync with the launch switch below); %%d = ACT kind
static const char* variant_kernel(int v) {
  switch (v) {
    case 0: return "gemm_kernel<%s, %s, 2, 2, 2, 2, 4, 4, false, %d>";
    case 4: return "gemm_kernel<%s, %s, 1, 3, 2, 2, 4, 4, false, %d>";
    case 5: return "gemm_kernel<%s, %s, 1, 4, 2, 2, 4, 4, false, %d>";
    case 12: return "gemm_kernel<%s, %s, 2, 3, 2, 2, 4, 2, false, %d>";
    case 13: return "gemm_kernel<%s, %s, 1, 4, 2, 2, 4, 2, false, %d>";
    case 14: return "gemm_kernel<%s, %s, 2, 2, 2, 2, 4, 4, true, %d>";
    case 16: return "gemm_kernel<%s, %s, 4, 1, 2, 2, 4, 4, false, %d>";
    case 22: return "gemm_kernel<%s, %s, 3, 1, 4, 2, 4, 4, false, %d>";
    case 24: return "gemm_kernel<%s, %s, 2, 2, 4, 1, 3, 4, false, %d>";
    case 25: return "gemm_kernel<%s, %s, 4, 1, 4, 1, 3, 4, false, %d>";
    case 26: return "gemm_kernel<%s, %s, 3, 1, 2, 2, 4, 8, false, %d, true>";
    case 27: return "gemm_kernel<%s, %s, 5, 1, 2, 2, 3, 4, false, %d, true>";
    case 28: return "gemm_kernel<%s, %s, 2, 1, 2, 4, 6, 4, false, %d, true>";
    case 31: return "gemm_kernel<%s, %s, 4, 1, 2, 2, 4, 4, true, %d, true>";
    case 32: return "gemm_kernel<%s, %s, 4, 1, 2, 2, 5, 4, false, %d, true>";
    default: return "gemm_kernel<%s, %s, 1, 3, 2, 2, 4, 4, true, %d>";
  }
}

extern "C" const char* icap_gemm_kernel_name(const icap_gemm_args* a) {
  static thread_local char buf[160];
  if (a == nullptr) return nullptr;
  GemmPlan pl;
  if (gemm_plan(*a, pl) != ICAP_OK) return nullptr;
  const char* ti = a->in_dtype == ICAP_BF16 ? "unsigned short" : a->in_dtype == ICAP_FP8_MX ? "icap::fp8_t" : "float";
  const char* tc = a->c_dtype == ICAP_BF16 ? "unsigned short" : "float";
  char fmt[96];
  if (pl.g256) {
    snprintf(buf, sizeof buf, "icap::gemm256_kernel<%s>", tc);
    return buf;
  }
  if (pl.g8p) {
    snprintf(buf, sizeof buf, "icap::gemm8p_kernel<%s, %d, %d>", tc, pl.g8p, pl.actk);
    return buf;
  }
  char inner[128];
  if (pl.skinny) {
    snprintf(fmt, sizeof fmt, "gemm_skinny_kernel<%%s, %%s, %d, 2, %d>", pl.nt, pl.sku);
    snprintf(inner, sizeof inner, fmt, ti, tc);
  } else {
    snprintf(inner, sizeof inner, variant_kernel(pl.variant), ti, tc, pl.actk);
  }
  snprintf(buf, sizeof buf, "icap::%s", inner);
  return buf;
}

extern "C" int icap_gemm_plan_info(const icap_gemm_args* a, int32_t* splits, int32_t* fused) {
  ICAP_REQUIRE(a != nullptr && splits != nullptr && fused != nullptr, "icap_gemm_plan_info: null pointer");
  GemmPlan pl;
  const int rc = gemm_plan(*a, pl);
  if (rc != ICAP_OK) return rc;
  *splits = pl.skinny || pl.g256 || pl.g8p ? 1 : pl.splits;
  *fused = pl.fused ? 1 : 0;
  return ICAP_OK;
}

extern "C" int icap_gemm_group(const icap_gemm_args* a, int32_t n, void* stream) {
  ICAP_REQUIRE(a != nullptr && n >= 1 && n <= ICAP_GEMM_GROUP_MAX, "icap_gemm_group: 1 ... 8 products");
  GemmGroup g;
  g.n = 0;
  g.tstart[0] = 0;
  for (int i = 0; i < n; ++i) {
    const icap_gemm_args& p = a[i];
    // (the general argument checks of a single product, then the group's own preconditions)
    GemmPlan pl;
    icap_gemm_args q = p;
    q.split_k = 1;
    q.path = 0;
    if (const int rc = gemm_plan(q, pl); rc != ICAP_OK) return rc;
    ICAP_REQUIRE(p.trans_ab && p.in_dtype == ICAP_BF16 && p.c_dtype == ICAP_F32,
                 "icap_gemm_group: K-outer (trans_ab) bf16 products with an fp32 C");
    ICAP_REQUIRE(p.act == ICAP_ACT_NONE && p.dact == ICAP_ACT_NONE && !p.bias && !p.resid && !p.aux && !p.ln_gamma &&
                     !p.ln_wsum && !p.ln_stats_in && !p.ln_stats_out && p.drop_p == 0.f && !p.m_dev,
                 "icap_gemm_group: plain products only (alpha, beta; no epilogue operands)");
    if (p.M == 0 || p.N == 0) continue;
    ICAP_REQUIRE(p.K > 0, "icap_gemm_group: K must be positive");
    const int k = g.n;
    g.a[k] = p;
    g.a[k].split_k = 1;
    g.a[k].tickets = nullptr;
    g.tiles_n[k] = (int)((p.N + GBN - 1) / GBN);
    g.nk[k] = (int)((p.K + 63) / 64);
    const int64_t tiles = ((p.M + GBM - 1) / GBM) * (int64_t)g.tiles_n[k];
    ICAP_REQUIRE(g.tstart[k] + tiles < (1ll << 30), "icap_gemm_group: too many tiles");
    g.tstart[k + 1] = g.tstart[k] + (int)tiles;
    ++g.n;
  }
  if (g.n == 0) return ICAP_OK;
  launch_group_kout(g, (int)device_cus(), reinterpret_cast<hipStream_t>(stream));
  return check_launch("icap_gemm_group");
}

extern "C" int icap_gemm(const icap_gemm_args* a, void* stream) {
  ICAP_REQUIRE(a != nullptr, "icap_gemm: null args");
  if (a->M == 0 || a->N == 0) return ICAP_OK;
  GemmPlan pl;
  const int prc = gemm_plan(*a, pl);
  if (prc != ICAP_OK) return prc;
  // the kernels take the in-launch combine exactly when tickets reach them: only for the plan that chose it (a
  // reduce-pass split must write its slabs, whatever the caller passed)
  icap_gemm_args pk = *a;
  if (!pl.fused) pk.tickets = nullptr;
  const icap_gemm_args& p = pk;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint32_t thr = pl.thr;
  const float inv_keep = pl.inv_keep;
  if (pl.skinny) {
    const dim3 sgrid = pl.grid, sblock = pl.block;
#define ICAP_SK(TI, TC, NT, U) hipLaunchKernelGGL((gemm_skinny_kernel<TI, TC, NT, 2, U>), sgrid, sblock, 0, s, p, thr, inv_keep)
#define ICAP_SKINNY_BF(TC)                                                                 \
  switch (pl.nt * 100 + pl.sku) {                                                          \
    case 103: ICAP_SK(bf16_t, TC, 1, 3); break;                                            \
    case 104: ICAP_SK(bf16_t, TC, 1, 4); break;                                            \
    case 106: ICAP_SK(bf16_t, TC, 1, 6); break;                                            \
    case 112: ICAP_SK(bf16_t, TC, 1, 12); break;                                           \
    case 203: ICAP_SK(bf16_t, TC, 2, 3); break;                                            \
    case 204: ICAP_SK(bf16_t, TC, 2, 4); break;                                            \
    case 206: ICAP_SK(bf16_t, TC, 2, 6); break;                                            \
    case 303: ICAP_SK(bf16_t, TC, 3, 3); break;                                            \
    case 304: ICAP_SK(bf16_t, TC, 3, 4); break;                                            \
    case 306: ICAP_SK(bf16_t, TC, 3, 6); break;                                            \
    case 403: ICAP_SK(bf16_t, TC, 4, 3); break;                                            \
    case 404: ICAP_SK(bf16_t, TC, 4, 4); break;                                            \
    default: ICAP_SK(bf16_t, TC, 4, 6); break;                                             \
  }
#define ICAP_SKINNY_F32(TC)                                                                \
  switch (pl.nt) {                                                                         \
    case 1: ICAP_SK(float, TC, 1, 6); break;                                               \
    case 2: ICAP_SK(float, TC, 2, 6); break;                                               \
    case 3: ICAP_SK(float, TC, 3, 6); break;                                               \
    default: ICAP_SK(float, TC, 4, 6); break;                                              \
  }
    if (p.in_dtype == ICAP_BF16) {
      if (p.c_dtype == ICAP_BF16) { ICAP_SKINNY_BF(bf16_t) } else { ICAP_SKINNY_BF(float) }
    } else {
      if (p.c_dtype == ICAP_BF16) { ICAP_SKINNY_F32(bf16_t) } else { ICAP_SKINNY_F32(float) }
    }
#undef ICAP_SKINNY_BF
#undef ICAP_SKINNY_F32
#undef ICAP_SK
    return check_launch("icap_gemm(skinny)");
  }
  if (pl.g256) return gemm256_launch(p, thr, inv_keep, s);
  if (pl.g8p) return gemm8p_launch(p, pl.g8p, pl.actk, thr, inv_keep, s);
  const int sp = pl.splits;
  // (the split-role variants walk K in its natural order: one round of tiles, no lockstep panel misses to stagger,
  // and automatic launches then equal forced ones and the tile path bitwise)
  const int skew = (pl.variant >= 26 && pl.variant <= 32) ? 0 : kskew_for(p, pl.nk_split);
  const int nks = pl.nk_split | (skew << 20) | (gemm_diag() << 28) | (gemm_acquire() << 30);
  const dim3 rgrid((unsigned)((p.M * (p.N / 4) + 255) / 256));
  if (pl.variant == 31) launch_tile_roles_kout(pl, p, nks, s);                       // gemm_tile_roles_kout.hip
  else if (pl.variant == 26) launch_tile_roles(pl, p, nks, s);                       // gemm_tile_roles.hip
  else if (pl.variant == 32) launch_tile_roles160(pl, p, nks, s);                    // gemm_tile_roles160.hip
  else if (pl.variant == 27) launch_tile_roles96(pl, p, nks, s);                     // gemm_tile_roles96.hip
  else if (pl.variant == 28) launch_tile_roles192(pl, p, nks, s);                    // gemm_tile_roles192.hip
  else if (pl.variant == 22) launch_tile_r256(pl, p, nks, s);                        // gemm_tile_r256.hip
  else if (pl.variant == 24 || pl.variant == 25) launch_tile_w192(pl, p, nks, s);   // gemm_tile_w192.hip
  else if (pl.actk >= ACT_LNS) launch_tile_ln(pl, p, nks, s);                      // gemm_tile_ln.hip
  else if (pl.actk >= ACT_FWD) launch_tile_act(pl, p, nks, s);                     // gemm_tile_act.hip
  else if (pl.variant == 14 || pl.variant == 15) launch_tile_kout(pl, p, nks, s);    // gemm_tile_kout.hip
  else if (p.in_dtype == ICAP_BF16) launch_tile_bf16(pl, p, nks, s);                 // gemm_tile_bf16.hip
  else if (p.in_dtype == ICAP_FP8_MX) launch_tile_mx(pl, p, nks, s);                 // gemm_tile_mx.hip
  else launch_tile_f32(pl, p, nks, s);                                               // gemm_tile_f32.hip
  if (sp > 1 && !pl.fused) {
    if (p.c_dtype == ICAP_BF16)
      hipLaunchKernelGGL((gemm_splitk_reduce<bf16_t>), rgrid, dim3(256), 0, s, p, sp, thr, inv_keep);
    else
      hipLaunchKernelGGL((gemm_splitk_reduce<float>), rgrid, dim3(256), 0, s, p, sp, thr, inv_keep);
  }
  return check_launch("icap_gemm");
}

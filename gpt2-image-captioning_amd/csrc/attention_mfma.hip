// bf16 MFMA attention for the short sequences of the captioning path (S <= 128, head_dim 64 / 96):
// GPT-2 (S=65, causal + key padding), CLIP (S=50), mapper (S=25, hd 96).
//
// One 4-wave workgroup per (batch, head). Every product is a v_mfma_f32_16x16x32_bf16 chain
// C[m][n] = sum_k A[m][k] B[n][k] whose operands are read as 16-byte k-contiguous fragments
// (lane l: row r0 + (l&15), k = k0 + 8(l>>4) .. +7):
//   forward   S = Q K^T (Q, K fragments straight from the fused QKV rows in HBM/L2),
//             softmax on the accumulator layout (row = 4(l>>4)+reg, key = l&15): row max / sum by
//             16-lane shuffles, P written to a per-wave LDS tile, O = P V with V^T staged in LDS.
//   backward  P recomputed from the saved log-sum-exp, dP = dO V^T, dS = P (dP - rowsum(P dP)),
//             dQ = dS K (K^T in LDS), dK = dS^T Q and dV = P^T dO (Q^T, dO^T, dS^T, P^T in LDS).
// LDS rows are padded to (Sp32 + 8) / hd-stride so the 16 lanes of a fragment read hit distinct
// 16-byte bank groups. Keys/queries are padded to multiples of 16 / 32 with zeros (masked scores,
// zero operands), so padding never reaches an output.
#include "common.h"

#include <math.h>

namespace icap {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

namespace amfma {

constexpr int MAXKT = 8;  // key tiles of 16 -> S <= 128

struct Geo {
  int S, H, hd, D, Sp16, Sp32, ldT;
  int64_t rsb, rss;
};

__device__ __forceinline__ int64_t trow(const Geo& g, int b, int s) { return (int64_t)b * g.rsb + (int64_t)s * g.rss; }

__device__ __forceinline__ f32x4_t mfma(const uint4& a, const uint4& b, f32x4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_t, a), __builtin_bit_cast(bf16x8_t, b), c,
                                                 0, 0, 0);
}

// fragment of a [rows][k] bf16 LDS matrix
__device__ __forceinline__ uint4 lfrag(const bf16_t* base, int ld, int r0, int k0, int lane) {
  return *reinterpret_cast<const uint4*>(base + (r0 + (lane & 15)) * ld + k0 + 8 * (lane >> 4));
}

// fragment of the head's [S][hd] slice at column col0 of a strided token matrix in global memory;
// rows >= S read as zeros
__device__ __forceinline__ uint4 gfrag(const bf16_t* mat, int64_t ld, int col0, const Geo& g, int b, int r0, int k0,
                                       int lane) {
  const int r = r0 + (lane & 15);
  const int rc = r < g.S ? r : g.S - 1;
  uint4 v = *reinterpret_cast<const uint4*>(mat + trow(g, b, rc) * ld + col0 + k0 + 8 * (lane >> 4));
  if (r >= g.S) v = make_uint4(0, 0, 0, 0);
  return v;
}

// dst[d][s] = src[s][col0 + d] for s < S (zeros for S <= s < Sp32), d < hd; 256 threads
__device__ __forceinline__ void stage_T(bf16_t* dst, int ld, const bf16_t* src, int64_t lds, int col0, const Geo& g,
                                        int b) {
  const int nc = g.hd >> 3;
  for (int idx = threadIdx.x; idx < g.Sp32 * nc; idx += blockDim.x) {
    const int s = idx / nc, c = idx - s * nc;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (s < g.S) v = *reinterpret_cast<const uint4*>(src + trow(g, b, s) * lds + col0 + 8 * c);
    const bf16_t* e = reinterpret_cast<const bf16_t*>(&v);
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[(8 * c + k) * ld + s] = e[k];
  }
}

__device__ __forceinline__ bool key_ok(int causal, const int32_t* km, const Geo& g, int b, int q, int key) {
  if (key >= g.S) return false;
  if (causal && key > q) return false;
  if (km && km[(int64_t)b * g.S + key] == 0) return false;
  return true;
}

__device__ __forceinline__ uint32_t pack2(float a, float b) {
  return (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
}

// softmax statistics over the 16 lanes that share (lane >> 4)
__device__ __forceinline__ float row16_max(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float row16_sum(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int HD>
__global__ __launch_bounds__(256) void fwd_kernel(icap_attn_args p, Geo g, uint32_t thr, float inv_keep) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sm[];
  constexpr int NKS = HD / 32;   // k-steps of QK^T
  constexpr int NDT = HD / 16;   // d tiles of O
  const int bh = blockIdx.x;
  const int b = bh / g.H, h = bh - b * g.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ldT = g.ldT;
  bf16_t* Vt = sm;                                   // [HD][ldT]
  bf16_t* Pw = sm + HD * ldT + wave * 16 * ldT;      // per wave [16][ldT]
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  stage_T(Vt, ldT, qkv, p.ld_qkv, 2 * g.D + h * HD, g, b);
  for (int i = lane; i < 16 * ldT; i += 64) Pw[i] = 0;
  __syncthreads();
  const uint64_t seed = thr ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  const uint64_t dbase = p.offset + (uint64_t)bh * g.S * g.S;
  const int nkt = g.Sp16 >> 4, nqt = g.Sp16 >> 4, nks2 = g.Sp32 >> 5;
  const int fr = lane & 15, fg = lane >> 4;
  bf16_t* out = reinterpret_cast<bf16_t*>(p.out);
  for (int qt = wave; qt < nqt; qt += 4) {
    uint4 qf[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) qf[ks] = gfrag(qkv, p.ld_qkv, h * HD, g, b, qt * 16, ks * 32, lane);
    f32x4_t s[MAXKT];
#pragma unroll
    for (int kt = 0; kt < MAXKT; ++kt) {
      s[kt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      if (kt < nkt) {
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
          s[kt] = mfma(qf[ks], gfrag(qkv, p.ld_qkv, g.D + h * HD, g, b, kt * 16, ks * 32, lane), s[kt]);
      }
    }
    // masked, scaled softmax per query row (rows 4fg+v of this q tile)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int q = qt * 16 + fg * 4 + v;
      float m = -INFINITY;
#pragma unroll
      for (int kt = 0; kt < MAXKT; ++kt) {
        if (kt < nkt) {
          const int key = kt * 16 + fr;
          const float x = key_ok(p.causal, p.key_mask, g, b, q, key) ? s[kt][v] * p.scale : -INFINITY;
          s[kt][v] = x;
          m = fmaxf(m, x);
        }
      }
      m = row16_max(m);
      float l = 0.f;
#pragma unroll
      for (int kt = 0; kt < MAXKT; ++kt) {
        if (kt < nkt) {
          const float e = (m == -INFINITY) ? 0.f : __expf(s[kt][v] - m);
          s[kt][v] = e;
          l += e;
        }
      }
      l = row16_sum(l);
      const float inv = l > 0.f ? 1.f / l : 0.f;
      if (fr == 0 && q < g.S && p.lse) p.lse[(int64_t)bh * g.S + q] = l > 0.f ? m + logf(l) : -INFINITY;
#pragma unroll
      for (int kt = 0; kt < MAXKT; ++kt) {
        if (kt < nkt) {
          const int key = kt * 16 + fr;
          float pv = s[kt][v] * inv;
          if (thr && q < g.S && key < g.S) pv *= drop_scale(seed, dbase + (uint64_t)q * g.S + key, thr, inv_keep);
          Pw[(fg * 4 + v) * ldT + key] = f2bf(pv);
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // O = P V
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      f32x4_t o = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      for (int ks = 0; ks < nks2; ++ks) o = mfma(lfrag(Pw, ldT, 0, ks * 32, lane), lfrag(Vt, ldT, dt * 16, ks * 32, lane), o);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int q = qt * 16 + fg * 4 + v;
        if (q < g.S) out[trow(g, b, q) * p.ld_out + h * HD + dt * 16 + fr] = f2bf(o[v]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

template <int HD>
__global__ __launch_bounds__(256) void bwd_kernel(icap_attn_args p, Geo g, uint32_t thr, float inv_keep) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sm[];
  constexpr int NKS = HD / 32;
  constexpr int NDT = HD / 16;
  const int bh = blockIdx.x;
  const int b = bh / g.H, h = bh - b * g.H;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ldT = g.ldT;
  bf16_t* Kt = sm;                        // [HD][ldT]   K^T  (dQ B operand)
  bf16_t* Qt = Kt + HD * ldT;             // [HD][ldT]   Q^T  (dK B operand)
  bf16_t* dOt = Qt + HD * ldT;            // [HD][ldT]   dO^T (dV B operand)
  bf16_t* dSt = dOt + HD * ldT;           // [Sp16][ldT] dS^T (dK A operand)
  bf16_t* Pdt = dSt + g.Sp16 * ldT;       // [Sp16][ldT] (dropped P)^T (dV A operand)
  bf16_t* dSw = Pdt + g.Sp16 * ldT + wave * 16 * ldT;  // per wave [16][ldT] dS rows (dQ A operand)
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  const bf16_t* dout = reinterpret_cast<const bf16_t*>(p.dout);
  stage_T(Kt, ldT, qkv, p.ld_qkv, g.D + h * HD, g, b);
  stage_T(Qt, ldT, qkv, p.ld_qkv, h * HD, g, b);
  stage_T(dOt, ldT, dout, p.ld_dout, h * HD, g, b);
  {
    uint4* z = reinterpret_cast<uint4*>(dSt);
    const int n16 = (2 * g.Sp16 * ldT) / 8;
    for (int i = threadIdx.x; i < n16; i += blockDim.x) z[i] = make_uint4(0, 0, 0, 0);
    for (int i = lane; i < 16 * ldT; i += 64) dSw[i] = 0;
  }
  __syncthreads();
  const uint64_t seed = thr ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  const uint64_t dbase = p.offset + (uint64_t)bh * g.S * g.S;
  const int nkt = g.Sp16 >> 4, nqt = g.Sp16 >> 4, nks2 = g.Sp32 >> 5;
  const int fr = lane & 15, fg = lane >> 4;
  bf16_t* dqkv = reinterpret_cast<bf16_t*>(p.dqkv);
  for (int qt = wave; qt < nqt; qt += 4) {
    uint4 qf[NKS], of[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      qf[ks] = gfrag(qkv, p.ld_qkv, h * HD, g, b, qt * 16, ks * 32, lane);
      of[ks] = gfrag(dout, p.ld_dout, h * HD, g, b, qt * 16, ks * 32, lane);
    }
    f32x4_t s[MAXKT], dp[MAXKT];
#pragma unroll
    for (int kt = 0; kt < MAXKT; ++kt) {
      s[kt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      dp[kt] = s[kt];
      if (kt < nkt) {
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          s[kt] = mfma(qf[ks], gfrag(qkv, p.ld_qkv, g.D + h * HD, g, b, kt * 16, ks * 32, lane), s[kt]);
          dp[kt] = mfma(of[ks], gfrag(qkv, p.ld_qkv, 2 * g.D + h * HD, g, b, kt * 16, ks * 32, lane), dp[kt]);
        }
      }
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int q = qt * 16 + fg * 4 + v;
      const float lse = q < g.S ? p.lse[(int64_t)bh * g.S + q] : -INFINITY;
      float delta = 0.f;
#pragma unroll
      for (int kt = 0; kt < MAXKT; ++kt) {
        if (kt < nkt) {
          const int key = kt * 16 + fr;
          float pv = 0.f;
          if (q < g.S && lse != -INFINITY && key_ok(p.causal, p.key_mask, g, b, q, key))
            pv = __expf(s[kt][v] * p.scale - lse);
          float d = dp[kt][v];
          float pd = pv;
          if (thr && q < g.S && key < g.S) {
            const float ms = drop_scale(seed, dbase + (uint64_t)q * g.S + key, thr, inv_keep);
            d *= ms;
            pd *= ms;
          }
          s[kt][v] = pv;
          dp[kt][v] = d;
          delta += pv * d;
          Pdt[key * ldT + qt * 16 + fg * 4 + v] = f2bf(pd);
        }
      }
      delta = row16_sum(delta);
#pragma unroll
      for (int kt = 0; kt < MAXKT; ++kt) {
        if (kt < nkt) {
          const int key = kt * 16 + fr;
          const float ds = s[kt][v] * (dp[kt][v] - delta);
          const bf16_t d16 = f2bf(ds);
          dSw[(fg * 4 + v) * ldT + key] = d16;
          dSt[key * ldT + qt * 16 + fg * 4 + v] = d16;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // dQ = scale * dS K
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      f32x4_t o = (f32x4_t){0.f, 0.f, 0.f, 0.f};
      for (int ks = 0; ks < nks2; ++ks) o = mfma(lfrag(dSw, ldT, 0, ks * 32, lane), lfrag(Kt, ldT, dt * 16, ks * 32, lane), o);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int q = qt * 16 + fg * 4 + v;
        if (q < g.S) dqkv[trow(g, b, q) * p.ld_dqkv + h * HD + dt * 16 + fr] = f2bf(o[v] * p.scale);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  __syncthreads();
  // dK = scale * dS^T Q,  dV = Pd^T dO   (rows = keys)
  for (int kt = wave; kt < nkt; kt += 4) {
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) {
      f32x4_t ak = (f32x4_t){0.f, 0.f, 0.f, 0.f}, av = ak;
      for (int ks = 0; ks < nks2; ++ks) {
        ak = mfma(lfrag(dSt, ldT, kt * 16, ks * 32, lane), lfrag(Qt, ldT, dt * 16, ks * 32, lane), ak);
        av = mfma(lfrag(Pdt, ldT, kt * 16, ks * 32, lane), lfrag(dOt, ldT, dt * 16, ks * 32, lane), av);
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int key = kt * 16 + fg * 4 + v;
        if (key < g.S) {
          bf16_t* rowp = dqkv + trow(g, b, key) * p.ld_dqkv;
          rowp[g.D + h * HD + dt * 16 + fr] = f2bf(ak[v] * p.scale);
          rowp[2 * g.D + h * HD + dt * 16 + fr] = f2bf(av[v]);
        }
      }
    }
  }
}

}  // namespace amfma

static inline int rup(int x, int m) { return (x + m - 1) / m * m; }

amfma::Geo mfma_geo(const icap_attn_args* a) {
  amfma::Geo g;
  g.S = a->S; g.H = a->H; g.hd = a->hd; g.D = a->H * a->hd;
  g.Sp16 = rup(a->S, 16); g.Sp32 = rup(a->S, 32); g.ldT = g.Sp32 + 8;
  g.rsb = a->row_stride_b; g.rss = a->row_stride_s;
  return g;
}

size_t mfma_fwd_lds(const amfma::Geo& g) { return 2 * ((size_t)g.hd * g.ldT + 4 * 16 * (size_t)g.ldT); }
size_t mfma_bwd_lds(const amfma::Geo& g) {
  return 2 * (3 * (size_t)g.hd * g.ldT + 2 * (size_t)g.Sp16 * g.ldT + 4 * 16 * (size_t)g.ldT);
}

bool mfma_attention_ok(const icap_attn_args* a, bool bwd) {
  if (a->dtype != ICAP_BF16 || (a->hd != 64 && a->hd != 96) || a->S > 16 * amfma::MAXKT) return false;
  if ((a->ld_qkv & 7) || (bwd && (a->ld_dout & 7))) return false;
  const amfma::Geo g = mfma_geo(a);
  return (bwd ? mfma_bwd_lds(g) : mfma_fwd_lds(g)) <= 160 * 1024;
}

template <typename K>
static void lds_limit(K kernel) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize,
                            160 * 1024);
}

int mfma_attention_launch(const icap_attn_args* a, bool bwd, uint32_t thr, float inv_keep, hipStream_t s) {
  const amfma::Geo g = mfma_geo(a);
  dim3 grid((unsigned)(a->B * a->H)), block(256);
  if (!bwd) {
    const size_t lds = mfma_fwd_lds(g);
    if (a->hd == 64) {
      static bool once = (lds_limit(amfma::fwd_kernel<64>), true); (void)once;
      hipLaunchKernelGGL(amfma::fwd_kernel<64>, grid, block, lds, s, *a, g, thr, inv_keep);
    } else {
      static bool once = (lds_limit(amfma::fwd_kernel<96>), true); (void)once;
      hipLaunchKernelGGL(amfma::fwd_kernel<96>, grid, block, lds, s, *a, g, thr, inv_keep);
    }
  } else {
    const size_t lds = mfma_bwd_lds(g);
    if (a->hd == 64) {
      static bool once = (lds_limit(amfma::bwd_kernel<64>), true); (void)once;
      hipLaunchKernelGGL(amfma::bwd_kernel<64>, grid, block, lds, s, *a, g, thr, inv_keep);
    } else {
      static bool once = (lds_limit(amfma::bwd_kernel<96>), true); (void)once;
      hipLaunchKernelGGL(amfma::bwd_kernel<96>, grid, block, lds, s, *a, g, thr, inv_keep);
    }
  }
  return check_launch(bwd ? "icap_attention_bwd(mfma)" : "icap_attention_fwd(mfma)");
}

}  // namespace icap

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

// S: tokens of this block's sequence (the launch's S, or seq_len[b] for packed sequences); Sst: the launch's S,
// the stride of the lse [B, H, S] and dropout [B, H, S, S] numbering; base / kmb: row of token 0 and its key-mask
// index (localize)
struct Geo {
  int S, H, hd, D, Sp16, Sp32, ldT;
  int64_t rsb, rss;
  int Sst;
  int64_t base, kmb;
  int slo, shi;  // length class of the launch: blocks whose sequence has slo < S <= shi (packed short / long pass)
};

__device__ __forceinline__ int64_t trow(const Geo& g, int b, int s) { return g.base + (int64_t)s * g.rss; }

// per-block sequence geometry (icap_attn_args.seq_off / seq_len: packed rows); false: empty sequence
__device__ __forceinline__ bool localize(Geo& g, const icap_attn_args& p, int b) {
  if (p.seq_len) {
    const int n = p.seq_len[b];
    g.S = n < g.Sst ? n : g.Sst;
    g.base = p.seq_off[b];
    g.kmb = p.seq_off[b];
    g.Sp16 = (g.S + 15) & ~15;
    g.Sp32 = (g.S + 31) & ~31;
  } else {
    g.base = (int64_t)b * g.rsb;
    g.kmb = (int64_t)b * g.Sst;
  }
  return g.S > g.slo && g.S <= g.shi;  // (slo >= 0: empty sequences do nothing)
}

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
  if (km && km[g.kmb + key] == 0) return false;
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
  if (!localize(g, p, b)) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int ldT = g.ldT;
  bf16_t* Vt = sm;                                   // [HD][ldT]
  bf16_t* Pw = sm + HD * ldT + wave * 16 * ldT;      // per wave [16][ldT]
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  stage_T(Vt, ldT, qkv, p.ld_qkv, 2 * g.D + h * HD, g, b);
  for (int i = lane; i < 16 * ldT; i += 64) Pw[i] = 0;
  __syncthreads();
  const uint64_t seed = thr ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  const uint64_t dbase = p.offset + (uint64_t)bh * g.Sst * g.Sst;
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
      if (fr == 0 && q < g.S && p.lse) p.lse[(int64_t)bh * g.Sst + q] = l > 0.f ? m + logf(l) : -INFINITY;
#pragma unroll
      for (int kt = 0; kt < MAXKT; ++kt) {
        if (kt < nkt) {
          const int key = kt * 16 + fr;
          float pv = s[kt][v] * inv;
          if (thr && q < g.S && key < g.S) pv *= drop_scale(seed, dbase + (uint64_t)q * g.Sst + key, thr, inv_keep);
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
  if (!localize(g, p, b)) return;
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
  const uint64_t dbase = p.offset + (uint64_t)bh * g.Sst * g.Sst;
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
      const float lse = q < g.S ? p.lse[(int64_t)bh * g.Sst + q] : -INFINITY;
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
            const float ms = drop_scale(seed, dbase + (uint64_t)q * g.Sst + key, thr, inv_keep);
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

// ---------------------------------------------------------------------------------------------------------
// Backward v2 (needs the forward output O: delta[q] = rowsum(dO o O) = rowsum(P o dP), dropout included).
// Q, K, V, dO of the head are staged ROW-major in LDS once (16-byte copies, rows padded to ldr_of(HD) halves: see
// below); no scalar transposes. Waves split by role:
//   waves [0, nt)   : one 16-key tile each -> dV^T = dO^T P_drop, dK^T = Q^T dS over all queries,
//   waves [nt, 2nt) : one 16-query tile each -> dQ^T = K^T dS^T over all keys,
// where the first products (S = Q K^T, dP = dO V^T, in whichever orientation puts the contraction index of the
// second product into the accumulator ROWS) come from row fragments, and the second products take the bf16
// accumulator tile as the B operand directly (two 16-row tiles = one 32-deep k step; element j of lane group g
// is row 4g+j / 16+4g+j-4) with the A operand read transposed by ds_read_b64_tr_b16 from the same row-major
// image (cdna_hip_programming.md "An accumulator tile as the next MFMA's operand", T10). Outputs come out with
// 4 consecutive head dims per lane (8-byte stores).
typedef short v4s_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s_t* lds_v4s_ptr;
// Row stride (halves) of the row-major Q / K / V / dO images: HD + 16. With the 64 four-byte banks and the lane
// groups of ds_read_b128 (4 x 16 lanes) and ds_read_b64_tr_b16 (2 x 32) (MI355X_MICROARCH.md "LDS"), a stride of
// HD + 8 put two rows of every 16-row fragment read (rowfrag) and of every 8-row transposed read (trfrag) on the
// same banks — 8 / 4 LDS cycles per wave-instruction for 4 / 2 conflict-free; HD + 16 (an odd multiple of 32 bytes
// past a multiple of 128) spreads them over all 64 banks for hd 64, 96 and 128 (round 5; the r04 PMC pass measured
// SQ_LDS_BANK_CONFLICT at 0.32-0.39 of these kernels' LDS cycles, profiles/r04_pmc_lds.txt). Measured: no change
// in time (B = 128, S = 65: forward 22.2 -> 22.1 µs, backward 45.1 -> 44.7; profiles/r05_attn_ldr_ab.txt) — the LDS
// was not what bounds these launches; kept for the conflict-free reads.
__host__ __device__ constexpr int ldr_of(int hd) { return hd + 16; }

template <int LDR>
__device__ __forceinline__ uint4 rowfrag(const bf16_t* base, int r0, int k0, int lane) {
  return *reinterpret_cast<const uint4*>(base + (r0 + (lane & 15)) * LDR + k0 + 8 * (lane >> 4));
}
// A operand [m = column c0 + (lane & 15)][k = 32-row block starting at r0] of a row-major LDS image, in the
// k order of an accumulator-tile B operand (element j of group g = row r0 + 4g + j, j < 4; r0 + 16 + 4g + j - 4)
template <int LDR>
__device__ __forceinline__ uint4 trfrag(const bf16_t* base, int r0, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const bf16_t* a0 = base + (r0 + 4 * g + (i >> 2)) * LDR + c0 + 4 * (i & 3);
  const bf16_t* a1 = a0 + 16 * LDR;
  const v4s_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_ptr)(a0));
  const v4s_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s_ptr)(a1));
  uint4 r;
  r.x = (uint32_t)(uint16_t)lo[0] | ((uint32_t)(uint16_t)lo[1] << 16);
  r.y = (uint32_t)(uint16_t)lo[2] | ((uint32_t)(uint16_t)lo[3] << 16);
  r.z = (uint32_t)(uint16_t)hi[0] | ((uint32_t)(uint16_t)hi[1] << 16);
  r.w = (uint32_t)(uint16_t)hi[2] | ((uint32_t)(uint16_t)hi[3] << 16);
  return r;
}

template <int HD>
__global__ __launch_bounds__(512) void bwd2_kernel(icap_attn_args p, Geo g, uint32_t thr, float inv_keep) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sm[];
  constexpr int LDR = ldr_of(HD);
  constexpr int NKS = HD / 32;  // 32-deep k steps over the head dim
  constexpr int NDT = HD / 16;  // 16-wide head-dim tiles of the outputs
  constexpr int CPR = HD / 8;   // 16-byte chunks per row
  const int bh = blockIdx.x;
  const int b = bh / g.H, h = bh - b * g.H;
  if (!localize(g, p, b)) return;
  const int Sp = g.Sp32, S = g.S, SS = g.Sst;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  const int nt = g.Sp16 >> 4;
  bf16_t* Qs = sm;
  bf16_t* Ks = Qs + Sp * LDR;
  bf16_t* Vs = Ks + Sp * LDR;
  bf16_t* dOs = Vs + g.Sp16 * LDR;  // V is only read by 16-row tiles below Sp16 (skipped past it in the dQ loop)
  float* lse_s = reinterpret_cast<float*>(dOs + Sp * LDR);
  float* delta_s = lse_s + Sp;
  uint8_t* kok_s = reinterpret_cast<uint8_t*>(delta_s + Sp);  // key allowed by the padding mask (and < S)
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  const bf16_t* dout = reinterpret_cast<const bf16_t*>(p.dout);
  const bf16_t* outp = reinterpret_cast<const bf16_t*>(p.out);
  // per-row lse / key mask: loaded here, stored to LDS after the staging loads below are issued, under the same
  // barrier (round 5: a barrier and a dependent round trip of their own before). Sp = Sp32 <= Sp16 + 16 <= blockDim
  // = 4 Sp16, so one row per thread.
  const int rr = threadIdx.x;
  float lse_r = -INFINITY;
  uint8_t kok_r = 0;
  if (rr < S) {
    lse_r = p.lse[(int64_t)bh * SS + rr];
    kok_r = (p.key_mask == nullptr || p.key_mask[g.kmb + rr] != 0) ? 1 : 0;
  }
  // CPR a power of two (HD 64 / 128): delta[q] = sum_d dO[q][d] O[q][d] fused into the staging loop, the CPR
  // chunk partials of a row summed across its CPR consecutive lanes (block size and the loop bound are multiples
  // of CPR, so a row's lanes are active together); otherwise one thread per query after it. Fixed order either way.
  constexpr bool FUSED_DELTA = (CPR & (CPR - 1)) == 0 && CPR <= 64;
  // Staging in batches of SIT rows-chunks per thread: every global load of a batch is issued before the first LDS
  // store, so the block waits out one memory round trip per batch instead of one per chunk (hd 64, S = 65: one
  // batch; it was three dependent round trips).
  constexpr int SIT = HD == 64 ? 4 : 2;
  const int nidx = Sp * CPR;
  for (int base = threadIdx.x; base < nidx; base += SIT * blockDim.x) {
    uint4 qa[SIT], ka[SIT], va[SIT], da[SIT], oa[SIT];
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
      const int idx = base + it * (int)blockDim.x;
      const int r = idx / CPR, c = idx - r * CPR;
      qa[it] = ka[it] = va[it] = da[it] = oa[it] = make_uint4(0, 0, 0, 0);
      if (idx < nidx && r < S) {
        const int64_t row = trow(g, b, r);
        const bf16_t* src = qkv + row * p.ld_qkv + h * HD + 8 * c;
        qa[it] = *reinterpret_cast<const uint4*>(src);
        ka[it] = *reinterpret_cast<const uint4*>(src + g.D);
        va[it] = *reinterpret_cast<const uint4*>(src + 2 * g.D);
        da[it] = *reinterpret_cast<const uint4*>(dout + row * p.ld_dout + h * HD + 8 * c);
        if (FUSED_DELTA) oa[it] = *reinterpret_cast<const uint4*>(outp + row * p.ld_out + h * HD + 8 * c);
      }
    }
#pragma unroll
    for (int it = 0; it < SIT; ++it) {
      const int idx = base + it * (int)blockDim.x;
      if (idx >= nidx) break;  // uniform over a row's CPR lanes (nidx and blockDim are multiples of CPR)
      const int r = idx / CPR, c = idx - r * CPR;
      *reinterpret_cast<uint4*>(Qs + r * LDR + 8 * c) = qa[it];
      *reinterpret_cast<uint4*>(Ks + r * LDR + 8 * c) = ka[it];
      if (r < g.Sp16) *reinterpret_cast<uint4*>(Vs + r * LDR + 8 * c) = va[it];
      *reinterpret_cast<uint4*>(dOs + r * LDR + 8 * c) = da[it];
      if constexpr (FUSED_DELTA) {
        const uint32_t dw[4] = {da[it].x, da[it].y, da[it].z, da[it].w}, ow[4] = {oa[it].x, oa[it].y, oa[it].z, oa[it].w};
        float part = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e)
          part += __uint_as_float(dw[e] << 16) * __uint_as_float(ow[e] << 16) +
                  __uint_as_float(dw[e] & 0xffff0000u) * __uint_as_float(ow[e] & 0xffff0000u);
#pragma unroll
        for (int off = 1; off < CPR; off <<= 1) part += __shfl_xor(part, off, 64);
        if (c == 0 && r < S) delta_s[r] = part;
      }
    }
  }
  if (rr < Sp) {
    lse_s[rr] = lse_r;
    kok_s[rr] = kok_r;
    if (rr >= S) delta_s[rr] = 0.f;  // (rows < S: written by the fused staging loop or the per-query sums below)
  }
  if constexpr (!FUSED_DELTA) {
    for (int r = threadIdx.x; r < S; r += blockDim.x) {
      const int64_t row = trow(g, b, r);
      const bf16_t* orow = outp + row * p.ld_out + h * HD;
      const bf16_t* drow = dout + row * p.ld_dout + h * HD;
      float acc = 0.f;
#pragma unroll
      for (int c = 0; c < CPR; ++c) {
        const uint4 o = *reinterpret_cast<const uint4*>(orow + 8 * c);
        const uint4 d = *reinterpret_cast<const uint4*>(drow + 8 * c);
        const uint32_t dw[4] = {d.x, d.y, d.z, d.w}, ow[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int e = 0; e < 4; ++e)
          acc += __uint_as_float(dw[e] << 16) * __uint_as_float(ow[e] << 16) +
                 __uint_as_float(dw[e] & 0xffff0000u) * __uint_as_float(ow[e] & 0xffff0000u);
      }
      delta_s[r] = acc;
    }
  }
  __syncthreads();
  auto kok = [&](int q, int key) { return kok_s[key] && !(p.causal && key > q); };
  const uint64_t seed = thr ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  const uint64_t dbase = p.offset + (uint64_t)bh * SS * SS;
  bf16_t* dqkv = reinterpret_cast<bf16_t*>(p.dqkv);
  const int npair = Sp >> 5;
  if (wave < nt) {
    // ---- dK, dV for keys [16 kt, 16 kt + 16): accumulators C[q][key] (lane = key, rows = 4 queries)
    const int kt = wave;
    const int key = kt * 16 + fr;
    uint4 kf[NKS], vf[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      kf[ks] = rowfrag<LDR>(Ks, kt * 16, ks * 32, lane);
      vf[ks] = rowfrag<LDR>(Vs, kt * 16, ks * 32, lane);
    }
    f32x4_t dv[NDT], dk[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) dv[dt] = dk[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int qp0 = p.causal ? (kt * 16) >> 5 : 0;  // earlier query pairs see none of these keys
    for (int qp = qp0; qp < npair; ++qp) {
      float pd[8], ds[8];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const int qt = 2 * qp + sub;
        f32x4_t sc = (f32x4_t){0.f, 0.f, 0.f, 0.f}, dp = sc;
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
          sc = mfma(rowfrag<LDR>(Qs, qt * 16, ks * 32, lane), kf[ks], sc);
          dp = mfma(rowfrag<LDR>(dOs, qt * 16, ks * 32, lane), vf[ks], dp);
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int q = qt * 16 + 4 * fg + v;
          const float lse = lse_s[q];
          float pv = 0.f;
          if (lse != -INFINITY && kok(q, key)) pv = __expf(sc[v] * p.scale - lse);
          float ms = 1.f;
          if (thr && q < S && key < S) ms = drop_scale(seed, dbase + (uint64_t)q * SS + key, thr, inv_keep);
          pd[sub * 4 + v] = pv * ms;
          ds[sub * 4 + v] = pv * (dp[v] * ms - delta_s[q]);
        }
      }
      uint4 xp, xs;
      xp.x = f2bf2(pd[0], pd[1]); xp.y = f2bf2(pd[2], pd[3]); xp.z = f2bf2(pd[4], pd[5]); xp.w = f2bf2(pd[6], pd[7]);
      xs.x = f2bf2(ds[0], ds[1]); xs.y = f2bf2(ds[2], ds[3]); xs.z = f2bf2(ds[4], ds[5]); xs.w = f2bf2(ds[6], ds[7]);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        dv[dt] = mfma(trfrag<LDR>(dOs, qp * 32, dt * 16, lane), xp, dv[dt]);
        dk[dt] = mfma(trfrag<LDR>(Qs, qp * 32, dt * 16, lane), xs, dk[dt]);
      }
    }
    if (key < S) {
      bf16_t* rowp = dqkv + trow(g, b, key) * p.ld_dqkv + h * HD;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) {
        const int d0 = dt * 16 + 4 * fg;
        *reinterpret_cast<uint2*>(rowp + g.D + d0) =
            make_uint2(f2bf2(dk[dt][0] * p.scale, dk[dt][1] * p.scale), f2bf2(dk[dt][2] * p.scale, dk[dt][3] * p.scale));
        *reinterpret_cast<uint2*>(rowp + 2 * g.D + d0) =
            make_uint2(f2bf2(dv[dt][0], dv[dt][1]), f2bf2(dv[dt][2], dv[dt][3]));
      }
    }
  }
  // one wave per 16-row tile runs both roles in turn (nt waves per block: 120 VGPRs and a 54 KB LDS image fit
  // three blocks per CU, where a wave per role held one 2 nt-wave block per CU)
  if (wave < nt) {
    // ---- dQ for queries [16 qt, 16 qt + 16): accumulators C[key][q] (lane = query, rows = 4 keys)
    const int qt = wave;
    const int q = qt * 16 + fr;
    uint4 qf[NKS], of[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      qf[ks] = rowfrag<LDR>(Qs, qt * 16, ks * 32, lane);
      of[ks] = rowfrag<LDR>(dOs, qt * 16, ks * 32, lane);
    }
    const float lse = lse_s[q], de = delta_s[q];
    f32x4_t dq[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) dq[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    const int kp1 = p.causal ? ((qt * 16 + 15) >> 5) + 1 : npair;  // later key pairs are all masked
    for (int kp = 0; kp < kp1 && kp < npair; ++kp) {
      float ds[8];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        const int kt = 2 * kp + sub;
        f32x4_t st = (f32x4_t){0.f, 0.f, 0.f, 0.f}, dpt = st;
        if (kt < nt) {  // key tiles past Sp16 are all padding (and V holds no rows for them)
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks) {
            st = mfma(rowfrag<LDR>(Ks, kt * 16, ks * 32, lane), qf[ks], st);
            dpt = mfma(rowfrag<LDR>(Vs, kt * 16, ks * 32, lane), of[ks], dpt);
          }
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int key = kt * 16 + 4 * fg + v;
          float pv = 0.f;
          if (lse != -INFINITY && kok(q, key)) pv = __expf(st[v] * p.scale - lse);
          float ms = 1.f;
          if (thr && q < S && key < S) ms = drop_scale(seed, dbase + (uint64_t)q * SS + key, thr, inv_keep);
          ds[sub * 4 + v] = pv * (dpt[v] * ms - de);
        }
      }
      uint4 xs;
      xs.x = f2bf2(ds[0], ds[1]); xs.y = f2bf2(ds[2], ds[3]); xs.z = f2bf2(ds[4], ds[5]); xs.w = f2bf2(ds[6], ds[7]);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) dq[dt] = mfma(trfrag<LDR>(Ks, kp * 32, dt * 16, lane), xs, dq[dt]);
    }
    if (q < S) {
      bf16_t* rowp = dqkv + trow(g, b, q) * p.ld_dqkv + h * HD;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
        *reinterpret_cast<uint2*>(rowp + dt * 16 + 4 * fg) =
            make_uint2(f2bf2(dq[dt][0] * p.scale, dq[dt][1] * p.scale), f2bf2(dq[dt][2] * p.scale, dq[dt][3] * p.scale));
    }
  }
}

// Forward v2: K and V of the head staged row-major in LDS (16-byte copies); one wave per 16-query tile.
// S^T = K Q^T puts the keys of a query in the accumulator ROWS (lane = query), so the masked softmax reduces
// over registers plus the 4 lane groups, and P^T (bf16, dropout applied) is the B operand of O^T = V^T P^T
// directly, with V^T read transposed (ds_read_b64_tr_b16) from the row-major image. Fully masked causal key
// tiles are skipped. Output rows come out 4 head dims per lane (8-byte stores).
template <int HD>
__global__ __launch_bounds__(512) void fwd2_kernel(icap_attn_args p, Geo g, uint32_t thr, float inv_keep) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sm[];
  constexpr int LDR = ldr_of(HD);
  constexpr int NKS = HD / 32;
  constexpr int NDT = HD / 16;
  constexpr int CPR = HD / 8;
  const int bh = blockIdx.x;
  const int b = bh / g.H, h = bh - b * g.H;
  if (!localize(g, p, b)) return;
  const int Sp = g.Sp32, S = g.S, SS = g.Sst;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  bf16_t* Ks = sm;
  bf16_t* Vs = Ks + Sp * LDR;
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  const int qt = wave;
  // Q fragments of this query tile straight from HBM/L2 (B operand: rows = queries), issued before the K / V
  // staging loads so both are one memory round trip (round 5: they were a second dependent trip after the barrier;
  // gfrag clamps its rows, so the waves past S load valid addresses and exit below)
  uint4 qf[NKS];
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) qf[ks] = gfrag(qkv, p.ld_qkv, h * HD, g, b, qt * 16, ks * 32, lane);
  for (int idx = threadIdx.x; idx < Sp * CPR; idx += blockDim.x) {
    const int r = idx / CPR, c = idx - r * CPR;
    uint4 k = make_uint4(0, 0, 0, 0), v = k;
    if (r < S) {
      const bf16_t* src = qkv + trow(g, b, r) * p.ld_qkv + g.D + h * HD + 8 * c;
      k = *reinterpret_cast<const uint4*>(src);
      v = *reinterpret_cast<const uint4*>(src + g.D);
    }
    *reinterpret_cast<uint4*>(Ks + r * LDR + 8 * c) = k;
    *reinterpret_cast<uint4*>(Vs + r * LDR + 8 * c) = v;
  }
  __syncthreads();
  if (qt * 16 >= S) return;  // (packed sequences shorter than the launch's S; no barrier follows)
  const int q = qt * 16 + fr;
  const int npair = Sp >> 5;
  const int kp1 = p.causal ? ((qt * 16 + 15) >> 5) + 1 : npair;
  const int np = kp1 < npair ? kp1 : npair;
  f32x4_t st[MAXKT];  // up to 8 key tiles of 16
#pragma unroll
  for (int t = 0; t < MAXKT; ++t) st[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
  float m = -INFINITY;
#pragma unroll
  for (int t = 0; t < MAXKT; ++t) {
    if (t < 2 * np) {
#pragma unroll
      for (int ks = 0; ks < NKS; ++ks) st[t] = mfma(rowfrag<LDR>(Ks, t * 16, ks * 32, lane), qf[ks], st[t]);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int key = t * 16 + 4 * fg + v;
        const float x = key_ok(p.causal, p.key_mask, g, b, q, key) ? st[t][v] * p.scale : -INFINITY;
        st[t][v] = x;
        m = fmaxf(m, x);
      }
    }
  }
  // row max / sum over the 4 lane groups that share this query
  m = fmaxf(m, __shfl_xor(m, 16, 64));
  m = fmaxf(m, __shfl_xor(m, 32, 64));
  float l = 0.f;
#pragma unroll
  for (int t = 0; t < MAXKT; ++t) {
    if (t < 2 * np) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const float e = (m == -INFINITY) ? 0.f : __expf(st[t][v] - m);
        st[t][v] = e;
        l += e;
      }
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  const float inv = l > 0.f ? 1.f / l : 0.f;
  if (fg == 0 && q < S && p.lse) p.lse[(int64_t)bh * SS + q] = l > 0.f ? m + logf(l) : -INFINITY;
  const uint64_t seed = thr ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  const uint64_t dbase = p.offset + (uint64_t)bh * SS * SS;
  f32x4_t o[NDT];
#pragma unroll
  for (int dt = 0; dt < NDT; ++dt) o[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kp = 0; kp < MAXKT / 2; ++kp) {
    if (kp < np) {
      float pv[8];
#pragma unroll
      for (int sub = 0; sub < 2; ++sub)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int key = (2 * kp + sub) * 16 + 4 * fg + v;
          float x = st[2 * kp + sub][v] * inv;
          if (thr && q < S && key < S) x *= drop_scale(seed, dbase + (uint64_t)q * SS + key, thr, inv_keep);
          pv[sub * 4 + v] = x;
        }
      uint4 xp;
      xp.x = f2bf2(pv[0], pv[1]); xp.y = f2bf2(pv[2], pv[3]); xp.z = f2bf2(pv[4], pv[5]); xp.w = f2bf2(pv[6], pv[7]);
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt) o[dt] = mfma(trfrag<LDR>(Vs, kp * 32, dt * 16, lane), xp, o[dt]);
    }
  }
  if (q < S) {
    bf16_t* rowp = reinterpret_cast<bf16_t*>(p.out) + trow(g, b, q) * p.ld_out + h * HD;
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt)
      *reinterpret_cast<uint2*>(rowp + dt * 16 + 4 * fg) = make_uint2(f2bf2(o[dt][0], o[dt][1]), f2bf2(o[dt][2], o[dt][3]));
  }
}

// Forward v3 for sequences past the 8 register-resident key tiles of v2 (ViT-L/14: S = 257): the same K/V LDS
// images and S^T / O^T accumulator layouts, with the keys walked in chunks of 8 tiles under an online softmax
// (running max / sum per query, O^T rescaled per lane since lane = query), and each wave looping over query
// tiles. P is exponentiated against the running max, rounded to bf16 unnormalised, and O is divided by the
// final sum; lse = max + log(sum) as in v2, so the backward recomputes the same probabilities.
template <int HD>
__global__ __launch_bounds__(HD == 64 ? 1024 : 512) void fwd3_kernel(icap_attn_args p, Geo g, uint32_t thr, float inv_keep) {
  extern __shared__ __attribute__((aligned(16))) bf16_t sm[];
  constexpr int LDR = ldr_of(HD);
  constexpr int NKS = HD / 32;
  constexpr int NDT = HD / 16;
  constexpr int CPR = HD / 8;
  const int bh = blockIdx.x;
  const int b = bh / g.H, h = bh - b * g.H;
  if (!localize(g, p, b)) return;
  const int Sp = g.Sp32, S = g.S, SS = g.Sst;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  bf16_t* Ks = sm;
  bf16_t* Vs = Ks + Sp * LDR;
  const bf16_t* qkv = reinterpret_cast<const bf16_t*>(p.qkv);
  for (int idx = threadIdx.x; idx < Sp * CPR; idx += blockDim.x) {
    const int r = idx / CPR, c = idx - r * CPR;
    uint4 k = make_uint4(0, 0, 0, 0), v = k;
    if (r < S) {
      const bf16_t* src = qkv + trow(g, b, r) * p.ld_qkv + g.D + h * HD + 8 * c;
      k = *reinterpret_cast<const uint4*>(src);
      v = *reinterpret_cast<const uint4*>(src + g.D);
    }
    *reinterpret_cast<uint4*>(Ks + r * LDR + 8 * c) = k;
    *reinterpret_cast<uint4*>(Vs + r * LDR + 8 * c) = v;
  }
  __syncthreads();
  const int nqt = g.Sp16 >> 4;
  const int nkt = Sp >> 4;  // key tiles incl. the zero rows up to Sp32 (pairs stay whole)
  const uint64_t seed = thr ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  const uint64_t dbase = p.offset + (uint64_t)bh * SS * SS;
  for (int qt = wave; qt < nqt; qt += nw) {
    const int q = qt * 16 + fr;
    uint4 qf[NKS];
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) qf[ks] = gfrag(qkv, p.ld_qkv, h * HD, g, b, qt * 16, ks * 32, lane);
    const int klim = p.causal ? (qt * 16 + 16 < S ? qt * 16 + 16 : S) : S;  // keys past it are all masked
    float m = -INFINITY, l = 0.f;
    f32x4_t o[NDT];
#pragma unroll
    for (int dt = 0; dt < NDT; ++dt) o[dt] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
    for (int c0 = 0; c0 < nkt && c0 * 16 < klim; c0 += MAXKT) {
      f32x4_t st[MAXKT];
      float mc = -INFINITY;
#pragma unroll
      for (int t = 0; t < MAXKT; ++t) {
        st[t] = (f32x4_t){0.f, 0.f, 0.f, 0.f};
        if (c0 + t < nkt) {
#pragma unroll
          for (int ks = 0; ks < NKS; ++ks) st[t] = mfma(rowfrag<LDR>(Ks, (c0 + t) * 16, ks * 32, lane), qf[ks], st[t]);
        }
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int key = (c0 + t) * 16 + 4 * fg + v;
          const float x = (c0 + t < nkt && key_ok(p.causal, p.key_mask, g, b, q, key)) ? st[t][v] * p.scale : -INFINITY;
          st[t][v] = x;
          mc = fmaxf(mc, x);
        }
      }
      mc = fmaxf(mc, __shfl_xor(mc, 16, 64));
      mc = fmaxf(mc, __shfl_xor(mc, 32, 64));
      const float mn = fmaxf(m, mc);
      const float alpha = (m == -INFINITY) ? 0.f : __expf(m - mn);
      m = mn;
      l *= alpha;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
        for (int v = 0; v < 4; ++v) o[dt][v] *= alpha;
#pragma unroll
      for (int kp = 0; kp < MAXKT / 2; ++kp) {
        if (c0 + 2 * kp < nkt) {
          float pv[8];
#pragma unroll
          for (int sub = 0; sub < 2; ++sub)
#pragma unroll
            for (int v = 0; v < 4; ++v) {
              const int key = (c0 + 2 * kp + sub) * 16 + 4 * fg + v;
              float e = (m == -INFINITY) ? 0.f : __expf(st[2 * kp + sub][v] - m);
              l += e;
              if (thr && q < S && key < S) e *= drop_scale(seed, dbase + (uint64_t)q * SS + key, thr, inv_keep);
              pv[sub * 4 + v] = e;
            }
          uint4 xp;
          xp.x = f2bf2(pv[0], pv[1]); xp.y = f2bf2(pv[2], pv[3]); xp.z = f2bf2(pv[4], pv[5]); xp.w = f2bf2(pv[6], pv[7]);
#pragma unroll
          for (int dt = 0; dt < NDT; ++dt) o[dt] = mfma(trfrag<LDR>(Vs, (c0 / 2 + kp) * 32, dt * 16, lane), xp, o[dt]);
        }
      }
    }
    l += __shfl_xor(l, 16, 64);
    l += __shfl_xor(l, 32, 64);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    if (fg == 0 && q < S && p.lse) p.lse[(int64_t)bh * SS + q] = l > 0.f ? m + logf(l) : -INFINITY;
    if (q < S) {
      bf16_t* rowp = reinterpret_cast<bf16_t*>(p.out) + trow(g, b, q) * p.ld_out + h * HD;
#pragma unroll
      for (int dt = 0; dt < NDT; ++dt)
        *reinterpret_cast<uint2*>(rowp + dt * 16 + 4 * fg) =
            make_uint2(f2bf2(o[dt][0] * inv, o[dt][1] * inv), f2bf2(o[dt][2] * inv, o[dt][3] * inv));
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
  g.Sst = a->S; g.base = 0; g.kmb = 0;
  g.slo = 0; g.shi = 1 << 30;
  return g;
}

// Packed sequences (seq_len) in a launch of S > SHORT_S tokens: the v2 kernels run as two passes, the sequences of
// at most SHORT_S tokens with LDS and waves sized for SHORT_S (many blocks per CU: one round over the grid), then the
// longer ones with the launch's sizing (the short ones exit at once). The caption batches of the train step are all
// short (prefix + caption up to its last target); the split only changes which blocks run, never the arithmetic.
// icap_attn_args.short_only: the caller knows no sequence is longer (the trainer, from the batch's labels on the
// host), so the second pass — ~3-4 us of workgroups that only exit (tools/ab/ln_attn_probe.py) — is not launched.
constexpr int SHORT_S = 32;
static bool packed_split(const icap_attn_args* a) { return a->seq_len != nullptr && a->S > SHORT_S; }
static amfma::Geo short_geo(amfma::Geo g) {
  g.slo = 0; g.shi = SHORT_S;
  g.Sp16 = SHORT_S; g.Sp32 = SHORT_S; g.ldT = g.Sp32 + 8;
  return g;
}

size_t mfma_fwd_lds(const amfma::Geo& g) { return 2 * ((size_t)g.hd * g.ldT + 4 * 16 * (size_t)g.ldT); }
size_t mfma_bwd_lds(const amfma::Geo& g) {
  return 2 * (3 * (size_t)g.hd * g.ldT + 2 * (size_t)g.Sp16 * g.ldT + 4 * 16 * (size_t)g.ldT);
}

size_t mfma_fwd2_lds(const amfma::Geo& g) { return 2 * 2 * (size_t)g.Sp32 * amfma::ldr_of(g.hd); }

static bool mfma_fwd2_ok(const icap_attn_args* a) {
  if ((a->ld_out & 3) || (a->ld_qkv & 7)) return false;
  if ((reinterpret_cast<uintptr_t>(a->out) & 7) || (reinterpret_cast<uintptr_t>(a->qkv) & 15)) return false;
  const amfma::Geo g = mfma_geo(a);
  return (g.Sp16 / 16) * 64 <= 512;
}

size_t mfma_bwd2_lds(const amfma::Geo& g) {
  return 2 * (3 * (size_t)g.Sp32 + (size_t)g.Sp16) * amfma::ldr_of(g.hd) + 2 * sizeof(float) * (size_t)g.Sp32 +
         (size_t)g.Sp32;
}

// v2 backward: needs O (delta), 16-byte aligned row segments, and 2 * Sp16/16 waves within the launch bound
static bool mfma_bwd2_ok(const icap_attn_args* a) {
  if (a->out == nullptr || (a->ld_out & 7) || (a->ld_dqkv & 7)) return false;
  if ((reinterpret_cast<uintptr_t>(a->out) | reinterpret_cast<uintptr_t>(a->qkv) |
       reinterpret_cast<uintptr_t>(a->dout) | reinterpret_cast<uintptr_t>(a->dqkv)) & 15)
    return false;
  const amfma::Geo g = mfma_geo(a);
  const int waves = g.Sp16 / 16;
  return waves * 64 <= 512 && mfma_bwd2_lds(g) <= 160 * 1024;
}

size_t mfma_fwd3_lds(const amfma::Geo& g) { return 2 * 2 * (size_t)g.Sp32 * amfma::ldr_of(g.hd); }

// long-sequence forward (v3): S past 8 key tiles, K/V of the whole sequence in LDS
static bool mfma_fwd3_ok(const icap_attn_args* a) {
  if (a->dtype != ICAP_BF16 || (a->hd != 64 && a->hd != 96) || a->S <= 16 * amfma::MAXKT) return false;
  if ((a->ld_out & 3) || (a->ld_qkv & 7)) return false;
  if ((reinterpret_cast<uintptr_t>(a->out) & 7) || (reinterpret_cast<uintptr_t>(a->qkv) & 15)) return false;
  return mfma_fwd3_lds(mfma_geo(a)) <= 160 * 1024;
}

bool mfma_attention_ok(const icap_attn_args* a, bool bwd) {
  if (!bwd && mfma_fwd3_ok(a)) return true;
  // head dim 128 (the mapper at gpt_dim 1024, BASELINE configs[3]): the transpose-free v2 kernels only
  if (a->dtype == ICAP_BF16 && a->hd == 128 && a->S <= 16 * amfma::MAXKT && !(a->ld_qkv & 7))
    return bwd ? ((a->ld_dout & 7) == 0 && mfma_bwd2_ok(a)) : mfma_fwd2_ok(a);
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
  if (!bwd && mfma_fwd3_ok(a)) {
    // waves: the fewest that cover the query tiles in an equal number of passes (at most 16)
    const int maxw = a->hd == 64 ? 16 : 8;  // (the hd-96 form is built for 512 threads: register budget)
    const int nqt = g.Sp16 / 16, passes = (nqt + maxw - 1) / maxw;
    const dim3 block3((unsigned)(64 * ((nqt + passes - 1) / passes)));
    const size_t lds3 = mfma_fwd3_lds(g);
    if (a->hd == 64) {
      static bool once = (lds_limit(amfma::fwd3_kernel<64>), true); (void)once;
      hipLaunchKernelGGL(amfma::fwd3_kernel<64>, grid, block3, lds3, s, *a, g, thr, inv_keep);
    } else {
      static bool once = (lds_limit(amfma::fwd3_kernel<96>), true); (void)once;
      hipLaunchKernelGGL(amfma::fwd3_kernel<96>, grid, block3, lds3, s, *a, g, thr, inv_keep);
    }
    return check_launch("icap_attention_fwd(mfma v3)");
  }
  if (!bwd && mfma_fwd2_ok(a)) {
    static bool once = (lds_limit(amfma::fwd2_kernel<64>), lds_limit(amfma::fwd2_kernel<128>),
                        lds_limit(amfma::fwd2_kernel<96>), true);
    (void)once;
    auto go = [&](const amfma::Geo& gg) {
      const size_t lds2 = mfma_fwd2_lds(gg);
      const dim3 block2((unsigned)(64 * (gg.Sp16 / 16)));
      if (a->hd == 64) hipLaunchKernelGGL(amfma::fwd2_kernel<64>, grid, block2, lds2, s, *a, gg, thr, inv_keep);
      else if (a->hd == 128) hipLaunchKernelGGL(amfma::fwd2_kernel<128>, grid, block2, lds2, s, *a, gg, thr, inv_keep);
      else hipLaunchKernelGGL(amfma::fwd2_kernel<96>, grid, block2, lds2, s, *a, gg, thr, inv_keep);
    };
    if (packed_split(a)) {
      go(short_geo(g));
      if (!a->short_only) {
        amfma::Geo gl = g;
        gl.slo = SHORT_S;
        go(gl);
      }
    } else {
      go(g);
    }
    return check_launch("icap_attention_fwd(mfma v2)");
  }
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
    if (mfma_bwd2_ok(a)) {
      static bool once = (lds_limit(amfma::bwd2_kernel<64>), lds_limit(amfma::bwd2_kernel<128>),
                          lds_limit(amfma::bwd2_kernel<96>), true);
      (void)once;
      auto go = [&](const amfma::Geo& gg) {
        const size_t lds2 = mfma_bwd2_lds(gg);
        const dim3 block2((unsigned)(64 * (gg.Sp16 / 16)));
        if (a->hd == 64) hipLaunchKernelGGL(amfma::bwd2_kernel<64>, grid, block2, lds2, s, *a, gg, thr, inv_keep);
        else if (a->hd == 128) hipLaunchKernelGGL(amfma::bwd2_kernel<128>, grid, block2, lds2, s, *a, gg, thr, inv_keep);
        else hipLaunchKernelGGL(amfma::bwd2_kernel<96>, grid, block2, lds2, s, *a, gg, thr, inv_keep);
      };
      if (packed_split(a)) {
        go(short_geo(g));
        if (!a->short_only) {
          amfma::Geo gl = g;
          gl.slo = SHORT_S;
          go(gl);
        }
      } else {
        go(g);
      }
      return check_launch("icap_attention_bwd(mfma v2)");
    }
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

// Multi-head softmax attention for the short sequences of the captioning path
// (GPT-2 S=65 causal+padding, CLIP S=50, mapper S=25 with head_dim 96).
//
// One workgroup per (batch, head) (forward: per query chunk when S x S overflows LDS): Q, K, V (and dO in backward) are staged once
// from HBM into LDS as fp32 (rows padded to hd+1 floats so column walks are
// bank-conflict free), the S x S score block lives in LDS, softmax row
// reductions use wave shuffles, and P.V / dS.K / dS^T.Q / P^T.dO are LDS dot
// products. At these sizes the attention core is ~1 % of the step FLOPs
// (0.156 of 11.2 GF/sample); the kernel is bound by its
// QKV/out HBM traffic, so it is written for coalesced loads, not for MFMA.
#include "common.h"

#include <math.h>

namespace icap {

// S: tokens of this block's sequence (seq_len[b] for packed sequences); Sst: the launch's S (lse / dropout
// numbering); base / kmb: row of token 0 and its key-mask index (attn_localize)
struct AttnGeom {
  int S, H, hd, D;
  int64_t rsb, rss;  // row strides (in rows) for batch and sequence
  int Sst;
  int64_t base, kmb;
};

__device__ __forceinline__ int64_t tok_row(const AttnGeom& g, int b, int s) { return g.base + (int64_t)s * g.rss; }

__device__ __forceinline__ bool attn_localize(AttnGeom& g, const icap_attn_args& p, int b) {
  if (p.seq_len) {
    const int n = p.seq_len[b];
    g.S = n < g.Sst ? n : g.Sst;
    g.base = p.seq_off[b];
    g.kmb = p.seq_off[b];
  } else {
    g.base = (int64_t)b * g.rsb;
    g.kmb = (int64_t)b * g.Sst;
  }
  return g.S > 0;
}

template <typename T>
__device__ __forceinline__ void stage_head(const T* src, int64_t ld, int col0, const AttnGeom& g, int b,
                                           float* dst, int dld, float mul) {
  const int nv = g.hd >> 2;  // float4 groups per row (hd % 4 == 0)
  for (int idx = threadIdx.x; idx < g.S * nv; idx += blockDim.x) {
    const int s = idx / nv, c = idx - s * nv;
    float v[4];
    io<T>::ld4(src + tok_row(g, b, s) * ld + col0 + 4 * c, v);
    float* d = dst + s * dld + 4 * c;
    d[0] = v[0] * mul; d[1] = v[1] * mul; d[2] = v[2] * mul; d[3] = v[3] * mul;
  }
}

__device__ __forceinline__ bool allowed(int causal, const int32_t* key_mask, int64_t kmb, int i, int j) {
  if (causal && j > i) return false;
  if (key_mask && key_mask[kmb + j] == 0) return false;
  return true;
}

// Query rows [q0, q0 + QT) of one (batch, head) per workgroup (blockIdx.y = chunk): K and V stay whole in LDS, the
// score block is QT x S. QT == S for the short sequences (one chunk); the towers' S=197/257 fp32 parity mode uses
// QT < S so the block fits the 160 KB LDS. Every row's arithmetic is the same whatever QT is.
template <typename T>
__global__ __launch_bounds__(256) void attn_fwd_kernel(icap_attn_args p, AttnGeom g, int QT, uint32_t thr, float inv_keep) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int bh = blockIdx.x;
  const int b = bh / g.H, h = bh - b * g.H;
  if (!attn_localize(g, p, b)) return;
  const int S = g.S, SS = g.Sst, hd = g.hd, ldp = hd + 1;
  const int q0 = blockIdx.y * QT, nq = min(QT, S - q0);
  if (nq <= 0) return;
  float* Ks = sm;
  float* Vs = Ks + S * ldp;
  float* Qs = Vs + S * ldp;
  float* P = Qs + QT * ldp;
  const T* qkv = reinterpret_cast<const T*>(p.qkv);
  stage_head<T>(qkv, p.ld_qkv, g.D + h * hd, g, b, Ks, ldp, 1.f);
  stage_head<T>(qkv, p.ld_qkv, 2 * g.D + h * hd, g, b, Vs, ldp, 1.f);
  {
    const int nv = hd >> 2;
    for (int idx = threadIdx.x; idx < nq * nv; idx += blockDim.x) {
      const int s = idx / nv, c = idx - s * nv;
      float v[4];
      io<T>::ld4(qkv + tok_row(g, b, q0 + s) * p.ld_qkv + h * hd + 4 * c, v);
      float* d = Qs + s * ldp + 4 * c;
      d[0] = v[0] * p.scale; d[1] = v[1] * p.scale; d[2] = v[2] * p.scale; d[3] = v[3] * p.scale;
    }
  }
  __syncthreads();

  for (int idx = threadIdx.x; idx < nq * S; idx += blockDim.x) {
    const int il = idx / S, j = idx - il * S;
    float s = -INFINITY;
    if (allowed(p.causal, p.key_mask, g.kmb, q0 + il, j)) {
      const float* q = Qs + il * ldp;
      const float* k = Ks + j * ldp;
      float a0 = 0.f, a1 = 0.f;
      for (int d = 0; d < hd; d += 2) {
        a0 = fmaf(q[d], k[d], a0);
        a1 = fmaf(q[d + 1], k[d + 1], a1);
      }
      s = a0 + a1;
    }
    P[idx] = s;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  const uint64_t drop_base = p.offset + (uint64_t)bh * SS * SS;
  const uint64_t seed = thr ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  for (int il = wv; il < nq; il += nwv) {
    const int i = q0 + il;
    float* row = P + il * S;
    float m = -INFINITY;
    for (int j = lane; j < S; j += 64) m = fmaxf(m, row[j]);
    m = wave_max(m);
    float l = 0.f;
    for (int j = lane; j < S; j += 64) l += (m == -INFINITY) ? 0.f : __expf(row[j] - m);
    l = wave_sum(l);
    const float inv = l > 0.f ? 1.f / l : 0.f;
    for (int j = lane; j < S; j += 64) {
      float pv = (m == -INFINITY) ? 0.f : __expf(row[j] - m) * inv;
      if (thr) pv *= drop_scale(seed, drop_base + (uint64_t)i * SS + j, thr, inv_keep);
      row[j] = pv;
    }
    if (lane == 0 && p.lse) p.lse[(int64_t)bh * SS + i] = (l > 0.f) ? m + logf(l) : -INFINITY;
  }
  __syncthreads();

  T* out = reinterpret_cast<T*>(p.out);
  for (int idx = threadIdx.x; idx < nq * hd; idx += blockDim.x) {
    const int il = idx / hd, d = idx - il * hd;
    const float* row = P + il * S;
    float a0 = 0.f, a1 = 0.f;
    int j = 0;
    for (; j + 1 < S; j += 2) {
      a0 = fmaf(row[j], Vs[j * ldp + d], a0);
      a1 = fmaf(row[j + 1], Vs[(j + 1) * ldp + d], a1);
    }
    if (j < S) a0 = fmaf(row[j], Vs[j * ldp + d], a0);
    io<T>::st(out + tok_row(g, b, q0 + il) * p.ld_out + h * hd + d, a0 + a1);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void attn_bwd_kernel(icap_attn_args p, AttnGeom g, uint32_t thr, float inv_keep) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  const int bh = blockIdx.x;
  const int b = bh / g.H, h = bh - b * g.H;
  if (!attn_localize(g, p, b)) return;
  const int S = g.S, SS = g.Sst, hd = g.hd, ldp = hd + 1;
  float* Qs = sm;
  float* Ks = Qs + S * ldp;
  float* Vs = Ks + S * ldp;
  float* dOs = Vs + S * ldp;
  float* P = dOs + S * ldp;   // P, then dropped P
  float* dS = P + S * S;      // dPd, then dS
  const T* qkv = reinterpret_cast<const T*>(p.qkv);
  stage_head<T>(qkv, p.ld_qkv, h * hd, g, b, Qs, ldp, p.scale);
  stage_head<T>(qkv, p.ld_qkv, g.D + h * hd, g, b, Ks, ldp, 1.f);
  stage_head<T>(qkv, p.ld_qkv, 2 * g.D + h * hd, g, b, Vs, ldp, 1.f);
  stage_head<T>(reinterpret_cast<const T*>(p.dout), p.ld_dout, h * hd, g, b, dOs, ldp, 1.f);
  __syncthreads();

  for (int idx = threadIdx.x; idx < S * S; idx += blockDim.x) {
    const int i = idx / S, j = idx - i * S;
    float pv = 0.f, dp = 0.f;
    const float lse = p.lse[(int64_t)bh * SS + i];
    if (allowed(p.causal, p.key_mask, g.kmb, i, j) && lse != -INFINITY) {
      const float* q = Qs + i * ldp;
      const float* k = Ks + j * ldp;
      const float* o = dOs + i * ldp;
      const float* v = Vs + j * ldp;
      float a0 = 0.f, a1 = 0.f, c0 = 0.f, c1 = 0.f;
      for (int d = 0; d < hd; d += 2) {
        a0 = fmaf(q[d], k[d], a0);
        a1 = fmaf(q[d + 1], k[d + 1], a1);
        c0 = fmaf(o[d], v[d], c0);
        c1 = fmaf(o[d + 1], v[d + 1], c1);
      }
      pv = __expf(a0 + a1 - lse);
      dp = c0 + c1;
    }
    P[idx] = pv;
    dS[idx] = dp;
  }
  __syncthreads();

  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  const uint64_t drop_base = p.offset + (uint64_t)bh * SS * SS;
  const uint64_t seed = thr ? eff_seed(p.seed, p.seed_ptr) : 0ull;
  for (int i = wv; i < S; i += nwv) {
    float* prow = P + i * S;
    float* drow = dS + i * S;
    float delta = 0.f;
    for (int j = lane; j < S; j += 64) {
      float dp = drow[j];
      if (thr) dp *= drop_scale(seed, drop_base + (uint64_t)i * SS + j, thr, inv_keep);
      drow[j] = dp;
      delta += prow[j] * dp;
    }
    delta = wave_sum(delta);
    for (int j = lane; j < S; j += 64) {
      const float pv = prow[j];
      drow[j] = pv * (drow[j] - delta);
      if (thr) prow[j] = pv * drop_scale(seed, drop_base + (uint64_t)i * SS + j, thr, inv_keep);
    }
  }
  __syncthreads();

  T* dqkv = reinterpret_cast<T*>(p.dqkv);
  for (int idx = threadIdx.x; idx < S * hd; idx += blockDim.x) {
    const int i = idx / hd, d = idx - i * hd;  // i: query row for dQ, key row for dK/dV
    float aq = 0.f, ak = 0.f, av = 0.f;
    for (int j = 0; j < S; ++j) {
      aq = fmaf(dS[i * S + j], Ks[j * ldp + d], aq);   // dQ_i = sum_j dS_ij K_j
      ak = fmaf(dS[j * S + i], Qs[j * ldp + d], ak);   // dK_i = sum_j dS_ji Qs_j
      av = fmaf(P[j * S + i], dOs[j * ldp + d], av);   // dV_i = sum_j Pd_ji dO_j
    }
    T* rowp = dqkv + tok_row(g, b, i) * p.ld_dqkv;
    io<T>::st(rowp + h * hd + d, aq * p.scale);
    io<T>::st(rowp + g.D + h * hd + d, ak);
    io<T>::st(rowp + 2 * g.D + h * hd + d, av);
  }
}

// one wave per (b, h); keys 0..pos from the position-major cache
template <typename T>
__global__ __launch_bounds__(64) void attn_decode_kernel(int B, int H, int hd, int pos, const T* __restrict__ cache,
                                                        int64_t ld, const int32_t* __restrict__ anc,
                                                        T* __restrict__ out, int64_t ld_out, float scale) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* q = sm;            // hd
  float* sc = sm + 128;     // pos+1 scores
  const int bh = blockIdx.x;
  const int b = bh / H, h = bh - b * H;
  const int D = H * hd;
  const int lane = threadIdx.x;
  const int n = pos + 1;
  const T* qrow = cache + ((int64_t)pos * B + b) * ld + h * hd;
  for (int d = lane; d < hd; d += 64) q[d] = io<T>::ld(qrow + d) * scale;
  __syncthreads();
  float m = -INFINITY;
  // row of key j: this row's own (b) or, in beam search, the cache row its history holds position j in
  auto src = [&](int j) -> int64_t { return anc ? (int64_t)anc[(int64_t)j * B + b] : (int64_t)b; };
  for (int j = lane; j < n; j += 64) {
    const T* krow = cache + ((int64_t)j * B + src(j)) * ld + D + h * hd;
    float a = 0.f;
    for (int d = 0; d < hd; d += 4) {
      float kv[4];
      io<T>::ld4(krow + d, kv);
      a = fmaf(q[d], kv[0], a);
      a = fmaf(q[d + 1], kv[1], a);
      a = fmaf(q[d + 2], kv[2], a);
      a = fmaf(q[d + 3], kv[3], a);
    }
    sc[j] = a;
    m = fmaxf(m, a);
  }
  m = wave_max(m);
  float l = 0.f;
  for (int j = lane; j < n; j += 64) {
    const float e = __expf(sc[j] - m);
    sc[j] = e;
    l += e;
  }
  l = wave_sum(l);
  __syncthreads();
  const float inv = 1.f / l;
  for (int d = lane; d < hd; d += 64) {
    float a = 0.f;
    for (int j = 0; j < n; ++j) a = fmaf(sc[j], io<T>::ld(cache + ((int64_t)j * B + src(j)) * ld + 2 * D + h * hd + d), a);
    io<T>::st(out + (int64_t)b * ld_out + h * hd + d, a * inv);
  }
}

// bf16, hd = 64 (every GPT-2 size): one wave per (b, h). The V rows of the first 8*TV keys go into registers
// before any score is computed (they do not depend on the scores), so the K and V reads of a short cache share
// one memory round trip; lane = key for the QK^T dots (8 x 16-byte loads per K row), lane = (key group kg = lane/8,
// 16-byte column chunk dc = lane%8) for P.V, the 8 key groups summed with cross-lane adds at the end.
template <int TV>
__global__ __launch_bounds__(64) void attn_decode64_kernel(int B, int H, int pos, const bf16_t* __restrict__ cache,
                                                          int64_t ld, const int32_t* __restrict__ anc,
                                                          bf16_t* __restrict__ out, int64_t ld_out, float scale) {
  extern __shared__ __attribute__((aligned(16))) float sm[];
  float* q = sm;         // 64
  float* sc = sm + 64;   // pos + 1 scores
  const int bh = blockIdx.x;
  const int b = bh / H, h = bh - b * H;
  const int D = H * 64;
  const int lane = threadIdx.x, kg = lane >> 3, dc = lane & 7;
  const int n = pos + 1;
  const int64_t rs = (int64_t)B * ld;  // elements from one position's row to the next
  const bf16_t* base = cache + (int64_t)b * ld + h * 64;
  // key j's row (relative to base): this row's own or, in beam search, the cache row holding its position j
  auto koff = [&](int j) -> int64_t { return j * rs + (anc ? ((int64_t)anc[(int64_t)j * B + b] - b) * ld : 0); };
  uint4 vr[TV];
#pragma unroll
  for (int t = 0; t < TV; ++t) {
    const int j = kg + 8 * t;
    vr[t] = j < n ? *reinterpret_cast<const uint4*>(base + koff(j) + 2 * D + dc * 8) : make_uint4(0u, 0u, 0u, 0u);
  }
  if (lane < 8) {
    float v[8];
    io<bf16_t>::ld8(base + (int64_t)pos * rs + lane * 8, v);
#pragma unroll
    for (int e = 0; e < 8; ++e) q[lane * 8 + e] = v[e] * scale;
  }
  __syncthreads();
  float m = -INFINITY;
  for (int j = lane; j < n; j += 64) {
    const bf16_t* kr = base + koff(j) + D;
    uint4 kk[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) kk[c] = *reinterpret_cast<const uint4*>(kr + 8 * c);
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const uint32_t w[4] = {kk[c].x, kk[c].y, kk[c].z, kk[c].w};
      const float4 q0 = *reinterpret_cast<const float4*>(q + 8 * c);
      const float4 q1 = *reinterpret_cast<const float4*>(q + 8 * c + 4);
      a0 = fmaf(q0.x, __uint_as_float(w[0] << 16), a0);
      a1 = fmaf(q0.y, __uint_as_float(w[0] & 0xffff0000u), a1);
      a0 = fmaf(q0.z, __uint_as_float(w[1] << 16), a0);
      a1 = fmaf(q0.w, __uint_as_float(w[1] & 0xffff0000u), a1);
      a0 = fmaf(q1.x, __uint_as_float(w[2] << 16), a0);
      a1 = fmaf(q1.y, __uint_as_float(w[2] & 0xffff0000u), a1);
      a0 = fmaf(q1.z, __uint_as_float(w[3] << 16), a0);
      a1 = fmaf(q1.w, __uint_as_float(w[3] & 0xffff0000u), a1);
    }
    const float s = a0 + a1;
    sc[j] = s;
    m = fmaxf(m, s);
  }
  m = wave_max(m);
  float l = 0.f;
  for (int j = lane; j < n; j += 64) {
    const float e = __expf(sc[j] - m);
    sc[j] = e;
    l += e;
  }
  l = wave_sum(l);
  __syncthreads();
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto add_row = [&](const uint4 v, float p) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      acc[2 * e] = fmaf(p, __uint_as_float(w[e] << 16), acc[2 * e]);
      acc[2 * e + 1] = fmaf(p, __uint_as_float(w[e] & 0xffff0000u), acc[2 * e + 1]);
    }
  };
#pragma unroll
  for (int t = 0; t < TV; ++t) {
    const int j = kg + 8 * t;
    if (j < n) add_row(vr[t], sc[j]);
  }
  for (int j = 8 * TV + kg; j < n; j += 8)  // keys past the prefetched ones (caches longer than 8*TV)
    add_row(*reinterpret_cast<const uint4*>(base + koff(j) + 2 * D + dc * 8), sc[j]);
#pragma unroll
  for (int o = 8; o < 64; o <<= 1)
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] += __shfl_xor(acc[e], o, 64);
  if (kg == 0) {
    const float inv = 1.f / l;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    io<bf16_t>::st8(out + (int64_t)b * ld_out + h * 64 + dc * 8, acc);
  }
}

// bf16 MFMA kernels (attention_mfma.hip); the fp32 parity mode and shapes they do not cover use the
// LDS/VALU kernels of this file. (diagnostic build) ICAP_ATTN_VALU=1 forces the VALU kernels.
bool mfma_attention_ok(const icap_attn_args* a, bool bwd);
int mfma_attention_launch(const icap_attn_args* a, bool bwd, uint32_t thr, float inv_keep, hipStream_t s);
static bool force_valu() {
  static const bool f = diag_env("ICAP_ATTN_VALU", 0) == 1;
  return f;
}

static size_t fwd_lds(int S, int hd, int QT) {
  return sizeof(float) * ((size_t)(2 * S + QT) * (hd + 1) + (size_t)QT * S);
}
static size_t bwd_lds(int S, int hd) { return sizeof(float) * ((size_t)4 * S * (hd + 1) + (size_t)2 * S * S); }
constexpr size_t LDS_CAP = 160 * 1024;

template <typename K>
static void raise_lds_limit(K kernel) {
  (void)hipFuncSetAttribute(reinterpret_cast<const void*>(kernel), hipFuncAttributeMaxDynamicSharedMemorySize, (int)LDS_CAP);
}

// Query rows per forward workgroup: the whole sequence when it fits, else the largest power of two that does
// (0 = K and V alone overflow LDS).
static int fwd_rows(int S, int hd) {
  if (fwd_lds(S, hd, S) <= LDS_CAP) return S;
  for (int qt = 128; qt >= 4; qt >>= 1)
    if (qt < S && fwd_lds(S, hd, qt) <= LDS_CAP) return qt;
  return 0;
}

static int check_attn(const icap_attn_args* a, bool bwd) {
  ICAP_REQUIRE(a != nullptr, "icap_attention: null args");
  ICAP_REQUIRE(a->dtype == ICAP_F32 || a->dtype == ICAP_BF16, "icap_attention: bad dtype");
  ICAP_REQUIRE(a->B >= 0 && a->S > 0 && a->H > 0 && a->hd > 0 && a->hd % 4 == 0, "icap_attention: bad geometry (hd % 4 == 0)");
  ICAP_REQUIRE(a->qkv && (bwd ? (a->dout && a->dqkv && a->lse) : (a->out != nullptr)), "icap_attention: null pointer");
  ICAP_REQUIRE(a->ld_qkv % 4 == 0, "icap_attention: ld_qkv must be a multiple of 4");
  ICAP_REQUIRE(a->drop_p >= 0.f && a->drop_p < 1.f, "icap_attention: drop_p out of range");
  ICAP_REQUIRE((a->seq_off == nullptr) == (a->seq_len == nullptr), "icap_attention: seq_off and seq_len go together");
  ICAP_REQUIRE(a->seq_off == nullptr || a->row_stride_s == 1, "icap_attention: packed sequences need row_stride_s 1");

  return ICAP_OK;
}

}  // namespace icap

using namespace icap;

extern "C" int icap_attention_fwd(const icap_attn_args* a, void* stream) {
  int rc = check_attn(a, false);
  if (rc) return rc;
  if (a->B == 0) return ICAP_OK;
  AttnGeom g{a->S, a->H, a->hd, a->H * a->hd, a->row_stride_b, a->row_stride_s, a->S, 0, 0};
  const uint32_t thr = a->drop_p > 0.f ? drop_threshold(a->drop_p) : 0u;
  const float inv_keep = a->drop_p > 0.f ? 1.f / (1.f - a->drop_p) : 1.f;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!force_valu() && mfma_attention_ok(a, false)) return mfma_attention_launch(a, false, thr, inv_keep, s);
  const int QT = fwd_rows(a->S, a->hd);
  ICAP_REQUIRE(QT > 0, "icap_attention: sequence/head too large for the LDS-resident kernel");
  const size_t lds = fwd_lds(a->S, a->hd, QT);
  dim3 grid((unsigned)(a->B * a->H), (unsigned)((a->S + QT - 1) / QT)), block(256);
  if (a->dtype == ICAP_BF16) {
    static bool once = (raise_lds_limit(attn_fwd_kernel<bf16_t>), true); (void)once;
    hipLaunchKernelGGL(attn_fwd_kernel<bf16_t>, grid, block, lds, s, *a, g, QT, thr, inv_keep);
  } else {
    static bool once = (raise_lds_limit(attn_fwd_kernel<float>), true); (void)once;
    hipLaunchKernelGGL(attn_fwd_kernel<float>, grid, block, lds, s, *a, g, QT, thr, inv_keep);
  }
  return check_launch("icap_attention_fwd");
}

extern "C" int icap_attention_bwd(const icap_attn_args* a, void* stream) {
  int rc = check_attn(a, true);
  if (rc) return rc;
  if (a->B == 0) return ICAP_OK;
  AttnGeom g{a->S, a->H, a->hd, a->H * a->hd, a->row_stride_b, a->row_stride_s, a->S, 0, 0};
  const uint32_t thr = a->drop_p > 0.f ? drop_threshold(a->drop_p) : 0u;
  const float inv_keep = a->drop_p > 0.f ? 1.f / (1.f - a->drop_p) : 1.f;
  const size_t lds = bwd_lds(a->S, a->hd);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (!force_valu() && mfma_attention_ok(a, true)) return mfma_attention_launch(a, true, thr, inv_keep, s);
  ICAP_REQUIRE(bwd_lds(a->S, a->hd) <= LDS_CAP, "icap_attention: sequence/head too large for the LDS-resident kernel");
  dim3 grid((unsigned)(a->B * a->H)), block(256);
  if (a->dtype == ICAP_BF16) {
    static bool once = (raise_lds_limit(attn_bwd_kernel<bf16_t>), true); (void)once;
    hipLaunchKernelGGL(attn_bwd_kernel<bf16_t>, grid, block, lds, s, *a, g, thr, inv_keep);
  } else {
    static bool once = (raise_lds_limit(attn_bwd_kernel<float>), true); (void)once;
    hipLaunchKernelGGL(attn_bwd_kernel<float>, grid, block, lds, s, *a, g, thr, inv_keep);
  }
  return check_launch("icap_attention_bwd");
}

extern "C" int icap_attention_decode_anc(int32_t dtype, int32_t B, int32_t H, int32_t hd, int32_t pos,
                                         const void* cache, int64_t ld_cache, const int32_t* anc, void* out,
                                         int64_t ld_out, float scale, void* stream) {
  ICAP_REQUIRE(hd > 0 && hd <= 128 && hd % 4 == 0, "icap_attention_decode: hd must be <= 128, multiple of 4");
  ICAP_REQUIRE(pos >= 0 && pos < 4096, "icap_attention_decode: pos out of range");
  ICAP_REQUIRE(cache && out, "icap_attention_decode: null pointer");
  if (B == 0) return ICAP_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dim3 grid((unsigned)(B * H)), block(64);
  const bool al = ((reinterpret_cast<uintptr_t>(cache) | reinterpret_cast<uintptr_t>(out)) & 15) == 0;
  if (dtype == ICAP_BF16 && hd == 64 && al && ld_cache % 8 == 0 && ld_out % 8 == 0) {
    const size_t lds = sizeof(float) * (64 + (size_t)pos + 1);
    hipLaunchKernelGGL(attn_decode64_kernel<16>, grid, block, lds, s, B, H, pos, (const bf16_t*)cache, ld_cache,
                       anc, (bf16_t*)out, ld_out, scale);
    return check_launch("icap_attention_decode");
  }
  const size_t lds = sizeof(float) * (128 + (size_t)pos + 1);
  if (dtype == ICAP_BF16)
    hipLaunchKernelGGL(attn_decode_kernel<bf16_t>, grid, block, lds, s, B, H, hd, pos, (const bf16_t*)cache, ld_cache,
                       anc, (bf16_t*)out, ld_out, scale);
  else
    hipLaunchKernelGGL(attn_decode_kernel<float>, grid, block, lds, s, B, H, hd, pos, (const float*)cache, ld_cache,
                       anc, (float*)out, ld_out, scale);
  return check_launch("icap_attention_decode");
}

extern "C" int icap_attention_decode(int32_t dtype, int32_t B, int32_t H, int32_t hd, int32_t pos,
                                     const void* cache, int64_t ld_cache, void* out, int64_t ld_out,
                                     float scale, void* stream) {
  return icap_attention_decode_anc(dtype, B, H, hd, pos, cache, ld_cache, nullptr, out, ld_out, scale, stream);
}

// Beam search over the KV-cached decoder: the definition is transformers' beam search
// (GPT2LMHeadModel.generate(num_beams=W, do_sample=False, early_stopping=False), HF/generation/utils.py:
// 3208-3540); the reference itself decodes greedy / top-p only (src/models.py:327-477).
//
// Rows: R = B*W decode rows, row r = b*W + i (beam i of caption b). Per step two launches:
//   beam_rowtop_kernel  one block per row: log-sum-exp of the row's V logits and its top K (K >= 2W) logits
//                       (descending, ties -> lower token id). The caption's top 2W candidates over W x V are
//                       among its rows' top 2W, so a row never needs more.
//   beam_update_kernel  one block per caption: candidate scores (logit - max) - log(sum) + running score, the
//                       top 2W, the next running beams, the finished-hypothesis merge, the early-stop heuristic,
//                       the running / finished token histories, the KV ancestry of the new rows and their next
//                       input embeddings. The serial bookkeeping (a few dozen candidates) runs on one lane; the
//                       copies on the whole block.
// KV ancestry: the cache keeps each row's K/V where the row computed it; anc[t*R + r] names the cache row holding
// position t of row r's history (icap_attention_decode_anc), so a beam reorder rewrites W*(pos+1) ints per caption
// instead of moving any cache bytes.
#include "common.h"

namespace icap {
namespace beam {
constexpr float NEG = -1.0e9f;  // transformers' "impossible" running / finished score
constexpr int NT = 256;
constexpr int KMAX = 16;        // K <= 16 (W <= 8)
constexpr int TMAX = 1024;      // cache positions (GPT-2 n_positions)

// workspace carve-up (all 4-byte words; offsets in words, each block 16-byte aligned)
struct Layout {
  int64_t run_score, run_seq, fin_score, fin_len, fin_seq, fin_cnt, done, anc, total;
};
__host__ __device__ inline int64_t up4(int64_t n) { return (n + 3) & ~3ll; }
__host__ __device__ inline Layout layout(int64_t B, int64_t W, int64_t T, int64_t L) {
  const int64_t R = B * W;
  Layout l;
  int64_t o = 0;
  l.run_score = o; o += up4(R);
  l.run_seq = o;   o += up4(R * L);
  l.fin_score = o; o += up4(R);
  l.fin_len = o;   o += up4(R);
  l.fin_seq = o;   o += up4(R * L);
  l.fin_cnt = o;   o += up4(B);
  l.done = o;      o += up4(B);
  l.anc = o;       o += up4(T * R);
  l.total = o;
  return l;
}

// candidate order: higher score first, then lower key (flat beam*V + token, or candidate rank)
__device__ __forceinline__ bool better(float a, int64_t ka, float b, int64_t kb) {
  return a > b || (a == b && ka < kb);
}
}  // namespace beam

template <typename T, int K>
__global__ __launch_bounds__(256) void beam_rowtop_kernel(int64_t V, const T* __restrict__ logits, int64_t ld,
                                                          float* __restrict__ top_val, int32_t* __restrict__ top_idx,
                                                          float* __restrict__ top_m, float* __restrict__ top_ls) {
  using namespace beam;
  __shared__ float sv[NT / 64];
  __shared__ int32_t si[NT / 64];
  __shared__ float sm[NT / 64], ss[NT / 64];
  const int64_t r = blockIdx.x;
  const T* row = logits + r * ld;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  float v[K];
  int32_t id[K];
#pragma unroll
  for (int k = 0; k < K; ++k) { v[k] = -INFINITY; id[k] = 0x7fffffff; }
  float m = -INFINITY, s = 0.f;
  // each thread walks its elements in increasing index order, so a strict '>' keeps the lower index on ties
  for (int64_t j = tid; j < V; j += NT) {
    const float x = io<T>::ld(row + j);
    if (x > m) { s = s * expf(m - x) + 1.f; m = x; } else { s += expf(x - m); }
    if (x > v[K - 1]) {  // insertion into the sorted register list (compile-time indices)
      float cv = x;
      int32_t ci = (int32_t)j;
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if (cv > v[k]) {
          const float tv = v[k]; const int32_t ti = id[k];
          v[k] = cv; id[k] = ci; cv = tv; ci = ti;
        }
      }
    }
  }
  // (max, sum) of the row
  float bm = m;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) bm = fmaxf(bm, __shfl_xor(bm, o, 64));
  float bs = m == -INFINITY ? 0.f : s * expf(m - bm);
  bs = wave_sum(bs);
  if (lane == 0) { sm[w] = bm; ss[w] = bs; }
  __syncthreads();
  float gm = sm[0];
#pragma unroll
  for (int q = 1; q < NT / 64; ++q) gm = fmaxf(gm, sm[q]);
  float gs = 0.f;
#pragma unroll
  for (int q = 0; q < NT / 64; ++q) gs += ss[q] * expf(sm[q] - gm);
  // top K of the block: K rounds of a block-wide max over every thread's list head
  int head = 0;
  for (int k = 0; k < K; ++k) {
    float hv = -INFINITY;
    int32_t hi = 0x7fffffff;
#pragma unroll
    for (int q = 0; q < K; ++q)
      if (q == head) { hv = v[q]; hi = id[q]; }
    float bv = hv;
    int32_t bi = hi;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ov = __shfl_xor(bv, o, 64);
      const int32_t oi = __shfl_xor(bi, o, 64);
      if (better(ov, oi, bv, bi)) { bv = ov; bi = oi; }
    }
    __syncthreads();  // the previous round's readers are done with sv / si
    if (lane == 0) { sv[w] = bv; si[w] = bi; }
    __syncthreads();
    float wv = sv[0];
    int32_t wi = si[0];
#pragma unroll
    for (int q = 1; q < NT / 64; ++q)
      if (better(sv[q], si[q], wv, wi)) { wv = sv[q]; wi = si[q]; }
    if (hi == wi && hv == wv) ++head;  // indices are unique: exactly one thread owns the winner
    if (tid == 0) {
      top_val[r * K + k] = wv;
      top_idx[r * K + k] = wi;
    }
  }
  if (tid == 0) {
    top_m[r] = gm;
    top_ls[r] = logf(gs);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void beam_update_kernel(icap_beam_args a, int step, int pos) {
  using namespace beam;
  const int b = blockIdx.x, tid = threadIdx.x;
  const int W = a.W, K = a.K, L = a.max_len;
  const int64_t R = (int64_t)a.B * W;
  const Layout lo = layout(a.B, W, a.T, L);
  float* wsf = reinterpret_cast<float*>(a.ws);
  int32_t* wsi = reinterpret_cast<int32_t*>(a.ws);
  float* run_score = wsf + lo.run_score + (int64_t)b * W;
  int32_t* run_seq = wsi + lo.run_seq + (int64_t)b * W * L;
  float* fin_score = wsf + lo.fin_score + (int64_t)b * W;
  int32_t* fin_len = wsi + lo.fin_len + (int64_t)b * W;
  int32_t* fin_seq = wsi + lo.fin_seq + (int64_t)b * W * L;
  int32_t* fin_cnt = wsi + lo.fin_cnt + b;
  int32_t* done = wsi + lo.done + b;
  int32_t* anc = wsi + lo.anc;

  __shared__ int32_t s_run[8 * TMAX / 8];  // old running histories, W x L (W * L <= 1024)
  __shared__ int32_t s_fin[8 * TMAX / 8];  // old finished histories
  __shared__ int32_t s_anc[8 * TMAX];      // this caption's ancestry columns, (pos + 1) x W
  __shared__ int32_t run_src[8], run_tok[8];
  __shared__ int32_t fin_src[8], fin_tok[8], fin_from_cand[8], fin_lenv[8];
  __shared__ float fin_sc[8];
  __shared__ int32_t n_fin;

  for (int e = tid; e < W * L; e += NT) {
    s_run[e] = run_seq[e];
    s_fin[e] = fin_seq[e];
  }
  for (int e = tid; e < (pos + 1) * W; e += NT) {
    const int t = e / W, i = e - t * W;
    s_anc[e] = anc[(int64_t)t * R + (int64_t)b * W + i];
  }
  if (tid == 0) {
    // 1. the caption's top 2W candidates over its W rows' top K
    float cs[2 * KMAX];
    int64_t ck[2 * KMAX];
    int32_t cbeam[2 * KMAX], ctok[2 * KMAX];
    const int C = 2 * W;
    for (int c = 0; c < C; ++c) { cs[c] = -INFINITY; ck[c] = INT64_MAX; cbeam[c] = 0; ctok[c] = 0; }
    for (int i = 0; i < W; ++i) {
      const int64_t rr = (int64_t)b * W + i;
      const float m = a.top_m[rr], ls = a.top_ls[rr], rs = run_score[i];
      for (int k = 0; k < K; ++k) {
        const float x = a.top_val[rr * K + k];
        const int32_t tok = a.top_idx[rr * K + k];
        if (x == -INFINITY) break;
        const float sc = ((x - m) - ls) + rs;  // log_softmax + running score (HF/generation/utils.py:3396-3401)
        const int64_t key = (int64_t)i * a.V + tok;
        if (!better(sc, key, cs[C - 1], ck[C - 1])) continue;
        int p = C - 1;  // insertion
        while (p > 0 && better(sc, key, cs[p - 1], ck[p - 1])) {
          cs[p] = cs[p - 1]; ck[p] = ck[p - 1]; cbeam[p] = cbeam[p - 1]; ctok[p] = ctok[p - 1];
          --p;
        }
        cs[p] = sc; ck[p] = key; cbeam[p] = i; ctok[p] = tok;
      }
    }
    // 2. stopping criteria per candidate: EOS, or the last token of the budget
    bool hit[2 * KMAX];
    for (int c = 0; c < C; ++c) hit[c] = ctok[c] == a.eos || step + 1 >= L;
    // 3. next running beams: best W after -1e9 on hitting candidates (:3131-3151)
    float rsc[2 * KMAX];
    bool taken[2 * KMAX];
    for (int c = 0; c < C; ++c) { rsc[c] = cs[c] + (hit[c] ? NEG : 0.f); taken[c] = false; }
    float new_rs[8];
    for (int i = 0; i < W; ++i) {
      int bc = -1;
      for (int c = 0; c < C; ++c)
        if (!taken[c] && (bc < 0 || better(rsc[c], c, rsc[bc], bc))) bc = c;
      taken[bc] = true;
      run_src[i] = cbeam[bc];
      run_tok[i] = ctok[bc];
      new_rs[i] = rsc[bc];
    }
    // 4. finished hypotheses: hitting candidates among the first W, length-normalised, merged (:3153-3206)
    int nf = *fin_cnt;
    float fs[16];
    int32_t fsrc[16], ftok[16], ffc[16], flen[16];
    for (int k = 0; k < nf; ++k) { fs[k] = fin_score[k]; fsrc[k] = k; ftok[k] = 0; ffc[k] = 0; flen[k] = fin_len[k]; }
    if (!*done) {
      const float norm = powf((float)(step + 1), a.length_penalty);
      for (int c = 0; c < W; ++c) {
        if (!hit[c]) continue;
        const float sc = cs[c] / norm;
        // insert after existing entries of equal score (the kept ones win ties)
        int p = nf;
        while (p > 0 && sc > fs[p - 1]) {
          fs[p] = fs[p - 1]; fsrc[p] = fsrc[p - 1]; ftok[p] = ftok[p - 1]; ffc[p] = ffc[p - 1]; flen[p] = flen[p - 1];
          --p;
        }
        fs[p] = sc; fsrc[p] = cbeam[c]; ftok[p] = ctok[c]; ffc[p] = 1; flen[p] = step + 1;
        ++nf;  // <= 2W <= 16 before the cut to W below
      }
      if (nf > W) nf = W;
    }
    for (int k = 0; k < nf; ++k) {
      fin_sc[k] = fs[k]; fin_src[k] = fsrc[k]; fin_tok[k] = ftok[k]; fin_from_cand[k] = ffc[k]; fin_lenv[k] = flen[k];
    }
    n_fin = nf;
    // 5. early-stop heuristic after this step (:3008-3053, early_stopping=False): sticky
    if (!*done && nf == W) {
      const float best_possible = new_rs[0] / powf((float)(step + 1), a.length_penalty);
      if (!(best_possible > fs[nf - 1])) *done = 1;
    }
    for (int i = 0; i < W; ++i) run_score[i] = new_rs[i];
    *fin_cnt = nf;
  }
  __syncthreads();
  // 6. histories: running beam i <- beam run_src[i] + run_tok[i]; finished slots from kept slots or candidates
  for (int e = tid; e < W * L; e += NT) {
    const int i = e / L, t = e - i * L;
    run_seq[e] = t < step ? s_run[run_src[i] * L + t] : (t == step ? run_tok[i] : a.eos);
  }
  const int nf = n_fin;
  for (int e = tid; e < nf * L; e += NT) {
    const int k = e / L, t = e - k * L;
    int32_t v;
    if (fin_from_cand[k]) v = t < step ? s_run[fin_src[k] * L + t] : (t == step ? fin_tok[k] : a.eos);
    else v = s_fin[fin_src[k] * L + t];
    fin_seq[e] = v;
  }
  if (tid < nf) {
    fin_score[tid] = fin_sc[tid];
    fin_len[tid] = fin_lenv[tid];
  }
  // 7. KV ancestry of the new rows: positions 0..pos from the parent row, position pos+1 their own row
  for (int e = tid; e < (pos + 1) * W; e += NT) {
    const int t = e / W, i = e - t * W;
    anc[(int64_t)t * R + (int64_t)b * W + i] = s_anc[t * W + run_src[i]];
  }
  if (pos + 1 < a.T && tid < W) anc[(int64_t)(pos + 1) * R + (int64_t)b * W + tid] = b * W + tid;
  // 8. next input embeddings: x[r] = wte[token] + wpe[min(pos + 1, n_positions - 1)]
  if (a.x) {
    const T* wte = reinterpret_cast<const T*>(a.wte);
    const T* wpe = reinterpret_cast<const T*>(a.wpe);
    T* x = reinterpret_cast<T*>(a.x);
    const int pn = pos + 1 < a.n_positions ? pos + 1 : a.n_positions - 1;
    for (int e = tid; e < W * a.D; e += NT) {
      const int i = e / a.D, d = e - i * a.D;
      io<T>::st(x + ((int64_t)b * W + i) * a.D + d,
                io<T>::ld(wte + (int64_t)run_tok[i] * a.D + d) + io<T>::ld(wpe + (int64_t)pn * a.D + d));
    }
  }
}

__global__ void beam_init_kernel(icap_beam_args a, int P) {
  using namespace beam;
  const Layout lo = layout(a.B, a.W, a.T, a.max_len);
  const int64_t R = (int64_t)a.B * a.W;
  float* wsf = reinterpret_cast<float*>(a.ws);
  int32_t* wsi = reinterpret_cast<int32_t*>(a.ws);
  const int64_t n = (int64_t)P * R;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e % R;
    wsi[lo.anc + e] = (int32_t)r;  // prefill: every row holds its own copy of the prefix
    if (e < R) {
      wsf[lo.run_score + r] = (r % a.W) == 0 ? 0.f : NEG;  // only beam 0 seeds candidates (:3318-3320)
      wsf[lo.fin_score + r] = NEG;
      wsi[lo.fin_len + r] = 0;
    }
    if (e < a.B) {
      wsi[lo.fin_cnt + e] = 0;
      wsi[lo.done + e] = 0;
    }
  }
}

__global__ void beam_finalize_kernel(icap_beam_args a, int64_t* __restrict__ out, int32_t* __restrict__ out_len) {
  using namespace beam;
  const Layout lo = layout(a.B, a.W, a.T, a.max_len);
  const int b = blockIdx.x;
  const int32_t* wsi = reinterpret_cast<const int32_t*>(a.ws);
  const int L = a.max_len;
  const int nf = wsi[lo.fin_cnt + b];
  // the best finished hypothesis (slot 0); a caption without one (a loop stopped before its budget) returns its
  // best running beam
  const int32_t* seq = nf > 0 ? wsi + lo.fin_seq + (int64_t)b * a.W * L : wsi + lo.run_seq + (int64_t)b * a.W * L;
  const int len = nf > 0 ? wsi[lo.fin_len + (int64_t)b * a.W] : a.max_len;
  for (int t = threadIdx.x; t < L; t += blockDim.x) out[(int64_t)b * L + t] = t < len ? seq[t] : a.eos;
  if (threadIdx.x == 0) out_len[b] = len;
}

}  // namespace icap

using namespace icap;

extern "C" size_t icap_beam_workspace_bytes(int32_t B, int32_t W, int32_t T, int32_t max_len) {
  if (B < 0 || W <= 0 || T <= 0 || max_len <= 0) return 0;
  return (size_t)beam::layout(B, W, T, max_len).total * 4;
}

extern "C" int icap_beam_layout(int32_t B, int32_t W, int32_t T, int32_t max_len, int64_t* word_offsets) {
  ICAP_REQUIRE(word_offsets != nullptr, "icap_beam_layout: null output");
  ICAP_REQUIRE(B >= 0 && W > 0 && T > 0 && max_len > 0, "icap_beam_layout: bad sizes");
  const beam::Layout l = beam::layout(B, W, T, max_len);
  const int64_t o[9] = {l.run_score, l.run_seq, l.fin_score, l.fin_len, l.fin_seq, l.fin_cnt, l.done, l.anc, l.total};
  for (int i = 0; i < 9; ++i) word_offsets[i] = o[i];
  return ICAP_OK;
}

static int beam_check(const icap_beam_args* a) {
  ICAP_REQUIRE(a != nullptr, "icap_beam: null args");
  ICAP_REQUIRE(a->W >= 1 && a->W <= 8, "icap_beam: num_beams must be in [1, 8]");
  ICAP_REQUIRE(a->K == 8 || a->K == 16, "icap_beam: K must be 8 (W <= 4) or 16 (W <= 8)");
  ICAP_REQUIRE(a->K >= 2 * a->W, "icap_beam: K must be >= 2 * num_beams");
  ICAP_REQUIRE(a->max_len >= 1 && a->W * a->max_len <= 1024, "icap_beam: num_beams * max_len must be <= 1024");
  ICAP_REQUIRE(a->T >= 1 && a->T <= 1024, "icap_beam: T (cache positions) must be in [1, 1024]");
  ICAP_REQUIRE(a->V >= 1, "icap_beam: V must be positive");
  ICAP_REQUIRE(a->ws != nullptr && (reinterpret_cast<uintptr_t>(a->ws) & 15) == 0, "icap_beam: workspace missing or misaligned");
  return ICAP_OK;
}

extern "C" int icap_beam_init(const icap_beam_args* a, int32_t P, void* stream) {
  const int rc = beam_check(a);
  if (rc != ICAP_OK) return rc;
  ICAP_REQUIRE(P >= 1 && P <= a->T, "icap_beam_init: prefix length out of range");
  if (a->B == 0) return ICAP_OK;
  const int64_t n = (int64_t)P * a->B * a->W;
  const unsigned g = (unsigned)((n + 255) / 256 < 1024 ? (n + 255) / 256 : 1024);
  hipLaunchKernelGGL(beam_init_kernel, dim3(g), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), *a, P);
  return check_launch("icap_beam_init");
}

extern "C" int icap_beam_rowtop(int32_t dtype, int64_t R, int64_t V, const void* logits, int64_t ld, int32_t K,
                                float* top_val, int32_t* top_idx, float* top_m, float* top_ls, void* stream) {
  ICAP_REQUIRE(logits && top_val && top_idx && top_m && top_ls, "icap_beam_rowtop: null pointer");
  ICAP_REQUIRE(K == 8 || K == 16, "icap_beam_rowtop: K must be 8 or 16");
  ICAP_REQUIRE(V >= 1 && V < (1ll << 31) && ld >= V, "icap_beam_rowtop: bad V / ld");
  if (R == 0) return ICAP_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const dim3 grid((unsigned)R), block(256);
  if (dtype == ICAP_BF16) {
    if (K == 8) hipLaunchKernelGGL((beam_rowtop_kernel<bf16_t, 8>), grid, block, 0, s, V, (const bf16_t*)logits, ld, top_val, top_idx, top_m, top_ls);
    else hipLaunchKernelGGL((beam_rowtop_kernel<bf16_t, 16>), grid, block, 0, s, V, (const bf16_t*)logits, ld, top_val, top_idx, top_m, top_ls);
  } else {
    if (K == 8) hipLaunchKernelGGL((beam_rowtop_kernel<float, 8>), grid, block, 0, s, V, (const float*)logits, ld, top_val, top_idx, top_m, top_ls);
    else hipLaunchKernelGGL((beam_rowtop_kernel<float, 16>), grid, block, 0, s, V, (const float*)logits, ld, top_val, top_idx, top_m, top_ls);
  }
  return check_launch("icap_beam_rowtop");
}

extern "C" int icap_beam_update(const icap_beam_args* a, int32_t step, int32_t pos, void* stream) {
  const int rc = beam_check(a);
  if (rc != ICAP_OK) return rc;
  ICAP_REQUIRE(a->top_val && a->top_idx && a->top_m && a->top_ls, "icap_beam_update: row tops missing");
  ICAP_REQUIRE(step >= 0 && step < a->max_len, "icap_beam_update: step out of range");
  ICAP_REQUIRE(pos >= 0 && pos < a->T, "icap_beam_update: pos out of range");
  ICAP_REQUIRE(a->x == nullptr || (a->wte && a->wpe && a->D > 0 && a->n_positions > 0),
               "icap_beam_update: x requires wte / wpe / D / n_positions");
  if (a->B == 0) return ICAP_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (a->dtype == ICAP_BF16)
    hipLaunchKernelGGL(beam_update_kernel<bf16_t>, dim3((unsigned)a->B), dim3(256), 0, s, *a, step, pos);
  else
    hipLaunchKernelGGL(beam_update_kernel<float>, dim3((unsigned)a->B), dim3(256), 0, s, *a, step, pos);
  return check_launch("icap_beam_update");
}

extern "C" int icap_beam_finalize(const icap_beam_args* a, int64_t* out, int32_t* out_len, void* stream) {
  const int rc = beam_check(a);
  if (rc != ICAP_OK) return rc;
  ICAP_REQUIRE(out && out_len, "icap_beam_finalize: null output");
  if (a->B == 0) return ICAP_OK;
  hipLaunchKernelGGL(beam_finalize_kernel, dim3((unsigned)a->B), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), *a,
                     out, out_len);
  return check_launch("icap_beam_finalize");
}

// HBM-bound kernels of the captioning path: input assembly, cross entropy,
// clip + AdamW, layout/reduction helpers, CLIP tower glue, greedy-decode glue.
#include "common.h"

#include <math.h>

namespace icap {

static inline hipStream_t S_(void* s) { return reinterpret_cast<hipStream_t>(s); }
static inline unsigned nblk(int64_t n, int per, int cap = 65535) {
  int64_t b = (n + per - 1) / per;
  if (b < 1) b = 1;
  if (b > cap) b = cap;
  return (unsigned)b;
}

// block-wide sum (256 threads)
__device__ __forceinline__ float block_sum256(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = red[0] + red[1] + red[2] + red[3];
  return r;
}

// ---------------------------------------------------------------- GPT-2 input
template <typename T>
__global__ void gpt2_embed_kernel(int B, int P, int L, int D, const T* __restrict__ prefix, int64_t pbs,
                                  const T* __restrict__ wte, const T* __restrict__ wpe,
                                  const int64_t* __restrict__ ids, T* __restrict__ x, uint32_t thr,
                                  float inv_keep, uint64_t seed0, const uint64_t* seed_ptr, uint64_t offset,
                                  const int32_t* __restrict__ seq_off, const int32_t* __restrict__ seq_len) {
  const int S = P + L, D4 = D >> 2;
  const uint64_t seed = thr ? eff_seed(seed0, seed_ptr) : 0ull;
  const int64_t total = (int64_t)B * S * D4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t prow = i / D4;  // padded (b, t) index
    const int c = (int)(i - prow * D4) * 4;
    const int b = (int)(prow / S), t = (int)(prow - (int64_t)b * S);
    int64_t row = prow;  // destination row
    if (seq_off) {       // packed: only the live prefix of the sequence, at its packed rows
      if (t >= seq_len[b]) continue;
      row = (int64_t)seq_off[b] + t;
    }
    float v[4], w[4];
    if (t < P) io<T>::ld4(prefix + (int64_t)b * pbs + (int64_t)t * D + c, v);
    else io<T>::ld4(wte + ids[(int64_t)b * L + (t - P)] * D + c, v);
    io<T>::ld4(wpe + (int64_t)t * D + c, w);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] += w[e];
      if (thr) v[e] *= drop_scale(seed, offset + (uint64_t)(row * D + c + e), thr, inv_keep);
    }
    io<T>::st4(x + row * D + c, v);
  }
}

// d(wte)[ids[b,t-P]] += dx[b*S+t] for caption rows (fp32 atomics; unfrozen GPT-2 only)
template <typename T>
__global__ void embed_scatter_kernel(int B, int P, int L, int D, const T* __restrict__ dx,
                                     const int64_t* __restrict__ ids, float* __restrict__ dwte) {
  const int S = P + L;
  const int64_t total = (int64_t)B * L * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / D;
    const int d = (int)(i - r * D);
    const int b = (int)(r / L), t = (int)(r - (int64_t)b * L);
    atomicAdd(dwte + ids[(int64_t)b * L + t] * D + d, io<T>::ld(dx + ((int64_t)b * S + P + t) * D + d));
  }
}

// One 1024-thread block; thread k owns the contiguous rows [k*per, (k+1)*per) so the target compaction is an
// exclusive scan of per-thread counts (wave shuffles + one LDS pass) and keeps row order.
__global__ __launch_bounds__(1024) void caption_prep_kernel(int B, int P, int L, const int64_t* __restrict__ mask,
                                                           const int64_t* __restrict__ labels, int32_t* key_mask,
                                                           int32_t* lab_shift, int32_t* n_valid, int32_t* row_slot,
                                                           int32_t* lab_c) {
  __shared__ int wsum[16];
  const int S = P + L, n = B * S;
  const int per = (n + 1023) / 1024;
  const int i0 = threadIdx.x * per;
  const int i1 = i0 + per < n ? i0 + per : n;
  auto label_at = [&](int i) {
    const int b = i / S, tn = i - b * S + 1;
    return (tn < S && tn >= P && labels) ? (int)labels[(int64_t)b * L + tn - P] : -100;
  };
  int cnt = 0;
  for (int i = i0; i < i1; ++i) {
    const int b = i / S, t = i - b * S;
    if (key_mask) key_mask[i] = (t < P || mask == nullptr) ? 1 : (mask[(int64_t)b * L + t - P] != 0 ? 1 : 0);
    const int lab = label_at(i);
    if (lab_shift) lab_shift[i] = lab;
    cnt += lab != -100 ? 1 : 0;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int woff = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    woff += k < w ? wsum[k] : 0;
    tot += wsum[k];
  }
  if (row_slot) {
    int slot = woff + incl - cnt;
    for (int i = i0; i < i1; ++i) {
      const int lab = label_at(i);
      if (lab != -100) {
        row_slot[i] = slot;
        if (lab_c) lab_c[slot] = lab;
        ++slot;
      } else {
        row_slot[i] = -1;
      }
    }
  }
  if (threadIdx.x == 0 && n_valid) *n_valid = tot;
}

// Packed token rows (icap_caption_pack): one 1024-thread block. Phase 1: per-sequence live length (the last
// position whose shifted label is a target, at least the P prefix rows) and an exclusive scan of the lengths
// (threads own contiguous sequences). Phase 2: the per-row arrays over the packed rows (threads own contiguous
// rows) and the target compaction, an exclusive scan over the same contiguous ownership as caption_prep_kernel,
// so the compacted rows keep row order — the order caption_prep_kernel gives them in the padded layout.
__device__ __forceinline__ int block_excl_scan1024(int cnt, int* wsum, int& total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int incl = cnt;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  __syncthreads();  // wsum reuse
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int woff = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    woff += k < w ? wsum[k] : 0;
    tot += wsum[k];
  }
  total = tot;
  return woff + incl - cnt;
}

__global__ __launch_bounds__(1024) void caption_pack_kernel(int B, int P, int L, const int64_t* __restrict__ mask,
                                                           const int64_t* __restrict__ labels, int32_t* seq_off,
                                                           int32_t* seq_len, int32_t* m_live, int32_t* key_mask,
                                                           int32_t* lab_shift, int32_t* n_valid, int32_t* row_slot,
                                                           int32_t* lab_c) {
  __shared__ int wsum[16];
  constexpr int PK_LDS = 2048;                   // sequences whose offsets / lengths phase 2 reads from LDS
  __shared__ int s_off[PK_LDS], s_len[PK_LDS];
  const int S = P + L, n = B * S;
  auto label_at = [&](int b, int t) {  // shifted label of position t of sequence b
    const int tn = t + 1;
    return (tn < S && tn >= P && labels) ? (int)labels[(int64_t)b * L + tn - P] : -100;
  };
  // phase 1: lengths + offsets. The last target of a sequence is found by one pass over all its positions whose
  // loads do not depend on each other (a backwards scan with an early exit made each label load wait for the one
  // before it: ~50 dependent round trips per caption, the kernel took ~34 us)
  const int bper = (B + 1023) / 1024;
  const int b0 = threadIdx.x * bper < B ? threadIdx.x * bper : B;
  const int b1 = b0 + bper < B ? b0 + bper : B;
  int cnt = 0;
  for (int b = b0; b < b1; ++b) {
    int len = P;
#pragma unroll 8
    for (int t = P; t < S; ++t)
      if (label_at(b, t) != -100) len = t + 1;
    seq_len[b] = len;
    if (b < PK_LDS) s_len[b] = len;
    cnt += len;
  }
  int mtot = 0;
  int off = block_excl_scan1024(cnt, wsum, mtot);
  for (int b = b0; b < b1; ++b) {
    seq_off[b] = off;
    if (b < PK_LDS) s_off[b] = off;
    off += b < PK_LDS ? s_len[b] : seq_len[b];
  }
  if (threadIdx.x == 0) *m_live = mtot;
  __syncthreads();  // seq_off / seq_len (and their LDS copies) visible to the whole block
  const bool lds = B <= PK_LDS;
  auto OFF = [&](int b) { return lds ? s_off[b] : seq_off[b]; };
  auto LEN = [&](int b) { return lds ? s_len[b] : seq_len[b]; };
  // phase 2: per packed row
  const int per = (n + 1023) / 1024;
  const int i0 = threadIdx.x * per < n ? threadIdx.x * per : n;
  const int i1 = i0 + per < n ? i0 + per : n;
  // sequence of the first row this thread owns (binary search over the offsets)
  int bb = 0;
  if (i0 < mtot) {
    int lo = 0, hi = B - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (OFF(mid) <= i0) lo = mid; else hi = mid - 1;
    }
    bb = lo;
  }
  int tcnt = 0;
  {
    int b = bb;
    for (int i = i0; i < i1; ++i) {
      int lab = -100, km = 0;
      if (i < mtot) {
        while (i >= OFF(b) + LEN(b)) ++b;  // skips empty sequences too
        const int t = i - OFF(b);
        km = (t < P || mask == nullptr) ? 1 : (mask[(int64_t)b * L + t - P] != 0 ? 1 : 0);
        lab = label_at(b, t);
      }
      key_mask[i] = km;
      lab_shift[i] = lab;
      tcnt += lab != -100 ? 1 : 0;
    }
  }
  int tot = 0;
  const int slot0 = block_excl_scan1024(tcnt, wsum, tot);
  if (row_slot) {
    int slot = slot0;
    for (int i = i0; i < i1; ++i) {
      const int lab = lab_shift[i];
      if (lab != -100) {
        row_slot[i] = slot;
        if (lab_c) lab_c[slot] = lab;
        ++slot;
      } else {
        row_slot[i] = -1;
      }
    }
  }
  if (threadIdx.x == 0 && n_valid) *n_valid = tot;
}

// The same outputs from several blocks, for B <= PK2_MAX (round 5: the one-block form above took ~32 us per step, a
// chain of dependent label loads and block scans on one CU). Every block runs phase 1 over ALL captions — one wave
// per caption, lanes over its 50 label positions, one ballot: live length, target count, target bit mask — and the
// two exclusive scans (offsets, target slots) in its own LDS, so no block waits for another; then each wave writes
// the rows of one caption of the block's share (lanes over positions; the slot of a target row is the caption's
// slot offset + the targets before it in the ballot), and the blocks stride over the dead rows [m_live, B S).
// Identical outputs to caption_pack_kernel (tests/test_pack_gpu.py compares both forms element by element).
constexpr int PK2_MAX = 2048;
constexpr int PK2_WAVES = 16;
__global__ __launch_bounds__(1024) void caption_pack2_kernel(int B, int P, int L, const int64_t* __restrict__ mask,
                                                            const int64_t* __restrict__ labels, int32_t* seq_off,
                                                            int32_t* seq_len, int32_t* m_live, int32_t* key_mask,
                                                            int32_t* lab_shift, int32_t* n_valid, int32_t* row_slot,
                                                            int32_t* lab_c) {
  __shared__ int wsum[16];
  __shared__ int s_len[PK2_MAX], s_off[PK2_MAX], s_tgt[PK2_MAX];
  const int S = P + L, n = B * S;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // position t's shifted label: labels[b, t + 1 - P] for P <= t + 1 < S (t = P - 1 + j, label j of the caption)
  auto label_at = [&](int b, int t) {
    const int tn = t + 1;
    return (tn < S && tn >= P && labels) ? (int)labels[(int64_t)b * L + tn - P] : -100;
  };
  // phase 1 (every block, all captions): live length P + (last target j >= 1), target count over j (t = P - 1 + j >= 0)
  for (int b = w; b < B; b += PK2_WAVES) {
    int jlast = 0, tg = 0;
    for (int j0 = 0; j0 < L; j0 += 64) {
      const int j = j0 + lane;
      const bool ok = j < L && P - 1 + j >= 0 && labels != nullptr && labels[(int64_t)b * L + j] != -100;
      const uint64_t bal = __ballot(ok);
      tg += __popcll(bal);
      if (bal) jlast = j0 + 63 - __clzll(bal);
    }
    if (lane == 0) {
      s_len[b] = P + (jlast >= 1 ? jlast : 0);
      s_tgt[b] = tg;
    }
  }
  __syncthreads();
  // the two exclusive scans over the captions: thread k owns captions [k c, k c + c)
  const int per = (B + 1023) / 1024;
  const int b0 = threadIdx.x * per < B ? threadIdx.x * per : B;
  const int b1 = b0 + per < B ? b0 + per : B;
  int cl = 0, ct = 0;
  for (int b = b0; b < b1; ++b) {
    cl += s_len[b];
    ct += s_tgt[b];
  }
  int mtot = 0, ttot = 0;
  int off = block_excl_scan1024(cl, wsum, mtot);
  int slot = block_excl_scan1024(ct, wsum, ttot);
  __syncthreads();  // every thread has read s_len / s_tgt for its sums
  for (int b = b0; b < b1; ++b) {
    const int l = s_len[b], tg = s_tgt[b];
    s_off[b] = off;
    s_tgt[b] = slot;  // now the caption's first target slot
    if (blockIdx.x == 0) {
      seq_off[b] = off;
      seq_len[b] = l;
    }
    off += l;
    slot += tg;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *m_live = mtot;
    if (n_valid) *n_valid = ttot;
  }
  __syncthreads();
  // phase 2: one wave per caption of this block's share
  for (int b = blockIdx.x * PK2_WAVES + w; b < B; b += gridDim.x * PK2_WAVES) {
    const int o = s_off[b], len = s_len[b];
    int sl = s_tgt[b];
    for (int t0 = 0; t0 < len; t0 += 64) {
      const int t = t0 + lane;
      int lab = -100, km = 0;
      if (t < len) {
        km = (t < P || mask == nullptr) ? 1 : (mask[(int64_t)b * L + t - P] != 0 ? 1 : 0);
        lab = label_at(b, t);
        key_mask[o + t] = km;
        lab_shift[o + t] = lab;
      }
      const bool tgt = lab != -100;
      const uint64_t bal = __ballot(tgt);
      if (row_slot && t < len) {
        const int mine = sl + __popcll(bal & ((1ull << lane) - 1ull));
        row_slot[o + t] = tgt ? mine : -1;
        if (tgt && lab_c) lab_c[mine] = lab;
      }
      sl += __popcll(bal);
    }
  }
  // the dead rows past the packed ones
  for (int i = mtot + blockIdx.x * 1024 + (int)threadIdx.x; i < n; i += gridDim.x * 1024) {
    key_mask[i] = 0;
    lab_shift[i] = -100;
    if (row_slot) row_slot[i] = -1;
  }
}

template <typename T>
__global__ void rows_unpack_kernel(int B, int P, int D, const T* __restrict__ src, const int32_t* __restrict__ seq_off,
                                   const int32_t* __restrict__ seq_len, T* __restrict__ dst, int64_t dbs) {
  const int D4 = D >> 2;
  const int64_t total = (int64_t)B * P * D4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / D4;
    const int c = (int)(i - r * D4) * 4;
    const int b = (int)(r / P), t = (int)(r - (int64_t)b * P);
    float v[4] = {0.f, 0.f, 0.f, 0.f};
    if (t < seq_len[b]) io<T>::ld4(src + ((int64_t)seq_off[b] + t) * D + c, v);
    io<T>::st4(dst + (int64_t)b * dbs + (int64_t)t * D + c, v);
  }
}

// ---------------------------------------------------------------- cross entropy
template <typename T>
__global__ __launch_bounds__(256) void ce_kernel(int64_t V, const T* __restrict__ logits, int64_t ld,
                                                const int32_t* __restrict__ labels,
                                                const int32_t* __restrict__ n_valid, float* __restrict__ loss_rows,
                                                T* dlogits, float grad_scale, const int32_t* __restrict__ rows_dev) {
  __shared__ float redm[4], reds[4];
  const int64_t r = blockIdx.x;
  if (rows_dev && r >= *rows_dev) return;  // compacted targets: this row does not exist
  const int y = labels[r];
  const T* x = logits + r * ld;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if (y < 0) {
    if (tid == 0) loss_rows[r] = 0.f;
    if (dlogits) {
      T* dx = dlogits + r * ld;
      for (int64_t j = tid; j < ld; j += 256) io<T>::st(dx + j, 0.f);
    }
    return;
  }
  // pass 1: online max / sum-exp per thread over float4 groups
  float m = -INFINITY, s = 0.f;
  const int64_t V4 = V >> 2;
  for (int64_t g = tid; g < V4; g += 256) {
    float v[4];
    io<T>::ld4(x + 4 * g, v);
    const float mx = fmaxf(fmaxf(v[0], v[1]), fmaxf(v[2], v[3]));
    if (mx > m) { s *= __expf(m - mx); m = mx; }
    s += __expf(v[0] - m) + __expf(v[1] - m) + __expf(v[2] - m) + __expf(v[3] - m);
  }
  for (int64_t j = 4 * V4 + tid; j < V; j += 256) {
    const float v = io<T>::ld(x + j);
    if (v > m) { s *= __expf(m - v); m = v; }
    s += __expf(v - m);
  }
  // combine (m, s) across the block
  float bm = wave_max(m);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - bm);
  s = wave_sum(s);
  if (lane == 0) { redm[w] = bm; reds[w] = s; }
  __syncthreads();
  float M = fmaxf(fmaxf(redm[0], redm[1]), fmaxf(redm[2], redm[3]));
  float Ssum = 0.f;
#pragma unroll
  for (int k = 0; k < 4; ++k) Ssum += reds[k] * __expf(redm[k] - M);
  const float lse = M + logf(Ssum);
  if (tid == 0) loss_rows[r] = lse - io<T>::ld(x + y);
  if (dlogits) {
    const float nv = (float)(*n_valid);
    const float sc = grad_scale / nv;
    T* dx = dlogits + r * ld;
    for (int64_t g = tid; g < V4; g += 256) {
      float v[4];
      io<T>::ld4(x + 4 * g, v);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int64_t j = 4 * g + e;
        v[e] = (__expf(v[e] - lse) - (j == y ? 1.f : 0.f)) * sc;
      }
      io<T>::st4(dx + 4 * g, v);
    }
    for (int64_t j = 4 * V4 + tid; j < ld; j += 256) {
      float v = 0.f;
      if (j < V) v = (__expf(io<T>::ld(x + j) - lse) - (j == y ? 1.f : 0.f)) * sc;
      io<T>::st(dx + j, v);
    }
  }
}

// bf16 logits, V <= 8 * 512 * R: the row is read from HBM ONCE into registers (R 16-byte groups per thread, all in
// flight together), then the block's online max / sum-exp and the dlogits pass both run from the registers
// (the two-pass kernel above reads the row twice: r01 PMC 541 MB per launch against 360 MB algorithmic).
template <int R>
__global__ __launch_bounds__(512) void ce_bf16_reg_kernel(int64_t V, const bf16_t* __restrict__ logits, int64_t ld,
                                                         const int32_t* __restrict__ labels,
                                                         const int32_t* __restrict__ n_valid,
                                                         float* __restrict__ loss_rows, bf16_t* dlogits,
                                                         float grad_scale, const int32_t* __restrict__ rows_dev) {
  constexpr int NT = 512, NW = NT / 64;
  __shared__ float redm[NW], reds[NW];
  const int64_t r = blockIdx.x;
  if (rows_dev && r >= *rows_dev) return;
  const int y = labels[r];
  const bf16_t* x = logits + r * ld;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int64_t V8 = V >> 3;
  if (y < 0) {
    if (tid == 0) loss_rows[r] = 0.f;
    if (dlogits) {
      bf16_t* dx = dlogits + r * ld;
      for (int64_t g = tid; g < (ld >> 3); g += NT) *reinterpret_cast<uint4*>(dx + 8 * g) = make_uint4(0u, 0u, 0u, 0u);
    }
    return;
  }
  uint4 wv[R];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    const int64_t g = tid + (int64_t)i * NT;
    wv[i] = g < V8 ? *reinterpret_cast<const uint4*>(x + 8 * g) : make_uint4(0xff80ff80u, 0xff80ff80u, 0xff80ff80u,
                                                                                  0xff80ff80u);  // -inf padding
  }
  float m = -INFINITY, s = 0.f;
#pragma unroll
  for (int i = 0; i < R; ++i) {
    float v[8];
    const uint32_t h[4] = {wv[i].x, wv[i].y, wv[i].z, wv[i].w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[2 * e] = __uint_as_float(h[e] << 16);
      v[2 * e + 1] = __uint_as_float(h[e] & 0xffff0000u);
    }
    float mx = v[0];
#pragma unroll
    for (int e = 1; e < 8; ++e) mx = fmaxf(mx, v[e]);
    if (mx > m) { s *= __expf(m - mx); m = mx; }
    if (m != -INFINITY) {
#pragma unroll
      for (int e = 0; e < 8; ++e) s += __expf(v[e] - m);
    }
  }
  for (int64_t j = 8 * V8 + tid; j < V; j += NT) {  // the last V % 8 logits
    const float v = bf2f(x[j]);
    if (v > m) { s *= __expf(m - v); m = v; }
    s += __expf(v - m);
  }
  const float bm = wave_max(m);
  s = (m == -INFINITY) ? 0.f : s * __expf(m - bm);
  s = wave_sum(s);
  if (lane == 0) { redm[w] = bm; reds[w] = s; }
  __syncthreads();
  float M = redm[0];
#pragma unroll
  for (int k = 1; k < NW; ++k) M = fmaxf(M, redm[k]);
  float Ssum = 0.f;
#pragma unroll
  for (int k = 0; k < NW; ++k) Ssum += reds[k] * __expf(redm[k] - M);
  const float lse = M + logf(Ssum);
  if (tid == 0) loss_rows[r] = lse - bf2f(x[y]);
  if (dlogits) {
    const float sc = grad_scale / (float)(*n_valid);
    bf16_t* dx = dlogits + r * ld;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t g = tid + (int64_t)i * NT;
      if (g < V8) {
        const uint32_t h[4] = {wv[i].x, wv[i].y, wv[i].z, wv[i].w};
        uint32_t o[4];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int64_t j = 8 * g + 2 * e;
          const float a = (__expf(__uint_as_float(h[e] << 16) - lse) - (j == y ? 1.f : 0.f)) * sc;
          const float b2 = (__expf(__uint_as_float(h[e] & 0xffff0000u) - lse) - (j + 1 == y ? 1.f : 0.f)) * sc;
          o[e] = f2bf2(a, b2);
        }
        *reinterpret_cast<uint4*>(dx + 8 * g) = make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
    for (int64_t j = 8 * V8 + tid; j < ld; j += NT) {  // V % 8 tail and the padding columns
      float v = 0.f;
      if (j < V) v = (__expf(bf2f(x[j]) - lse) - (j == y ? 1.f : 0.f)) * sc;
      dx[j] = f2bf(v);
    }
  }
}

__global__ void ce_reduce_kernel(int64_t rows, const float* __restrict__ loss_rows, const int32_t* n_valid,
                                 float* loss, const int32_t* __restrict__ rows_dev) {
  __shared__ double red[256];
  if (rows_dev && *rows_dev < rows) rows = *rows_dev;
  double a = 0.0;
  for (int64_t i = threadIdx.x; i < rows; i += 256) a += (double)loss_rows[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) *loss = (float)(red[0] / (double)(*n_valid));
}

// ---------------------------------------------------------------- norm / AdamW
constexpr int SQ_BLOCKS = 1024;

__global__ __launch_bounds__(256) void sqnorm_partial_kernel(int64_t n, const float* __restrict__ x, float* partial) {
  __shared__ float red[4];
  float a = 0.f;
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    const float4 v = reinterpret_cast<const float4*>(x)[i];
    a += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  if (blockIdx.x == 0)
    for (int64_t i = 4 * n4 + threadIdx.x; i < n; i += 256) a += x[i] * x[i];
  a = block_sum256(a, red);
  if (threadIdx.x == 0) partial[blockIdx.x] = a;
}

struct AdamState {  // 64-byte device state, see icap.h
  int64_t step;
  float norm, clip, lr, step_size, bc2_sqrt, decay;
  float pad[8];
};

__global__ void adam_finalize_kernel(int nparts, const float* __restrict__ partial, AdamState* st, float* sq_out,
                                     float lr0, float beta1, float beta2, float wd, float max_norm,
                                     int64_t warmup, int64_t total) {
  __shared__ double red[256];
  double a = 0.0;
  for (int i = threadIdx.x; i < nparts; i += 256) a += (double)partial[i];
  red[threadIdx.x] = a;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x != 0) return;
  if (sq_out) { *sq_out = (float)red[0]; return; }
  const float norm = (float)sqrt(red[0]);
  // TORCH/nn/utils/clip_grad.py:165-169: coef = max_norm / (norm + 1e-6), clamped to 1
  float clip = 1.f;
  if (max_norm > 0.f) {
    clip = max_norm / (norm + 1e-6f);
    if (clip > 1.f) clip = 1.f;
  }
  const int64_t k = st->step;
  // HF/optimization.py:101-107 linear schedule with warmup
  double lam;
  if (k < warmup) lam = (double)k / (double)(warmup > 1 ? warmup : 1);
  else {
    const double den = (double)((total - warmup) > 1 ? (total - warmup) : 1);
    lam = (double)(total - k) / den;
    if (lam < 0.0) lam = 0.0;
  }
  const double lr = (double)lr0 * lam;
  const double t = (double)(k + 1);
  const double bc1 = 1.0 - pow((double)beta1, t);
  const double bc2 = 1.0 - pow((double)beta2, t);
  st->norm = norm;
  st->clip = clip;
  st->lr = (float)lr;
  st->step_size = (float)(lr / bc1);
  st->bc2_sqrt = (float)sqrt(bc2);
  st->decay = (float)(1.0 - lr * (double)wd);
  st->step = k + 1;
}

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, float clip, float decay, float w1,
                                         float b2, float w2, float step_size, float bc2s, float eps) {
  g *= clip;
  p *= decay;
  m = m + w1 * (g - m);        // exp_avg.lerp_(grad, 1-beta1)
  v = v * b2 + w2 * (g * g);   // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1-beta2)
  const float denom = sqrtf(v) / bc2s + eps;
  p = p + (-step_size) * (m / denom);
}

__global__ __launch_bounds__(256) void adam_update_kernel(int64_t n, float* __restrict__ P, const float* __restrict__ G,
                                                         float* __restrict__ M1, float* __restrict__ M2,
                                                         bf16_t* __restrict__ out16, const AdamState* __restrict__ st,
                                                         float beta1, float beta2, float eps) {
  const float clip = st->clip, decay = st->decay, step_size = st->step_size, bc2s = st->bc2_sqrt;
  const float w1 = 1.f - beta1, w2 = 1.f - beta2;
  const int64_t n4 = n >> 2;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 p = reinterpret_cast<float4*>(P)[i];
    const float4 g = reinterpret_cast<const float4*>(G)[i];
    float4 m = reinterpret_cast<float4*>(M1)[i];
    float4 v = reinterpret_cast<float4*>(M2)[i];
    adam_one(p.x, g.x, m.x, v.x, clip, decay, w1, beta2, w2, step_size, bc2s, eps);
    adam_one(p.y, g.y, m.y, v.y, clip, decay, w1, beta2, w2, step_size, bc2s, eps);
    adam_one(p.z, g.z, m.z, v.z, clip, decay, w1, beta2, w2, step_size, bc2s, eps);
    adam_one(p.w, g.w, m.w, v.w, clip, decay, w1, beta2, w2, step_size, bc2s, eps);
    reinterpret_cast<float4*>(P)[i] = p;
    reinterpret_cast<float4*>(M1)[i] = m;
    reinterpret_cast<float4*>(M2)[i] = v;
    if (out16) {
      const float o[4] = {p.x, p.y, p.z, p.w};
      io<bf16_t>::st4(out16 + 4 * i, o);
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t i = 4 * n4 + threadIdx.x; i < n; i += 256) {
      float p = P[i], m = M1[i], v = M2[i];
      adam_one(p, G[i], m, v, clip, decay, w1, beta2, w2, step_size, bc2s, eps);
      P[i] = p; M1[i] = m; M2[i] = v;
      if (out16) out16[i] = f2bf(p);
    }
  }
}

// ---------------------------------------------------------------- layout helpers
template <typename T>
__global__ __launch_bounds__(256) void transpose_kernel(int64_t rows, int64_t cols, const T* __restrict__ src,
                                                       int64_t lds, T* __restrict__ dst, int64_t ldd,
                                                       int64_t rows_pad) {
  __shared__ T tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t r = r0 + i, c = c0 + tx;
    T v = (T)0;
    if (r < rows && c < cols) v = src[r * lds + c];
    tile[i][tx] = v;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, r = r0 + tx;
    if (c < cols && r < rows_pad) dst[c * ldd + r] = tile[tx][i];
  }
}

template <typename T>
__global__ __launch_bounds__(256) void colsum_kernel(int64_t M, int64_t N, const T* __restrict__ src, int64_t ld,
                                                    int64_t rows_per_chunk, float* __restrict__ partial) {
  __shared__ float red[4][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + tx;
  const int64_t m0 = (int64_t)blockIdx.y * rows_per_chunk;
  int64_t m1 = m0 + rows_per_chunk;
  if (m1 > M) m1 = M;
  float a = 0.f;
  if (c < N)
    for (int64_t m = m0 + ty; m < m1; m += 4) a += io<T>::ld(src + m * ld + c);
  red[ty][tx] = a;
  __syncthreads();
  if (ty == 0 && c < N) partial[(int64_t)blockIdx.y * N + c] = red[0][tx] + red[1][tx] + red[2][tx] + red[3][tx];
}

// 16-bit transpose with 16-byte accesses on both sides: 64x64 tile through LDS (row stride 68 halves, so the
// column gathers of the write phase are at most 2-way bank conflicted). Needs cols % 8 == 0, lds/ldd % 8 == 0,
// 16-byte aligned src/dst and rows_pad % 64 == 0 (checked by the host).
constexpr int T16_TLD = 68;
__device__ __forceinline__ void transpose16_tile(int64_t rows, int64_t cols, const uint16_t* __restrict__ src,
                                                 int64_t lds, uint16_t* __restrict__ dst, int64_t ldd, int64_t r0,
                                                 int64_t c0, uint16_t* tile) {
  constexpr int TLD = T16_TLD;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = threadIdx.x + 256 * h;
    const int r = idx >> 3, ch = idx & 7;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (r0 + r < rows && c0 + 8 * ch < cols) v = *reinterpret_cast<const uint4*>(src + (r0 + r) * lds + c0 + 8 * ch);
    uint2* t = reinterpret_cast<uint2*>(&tile[r * TLD + 8 * ch]);
    t[0] = make_uint2(v.x, v.y);
    t[1] = make_uint2(v.z, v.w);
  }
  __syncthreads();
  // read phase: a wave takes one 8-row group rq of all 64 columns (lane = column), so its 16-bit LDS reads hit 32
  // consecutive dwords (no bank conflict; 8 lanes per column at 8-row spacing were 4-way: 0.67 of the kernel's LDS
  // cycles, profiles/r04_pmc_lds.txt); each lane still stores 16 contiguous bytes of its output row
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int idx = threadIdx.x + 256 * h;
    const int c = idx & 63, rq = idx >> 6;
    if (c0 + c >= cols) continue;
    uint32_t w[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      w[e] = (uint32_t)tile[(8 * rq + 2 * e) * TLD + c] | ((uint32_t)tile[(8 * rq + 2 * e + 1) * TLD + c] << 16);
    *reinterpret_cast<uint4*>(dst + (c0 + c) * ldd + r0 + 8 * rq) = make_uint4(w[0], w[1], w[2], w[3]);
  }
}

__global__ __launch_bounds__(256) void transpose16_vec_kernel(int64_t rows, int64_t cols, const uint16_t* __restrict__ src,
                                                              int64_t lds, uint16_t* __restrict__ dst, int64_t ldd) {
  __shared__ __attribute__((aligned(16))) uint16_t tile[64 * T16_TLD];
  transpose16_tile(rows, cols, src, lds, dst, ldd, (int64_t)blockIdx.y * 64, (int64_t)blockIdx.x * 64, tile);
}

// Several bf16 transposes in one launch (the trained mapper's transposed weight copies after every optimizer step:
// 32 launches of 3-25 µs before): block b works on tile b - off[i] of the item i whose tile range holds b.
constexpr int T16_BATCH = 32;
struct Transpose16Batch {
  int n;
  int64_t off[T16_BATCH + 1];
  const uint16_t* src[T16_BATCH];
  uint16_t* dst[T16_BATCH];
  int64_t rows[T16_BATCH], cols[T16_BATCH], lds[T16_BATCH], ldd[T16_BATCH];
};
__global__ __launch_bounds__(256) void transpose16_batch_kernel(Transpose16Batch b) {
  __shared__ __attribute__((aligned(16))) uint16_t tile[64 * T16_TLD];
  const int64_t bid = blockIdx.x;
  int i = 0;
  while (i + 1 < b.n && bid >= b.off[i + 1]) ++i;  // block-uniform
  const int64_t t = bid - b.off[i];
  const int64_t tx = (b.cols[i] + 63) / 64;
  const int64_t ty = t / tx;
  transpose16_tile(b.rows[i], b.cols[i], b.src[i], b.lds[i], b.dst[i], b.ldd[i], ty * 64, (t - ty * tx) * 64, tile);
}

// column sums, 4 columns per lane (16-byte / 8-byte row segments), 4 waves over the rows of a chunk
template <typename T>
__global__ __launch_bounds__(256) void colsum4_kernel(int64_t M, int64_t N, const T* __restrict__ src, int64_t ld,
                                                     int64_t rows_per_chunk, float* __restrict__ partial) {
  __shared__ float4 red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c = ((int64_t)blockIdx.x * 64 + lane) * 4;
  const int64_t m0 = (int64_t)blockIdx.y * rows_per_chunk;
  int64_t m1 = m0 + rows_per_chunk;
  if (m1 > M) m1 = M;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < N) {
#pragma unroll 4
    for (int64_t m = m0 + w; m < m1; m += 4) {
      float v[4];
      io<T>::ld4(src + m * ld + c, v);
      a[0] += v[0]; a[1] += v[1]; a[2] += v[2]; a[3] += v[3];
    }
  }
  red[w][lane] = make_float4(a[0], a[1], a[2], a[3]);
  __syncthreads();
  if (w == 0 && c < N) {
    float4 t = red[0][lane];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 u = red[k][lane];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    *reinterpret_cast<float4*>(partial + (int64_t)blockIdx.y * N + c) = t;
  }
}

// 64 columns per block, 16 waves over the chunk partials in a fixed order (deterministic)
__global__ __launch_bounds__(1024) void colsum_reduce_kernel(int64_t N, int nchunks, const float* __restrict__ partial,
                                                            float* out, int acc) {
  __shared__ float red[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + tx;
  float a = 0.f;
  if (c < N) {
#pragma unroll 4
    for (int i = ty; i < nchunks; i += 16) a += partial[(int64_t)i * N + c];
  }
  red[ty][tx] = a;
  __syncthreads();
  if (ty == 0 && c < N) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][tx];
    out[c] = acc ? out[c] + s : s;
  }
}

// Batched column sums: the items' columns are laid end to end (item i at column base[i] of the partial rows);
// block (x, y) sums 256 columns of one item over row chunk y with the colsum4 loop, so each column's partial is
// the same float sequence as icap_colsum's.
struct ColsumBatch {
  int n;
  int64_t blk[ICAP_COLSUM_BATCH + 1];   // first x-block of each item (256 columns per block)
  int64_t base[ICAP_COLSUM_BATCH + 1];  // first partial column of each item; base[n] = total columns
  const void* src[ICAP_COLSUM_BATCH];
  int64_t ld[ICAP_COLSUM_BATCH], N[ICAP_COLSUM_BATCH];
  float* out[ICAP_COLSUM_BATCH];
};
template <typename T>
__global__ __launch_bounds__(256) void colsum4_batch_kernel(ColsumBatch b, int64_t M, int64_t rows_per_chunk,
                                                           float* __restrict__ partial) {
  __shared__ float4 red[4][64];
  const int64_t bx = blockIdx.x;
  int i = 0;
  while (i + 1 < b.n && bx >= b.blk[i + 1]) ++i;  // block-uniform
  const T* __restrict__ src = reinterpret_cast<const T*>(b.src[i]);
  const int64_t N = b.N[i], ld = b.ld[i];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t c = ((bx - b.blk[i]) * 64 + lane) * 4;
  const int64_t m0 = (int64_t)blockIdx.y * rows_per_chunk;
  int64_t m1 = m0 + rows_per_chunk;
  if (m1 > M) m1 = M;
  float a[4] = {0.f, 0.f, 0.f, 0.f};
  if (c < N) {
#pragma unroll 4
    for (int64_t m = m0 + w; m < m1; m += 4) {
      float v[4];
      io<T>::ld4(src + m * ld + c, v);
      a[0] += v[0]; a[1] += v[1]; a[2] += v[2]; a[3] += v[3];
    }
  }
  red[w][lane] = make_float4(a[0], a[1], a[2], a[3]);
  __syncthreads();
  if (w == 0 && c < N) {
    float4 t = red[0][lane];
#pragma unroll
    for (int k = 1; k < 4; ++k) {
      const float4 u = red[k][lane];
      t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
    }
    *reinterpret_cast<float4*>(partial + (int64_t)blockIdx.y * b.base[b.n] + b.base[i] + c) = t;
  }
}

// colsum_reduce_kernel over the concatenated columns; each column finds its item (the items' N are multiples of 4,
// not of 64, so a block may straddle two items)
__global__ __launch_bounds__(1024) void colsum_reduce_batch_kernel(ColsumBatch b, int nchunks,
                                                                  const float* __restrict__ partial, int acc) {
  __shared__ float red[16][64];
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  const int64_t Nt = b.base[b.n];
  const int64_t c = (int64_t)blockIdx.x * 64 + tx;
  float a = 0.f;
  if (c < Nt) {
#pragma unroll 4
    for (int k = ty; k < nchunks; k += 16) a += partial[(int64_t)k * Nt + c];
  }
  red[ty][tx] = a;
  __syncthreads();
  if (ty == 0 && c < Nt) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][tx];
    int i = 0;
    while (i + 1 < b.n && c >= b.base[i + 1]) ++i;
    float* o = b.out[i] + (c - b.base[i]);
    *o = acc ? *o + s : s;
  }
}

template <typename TS, typename TD>
__global__ void map2d_kernel(int64_t M, int64_t N, const TS* __restrict__ src, int64_t lds, TD* __restrict__ dst,
                             int64_t ldd, uint32_t thr, float inv_keep, uint64_t seed0, const uint64_t* seed_ptr,
                             uint64_t offset) {
  const int64_t total = M * N;
  const uint64_t seed = thr ? eff_seed(seed0, seed_ptr) : 0ull;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t m = i / N, n = i - m * N;
    float v = io<TS>::ld(src + m * lds + n);
    if (thr) v *= drop_scale(seed, offset + (uint64_t)i, thr, inv_keep);
    io<TD>::st(dst + m * ldd + n, v);
  }
}

__global__ void counter_inc_kernel(uint64_t* c) {
  if (threadIdx.x == 0) *c += 1;
}

template <typename T>
__global__ void broadcast_rows_kernel(int B, int64_t R, int64_t D, const float* __restrict__ src, T* __restrict__ dst,
                                      int64_t bs) {
  const int64_t per = R * D, total = (int64_t)B * per;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / per, k = i - b * per;
    io<T>::st(dst + b * bs + k, src[k]);
  }
}

// ---------------------------------------------------------------- CLIP glue
template <typename T>
__global__ void im2col_kernel(int B, int C, int HW, int p, const float* __restrict__ px, T* __restrict__ out) {
  const int G = HW / p;
  const int K = C * p * p;
  const int p4 = p >> 2;
  const int64_t total = (int64_t)B * G * G * C * p * p4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t t = i;
    const int kx4 = (int)(t % p4); t /= p4;
    const int ky = (int)(t % p); t /= p;
    const int c = (int)(t % C); t /= C;
    const int gx = (int)(t % G); t /= G;
    const int gy = (int)(t % G); t /= G;
    const int b = (int)t;
    const float4 v = *reinterpret_cast<const float4*>(px + (((int64_t)b * C + c) * HW + gy * p + ky) * HW + gx * p + 4 * kx4);
    const float o[4] = {v.x, v.y, v.z, v.w};
    const int64_t row = ((int64_t)b * G + gy) * G + gx;
    io<T>::st4(out + row * K + c * p * p + ky * p + 4 * kx4, o);
  }
}

// any patch size (ViT-L/14: p = 14, C p p = 588): one thread per element of the 8-padded patch row, pad zeros
template <typename T>
__global__ void im2col_any_kernel(int B, int C, int HW, int p, int Kp, const float* __restrict__ px,
                                  T* __restrict__ out) {
  const int G = HW / p;
  const int K = C * p * p;
  const int64_t total = (int64_t)B * G * G * Kp;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / Kp;
    const int col = (int)(i - row * Kp);
    float v = 0.f;
    if (col < K) {
      const int c = col / (p * p), r = col - c * p * p, ky = r / p, kx = r - ky * p;
      const int64_t b = row / (G * G);
      const int gy = (int)((row - b * G * G) / G), gx = (int)(row - b * G * G - (int64_t)gy * G);
      v = px[((b * C + c) * HW + gy * p + ky) * HW + gx * p + kx];
    }
    io<T>::st(out + i, v);
  }
}

template <typename T>
__global__ void vit_embed_kernel(int B, int G2, int NP, int D, const T* __restrict__ pe, const float* __restrict__ pfx,
                                 const float* __restrict__ pos, T* __restrict__ x) {
  const int S = G2 + NP;
  const int64_t total = (int64_t)B * S * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / D;
    const int d = (int)(i - row * D);
    const int b = (int)(row / S), t = (int)(row - (int64_t)b * S);
    const float v = (t < NP) ? pfx[(int64_t)t * D + d] : io<T>::ld(pe + ((int64_t)b * G2 + t - NP) * D + d);
    io<T>::st(x + i, pos ? v + pos[(int64_t)t * D + d] : v);
  }
}

// Rotary position embedding of the patch tokens (HF/models/dinov3_vit/modeling_dinov3_vit.py:203-268): for rows
// t >= NP of every image and every head, q and k (columns [0, H hd) and [H hd, 2 H hd) of the fused QKV row) become
// x * cos + rotate_half(x) * sin with rotate_half(x) = (-x[hd/2:], x[:hd/2]); cos / sin: fp32 [S - NP, hd]. One
// thread per (row, q|k, head, i < hd/2) pair updates elements i and i + hd/2 in place.
template <typename T>
__global__ void rope_patches_kernel(int B, int S, int NP, int H, int hd, T* __restrict__ qkv, int64_t ld,
                                    const float* __restrict__ cs, const float* __restrict__ sn) {
#pragma clang fp contract(off)
  const int half = hd >> 1;
  const int P = S - NP;
  const int64_t total = (int64_t)B * P * 2 * H * half;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int j = (int)(i % half);
    int64_t r = i / half;
    const int hq = (int)(r % (2 * H));  // q heads 0..H-1, then k heads
    r /= (2 * H);
    const int p = (int)(r % P);
    const int b = (int)(r / P);
    T* v = qkv + ((int64_t)b * S + NP + p) * ld + (int64_t)hq * hd;
    const float x1 = io<T>::ld(v + j), x2 = io<T>::ld(v + j + half);
    const float* c = cs + (int64_t)p * hd;
    const float* s = sn + (int64_t)p * hd;
    io<T>::st(v + j, x1 * c[j] + (-x2) * s[j]);
    io<T>::st(v + j + half, x2 * c[j + half] + x1 * s[j + half]);
  }
}

template <typename T>
__global__ void l2norm_kernel(int64_t rows, int64_t D, const T* __restrict__ x, int64_t ldx, float* __restrict__ out,
                              int64_t ldo) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= rows) return;
  float s = 0.f;
  for (int64_t d = lane; d < D; d += 64) {
    const float v = io<T>::ld(x + r * ldx + d);
    s += v * v;
  }
  s = wave_sum(s);
  const float inv = 1.f / sqrtf(s);
  for (int64_t d = lane; d < D; d += 64) out[r * ldo + d] = io<T>::ld(x + r * ldx + d) * inv;
}

// ---------------------------------------------------------------- greedy decode glue
// argmax order of torch.argmax: NaN beats everything, ties (and NaN vs NaN) -> smallest index
__device__ __forceinline__ bool argmax_better(float v, int64_t j, float best, int64_t bi) {
  if (v != v) return best == best || j < bi;
  if (best != best) return false;
  return v > best || (v == best && j < bi);
}

template <typename T>
__global__ __launch_bounds__(1024) void greedy_next_kernel(int64_t V, const T* __restrict__ logits, int64_t ld,
                                                         int64_t eos, const int64_t* __restrict__ forced,
                                                         int32_t* finished, int64_t* tokens,
                                                         int64_t ld_tokens, int step, const T* __restrict__ wte,
                                                         const T* __restrict__ wpe, int pos, int D, T* __restrict__ x,
                                                         int vec) {
  // one 1024-thread block per row: 4-wide vector loads keep ~12 loads in flight per thread (the previous
  // 256-thread scalar loop was latency bound at ~67 us per decode step for B=128)
  constexpr int NT = 1024, NW = NT / 64;
  __shared__ float rv[NW];
  __shared__ int64_t ri[NW];
  __shared__ int64_t nxt;
  const int b = blockIdx.x;
  const T* row = logits + (int64_t)b * ld;
  float best = -INFINITY;
  int64_t bi = V;  // sentinel
  auto consider = [&](float v, int64_t j) {
    if (argmax_better(v, j, best, bi)) { best = v; bi = j; }
  };
  int64_t j0 = 0;
  if constexpr (sizeof(T) == 2) {
    if (vec == 2) {
      // 16-byte loads, eight per thread in flight at once (a 50,304-logit row is one pass). Each thread visits its
      // logits in increasing index order, so a strict `>` keeps its first maximum (3 VALU ops per logit instead
      // of the NaN-aware 64-bit compare); a NaN anywhere in the row sends the block to the exact loop below.
      const int64_t V8 = V >> 3;
      float fb = -INFINITY;
      int fi = (int)V;
      bool nan = false;
      for (int64_t q0 = threadIdx.x; q0 < V8; q0 += 8 * NT) {
        uint4 w[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int64_t q = q0 + (int64_t)u * NT;
          w[u] = q < V8 ? *reinterpret_cast<const uint4*>(row + 8 * q) : make_uint4(0xff80ff80u, 0xff80ff80u,
                                                                                  0xff80ff80u, 0xff80ff80u);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int jb = (int)(8 * (q0 + (int64_t)u * NT));
          const uint32_t h[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float v0 = __uint_as_float(h[e] << 16), v1 = __uint_as_float(h[e] & 0xffff0000u);
            nan |= (v0 != v0) | (v1 != v1);
            if (v0 > fb) { fb = v0; fi = jb + 2 * e; }
            if (v1 > fb) { fb = v1; fi = jb + 2 * e + 1; }
          }
        }
      }
      if (__syncthreads_or(nan)) {
        for (int64_t q = threadIdx.x; q < V8; q += NT) {
          float v[8];
          io<T>::ld8(row + 8 * q, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) consider(v[e], 8 * q + e);
        }
      } else {
        best = fb;
        bi = fi < V ? fi : V;
      }
      j0 = V8 << 3;
    }
  }
  if (vec == 1) {
    const int64_t V4 = V >> 2;
#pragma unroll 4
    for (int64_t q = threadIdx.x; q < V4; q += NT) {
      float v[4];
      io<T>::ld4(row + 4 * q, v);
#pragma unroll
      for (int e = 0; e < 4; ++e) consider(v[e], 4 * q + e);
    }
    j0 = V4 << 2;
  }
  for (int64_t j = j0 + threadIdx.x; j < V; j += NT) consider(io<T>::ld(row + j), j);
  // wave argmax (ties -> smallest index)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int64_t oi = __shfl_xor(bi, o, 64);
    if (argmax_better(ov, oi, best, bi)) { best = ov; bi = oi; }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { rv[w] = best; ri[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float bv = rv[0];
    int64_t bj = ri[0];
    for (int k = 1; k < NW; ++k)
      if (argmax_better(rv[k], ri[k], bv, bj)) { bv = rv[k]; bj = ri[k]; }
    if (bj >= V) bj = 0;
    if (forced) bj = forced[b];
    int fin = finished[b];
    if (fin) bj = eos;
    if (bj == eos) fin = 1;
    finished[b] = fin;
    tokens[(int64_t)b * ld_tokens + step] = bj;
    nxt = bj;
  }
  __syncthreads();
  if (x) {
    const int64_t id = nxt;
    for (int d = threadIdx.x; d < D; d += NT)
      io<T>::st(x + (int64_t)b * D + d, io<T>::ld(wte + id * D + d) + io<T>::ld(wpe + (int64_t)pos * D + d));
  }
}

// Split form (round 5): a 1024-thread block per row left half the CUs idle at B = 128 and read its 100 KB row at
// one CU's intake (11 µs per decode step). Here GS blocks of 256 threads per row each take a contiguous column
// range and leave (max, first index) in the row's x slot (D elements, free until the finish kernel rewrites it),
// and a second launch takes the partials in range order (the first maximum wins: the same token as the single
// block, NaN and ties included) and does the latch and the embedding of the next token.
constexpr int GSPLIT = 8;
template <typename T>
__global__ __launch_bounds__(256) void greedy_part_kernel(int64_t V, const T* __restrict__ logits, int64_t ld,
                                                        int64_t chunk, T* __restrict__ x, int D, int vec) {
  constexpr int NT = 256, NW = NT / 64;
  __shared__ float rv[NW];
  __shared__ int64_t ri[NW];
  const int b = blockIdx.y, sidx = blockIdx.x;
  const int64_t c0 = (int64_t)sidx * chunk, c1 = c0 + chunk < V ? c0 + chunk : V;
  const T* row = logits + (int64_t)b * ld;
  float best = -INFINITY;
  int64_t bi = V;
  auto consider = [&](float v, int64_t j) {
    if (argmax_better(v, j, best, bi)) { best = v; bi = j; }
  };
  int64_t j0 = c0;
  if constexpr (sizeof(T) == 2) {
    if (vec == 2) {  // c0 % 8 == 0 (chunk is a multiple of 8): 16-byte loads, first maximum per thread by strict >
      const int64_t q0b = c0 >> 3, q1 = c1 >> 3;
      float fb = -INFINITY;
      int64_t fi = V;
      bool nan = false;
      for (int64_t q = q0b + threadIdx.x; q < q1; q += NT) {
        const uint4 w = *reinterpret_cast<const uint4*>(row + 8 * q);
        const uint32_t h[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v0 = __uint_as_float(h[e] << 16), v1 = __uint_as_float(h[e] & 0xffff0000u);
          nan |= (v0 != v0) | (v1 != v1);
          if (v0 > fb) { fb = v0; fi = 8 * q + 2 * e; }
          if (v1 > fb) { fb = v1; fi = 8 * q + 2 * e + 1; }
        }
      }
      if (__syncthreads_or(nan)) {
        for (int64_t q = q0b + threadIdx.x; q < q1; q += NT) {
          float v[8];
          io<T>::ld8(row + 8 * q, v);
#pragma unroll
          for (int e = 0; e < 8; ++e) consider(v[e], 8 * q + e);
        }
      } else {
        best = fb;
        bi = fi;
      }
      j0 = q1 << 3;
    }
  }
  for (int64_t j = j0 + threadIdx.x; j < c1; j += NT) consider(io<T>::ld(row + j), j);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ov = __shfl_xor(best, o, 64);
    const int64_t oi = __shfl_xor(bi, o, 64);
    if (argmax_better(ov, oi, best, bi)) { best = ov; bi = oi; }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { rv[w] = best; ri[w] = bi; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float bv = rv[0];
    int64_t bj = ri[0];
    for (int k = 1; k < NW; ++k)
      if (argmax_better(rv[k], ri[k], bv, bj)) { bv = rv[k]; bj = ri[k]; }
    int32_t* slot = reinterpret_cast<int32_t*>(x + (int64_t)b * D) + 2 * sidx;
    slot[0] = __float_as_int(bv);
    slot[1] = (int32_t)(bj < V ? bj : V);
  }
}

template <typename T>
__global__ __launch_bounds__(256) void greedy_finish_kernel(int64_t V, int nsplit, int64_t eos,
                                                          const int64_t* __restrict__ forced, int32_t* finished,
                                                          int64_t* tokens, int64_t ld_tokens, int step,
                                                          const T* __restrict__ wte, const T* __restrict__ wpe,
                                                          int pos, int D, T* __restrict__ x) {
  __shared__ int64_t nxt;
  const int b = blockIdx.x;
  if (threadIdx.x == 0) {
    const int32_t* slot = reinterpret_cast<const int32_t*>(x + (int64_t)b * D);
    float bv = -INFINITY;
    int64_t bj = V;
    for (int k = 0; k < nsplit; ++k) {
      const float v = __int_as_float(slot[2 * k]);
      const int64_t j = slot[2 * k + 1];
      if (argmax_better(v, j, bv, bj)) { bv = v; bj = j; }
    }
    if (bj >= V) bj = 0;
    if (forced) bj = forced[b];
    int fin = finished[b];
    if (fin) bj = eos;
    if (bj == eos) fin = 1;
    finished[b] = fin;
    tokens[(int64_t)b * ld_tokens + step] = bj;
    nxt = bj;
  }
  __syncthreads();
  const int64_t id = nxt;
  for (int d = threadIdx.x; d < D; d += blockDim.x)
    io<T>::st(x + (int64_t)b * D + d, io<T>::ld(wte + id * D + d) + io<T>::ld(wpe + (int64_t)pos * D + d));
}

template <typename T>
__global__ void add_position_kernel(int B, int npos, int D, const T* __restrict__ src, int64_t sbs, int64_t sts,
                                    const T* __restrict__ wpe, int pos0, T* __restrict__ x) {
  const int64_t total = (int64_t)npos * B * D;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / D;
    const int d = (int)(i - row * D);
    const int t = (int)(row / B), b = (int)(row - (int64_t)t * B);
    const float v = io<T>::ld(src + (int64_t)b * sbs + (int64_t)t * sts + d) + io<T>::ld(wpe + (int64_t)(pos0 + t) * D + d);
    io<T>::st(x + i, v);
  }
}


// ---- nucleus (top-p) sampling: src/models.py:400-449 ---------------------------------
// One 512-thread block per row. The row lives in registers, NPT elements per thread (index k*512 + tid), as a
// fixed-point probability q = trunc(float(e) * float(2^31 / Z)) of the temperature-scaled logit l = logit / T,
// e = expf(l - max), Z = sum(trunc(e * 2^40)) / 2^40: one register per element, 100 per lane for GPT-2's
// vocabulary within the 256 VGPRs a 512-thread block allows (1024 threads cap a lane at 128 and spilled). Every mass below is an exact integer sum, so nothing depends on the
// reduction order (deterministic; oracle/icap_oracle.py topp_sample_fixed restates it in numpy).
// The reference filter (sort descending, cumsum(softmax), remove where cumsum > top_p, shifted right by one)
// keeps ranks 0..r, r = the first rank whose inclusive cumsum exceeds top_p. Ranks here run by descending q
// and, among equal q, ascending index (a stable sort): equal logits tie exactly as in the reference; distinct
// logits whose probabilities differ by less than 2^-31 also tie here (documented deviation 1). Tokens whose
// probability is below 2^-31 get q = 0 and are never drawn, even with top_p >= 1 (documented deviation 2: the
// reference's multinomial would draw such a token with probability < 2^-31 per row and step).
// K* = min{K : mass(q > K) <= T} (bisection over q) is the q of rank r; of the c tokens tied at K* the first
// (T - A) / K* + 1 by index are kept, A = mass(q > K*). The draw is an inverse CDF over the kept tokens in vocabulary order with
// u = hash32(seed, step << 32 | row) / 2^32: torch.multinomial's stream is not reproducible across devices,
// its distribution (softmax over the kept logits) is what is matched.
namespace topp {
constexpr int NT = 512, NW = NT / 64;
// q as an opaque 32-bit value inside a loop: keeps the compiler from hoisting 64-bit zero-extended copies of
// the whole register-resident row out of the bisection loops (that doubled the row's registers and spilled)
__device__ __forceinline__ uint32_t opaque(uint32_t v) {
  asm volatile("" : "+v"(v));
  return v;
}
// block-wide sum, result in every thread; callers alternate `buf` between consecutive calls so one barrier
// per call suffices (a buffer is rewritten only after the next call's barrier, which follows every read of it)
__device__ __forceinline__ uint64_t block_sum(uint64_t v, uint64_t* buf) {
  unsigned long long x = v;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) x += __shfl_xor(x, o, 64);
  if ((threadIdx.x & 63) == 0) buf[threadIdx.x >> 6] = x;
  __syncthreads();
  uint64_t s = 0;
#pragma unroll
  for (int w = 0; w < NW; ++w) s += buf[w];
  return s;
}
}  // namespace topp

template <typename T, int NPT>
__global__ __launch_bounds__(512) void topp_sample_kernel(int64_t V, const T* __restrict__ logits, int64_t ld,
                                                         float temperature, float top_p,
                                                         const int32_t* __restrict__ finished, uint64_t seed,
                                                         const uint64_t* __restrict__ seed_ptr, int step, int64_t eos,
                                                         int64_t* __restrict__ out) {
  using namespace topp;
  __shared__ uint64_t sbuf[2][NW];
  __shared__ float fbuf[NW];
  const int b = blockIdx.x, tid = threadIdx.x;
  // finished rows: the reference samples from zeroed logits and then overwrites the draw with EOS (:410,:456)
  if (finished && finished[b]) {
    if (tid == 0) out[b] = eos;
    return;
  }
  const T* row = logits + (int64_t)b * ld;
  uint32_t q[NPT];
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const int64_t j = (int64_t)k * NT + tid;
    const float l = j < V ? io<T>::ld(row + j) / temperature : -INFINITY;
    q[k] = __float_as_uint(l);
    m = fmaxf(m, l);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((tid & 63) == 0) fbuf[tid >> 6] = m;
  __syncthreads();
  m = fbuf[0];
#pragma unroll
  for (int w = 1; w < NW; ++w) m = fmaxf(m, fbuf[w]);
  // Z as an exact 2^-40 fixed-point sum (order independent, so q below is reproducible bit for bit)
  uint64_t zi = 0;
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const float e = expf(__uint_as_float(q[k]) - m);
    q[k] = __float_as_uint(e);
    zi += (uint64_t)((double)e * 1099511627776.0);
  }
  int ci = 0;
  zi = block_sum(zi, sbuf[ci]);
  ci ^= 1;
  const double z = (double)zi * (1.0 / 1099511627776.0);
  if (!(z > 0.0)) {  // every logit -inf / NaN: nothing to sample
    if (tid == 0) out[b] = 0;
    return;
  }
  const float scale = (float)(2147483648.0 / z);
#pragma unroll
  for (int k = 0; k < NPT; ++k) q[k] = (uint32_t)(__uint_as_float(q[k]) * scale);

  uint32_t kstar = 0, jt = (uint32_t)V;
  if (top_p < 1.0f) {
    const uint64_t thr = (uint64_t)((double)top_p * 2147483648.0);
    uint32_t lo = 0, hi = 0x80000000u;  // q <= 2^31; invariant: mass(q > hi) <= thr
    while (lo < hi) {
      const uint32_t mid = lo + ((hi - lo) >> 1);
      uint64_t s = 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const uint32_t v = opaque(q[k]);
        s += v > mid ? v : 0u;
      }
      s = block_sum(s, sbuf[ci]);
      ci ^= 1;
      if (s <= thr) hi = mid; else lo = mid + 1;
    }
    kstar = lo;
    if (kstar != 0) {  // kstar == 0: every positive-mass token fits under top_p, everything stays
      uint64_t a = 0, c = 0;
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const uint32_t v = opaque(q[k]);
        a += v > kstar ? v : 0u;
        c += v == kstar ? 1u : 0u;
      }
      a = block_sum(a, sbuf[ci]); ci ^= 1;
      c = block_sum(c, sbuf[ci]); ci ^= 1;
      const uint64_t qs = kstar;
      const uint64_t ntie = (thr - a) / qs + 1;
      if (ntie < c) {  // keep the ntie lowest indices of the tie group: jt = min{J : count(tie, j < J) >= ntie}
        uint32_t jlo = 1, jhi = (uint32_t)V;
        while (jlo < jhi) {
          const uint32_t mid = jlo + ((jhi - jlo) >> 1);
          const int lim = (int)mid - tid;  // j = k*NT + tid < mid  <=>  k*NT < lim (no per-element index registers)
          uint64_t s = 0;
#pragma unroll
          for (int k = 0; k < NPT; ++k) s += (opaque(q[k]) == kstar && k * NT < lim) ? 1u : 0u;
          s = block_sum(s, sbuf[ci]);
          ci ^= 1;
          if (s >= ntie) jhi = mid; else jlo = mid + 1;
        }
        jt = jlo;
      }
    }
  }
  uint64_t keep[(NPT + 63) / 64] = {}, tot = 0;  // bit k: element k of this thread is in the nucleus
#pragma unroll
  for (int k = 0; k < NPT; ++k) {
    const uint32_t v = opaque(q[k]);
    const bool kk = v > kstar || (v == kstar && k * NT < (int)jt - tid);
    keep[k >> 6] |= (uint64_t)kk << (k & 63);
    tot += kk ? v : 0u;
  }
  tot = block_sum(tot, sbuf[ci]);
  ci ^= 1;
  const uint32_t u = hash32(eff_seed(seed, seed_ptr), ((uint64_t)(uint32_t)step << 32) | (uint32_t)b);
  const uint64_t target = (tot * (uint64_t)u) >> 32;  // tot <= 2^31: no overflow; target < tot
  uint32_t jlo = 1, jhi = (uint32_t)V;  // min{J : kept mass of j < J  > target}
  while (jlo < jhi) {
    const uint32_t mid = jlo + ((jhi - jlo) >> 1);
    const int lim = (int)mid - tid;
    uint64_t s = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const uint32_t v = opaque(q[k]);
      s += (((keep[k >> 6] >> (k & 63)) & 1) && k * NT < lim) ? v : 0u;
    }
    s = block_sum(s, sbuf[ci]);
    ci ^= 1;
    if (s > target) jhi = mid; else jlo = mid + 1;
  }
  if (tid == 0) out[b] = tot ? (int64_t)(jlo - 1) : 0;
}

}  // namespace icap

using namespace icap;

// launch KERNEL<T> with every typed pointer argument cast to T* via the TP()/CTP() helpers
#define DISPATCH_T(dtype, BODY)                       \
  do {                                                \
    if ((dtype) == ICAP_BF16) {                       \
      typedef bf16_t T;                               \
      BODY;                                           \
    } else if ((dtype) == ICAP_F32) {                 \
      typedef float T;                                \
      BODY;                                           \
    } else {                                          \
      set_error("bad dtype");                         \
      return ICAP_ERR_ARG;                            \
    }                                                 \
  } while (0)
#define TP(x) reinterpret_cast<T*>(x)
#define CTP(x) reinterpret_cast<const T*>(x)

extern "C" int icap_gpt2_embed(int32_t dtype, int32_t B, int32_t P, int32_t L, int32_t D, const void* prefix,
                               int64_t prefix_bstride, const void* wte, const void* wpe, const int64_t* ids, void* x,
                               float drop_p, uint64_t seed, uint64_t offset, const uint64_t* seed_ptr,
                               const int32_t* seq_off, const int32_t* seq_len, void* stream) {
  ICAP_REQUIRE(D % 4 == 0 && B >= 0 && P >= 0 && L >= 0, "icap_gpt2_embed: bad geometry");
  ICAP_REQUIRE((seq_off == nullptr) == (seq_len == nullptr), "icap_gpt2_embed: seq_off and seq_len go together");
  ICAP_REQUIRE(x && wpe && (P == 0 || prefix) && (L == 0 || (wte && ids)), "icap_gpt2_embed: null pointer");
  ICAP_REQUIRE(prefix_bstride % 4 == 0, "icap_gpt2_embed: prefix_bstride must be a multiple of 4");
  const int64_t n = (int64_t)B * (P + L) * (D / 4);
  if (n == 0) return ICAP_OK;
  const uint32_t thr = drop_p > 0.f ? drop_threshold(drop_p) : 0u;
  const float ik = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  if (dtype == ICAP_BF16)
    hipLaunchKernelGGL(gpt2_embed_kernel<bf16_t>, dim3(nblk(n, 256, 8192)), dim3(256), 0, S_(stream), B, P, L, D,
                       (const bf16_t*)prefix, prefix_bstride, (const bf16_t*)wte, (const bf16_t*)wpe, ids, (bf16_t*)x,
                       thr, ik, seed, seed_ptr, offset, seq_off, seq_len);
  else
    hipLaunchKernelGGL(gpt2_embed_kernel<float>, dim3(nblk(n, 256, 8192)), dim3(256), 0, S_(stream), B, P, L, D,
                       (const float*)prefix, prefix_bstride, (const float*)wte, (const float*)wpe, ids, (float*)x,
                       thr, ik, seed, seed_ptr, offset, seq_off, seq_len);
  return check_launch("icap_gpt2_embed");
}

extern "C" int icap_caption_prep(int32_t B, int32_t P, int32_t L, const int64_t* mask, const int64_t* labels,
                                 int32_t* key_mask, int32_t* labels_shift, int32_t* n_valid, int32_t* row_slot,
                                 int32_t* labels_compact, void* stream) {
  ICAP_REQUIRE(B >= 0 && P >= 0 && L >= 0, "icap_caption_prep: bad geometry");
  ICAP_REQUIRE((int64_t)B * (P + L) < (1ll << 30), "icap_caption_prep: too many rows");
  ICAP_REQUIRE((row_slot == nullptr) == (labels_compact == nullptr), "icap_caption_prep: row_slot and labels_compact go together");
  hipLaunchKernelGGL(caption_prep_kernel, dim3(1), dim3(1024), 0, S_(stream), B, P, L, mask, labels, key_mask,
                     labels_shift, n_valid, row_slot, labels_compact);
  return check_launch("icap_caption_prep");
}

extern "C" int icap_caption_pack(int32_t B, int32_t P, int32_t L, const int64_t* mask, const int64_t* labels,
                                 int32_t* seq_off, int32_t* seq_len, int32_t* m_live, int32_t* key_mask,
                                 int32_t* labels_shift, int32_t* n_valid, int32_t* row_slot, int32_t* labels_compact,
                                 void* stream) {
  ICAP_REQUIRE(B >= 1 && P >= 0 && L >= 0, "icap_caption_pack: bad geometry");
  ICAP_REQUIRE((int64_t)B * (P + L) < (1ll << 30), "icap_caption_pack: too many rows");
  ICAP_REQUIRE(seq_off && seq_len && m_live && key_mask && labels_shift, "icap_caption_pack: null pointer");
  ICAP_REQUIRE((row_slot == nullptr) == (labels_compact == nullptr), "icap_caption_pack: row_slot and labels_compact go together");
  if (B <= PK2_MAX) {
    const int nb = (B + PK2_WAVES - 1) / PK2_WAVES;
    hipLaunchKernelGGL(caption_pack2_kernel, dim3(nb), dim3(1024), 0, S_(stream), B, P, L, mask, labels, seq_off,
                       seq_len, m_live, key_mask, labels_shift, n_valid, row_slot, labels_compact);
  } else {
    hipLaunchKernelGGL(caption_pack_kernel, dim3(1), dim3(1024), 0, S_(stream), B, P, L, mask, labels, seq_off,
                       seq_len, m_live, key_mask, labels_shift, n_valid, row_slot, labels_compact);
  }
  return check_launch("icap_caption_pack");
}

extern "C" int icap_rows_unpack(int32_t dtype, int32_t B, int32_t P, int32_t D, const void* src, const int32_t* seq_off,
                                const int32_t* seq_len, void* dst, int64_t dst_bstride, void* stream) {
  ICAP_REQUIRE(B >= 0 && P >= 0 && D > 0 && D % 4 == 0 && dst_bstride % 4 == 0, "icap_rows_unpack: bad geometry");
  ICAP_REQUIRE(src && seq_off && seq_len && dst, "icap_rows_unpack: null pointer");
  const int64_t n = (int64_t)B * P * (D / 4);
  if (n == 0) return ICAP_OK;
  if (dtype == ICAP_BF16)
    hipLaunchKernelGGL(rows_unpack_kernel<bf16_t>, dim3(nblk(n, 256, 4096)), dim3(256), 0, S_(stream), B, P, D,
                       (const bf16_t*)src, seq_off, seq_len, (bf16_t*)dst, dst_bstride);
  else
    hipLaunchKernelGGL(rows_unpack_kernel<float>, dim3(nblk(n, 256, 4096)), dim3(256), 0, S_(stream), B, P, D,
                       (const float*)src, seq_off, seq_len, (float*)dst, dst_bstride);
  return check_launch("icap_rows_unpack");
}

extern "C" size_t icap_cross_entropy_workspace_bytes(int64_t rows) {
  return (size_t)(rows > 0 ? rows : 1) * sizeof(float);
}

extern "C" int icap_cross_entropy(int32_t dtype, int64_t rows, int64_t V, const void* logits, int64_t ld,
                                  const int32_t* labels, const int32_t* n_valid, float* loss, void* dlogits,
                                  float grad_scale, void* workspace, const int32_t* rows_dev, void* stream) {
  ICAP_REQUIRE(logits && labels && n_valid && loss && workspace, "icap_cross_entropy: null pointer");
  ICAP_REQUIRE(V > 0 && ld >= V && ld % 4 == 0, "icap_cross_entropy: ld must be >= V and a multiple of 4");
  if (rows <= 0) return ICAP_OK;
  ICAP_REQUIRE(rows < (1ll << 31), "icap_cross_entropy: too many rows");
  float* lrows = reinterpret_cast<float*>(workspace);
  const bool reg = dtype == ICAP_BF16 && V <= 8 * 512 * 13 && ld % 8 == 0 &&
                   (reinterpret_cast<uintptr_t>(logits) & 15) == 0 &&
                   (dlogits == nullptr || (reinterpret_cast<uintptr_t>(dlogits) & 15) == 0);
  if (reg) {
    hipLaunchKernelGGL(ce_bf16_reg_kernel<13>, dim3((unsigned)rows), dim3(512), 0, S_(stream), V,
                       reinterpret_cast<const bf16_t*>(logits), ld, labels, n_valid, lrows,
                       reinterpret_cast<bf16_t*>(dlogits), grad_scale, rows_dev);
  } else {
    DISPATCH_T(dtype, hipLaunchKernelGGL(ce_kernel<T>, dim3((unsigned)rows), dim3(256), 0, S_(stream), V, CTP(logits),
                                         ld, labels, n_valid, lrows, TP(dlogits), grad_scale, rows_dev));
  }
  int rc = check_launch("icap_cross_entropy");
  if (rc) return rc;
  hipLaunchKernelGGL(ce_reduce_kernel, dim3(1), dim3(256), 0, S_(stream), rows, lrows, n_valid, loss, rows_dev);
  return check_launch("icap_cross_entropy(reduce)");
}

extern "C" size_t icap_adamw_workspace_bytes(int64_t n) {
  (void)n;
  return SQ_BLOCKS * sizeof(float);
}

static int sq_partials(int64_t n, const float* x, float* partial, hipStream_t s, int* nparts) {
  const int nb = (int)nblk(n / 4 + 1, 256, SQ_BLOCKS);
  hipLaunchKernelGGL(sqnorm_partial_kernel, dim3(nb), dim3(256), 0, s, n, x, partial);
  *nparts = nb;
  return check_launch("sqnorm");
}

extern "C" int icap_sqnorm(int64_t n, const float* x, float* out, void* workspace, void* stream) {
  ICAP_REQUIRE(x && out && workspace, "icap_sqnorm: null pointer");
  ICAP_REQUIRE((reinterpret_cast<uintptr_t>(x) & 15) == 0, "icap_sqnorm: x must be 16-byte aligned");
  int np = 0;
  float* partial = reinterpret_cast<float*>(workspace);
  int rc = sq_partials(n, x, partial, S_(stream), &np);
  if (rc) return rc;
  hipLaunchKernelGGL(adam_finalize_kernel, dim3(1), dim3(256), 0, S_(stream), np, partial, (AdamState*)nullptr, out,
                     0.f, 0.f, 0.f, 0.f, 0.f, (int64_t)0, (int64_t)0);
  return check_launch("icap_sqnorm");
}

extern "C" int icap_adamw_step(const icap_adamw_args* a, void* workspace, void* stream) {
  ICAP_REQUIRE(a && workspace, "icap_adamw_step: null args/workspace");
  ICAP_REQUIRE(a->params && a->grads && a->exp_avg && a->exp_avg_sq && a->state, "icap_adamw_step: null pointer");
  ICAP_REQUIRE(((reinterpret_cast<uintptr_t>(a->params) | reinterpret_cast<uintptr_t>(a->grads) |
                 reinterpret_cast<uintptr_t>(a->exp_avg) | reinterpret_cast<uintptr_t>(a->exp_avg_sq)) & 15) == 0,
               "icap_adamw_step: buffers must be 16-byte aligned");
  ICAP_REQUIRE(a->bf16_out == nullptr || (reinterpret_cast<uintptr_t>(a->bf16_out) & 7) == 0,
               "icap_adamw_step: bf16_out must be 8-byte aligned");
  if (a->n <= 0) return ICAP_OK;
  hipStream_t s = S_(stream);
  float* partial = reinterpret_cast<float*>(workspace);
  int np = 0;
  int rc = sq_partials(a->n, a->grads, partial, s, &np);
  if (rc) return rc;
  hipLaunchKernelGGL(adam_finalize_kernel, dim3(1), dim3(256), 0, s, np, partial, (AdamState*)a->state,
                     (float*)nullptr, a->lr, a->beta1, a->beta2, a->weight_decay, a->max_norm, a->num_warmup_steps,
                     a->num_training_steps);
  rc = check_launch("icap_adamw_step(finalize)");
  if (rc) return rc;
  hipLaunchKernelGGL(adam_update_kernel, dim3(nblk(a->n / 4 + 1, 256, 4096)), dim3(256), 0, s, a->n, a->params,
                     a->grads, a->exp_avg, a->exp_avg_sq, (bf16_t*)a->bf16_out, (const AdamState*)a->state, a->beta1,
                     a->beta2, a->eps);
  return check_launch("icap_adamw_step(update)");
}

extern "C" int icap_transpose(int32_t dtype, int64_t rows, int64_t cols, const void* src, int64_t lds, void* dst,
                              int64_t ldd, int64_t rows_pad, void* stream) {
  ICAP_REQUIRE(src && dst && rows_pad >= rows, "icap_transpose: bad args");
  if (rows_pad == 0 || cols == 0) return ICAP_OK;
  dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows_pad + 63) / 64));
  ICAP_REQUIRE(grid.y < 65536, "icap_transpose: too many rows");
  const bool vec = dtype == ICAP_BF16 && cols % 8 == 0 && lds % 8 == 0 && ldd % 8 == 0 && rows_pad % 64 == 0 &&
                   (reinterpret_cast<uintptr_t>(src) & 15) == 0 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0;
  if (vec)
    hipLaunchKernelGGL(transpose16_vec_kernel, grid, dim3(256), 0, S_(stream), rows, cols, (const uint16_t*)src, lds,
                       (uint16_t*)dst, ldd);
  else if (dtype == ICAP_BF16)
    hipLaunchKernelGGL(transpose_kernel<uint16_t>, grid, dim3(256), 0, S_(stream), rows, cols, (const uint16_t*)src,
                       lds, (uint16_t*)dst, ldd, rows_pad);
  else
    hipLaunchKernelGGL(transpose_kernel<uint32_t>, grid, dim3(256), 0, S_(stream), rows, cols, (const uint32_t*)src,
                       lds, (uint32_t*)dst, ldd, rows_pad);
  return check_launch("icap_transpose");
}

extern "C" int icap_transpose_batch(int32_t n, const icap_transpose_item* items, void* stream) {
  ICAP_REQUIRE(n >= 0 && (n == 0 || items), "icap_transpose_batch: bad args");
  for (int32_t i0 = 0; i0 < n; i0 += T16_BATCH) {
    const int m = n - i0 < T16_BATCH ? n - i0 : T16_BATCH;
    Transpose16Batch b;
    b.n = 0;
    b.off[0] = 0;
    for (int j = 0; j < m; ++j) {
      const icap_transpose_item& it = items[i0 + j];
      ICAP_REQUIRE(it.src && it.dst && it.rows >= 0 && it.cols >= 0, "icap_transpose_batch: bad item");
      if (it.rows == 0 || it.cols == 0) continue;
      const bool vec = it.cols % 8 == 0 && it.lds % 8 == 0 && it.ldd % 8 == 0 && it.rows % 64 == 0 &&
                       it.lds >= it.cols && it.ldd >= it.rows && (reinterpret_cast<uintptr_t>(it.src) & 15) == 0 &&
                       (reinterpret_cast<uintptr_t>(it.dst) & 15) == 0;
      if (!vec) {  // (the batched form is the 16-byte tile path only)
        const int rc = icap_transpose(ICAP_BF16, it.rows, it.cols, it.src, it.lds, it.dst, it.ldd, it.rows, stream);
        if (rc) return rc;
        continue;
      }
      const int k = b.n++;
      b.src[k] = static_cast<const uint16_t*>(it.src);
      b.dst[k] = static_cast<uint16_t*>(it.dst);
      b.rows[k] = it.rows; b.cols[k] = it.cols; b.lds[k] = it.lds; b.ldd[k] = it.ldd;
      b.off[k + 1] = b.off[k] + ((it.cols + 63) / 64) * (it.rows / 64);
    }
    if (b.n == 0) continue;
    ICAP_REQUIRE(b.off[b.n] < (1ll << 31), "icap_transpose_batch: too many tiles");
    hipLaunchKernelGGL(transpose16_batch_kernel, dim3((unsigned)b.off[b.n]), dim3(256), 0, S_(stream), b);
    const int rc = check_launch("icap_transpose_batch");
    if (rc) return rc;
  }
  return ICAP_OK;
}

static int64_t colsum_chunks(int64_t M) {
  int64_t c = (M + 31) / 32;
  if (c > 64) c = 64;
  if (c < 1) c = 1;
  return c;
}

extern "C" size_t icap_colsum_workspace_bytes(int64_t M, int64_t N) {
  return (size_t)colsum_chunks(M) * (size_t)(N > 0 ? N : 1) * sizeof(float);
}

extern "C" int icap_colsum(int32_t dtype, int64_t M, int64_t N, const void* src, int64_t ld, float* out,
                           int32_t accumulate, void* workspace, void* stream) {
  ICAP_REQUIRE(src && out && workspace, "icap_colsum: null pointer");
  if (N == 0) return ICAP_OK;
  const int64_t ch = colsum_chunks(M);
  const int64_t rpc = (M + ch - 1) / ch;
  float* partial = reinterpret_cast<float*>(workspace);
  const int es = dtype == ICAP_BF16 ? 2 : 4;
  if (N % 4 == 0 && ld % 4 == 0 && (reinterpret_cast<uintptr_t>(src) % (4 * es)) == 0) {
    dim3 grid4((unsigned)((N + 255) / 256), (unsigned)ch);
    DISPATCH_T(dtype, hipLaunchKernelGGL(colsum4_kernel<T>, grid4, dim3(256), 0, S_(stream), M, N, CTP(src), ld,
                                         rpc > 0 ? rpc : 1, partial));
  } else {
    dim3 grid((unsigned)((N + 63) / 64), (unsigned)ch);
    DISPATCH_T(dtype, hipLaunchKernelGGL(colsum_kernel<T>, grid, dim3(256), 0, S_(stream), M, N, CTP(src), ld,
                                         rpc > 0 ? rpc : 1, partial));
  }
  int rc = check_launch("icap_colsum");
  if (rc) return rc;
  hipLaunchKernelGGL(colsum_reduce_kernel, dim3((unsigned)((N + 63) / 64)), dim3(1024), 0, S_(stream), N, (int)ch,
                     partial, out, accumulate);
  return check_launch("icap_colsum(reduce)");
}

extern "C" int icap_colsum_batch(int32_t dtype, int64_t M, int32_t n, const icap_colsum_item* items,
                                 int32_t accumulate, void* workspace, void* stream) {
  ICAP_REQUIRE(n >= 0 && n <= ICAP_COLSUM_BATCH, "icap_colsum_batch: 0 <= n <= ICAP_COLSUM_BATCH");
  ICAP_REQUIRE(n == 0 || (items && workspace), "icap_colsum_batch: null pointer");
  ICAP_REQUIRE(M >= 0, "icap_colsum_batch: M < 0");
  const int es = dtype == ICAP_BF16 ? 2 : 4;
  ColsumBatch b{};
  b.n = 0;
  for (int i = 0; i < n; ++i) {
    const icap_colsum_item& it = items[i];
    ICAP_REQUIRE(it.src && it.out, "icap_colsum_batch: null item pointer");
    ICAP_REQUIRE(it.N >= 0 && it.N % 4 == 0 && it.ld % 4 == 0 && it.ld >= it.N &&
                     reinterpret_cast<uintptr_t>(it.src) % (4 * es) == 0,
                 "icap_colsum_batch: items need N % 4 == 0, ld % 4 == 0, ld >= N and a 4-element aligned src");
    if (it.N == 0) continue;
    const int k = b.n++;
    b.src[k] = it.src; b.ld[k] = it.ld; b.N[k] = it.N; b.out[k] = it.out;
    b.blk[k + 1] = b.blk[k] + (it.N + 255) / 256;
    b.base[k + 1] = b.base[k] + it.N;
  }
  if (b.n == 0) return ICAP_OK;
  const int64_t ch = colsum_chunks(M);
  const int64_t rpc = (M + ch - 1) / ch;
  float* partial = reinterpret_cast<float*>(workspace);
  DISPATCH_T(dtype, hipLaunchKernelGGL(colsum4_batch_kernel<T>, dim3((unsigned)b.blk[b.n], (unsigned)ch), dim3(256),
                                       0, S_(stream), b, M, rpc > 0 ? rpc : 1, partial));
  int rc = check_launch("icap_colsum_batch");
  if (rc) return rc;
  hipLaunchKernelGGL(colsum_reduce_batch_kernel, dim3((unsigned)((b.base[b.n] + 63) / 64)), dim3(1024), 0,
                     S_(stream), b, (int)ch, partial, accumulate);
  return check_launch("icap_colsum_batch(reduce)");
}

extern "C" int icap_dropout_apply(int32_t dtype, int64_t M, int64_t N, const void* src, int64_t lds, void* dst,
                                  int64_t ldd, float drop_p, uint64_t seed, uint64_t offset,
                                  const uint64_t* seed_ptr, void* stream) {
  ICAP_REQUIRE(src && dst && drop_p >= 0.f && drop_p < 1.f, "icap_dropout_apply: bad args");
  if (M * N == 0) return ICAP_OK;
  const uint32_t thr = drop_p > 0.f ? drop_threshold(drop_p) : 0u;
  const float ik = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  DISPATCH_T(dtype, hipLaunchKernelGGL((map2d_kernel<T, T>), dim3(nblk(M * N, 256, 8192)), dim3(256), 0, S_(stream),
                                       M, N, CTP(src), lds, TP(dst), ldd, thr, ik, seed, seed_ptr, offset));
  return check_launch("icap_dropout_apply");
}

extern "C" int icap_convert(int32_t src_dtype, int32_t dst_dtype, int64_t M, int64_t N, const void* src, int64_t lds,
                            void* dst, int64_t ldd, void* stream) {
  ICAP_REQUIRE(src && dst, "icap_convert: null pointer");
  if (M * N == 0) return ICAP_OK;
  const dim3 g(nblk(M * N, 256, 8192)), b(256);
  if (src_dtype == ICAP_F32 && dst_dtype == ICAP_BF16)
    hipLaunchKernelGGL((map2d_kernel<float, bf16_t>), g, b, 0, S_(stream), M, N, (const float*)src, lds, (bf16_t*)dst,
                       ldd, 0u, 1.f, (uint64_t)0, (const uint64_t*)nullptr, (uint64_t)0);
  else if (src_dtype == ICAP_BF16 && dst_dtype == ICAP_F32)
    hipLaunchKernelGGL((map2d_kernel<bf16_t, float>), g, b, 0, S_(stream), M, N, (const bf16_t*)src, lds, (float*)dst,
                       ldd, 0u, 1.f, (uint64_t)0, (const uint64_t*)nullptr, (uint64_t)0);
  else if (src_dtype == ICAP_F32 && dst_dtype == ICAP_F32)
    hipLaunchKernelGGL((map2d_kernel<float, float>), g, b, 0, S_(stream), M, N, (const float*)src, lds, (float*)dst,
                       ldd, 0u, 1.f, (uint64_t)0, (const uint64_t*)nullptr, (uint64_t)0);
  else if (src_dtype == ICAP_BF16 && dst_dtype == ICAP_BF16)
    hipLaunchKernelGGL((map2d_kernel<bf16_t, bf16_t>), g, b, 0, S_(stream), M, N, (const bf16_t*)src, lds,
                       (bf16_t*)dst, ldd, 0u, 1.f, (uint64_t)0, (const uint64_t*)nullptr, (uint64_t)0);
  else {
    set_error("icap_convert: bad dtype");
    return ICAP_ERR_ARG;
  }
  return check_launch("icap_convert");
}

extern "C" int icap_broadcast_rows(int32_t dtype, int32_t B, int64_t R, int64_t D, const float* src, void* dst,
                                   int64_t dst_bstride, void* stream) {
  ICAP_REQUIRE(src && dst, "icap_broadcast_rows: null pointer");
  if ((int64_t)B * R * D == 0) return ICAP_OK;
  DISPATCH_T(dtype, hipLaunchKernelGGL(broadcast_rows_kernel<T>, dim3(nblk((int64_t)B * R * D, 256, 8192)), dim3(256),
                                       0, S_(stream), B, R, D, src, TP(dst), dst_bstride));
  return check_launch("icap_broadcast_rows");
}

extern "C" int icap_im2col_patches(int32_t dtype, int32_t B, int32_t C, int32_t HW, int32_t patch, const float* pixels,
                                   void* patches, void* stream) {
  ICAP_REQUIRE(pixels && patches, "icap_im2col_patches: null pointer");
  ICAP_REQUIRE(patch > 0 && HW % patch == 0, "icap_im2col_patches: patch must divide HW");
  const int G = HW / patch;
  const int K = C * patch * patch, Kp = (K + 7) / 8 * 8;
  if (patch % 4 != 0 || Kp != K) {  // rows of Kp elements (zero pad) so the patch GEMM keeps K % 8 == 0
    const int64_t n = (int64_t)B * G * G * Kp;
    if (n == 0) return ICAP_OK;
    DISPATCH_T(dtype, hipLaunchKernelGGL(im2col_any_kernel<T>, dim3(nblk(n, 256, 8192)), dim3(256), 0, S_(stream), B,
                                         C, HW, patch, Kp, pixels, TP(patches)));
    return check_launch("icap_im2col_patches");
  }
  const int64_t n = (int64_t)B * G * G * C * patch * (patch / 4);
  if (n == 0) return ICAP_OK;
  DISPATCH_T(dtype, hipLaunchKernelGGL(im2col_kernel<T>, dim3(nblk(n, 256, 8192)), dim3(256), 0, S_(stream), B, C, HW,
                                       patch, pixels, TP(patches)));
  return check_launch("icap_im2col_patches");
}

extern "C" int icap_vit_embed(int32_t dtype, int32_t B, int32_t G2, int32_t D, const void* patch_emb, const float* cls,
                              const float* pos, void* x, void* stream) {
  ICAP_REQUIRE(patch_emb && cls && pos && x, "icap_vit_embed: null pointer");
  const int64_t n = (int64_t)B * (G2 + 1) * D;
  if (n == 0) return ICAP_OK;
  DISPATCH_T(dtype, hipLaunchKernelGGL(vit_embed_kernel<T>, dim3(nblk(n, 256, 8192)), dim3(256), 0, S_(stream), B, G2,
                                       1, D, CTP(patch_emb), cls, pos, TP(x)));
  return check_launch("icap_vit_embed");
}

extern "C" int icap_prefix_embed(int32_t dtype, int32_t B, int32_t G2, int32_t NP, int32_t D, const void* patch_emb,
                                 const float* prefix, const float* pos, void* x, void* stream) {
  ICAP_REQUIRE(patch_emb && prefix && x, "icap_prefix_embed: null pointer");
  ICAP_REQUIRE(B >= 0 && G2 >= 0 && NP >= 1 && D > 0, "icap_prefix_embed: bad geometry");
  const int64_t n = (int64_t)B * (G2 + NP) * D;
  if (n == 0) return ICAP_OK;
  DISPATCH_T(dtype, hipLaunchKernelGGL(vit_embed_kernel<T>, dim3(nblk(n, 256, 8192)), dim3(256), 0, S_(stream), B, G2,
                                       NP, D, CTP(patch_emb), prefix, pos, TP(x)));
  return check_launch("icap_prefix_embed");
}

// bf16 form: one thread per (row, q|k, head, 8-element chunk of the first half): two 16-byte loads (elements
// [8c, 8c + 8) and their partners + hd/2), 16-byte stores; the same per-element arithmetic as rope_patches_kernel
__global__ void rope_patches8_kernel(int B, int S, int NP, int H, int hd, bf16_t* __restrict__ qkv, int64_t ld,
                                     const float* __restrict__ cs, const float* __restrict__ sn) {
#pragma clang fp contract(off)
  const int half = hd >> 1, nc = half >> 3;
  const int P = S - NP;
  const int64_t total = (int64_t)B * P * 2 * H * nc;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % nc);
    int64_t r = i / nc;
    const int hq = (int)(r % (2 * H));
    r /= (2 * H);
    const int p = (int)(r % P);
    const int b = (int)(r / P);
    bf16_t* v = qkv + ((int64_t)b * S + NP + p) * ld + (int64_t)hq * hd + 8 * c;
    float x1[8], x2[8], cl[8], sl[8], ch[8], sh[8], o1[8], o2[8];
    io<bf16_t>::ld8(v, x1);
    io<bf16_t>::ld8(v + half, x2);
    const float* cp = cs + (int64_t)p * hd + 8 * c;
    const float* sp = sn + (int64_t)p * hd + 8 * c;
    io<float>::ld8(cp, cl);
    io<float>::ld8(sp, sl);
    io<float>::ld8(cp + half, ch);
    io<float>::ld8(sp + half, sh);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      o1[e] = x1[e] * cl[e] + (-x2[e]) * sl[e];
      o2[e] = x2[e] * ch[e] + x1[e] * sh[e];
    }
    io<bf16_t>::st8(v, o1);
    io<bf16_t>::st8(v + half, o2);
  }
}

extern "C" int icap_rope_patches(int32_t dtype, int32_t B, int32_t S, int32_t NP, int32_t H, int32_t hd, void* qkv,
                                 int64_t ld_qkv, const float* cos_t, const float* sin_t, void* stream) {
  ICAP_REQUIRE(qkv && cos_t && sin_t, "icap_rope_patches: null pointer");
  ICAP_REQUIRE(B >= 0 && S > NP && NP >= 0 && H > 0 && hd > 0 && hd % 2 == 0 && ld_qkv >= 2ll * H * hd,
               "icap_rope_patches: bad geometry");
  const int64_t n = (int64_t)B * (S - NP) * H * hd;
  if (n == 0) return ICAP_OK;
  if (dtype == ICAP_BF16 && hd % 16 == 0 && ld_qkv % 8 == 0 && (reinterpret_cast<uintptr_t>(qkv) & 15) == 0 &&
      (reinterpret_cast<uintptr_t>(cos_t) & 15) == 0 && (reinterpret_cast<uintptr_t>(sin_t) & 15) == 0) {
    const int64_t n8 = n / 8;  // one thread per 8 pairs
    hipLaunchKernelGGL(rope_patches8_kernel, dim3(nblk(n8, 256, 8192)), dim3(256), 0, S_(stream), B, S, NP, H, hd,
                       reinterpret_cast<bf16_t*>(qkv), ld_qkv, cos_t, sin_t);
    return check_launch("icap_rope_patches");
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(rope_patches_kernel<T>, dim3(nblk(n, 256, 8192)), dim3(256), 0, S_(stream), B,
                                       S, NP, H, hd, TP(qkv), ld_qkv, cos_t, sin_t));
  return check_launch("icap_rope_patches");
}

extern "C" int icap_l2norm_rows(int32_t dtype, int64_t rows, int64_t D, const void* x, int64_t ldx, float* out,
                                int64_t ldo, void* stream) {
  ICAP_REQUIRE(x && out, "icap_l2norm_rows: null pointer");
  if (rows == 0) return ICAP_OK;
  DISPATCH_T(dtype, hipLaunchKernelGGL(l2norm_kernel<T>, dim3((unsigned)((rows + 3) / 4)), dim3(256), 0, S_(stream),
                                       rows, D, CTP(x), ldx, out, ldo));
  return check_launch("icap_l2norm_rows");
}

extern "C" int icap_greedy_next(int32_t dtype, int32_t B, int64_t V, const void* logits, int64_t ld, int64_t eos,
                                const int64_t* forced, int32_t* finished, int64_t* tokens, int64_t ld_tokens, int32_t step, const void* wte,
                                const void* wpe, int32_t pos, int32_t D, void* x, void* stream) {
  ICAP_REQUIRE(logits && finished && tokens, "icap_greedy_next: null pointer");
  ICAP_REQUIRE(x == nullptr || (wte && wpe), "icap_greedy_next: x requires wte/wpe");
  if (B == 0) return ICAP_OK;
  const int es = dtype == ICAP_BF16 ? 2 : 4;
  const uintptr_t lp = reinterpret_cast<uintptr_t>(logits);
  const int vec = (es == 2 && ld % 8 == 0 && lp % 16 == 0) ? 2 : (ld % 4 == 0 && lp % (4 * es) == 0) ? 1 : 0;
  // split form when the next-token embedding row can hold the partials (8 bytes per split)
  const int64_t chunk = ((V + GSPLIT - 1) / GSPLIT + 7) / 8 * 8;
  if (x && (int64_t)D * es >= 8 * GSPLIT && (reinterpret_cast<uintptr_t>(x) & 7) == 0 && (D * es) % 8 == 0 &&
      V >= 8 * GSPLIT) {
    const int nsplit = (int)((V + chunk - 1) / chunk);
    DISPATCH_T(dtype, hipLaunchKernelGGL(greedy_part_kernel<T>, dim3((unsigned)nsplit, (unsigned)B), dim3(256), 0,
                                         S_(stream), V, CTP(logits), ld, chunk, TP(x), D, vec));
    DISPATCH_T(dtype, hipLaunchKernelGGL(greedy_finish_kernel<T>, dim3((unsigned)B), dim3(256), 0, S_(stream), V,
                                         nsplit, eos, forced, finished, tokens, ld_tokens, step, CTP(wte), CTP(wpe),
                                         pos, D, TP(x)));
    return check_launch("icap_greedy_next(split)");
  }
  DISPATCH_T(dtype, hipLaunchKernelGGL(greedy_next_kernel<T>, dim3((unsigned)B), dim3(1024), 0, S_(stream), V,
                                       CTP(logits), ld, eos, forced, finished, tokens, ld_tokens, step, CTP(wte), CTP(wpe),
                                       pos, D, TP(x), vec));
  return check_launch("icap_greedy_next");
}

extern "C" int icap_topp_sample(int32_t dtype, int32_t B, int64_t V, const void* logits, int64_t ld, float temperature,
                                float top_p, const int32_t* finished, uint64_t seed, const uint64_t* seed_ptr,
                                int32_t step, int64_t eos, int64_t* out, void* stream) {
  ICAP_REQUIRE(logits && out, "icap_topp_sample: null pointer");
  ICAP_REQUIRE(V > 0 && V <= 64 * 1024 && ld >= V, "icap_topp_sample: need 0 < V <= 65536 and ld >= V");
  ICAP_REQUIRE(temperature > 0.f, "icap_topp_sample: temperature must be > 0 (0 is the greedy branch)");
  if (B == 0) return ICAP_OK;
  if (V <= 100 * 512) {
    DISPATCH_T(dtype, hipLaunchKernelGGL((topp_sample_kernel<T, 100>), dim3((unsigned)B), dim3(512), 0, S_(stream), V,
                                         CTP(logits), ld, temperature, top_p, finished, seed, seed_ptr, step, eos, out));
  } else {
    DISPATCH_T(dtype, hipLaunchKernelGGL((topp_sample_kernel<T, 128>), dim3((unsigned)B), dim3(512), 0, S_(stream), V,
                                         CTP(logits), ld, temperature, top_p, finished, seed, seed_ptr, step, eos, out));
  }
  return check_launch("icap_topp_sample");
}

extern "C" int icap_add_position(int32_t dtype, int32_t B, int32_t npos, int32_t D, const void* src,
                                 int64_t src_bstride, int64_t src_tstride, const void* wpe, int32_t pos0, void* x,
                                 void* stream) {
  ICAP_REQUIRE(src && wpe && x, "icap_add_position: null pointer");
  const int64_t n = (int64_t)npos * B * D;
  if (n == 0) return ICAP_OK;
  DISPATCH_T(dtype, hipLaunchKernelGGL(add_position_kernel<T>, dim3(nblk(n, 256, 8192)), dim3(256), 0, S_(stream), B,
                                       npos, D, CTP(src), src_bstride, src_tstride, CTP(wpe), pos0, TP(x)));
  return check_launch("icap_add_position");
}

extern "C" int icap_counter_increment(uint64_t* counter, void* stream) {
  ICAP_REQUIRE(counter, "icap_counter_increment: null pointer");
  hipLaunchKernelGGL(counter_inc_kernel, dim3(1), dim3(64), 0, S_(stream), counter);
  return check_launch("icap_counter_increment");
}

extern "C" int icap_embedding_scatter_add(int32_t dtype, int32_t B, int32_t P, int32_t L, int32_t D, const void* dx,
                                          const int64_t* ids, float* dwte, void* stream) {
  ICAP_REQUIRE(dx && ids && dwte, "icap_embedding_scatter_add: null pointer");
  const int64_t n = (int64_t)B * L * D;
  if (n == 0) return ICAP_OK;
  DISPATCH_T(dtype, hipLaunchKernelGGL(embed_scatter_kernel<T>, dim3(nblk(n, 256, 8192)), dim3(256), 0, S_(stream), B,
                                       P, L, D, CTP(dx), ids, dwte));
  return check_launch("icap_embedding_scatter_add");
}

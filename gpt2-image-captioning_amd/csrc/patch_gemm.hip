// Patch embedding as one GEMM that gathers its A operand from the pixel tensor (no im2col buffer).
//
// Reference: the ViT patch Conv2d (stride = kernel = p) of HF CLIP (modeling_clip.py:148-154,209-217: no bias, then
// [CLS || patches] + position embedding), ViT (modeling_vit.py: bias, CLS, positions) and DINOv3
// (modeling_dinov3_vit.py:75-92: bias, [CLS || registers || patches], no absolute positions), reached through
// src/embeddings/clip.py:132, vit.py:120, dino.py:166.
//
// out[b*S + NP + p][n] = sum_k pixel(b, p, k) W[n][k] (+ bias[n]) (+ pos[NP + p][n])     (patch rows)
// out[b*S + r][n]      = prefix[r][n] (+ pos[r][n])                                       (r < NP: CLS, registers)
// with k = (c, ky, kx) in the Conv2d weight's own order, S = NP + G^2.
//
// Before round 5 the bf16 path wrote the [B G^2, C p p] patch matrix (icap_im2col_patches: 77 MB of fp32 pixels read
// and 38.5 MB of bf16 patches written at B = 128) and a second launch (icap_vit_embed) added the CLS / position rows.
// Here each 128 x 128 output tile stages its 64-deep K slices through LDS itself: the weights [N][Kp] bf16 as 16-byte
// chunks, the pixels fp32 as 8-element runs of one pixel row (p % 8 == 0: two 16-byte loads per run, converted to
// one 16-byte bf16 chunk; otherwise per element) — both into the XOR-swizzled 128-byte LDS rows the tile GEMM uses
// (cdna_hip_programming.md §5.5 T2), register-staged (loads for slice k+1 issued before the MFMAs of slice k, written
// to the other LDS buffer after them: T14). 4 waves of 64 x 64 (16x16x32 bf16 MFMA), accumulators staged through
// LDS in the epilogue so every store is 16 bytes, bias / position added in fp32 and rounded once.
#include "gemm_common.h"

namespace icap {

struct PatchArgs {
  int B, C, HW, p, G, G2, NP, S, N, K, Kp;
  float inv_p, inv_pp;    // 1 / p, 1 / p^2 (k -> (c, ky, kx) without integer division: exact for k < 2^20)
  const float* px;        // [B, C, HW, HW] fp32
  const bf16_t* w;        // [N][ldw] bf16, columns k >= K zero
  int64_t ldw;
  const float* bias;      // [N] or null
  const float* pos;       // [S][N] fp32 or null
  const float* prefix;    // [NP][N] fp32 (NP > 0)
  bf16_t* out;            // [B*S][ldo]
  int64_t ldo;
};

constexpr int PG_BK = 64;          // K per LDS slice (one 128-byte bf16 row)
constexpr int PG_STB = 2 * 128 * GROWB;  // bytes per slice: A 128 rows + B 128 rows

// RUN: 8 = p % 8 == 0 (an 8-element K chunk is one 32-byte pixel run: two 16-byte loads), 2 = p even (four 8-byte
// pixel pairs, each inside one pixel row), 1 = per element
template <int RUN>
__global__ __launch_bounds__(256, 2) void patch_gemm_kernel(PatchArgs a) {
  constexpr bool RUN8 = RUN == 8;
  __shared__ __attribute__((aligned(16))) char smem[2 * PG_STB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;
  const int64_t M = (int64_t)a.B * a.G2;
  const int tiles_n = (a.N + 127) / 128;
  const int nwg = gridDim.x;
  // XCD-aware bijective remap (T1): the blocks of one XCD take consecutive tiles, i.e. the column tiles of one patch
  // row panel, whose pixel slices they then share in that XCD's L2
  const int bid = blockIdx.x, xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tm = wgid / tiles_n, tn = wgid - tm * tiles_n;
  const int64_t m0 = (int64_t)tm * 128;
  const int n0 = tn * 128;

  // this thread's staging chunks: chunk c = j * 256 + tid (j < 4) -> tile row c >> 3, K chunk tid & 7 (8 elements).
  // Buffer loads, branch-free: rows past M / N and K past K (pixels) / Kp (weights) get an offset beyond the
  // descriptor's range, which the hardware answers with zeros. The pixel descriptor starts at the tile's first image
  // (a tile spans <= 128 / G^2 + 2 images), so 32-bit byte offsets suffice for any batch.
  const int kc = tid & 7;
  const int HW2 = a.HW * a.HW, pp = a.p * a.p;
  const int64_t img = (int64_t)a.C * HW2;  // pixels per image
  const int64_t b_first = m0 / a.G2;
  const int64_t px_left = ((int64_t)a.B - b_first) * img * 4;
  const __amdgpu_buffer_rsrc_t rpx = make_rsrc(a.px + b_first * img, (uint64_t)px_left);
  uint32_t rowoff[4];  // byte offset (from the tile's first image) of patch (b, py, px) of the A rows staged here
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t m = m0 + j * 32 + (tid >> 3);
    if (m < M) {
      const int b = (int)(m / a.G2), pi = (int)(m - (int64_t)b * a.G2);
      const int py = pi / a.G, pxi = pi - py * a.G;
      rowoff[j] = (uint32_t)(((b - b_first) * img + (int64_t)py * a.p * a.HW + pxi * a.p) * 4);
    } else {
      rowoff[j] = OOB;
    }
  }
  const int nrows = a.N - n0 < 128 ? a.N - n0 : 128;
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(a.w + (int64_t)n0 * a.ldw, (uint64_t)((nrows - 1) * a.ldw + a.Kp) * 2);
  uint32_t woff[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = j * 32 + (tid >> 3);
    woff[j] = n < nrows ? (uint32_t)(n * a.ldw * 2) : OOB;
  }

  // A slice in registers, raw: 4 rows x 8 fp32 pixels and 4 rows x one 16-byte bf16 weight chunk per thread. Two
  // sets (even / odd slices): the loads of slice k + 2 are issued in iteration k, right after slice k + 1 left its set
  // for LDS, so each load has two slices of MFMAs to land (round 5: with one set, issued one slice ahead, every
  // k-step waited out an HBM round trip — 172 us for the CLIP-B/32 embed at B = 128, profiles/r05_kstats_*.txt).
  struct Raw {
    float v[4][8];
    uint4 b[4];
  };
  auto load_raw = [&](int kt, Raw& r) __attribute__((always_inline)) {
    const int k0 = kt * PG_BK + kc * 8;
#pragma unroll
    for (int j = 0; j < 4; ++j) r.b[j] = bload(rw, k0 < a.Kp ? woff[j] + (uint32_t)k0 * 2 : OOB);
    if constexpr (RUN8) {  // p % 8 == 0, HW % 8 == 0, K % 8 == 0: the 8 elements are one 32-byte pixel run
      const bool kin = k0 < a.K;
      const int cc = k0 / pp, rem = k0 - cc * pp, ky = rem / a.p, kx = rem - ky * a.p;
      const uint32_t koff = (uint32_t)(((int64_t)cc * HW2 + (int64_t)ky * a.HW + kx) * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t o = (kin && rowoff[j] != OOB) ? rowoff[j] + koff : OOB;
        const uint4 lo = bload(rpx, o), hi = bload(rpx, o == OOB ? OOB : o + 16);
        r.v[j][0] = __uint_as_float(lo.x), r.v[j][1] = __uint_as_float(lo.y);
        r.v[j][2] = __uint_as_float(lo.z), r.v[j][3] = __uint_as_float(lo.w);
        r.v[j][4] = __uint_as_float(hi.x), r.v[j][5] = __uint_as_float(hi.y);
        r.v[j][6] = __uint_as_float(hi.z), r.v[j][7] = __uint_as_float(hi.w);
      }
    } else if constexpr (RUN == 2) {  // even p (ViT-L/14): 4 pixel pairs, (kx, kx + 1) with kx even in one row
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const int k = k0 + e;
        const bool kin = k < a.K;
        const int cc = (int)(((float)k + 0.5f) * a.inv_pp), rem = k - cc * pp;
        const int ky = (int)(((float)rem + 0.5f) * a.inv_p), kx = rem - ky * a.p;
        const uint32_t koff = (uint32_t)(((int64_t)cc * HW2 + (int64_t)ky * a.HW + kx) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint2 w = __builtin_bit_cast(uint2, __builtin_amdgcn_raw_buffer_load_b64(
                                                        rpx, (kin && rowoff[j] != OOB) ? rowoff[j] + koff : OOB, 0, 0));
          r.v[j][e] = __uint_as_float(w.x);
          r.v[j][e + 1] = __uint_as_float(w.y);
        }
      }
    } else {  // general patch size: element by element, k >= K zero
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int k = k0 + e;
        const bool kin = k < a.K;
        const int cc = kin ? (int)(((float)k + 0.5f) * a.inv_pp) : 0, rem = k - cc * pp;
        const int ky = (int)(((float)rem + 0.5f) * a.inv_p), kx = rem - ky * a.p;
        const uint32_t koff = (uint32_t)(((int64_t)cc * HW2 + (int64_t)ky * a.HW + kx) * 4);
#pragma unroll
        for (int j = 0; j < 4; ++j)
          r.v[j][e] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                                                    rpx, (kin && rowoff[j] != OOB) ? rowoff[j] + koff : OOB, 0, 0));
      }
    }
  };
  auto store_raw = [&](const Raw& r, int s) __attribute__((always_inline)) {  // convert to bf16, into LDS buffer s
    char* As = smem + s * PG_STB;
    char* Bs = As + 128 * GROWB;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = j * 32 + (tid >> 3);
      *reinterpret_cast<uint4*>(As + lds_off(row, kc)) =
          make_uint4(f2bf2(r.v[j][0], r.v[j][1]), f2bf2(r.v[j][2], r.v[j][3]), f2bf2(r.v[j][4], r.v[j][5]),
                     f2bf2(r.v[j][6], r.v[j][7]));
      *reinterpret_cast<uint4*>(Bs + lds_off(row, kc)) = r.b[j];
    }
  };

  f32x4_t acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = (f32x4_t){0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int cur) __attribute__((always_inline)) {
    const char* As = smem + cur * PG_STB;
    const char* Bs = As + 128 * GROWB;
    uint4 af[2][4], bfr[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int ch = ks * 4 + fg;
#pragma unroll
      for (int i = 0; i < 4; ++i) af[ks][i] = *reinterpret_cast<const uint4*>(As + lds_off(wm * 64 + i * 16 + fr, ch));
#pragma unroll
      for (int j = 0; j < 4; ++j) bfr[ks][j] = *reinterpret_cast<const uint4*>(Bs + lds_off(wn * 64 + j * 16 + fr, ch));
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) mfma_chunk<bf16_t>(acc[i][j], af[ks][i], bfr[ks][j]);
  };

  // K slices, rounded up to an even count: every iteration then issues, stores and loads unconditionally (slices past
  // Kp load zeros through the range check). A conditional load made hipcc's wait counting assume the newest loads
  // could be the ones a store needs, and wait for all of them (vmcnt(0)) in every iteration.
  const int nk = ((a.Kp + PG_BK - 1) / PG_BK + 1) & ~1;
  Raw r0, r1;  // slices 0, 2, 4, ... in r0; 1, 3, 5, ... in r1
  load_raw(0, r0);
  load_raw(1, r1);
  store_raw(r0, 0);
  load_raw(2, r0);
  __syncthreads();
  // iteration kt: MFMAs on LDS buffer kt & 1; slice kt + 1 (in its register set since iteration kt - 2) into the
  // other buffer, which every wave finished reading before the previous barrier; slice kt + 3 loaded into that set
  auto iter = [&](int kt, Raw& nxt) __attribute__((always_inline)) {
    compute(kt & 1);
    store_raw(nxt, (kt & 1) ^ 1);
    load_raw(kt + 3, nxt);
    __syncthreads();
  };
  for (int kt = 0; kt < nk; kt += 2) {
    iter(kt, r1);
    iter(kt + 1, r0);
  }

  // prefix rows (CLS / registers): the blocks of the first row panel write them for their columns
  if (tm == 0) {
    const int rows = a.B * a.NP;
    for (int idx = tid; idx < rows * 16; idx += 256) {
      const int rr = idx >> 4, c8 = (idx & 15) * 8;
      const int b = rr / a.NP, t = rr - b * a.NP;
      const int n = n0 + c8;
      if (n + 8 <= a.N) {
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          v[e] = a.prefix[(int64_t)t * a.N + n + e] + (a.pos ? a.pos[(int64_t)t * a.N + n + e] : 0.f);
        io<bf16_t>::st8(a.out + ((int64_t)b * a.S + t) * a.ldo + n, v);
      } else {
        for (int e = 0; e < 8 && n + e < a.N; ++e)
          io<bf16_t>::st(a.out + ((int64_t)b * a.S + t) * a.ldo + n + e,
                         a.prefix[(int64_t)t * a.N + n + e] + (a.pos ? a.pos[(int64_t)t * a.N + n + e] : 0.f));
      }
    }
  }

  // epilogue: each wave stages 32 of its 64 accumulator rows at a time through LDS (the stage buffers are free after
  // the loop's last barrier), then every lane stores 8 consecutive columns of one row (16 bytes)
  constexpr int ELD = 64 + 4;
  float* cs = reinterpret_cast<float*>(smem) + wave * (32 * ELD);
  const int er = lane >> 3, ec = (lane & 7) * 8;
  const int col = n0 + wn * 64 + ec;
  float bw[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bw[e] = (a.bias && col + e < a.N) ? a.bias[col + e] : 0.f;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii)
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) cs[(ii * 16 + fg * 4 + v) * ELD + j * 16 + fr] = acc[2 * h + ii][j][v];
    __syncthreads();
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int lr = t * 8 + er;
      const int64_t m = m0 + wm * 64 + h * 32 + lr;
      if (m < M) {
        const int b = (int)(m / a.G2), pi = (int)(m - (int64_t)b * a.G2);
        const int64_t orow = (int64_t)b * a.S + a.NP + pi;
        float x[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) x[e] = cs[lr * ELD + ec + e] + bw[e];
        if (a.pos) {
          const float* pr = a.pos + (int64_t)(a.NP + pi) * a.N + col;
#pragma unroll
          for (int e = 0; e < 8; ++e) x[e] += (col + e < a.N) ? pr[e] : 0.f;
        }
        if (col + 8 <= a.N) {
          io<bf16_t>::st8(a.out + orow * a.ldo + col, x);
        } else {
          for (int e = 0; e < 8 && col + e < a.N; ++e) io<bf16_t>::st(a.out + orow * a.ldo + col + e, x[e]);
        }
      }
    }
    __syncthreads();
  }
}

}  // namespace icap

using namespace icap;

extern "C" int icap_patch_embed(int32_t B, int32_t C, int32_t HW, int32_t patch, int32_t NP, int32_t N,
                                const float* pixels, const void* w, int64_t ldw, int32_t Kp, const float* bias,
                                const float* pos, const float* prefix, void* out, int64_t ldo, void* stream) {
  ICAP_REQUIRE(pixels && w && out, "icap_patch_embed: null pointer");
  ICAP_REQUIRE(B >= 0 && C >= 1 && patch >= 1 && HW >= patch && HW % patch == 0 && N >= 1 && NP >= 0,
               "icap_patch_embed: bad geometry (HW must be a multiple of patch)");
  const int K = C * patch * patch;
  ICAP_REQUIRE(Kp >= K && Kp % 8 == 0 && ldw >= Kp && ldw % 8 == 0 && ldo >= N && ldo % 8 == 0,
               "icap_patch_embed: Kp >= C p p, Kp / ldw / ldo multiples of 8");
  ICAP_REQUIRE((reinterpret_cast<uintptr_t>(w) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(pixels) & 15) == 0,
               "icap_patch_embed: pixels, w and out must be 16-byte aligned");
  ICAP_REQUIRE(NP == 0 || prefix != nullptr, "icap_patch_embed: NP > 0 needs prefix rows");
  ICAP_REQUIRE((int64_t)B * C * HW * HW < (1ll << 40), "icap_patch_embed: too many pixels");
  if (B == 0) return ICAP_OK;
  PatchArgs a;
  a.B = B, a.C = C, a.HW = HW, a.p = patch, a.G = HW / patch, a.G2 = a.G * a.G, a.NP = NP, a.S = NP + a.G2;
  a.N = N, a.K = K, a.Kp = Kp, a.px = pixels, a.w = reinterpret_cast<const bf16_t*>(w), a.ldw = ldw;
  a.bias = bias, a.pos = pos, a.prefix = prefix, a.out = reinterpret_cast<bf16_t*>(out), a.ldo = ldo;
  const int64_t M = (int64_t)B * a.G2;
  const int64_t tiles = ((M + 127) / 128) * ((N + 127) / 128);
  ICAP_REQUIRE(tiles < (1ll << 30), "icap_patch_embed: too many tiles");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  a.inv_p = 1.f / (float)patch, a.inv_pp = 1.f / (float)(patch * patch);
  ICAP_REQUIRE(K < (1 << 20), "icap_patch_embed: C p p must stay below 2^20");
  if (patch % 8 == 0 && HW % 8 == 0) hipLaunchKernelGGL(patch_gemm_kernel<8>, dim3((unsigned)tiles), dim3(256), 0, s, a);
  else if (patch % 2 == 0) hipLaunchKernelGGL(patch_gemm_kernel<2>, dim3((unsigned)tiles), dim3(256), 0, s, a);
  else hipLaunchKernelGGL(patch_gemm_kernel<1>, dim3((unsigned)tiles), dim3(256), 0, s, a);
  return check_launch("icap_patch_embed");
}

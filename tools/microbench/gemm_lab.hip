// GEMM main-loop lab (round 6): C[M,N] = A[M,K] . B[N,K]^T, bf16 operands, fp32 accumulate, bf16 C, on the
// packed train step's shapes. Three main-loop structures on the same tiles, LDS-DMA ring of NST stages, one barrier
// per 64-deep k-step, fragments of the next 32-deep substep read during the current substep's MFMAs:
//   MODE 0 (burst): 4 waves; each k-step's DMA for stage k+NST-1 issued as a burst after the barrier
//   MODE 1 (inter): 4 waves; the same DMA pieces spread between the first substep's MFMAs
//   MODE 2 (roles): 8 waves; waves 0-3 only read fragments and issue MFMAs (one per SIMD), waves 4-7 only issue the
//                   DMA and wait for it (one per SIMD), so the DMA issue cost sits beside the MFMA stream
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 gemm_lab.hip -o gemm_lab ; run: ./gemm_lab
#include <hip/hip_runtime.h>

#include <cmath>
#include <utility>
#include <cstring>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint16_t bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_u(const void* base, uint64_t bytes) {
  const uint64_t b = reinterpret_cast<uint64_t>(base);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)b);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(b >> 32));
  const uint32_t n = __builtin_amdgcn_readfirstlane(bytes > 0x7fffffffull ? 0x7fffffffu : (uint32_t)bytes);
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, (int)n,
                                           0x00020000);
}
// lds: the LDS byte address (an integer: a generic pointer of value 0 would be cast to the LDS null, -1)
__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff, uint32_t soff) {
  typedef __attribute__((address_space(3))) void* lds_ptr_t;
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)(uintptr_t)lds, 16, voff, soff, 0, 0);
}
template <int OFF>
__device__ __forceinline__ void ldsr(u32x4& d, uint32_t a) {
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(d) : "v"(a), "n"(OFF));
}
template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// wait until at most c * P of this wave's DMA instructions are outstanding (c = 0 .. 3)
template <int P>
__device__ __forceinline__ void wait_vm_stages(int c) {
  if (c >= 3) wait_vm<3 * P>();
  else if (c == 2) wait_vm<2 * P>();
  else if (c == 1) wait_vm<P>();
  else wait_vm<0>();
}
__device__ __forceinline__ void mfma(f32x4& acc, const u32x4& a, const u32x4& b) {
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0,
                                                0, 0);
}

template <int TM, int TN, int NST, int MODE>
__global__ __launch_bounds__(MODE == 2 ? 512 : 256, 1) void lab_kernel(const bf16* __restrict__ A,
                                                                       const bf16* __restrict__ B, bf16* __restrict__ C,
                                                                       int M, int N, int K) {
  constexpr int BM = 32 * TM, BN = 32 * TN;
  constexpr int STB = (BM + BN) * 128;
  constexpr int P = TM + TN;  // DMA pieces (1 KiB) per loading wave per stage: (BM + BN) / 8 pieces over 4 waves
  constexpr int LDC = BN + 8;
  static_assert(NST * STB <= 160 * 1024, "LDS");
  static_assert(BM * LDC * 2 <= NST * STB, "epilogue tile");
  static_assert(NST - 2 <= 3 && 3 * P < 64, "vmcnt");
  __shared__ __attribute__((aligned(16))) char smem[NST * STB];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tiles_n = N / BN;
  const int nwg = (M / BM) * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int tm = wgid / tiles_n, tn = wgid - tm * tiles_n;
  const bf16* Ab = A + (size_t)tm * BM * K;
  const bf16* Bb = B + (size_t)tn * BN * K;
  const __amdgpu_buffer_rsrc_t ra = rsrc_u(Ab, (uint64_t)BM * K * 2);
  const __amdgpu_buffer_rsrc_t rb = rsrc_u(Bb, (uint64_t)BN * K * 2);
  const int nk = K / 64;
  const bool is_loader = MODE == 2 ? wave >= 4 : true;
  const bool is_mfma = MODE == 2 ? wave < 4 : true;
  const int lw = MODE == 2 ? (wave & 3) : wave;
  // piece i of loader lw = stack piece q = i * 4 + lw (A pieces: i < TM): rows 8 q .. 8 q + 7 of [A tile; B tile];
  // lane l -> row 8 q + (l >> 3), physical chunk l & 7 holding logical K chunk (l & 7) ^ (row & 7)
  uint32_t voff[P];
#pragma unroll
  for (int i = 0; i < P; ++i) {
    const int qq = i * 4 + lw;
    const int row = (i < TM ? qq : qq - BM / 8) * 8 + (lane >> 3);
    voff[i] = (uint32_t)(row * K + (((lane & 7) ^ (lane >> 3)) * 8)) * 2;
  }
  const uint32_t sbase = (uint32_t)reinterpret_cast<uintptr_t>(smem);
  auto issue_piece = [&](int i, int kt, int slot) __attribute__((always_inline)) {
    // stages past K load nothing (offset beyond num_records): the loop issues every stage unconditionally
    const uint32_t soff = __builtin_amdgcn_readfirstlane(kt < nk ? (uint32_t)kt * 128u : 0x80000000u);
    // (the LDS base goes to M0: readfirstlane so hipcc sees it wave-uniform and emits no waterfall loop)
    const uint32_t lds = __builtin_amdgcn_readfirstlane(sbase + (uint32_t)(slot * STB + (i * 4 + lw) * 1024));
    dma16s(i < TM ? ra : rb, lds, voff[i], soff);
  };
  auto issue_stage = [&](int kt, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < P; ++i) issue_piece(i, kt, slot);
  };

  // consumer state
  const int wm = (wave & 3) >> 1, wn = wave & 1;
  const int fr = lane & 15, fg = lane >> 4;
  uint32_t la[2], lb[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    const uint32_t sw = (uint32_t)(((ks * 4 + fg) ^ (fr & 7)) << 4);
    la[ks] = (uint32_t)((wm * 16 * TM + fr) * 128) + sw;
    lb[ks] = (uint32_t)((wn * 16 * TN + fr) * 128) + sw;
  }
  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  u32x4 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
  auto read0 = [&](int slot) __attribute__((always_inline)) {
    const uint32_t a = sbase + (uint32_t)(slot * STB) + la[0], b = sbase + (uint32_t)(slot * STB) + lb[0];
    [&]<int... I>(std::integer_sequence<int, I...>) { (ldsr<I * 2048>(fa0[I], a), ...); }(std::make_integer_sequence<int, TM>{});
    [&]<int... J>(std::integer_sequence<int, J...>) { (ldsr<BM * 128 + J * 2048>(fb0[J], b), ...); }(std::make_integer_sequence<int, TN>{});
  };
  auto read1 = [&](int slot) __attribute__((always_inline)) {
    const uint32_t a = sbase + (uint32_t)(slot * STB) + la[1], b = sbase + (uint32_t)(slot * STB) + lb[1];
    [&]<int... I>(std::integer_sequence<int, I...>) { (ldsr<I * 2048>(fa1[I], a), ...); }(std::make_integer_sequence<int, TM>{});
    [&]<int... J>(std::integer_sequence<int, J...>) { (ldsr<BM * 128 + J * 2048>(fb1[J], b), ...); }(std::make_integer_sequence<int, TN>{});
  };
  auto wait0 = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(fa0[i]));
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(fb0[j]));
    __builtin_amdgcn_sched_barrier(0);
  };
  auto wait1 = [&]() __attribute__((always_inline)) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < TM; ++i) asm volatile("" : "+v"(fa1[i]));
#pragma unroll
    for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(fb1[j]));
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mfmas0 = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) mfma(acc[i][j], fa0[i], fb0[j]);
  };
  auto mfmas1 = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) mfma(acc[i][j], fa1[i], fb1[j]);
  };
  // MFMAs of substep 0 with the P pieces of stage kt spread between them (MODE 1): one piece after every
  // (TM TN) / P MFMAs, the order pinned by sched_barrier
  auto mfmas0_inter = [&](int kt, int slot) __attribute__((always_inline)) {
    constexpr int NM = TM * TN;
#pragma unroll
    for (int m = 0; m < NM; ++m) {
      mfma(acc[m / TN][m % TN], fa0[m / TN], fb0[m % TN]);
      if ((m * P) / NM != ((m + 1) * P) / NM) issue_piece((m * P) / NM, kt, slot);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  if constexpr (MODE == 2) {
    if (is_loader) {
      for (int s = 0; s < NST - 1; ++s) issue_stage(s, s);
      wait_vm<(NST - 2) * P>();
      __builtin_amdgcn_s_barrier();
      for (int kt = 0; kt < nk; ++kt) {
        issue_stage(kt + NST - 1, (kt + NST - 1) % NST);
        wait_vm<(NST - 2) * P>();  // stage kt + 1 landed
        __builtin_amdgcn_s_barrier();
      }
    } else {
      __builtin_amdgcn_s_barrier();
      read0(0);
      for (int kt = 0; kt < nk; ++kt) {
        const int slot = kt % NST;
        wait0();
        read1(slot);
        mfmas0();
        wait1();
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        if (kt + 1 < nk) read0((kt + 1) % NST);
        mfmas1();
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else {
    for (int s = 0; s < NST - 1; ++s) issue_stage(s, s);
    wait_vm<(NST - 2) * P>();
    __builtin_amdgcn_s_barrier();
    read0(0);
    for (int kt = 0; kt < nk; ++kt) {
      const int slot = kt % NST;
      const int nslot = (kt + NST - 1) % NST;
      wait0();
      read1(slot);
      if constexpr (MODE == 0) {
        issue_stage(kt + NST - 1, nslot);
        __builtin_amdgcn_sched_barrier(0);
        mfmas0();
      } else {
        mfmas0_inter(kt + NST - 1, nslot);
      }
      wait1();
      wait_vm<(NST - 2) * P>();  // stage kt + 1 landed
      __builtin_amdgcn_s_barrier();
      __builtin_amdgcn_sched_barrier(0);
      if (kt + 1 < nk) read0((kt + 1) % NST);
      mfmas1();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  (void)is_mfma;
  // epilogue (lab only): bf16 tile through LDS, 16-byte coalesced stores by every thread
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  bf16* ct = reinterpret_cast<bf16*>(smem);
  if (MODE != 2 || wave < 4) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int v = 0; v < 4; ++v) {
          const int row = wm * 16 * TM + i * 16 + 4 * fg + v, col = wn * 16 * TN + j * 16 + fr;
          ct[row * LDC + col] = __builtin_bit_cast(bf16, (__bf16)acc[i][j][v]);
        }
  }
  __syncthreads();
  constexpr int NT = MODE == 2 ? 512 : 256;
  constexpr int CPR = BN / 8;
  for (int c = tid; c < BM * CPR; c += NT) {
    const int row = c / CPR, cc = c - row * CPR;
    const uint4 v = *reinterpret_cast<const uint4*>(ct + row * LDC + cc * 8);
    *reinterpret_cast<uint4*>(C + (size_t)(tm * BM + row) * N + tn * BN + cc * 8) = v;
  }
}

__global__ void ref_kernel(const bf16* A, const bf16* B, float* C, int M, int N, int K) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x, row = blockIdx.y;
  if (col >= N) return;
  float s = 0.f;
  for (int k = 0; k < K; ++k)
    s += __uint_as_float((uint32_t)A[(size_t)row * K + k] << 16) * __uint_as_float((uint32_t)B[(size_t)col * K + k] << 16);
  C[(size_t)row * N + col] = s;
}

static uint64_t rng = 0x1234567887654321ull;
static bf16 rand_bf16() {
  rng = rng * 6364136223846793005ull + 1442695040888963407ull;
  const float f = (float)((rng >> 40) & 0xffffff) / (float)0x1000000 * 2.f - 1.f;  // [-1, 1)
  uint32_t u;
  memcpy(&u, &f, 4);
  return (bf16)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

typedef void (*kfn_t)(const bf16*, const bf16*, bf16*, int, int, int);
struct Variant {
  const char* name;
  kfn_t fn;
  int bm, bn, threads;
};

template <int TM, int TN, int NST, int MODE>
Variant mk(const char* name) {
  return Variant{name, (kfn_t)lab_kernel<TM, TN, NST, MODE>, 32 * TM, 32 * TN, MODE == 2 ? 512 : 256};
}

static float time_variant(const Variant& v, const bf16* A, const bf16* B, bf16* C, int M, int N, int K) {
  const dim3 grid((M / v.bm) * (N / v.bn)), block(v.threads);
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(v.fn, grid, block, 0, 0, A, B, C, M, N, K);
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  const int reps = 20;
  for (int t = 0; t < 7; ++t) {
    CHECK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(v.fn, grid, block, 0, 0, A, B, C, M, N, K);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  CHECK(hipGetLastError());
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return best * 1000.f / reps;
}

static void run_group(const char* title, std::vector<Variant> vs, int M, int N, std::vector<int> Ks) {
  printf("== %s: M %d N %d\n", title, M, N);
  for (int K : Ks) {
    std::vector<bf16> ha((size_t)M * K), hb((size_t)N * K);
    for (auto& x : ha) x = rand_bf16();
    for (auto& x : hb) x = rand_bf16();
    bf16 *A, *B, *C;
    float* R;
    CHECK(hipMalloc(&A, ha.size() * 2));
    CHECK(hipMalloc(&B, hb.size() * 2));
    CHECK(hipMalloc(&C, (size_t)M * N * 2));
    CHECK(hipMalloc(&R, (size_t)M * N * 4));
    CHECK(hipMemcpy(A, ha.data(), ha.size() * 2, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(B, hb.data(), hb.size() * 2, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(ref_kernel, dim3((N + 255) / 256, M), dim3(256), 0, 0, A, B, R, M, N, K);
    CHECK(hipDeviceSynchronize());
    std::vector<float> hr((size_t)M * N);
    CHECK(hipMemcpy(hr.data(), R, hr.size() * 4, hipMemcpyDeviceToHost));
    printf("  K %5d:", K);
    for (const Variant& v : vs) {
      CHECK(hipMemset(C, 0xff, (size_t)M * N * 2));
      const float us = time_variant(v, A, B, C, M, N, K);
      std::vector<bf16> hc((size_t)M * N);
      CHECK(hipMemcpy(hc.data(), C, hc.size() * 2, hipMemcpyDeviceToHost));
      double maxerr = 0.0;
      size_t bad = 0, nan = 0;
      int shown = 0;
      for (size_t e = 0; e < hc.size(); ++e) {
        const float c = __builtin_bit_cast(float, (uint32_t)hc[e] << 16);
        const double err = std::fabs((double)c - (double)hr[e]);
        const double tol = 0.02 * std::sqrt((double)K / 3.0) + 0.01 * std::fabs((double)hr[e]);
        if (!(err <= tol)) {
          ++bad;
          if (std::isnan(c)) ++nan;
          if (shown < 6 && K == Ks[0]) {
            printf("\n    bad (%zu, %zu): %g vs %g", e / N, e % N, c, hr[e]);
            ++shown;
          }
        }
        if (err > maxerr || std::isnan(err)) maxerr = err;
      }
      printf("  %s %7.2f us (%4.0f TF/s)%s", v.name, us, 2.0 * M * N * K / us / 1e6, bad ? " BAD" : "");
      if (bad) printf("[%zu (nan %zu) maxerr %.3g]", bad, nan, maxerr);
    }
    printf("\n");
    fflush(stdout);
    hipFree(A);
    hipFree(B);
    hipFree(C);
    hipFree(R);
  }
}

int main(int argc, char** argv) {
  const int which = argc > 1 ? atoi(argv[1]) : 0;
  if (which == 9) {
    run_group("check", {mk<4, 8, 3, 0>("burst"), mk<4, 8, 3, 2>("roles")}, 256, 512, {64, 128, 768});
    return 0;
  }
  if (which == 0 || which == 1)
    run_group("128x256 tiles (64x128 per MFMA wave), 3-stage ring",
              {mk<4, 8, 3, 0>("burst"), mk<4, 8, 3, 1>("inter"), mk<4, 8, 3, 2>("roles")}, 3584, 2304,
              {768, 1536, 3072, 6144});
  if (which == 0 || which == 2)
    run_group("128x96 tiles (64x48 per MFMA wave)",
              {mk<4, 3, 4, 0>("burst4"), mk<4, 3, 4, 1>("inter4"), mk<4, 3, 4, 2>("roles4"), mk<4, 3, 5, 2>("roles5"),
               mk<4, 3, 5, 1>("inter5")},
              3584, 768, {768, 2304, 3072});
  return 0;
}

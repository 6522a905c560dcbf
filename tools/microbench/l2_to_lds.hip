// Microbenchmark: L2-resident operand bytes moved into LDS per CU per clock, LDS-DMA (buffer_load ... lds)
// vs register staging (buffer_load_dwordx4 -> ds_write_b128), in the GEMM's 32 KiB-per-block-stage pattern.
// Build: hipcc --offload-arch=gfx950 -O3 l2_to_lds.hip -o l2_to_lds ; run: ./l2_to_lds
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int STAGE = 32768;  // bytes per block-stage (A + B tiles of a 128x128x64 bf16 k-step)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)n, 0x00020000);
}

template <int MODE>  // 0 = LDS-DMA, 1 = register staging
__global__ __launch_bounds__(256) void stream_kernel(const char* src, uint32_t span, int iters, float* sink) {
  __shared__ __attribute__((aligned(16))) char lds[STAGE];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  // each block walks its own 32 KiB-aligned window of the (L2-resident) source
  const uint32_t base = (uint32_t)((blockIdx.x * 7919u) % (span / STAGE)) * STAGE;
  const __amdgpu_buffer_rsrc_t r = rsrc(src, span);
  float acc = 0.f;
  for (int it = 0; it < iters; ++it) {
    const uint32_t off = (base + (uint32_t)it * STAGE) % span;
    if (MODE == 0) {
      typedef __attribute__((address_space(3))) void* lds_ptr_t;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        char* dst = lds + (wave * 8 + i) * 1024;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_ptr_t)dst, 16, off + (wave * 8 + i) * 1024 + lane * 16, 0, 0, 0);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      uint4 v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i)
        v[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off + (wave * 8 + i) * 1024 + lane * 16, 0, 0));
#pragma unroll
      for (int i = 0; i < 8; ++i) *reinterpret_cast<uint4*>(lds + (wave * 8 + i) * 1024 + lane * 16) = v[i];
    }
    __syncthreads();
    acc += __uint_as_float(*reinterpret_cast<const uint32_t*>(lds + ((threadIdx.x * 16 + it * 64) & (STAGE - 1))) & 0x3f800000u);
    __syncthreads();
  }
  if (acc == 12345.f) sink[0] = acc;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const uint32_t spans[2] = {4u << 20, 64u << 20};  // L2-resident per XCD / MALL-resident
  char* src;
  float* sink;
  hipMalloc(&src, 64u << 20);
  hipMemset(src, 1, 64u << 20);
  hipMalloc(&sink, 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 256;
  for (uint32_t span : spans)
    for (int bpc = 1; bpc <= 4; bpc *= 2)
      for (int mode = 0; mode < 2; ++mode) {
        const int blocks = cus * bpc;
        auto launch = [&]() {
          if (mode == 0) hipLaunchKernelGGL(stream_kernel<0>, dim3(blocks), dim3(256), 0, 0, src, span, iters, sink);
          else hipLaunchKernelGGL(stream_kernel<1>, dim3(blocks), dim3(256), 0, 0, src, span, iters, sink);
        };
        launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0.f;
        hipEventElapsedTime(&ms, e0, e1);
        const double bytes = 5.0 * blocks * (double)iters * STAGE;
        printf("span %3u MiB  blocks/CU %d  %-12s  %7.1f GB/s chip  %6.1f GB/s per CU\n", span >> 20, bpc,
               mode == 0 ? "LDS-DMA" : "reg+ds_write", bytes / ms / 1e6, bytes / ms / 1e6 / cus);
      }
  return 0;
}

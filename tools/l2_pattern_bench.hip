// Per-CU read rate of the skinny GEMM's operand access shapes (diagnostic, not part of the library).
// One 512-thread block per CU, every wave keeping NL 16-byte-per-lane loads in flight, summing them so nothing is
// dead code. Shapes (one wave-instruction = 1 KiB):
//   0: 16 rows x 64 B   (the skinny kernel's MFMA-fragment loads: lane = (row l&15, 16-B chunk l>>4))
//   1:  8 rows x 128 B  (lane = (row l>>3, chunk l&7))
//   2:  4 rows x 256 B
//   3:  1 row  x 1 KiB  (fully contiguous)
// Every block reads the same `rows x row_bytes` panel (L2-resident after the first touch: the decode GEMM's A) or,
// with distinct=1, its own panel (the W slabs).
// Build: hipcc --offload-arch=gfx950 -O3 tools/l2_pattern_bench.hip -o tools/l2_pattern_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

template <int SHAPE, int NL>
__global__ __launch_bounds__(512) void rd(const char* __restrict__ base, int64_t row_bytes, int rows, int distinct,
                                          float* __restrict__ sink, int rot) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const char* panel = base + (distinct ? (int64_t)blockIdx.x * rows * row_bytes : 0);
  constexpr int RPI = SHAPE == 0 ? 16 : SHAPE == 1 ? 8 : SHAPE == 2 ? 4 : 1;  // rows per instruction
  constexpr int CPR = 64 / RPI;                                              // 16-B chunks per row per instr
  const int r = lane / CPR, c = lane % CPR;
  const int64_t seg = CPR * 16;                    // bytes of one row per instruction
  const int64_t nseg = row_bytes / seg;            // segments along a row
  const int64_t ninstr = (rows / RPI) * nseg;      // instructions to cover the panel
  uint32_t acc = 0;
  for (int64_t i0 = wave; i0 < ninstr; i0 += 8 * NL) {
    uint4 v[NL];
#pragma unroll
    for (int u = 0; u < NL; ++u) {
      const int64_t i = i0 + 8 * u;
      if (i < ninstr) {
        // rot: each block starts its sweep at a different segment (spreads concurrent blocks over L2 channels)
        const int64_t sg0 = i % nseg, rg = i / nseg;
        const int64_t sg = rot ? (sg0 + (int64_t)blockIdx.x * rot) % nseg : sg0;
        v[u] = *reinterpret_cast<const uint4*>(panel + (rg * RPI + r) * row_bytes + sg * seg + c * 16);
      } else {
        v[u] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < NL; ++u) acc += v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) sink[blockIdx.x] = 1.f;
}

template <int SHAPE>
static float run(const char* buf, int64_t row_bytes, int rows, int distinct, int blocks, float* sink, int rot) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL((rd<SHAPE, 32>), dim3(blocks), dim3(512), 0, 0, buf, row_bytes, rows, distinct, sink, rot);
  const int reps = 50;
  hipEventRecord(e0);
  for (int w = 0; w < reps; ++w)
    hipLaunchKernelGGL((rd<SHAPE, 32>), dim3(blocks), dim3(512), 0, 0, buf, row_bytes, rows, distinct, sink, rot);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / reps;
}

int main() {
  const int blocks = 256;
  const int rows = 32;
  char* buf;
  float* sink;
  const int64_t maxb = (int64_t)blocks * rows * 6144;
  if (hipMalloc(&buf, maxb) != hipSuccess || hipMalloc(&sink, blocks * 4) != hipSuccess) return 1;
  hipMemset(buf, 1, maxb);
  printf("shape rows row_bytes distinct rot us/launch  KB/block  GB/s/CU\n");
  for (int distinct = 0; distinct < 2; ++distinct)
    for (int rot : {0, 1, 3})
    for (int64_t rb : {1536, 6144}) {
      for (int shape = 0; shape < 4; shape += 3) {
        float us = 0;
        switch (shape) {
          case 0: us = run<0>(buf, rb, rows, distinct, blocks, sink, rot); break;
          default: us = run<3>(buf, rb, rows, distinct, blocks, sink, rot); break;
        }
        const double kb = rows * rb / 1024.0;
        printf("%5d %4d %9lld %8d %3d %10.2f %9.1f %8.1f\n", shape, rows, (long long)rb, distinct, rot, us, kb,
               rows * rb / (us * 1e3));
      }
    }
  // empty-kernel floor
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  for (int w = 0; w < 50; ++w) hipLaunchKernelGGL((rd<0, 32>), dim3(blocks), dim3(512), 0, 0, buf, 0, 0, 0, sink, 0);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  printf("empty launch: %.2f us\n", ms * 1e3 / 50);
  return 0;
}

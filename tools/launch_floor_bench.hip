// Per-kernel cost floor on MI355X (diagnostic, not part of the library): back-to-back launches of an empty
// kernel captured in one HIP graph, for several grid / block shapes, and with a small store per block (a kernel
// that leaves dirty lines for the end-of-kernel release).
// Build: hipcc --offload-arch=gfx950 -O3 tools/launch_floor_bench.hip -o /tmp/lfb
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void empty_kernel(float* out, int store) {
  if (store && threadIdx.x == 0) out[blockIdx.x] = 1.f;
}

static float time_graph(int blocks, int threads, int store, float* out, int reps) {
  hipStream_t s;
  (void)hipStreamCreate(&s);
  hipGraph_t g;
  hipGraphExec_t ge;
  (void)hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(empty_kernel, dim3(blocks), dim3(threads), 0, s, out, store);
  (void)hipStreamEndCapture(s, &g);
  (void)hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  (void)hipGraphLaunch(ge, s);
  (void)hipStreamSynchronize(s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  (void)hipGraphLaunch(ge, s);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipGraphExecDestroy(ge);
  (void)hipGraphDestroy(g);
  (void)hipStreamDestroy(s);
  return ms * 1e3f / reps;
}

int main() {
  float* out;
  if (hipMalloc(&out, 1 << 20) != hipSuccess) return 1;
  printf("blocks threads store  us/kernel (graph of 200)\n");
  for (int store = 0; store < 2; ++store)
    for (int blocks : {1, 64, 256, 1024})
      for (int threads : {64, 256, 512, 1024})
        printf("%6d %7d %5d %10.2f\n", blocks, threads, store, time_graph(blocks, threads, store, out, 200));
  return 0;
}

// LDS poison: fills (up to) all of every CU's LDS with 0xFF bytes (NaN as fp32 and bf16), so a later kernel
// that reads LDS it never wrote sees NaN instead of the previous kernel's leftovers (tools/lds_poison_check.py).
#include <hip/hip_runtime.h>
extern "C" __global__ __launch_bounds__(256) void lds_poison_kernel() {
  extern __shared__ uint4 lds[];
  const int n = 65536 / 16;
  for (int i = threadIdx.x; i < n; i += 256) lds[i] = make_uint4(~0u, ~0u, ~0u, ~0u);
  __syncthreads();
}
extern "C" int lds_poison(void* stream, int blocks) {
  hipLaunchKernelGGL(lds_poison_kernel, dim3(blocks), dim3(256), 65536, (hipStream_t)stream);
  return (int)hipGetLastError();
}

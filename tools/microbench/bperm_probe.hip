// Cross-lane sums under co-scheduled work (diagnostic; tools/ab/bperm_probe.py).
//
// det_probe5 showed the mapper's LayerNorm backward giving different outputs for identical inputs, launched twice
// back to back on one stream, while the side stream ran the K-outer weight-gradient GEMMs. Its only cross-lane
// operations are the half-wave sums (__shfl_xor 16..1 -> ds_bpermute_b32). This victim kernel does nothing else:
// each half-wave sums 32 small integers (exact in fp32 in any order) with the same butterfly, over many rounds, and
// counts every result that differs from the known total. Run it alone and beside other kernels on another stream.
#include <hip/hip_runtime.h>
#include <stdint.h>

__device__ __forceinline__ float half_sum_bperm(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// mode 0: ds_bpermute butterfly (what __shfl_xor lowers to); mode 1: DPP / permlane butterfly
__device__ __forceinline__ float half_sum_dpp(float v) {
  // xor 1, xor 2 inside a quad (quad_perm), then row_half_mirror (lane i <-> 7 - i within 8), row_mirror (i <-> 15 - i
  // within 16), then the two 16-lane rows of each half-wave via v_permlane16_swap
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, false));  // [2,3,0,1]
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x141, 0xF, 0xF, false)); // half mirror
  v += __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false)); // row mirror
  // v_permlane16_swap(vdst = v, vsrc = v): vdst's odd rows <-> vsrc's even rows, so the two results hold
  // (row 2i, row 2i) and (row 2i+1, row 2i+1) of each row pair: their sum is the half-wave total in every lane
  const auto sw = __builtin_amdgcn_permlane16_swap(__builtin_bit_cast(unsigned, v), __builtin_bit_cast(unsigned, v),
                                                   false, false);
  return __builtin_bit_cast(float, (unsigned)sw[0]) + __builtin_bit_cast(float, (unsigned)sw[1]);
}

extern "C" __global__ __launch_bounds__(256) void bperm_victim(int rounds, int mode, uint32_t* errs, uint32_t* first) {
  const int lane = threadIdx.x & 63;
  const int hl = lane & 31;
  uint32_t bad = 0;
  for (int r = 0; r < rounds; ++r) {
    const int base = (blockIdx.x * 131 + r * 17) & 1023;
    const float v = (float)(base + hl * 3);           // exact small integers
    const float want = (float)(32 * base + 3 * 496);  // sum over hl = 0..31 of (base + 3 hl)
    const float got = mode == 0 ? half_sum_bperm(v) : half_sum_dpp(v);
    if (got != want) {
      ++bad;
      if (bad == 1) atomicCAS(first, 0u, (uint32_t)(blockIdx.x * 256 + threadIdx.x + 1));
    }
  }
  if (bad) atomicAdd(errs, bad);
}

extern "C" int bperm_launch(int blocks, int rounds, int mode, uint32_t* errs, uint32_t* first, void* stream) {
  hipLaunchKernelGGL(bperm_victim, dim3(blocks), dim3(256), 0, (hipStream_t)stream, rounds, mode, errs, first);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}

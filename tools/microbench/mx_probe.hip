// Operand / scale lane maps of gfx950's block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4 (e4m3 A and B), found
// from random data: one wave runs the MFMA on random e4m3 register contents and random E8M0 scale bytes, and the
// raw inputs and outputs are written to a file; tools/mx_probe_check.py then tests layout hypotheses against them
// on the host (exact: every product and partial sum is a dyadic rational well inside fp32's range).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <cmath>

typedef int v8i __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));

template <int OSA, int OSB>
__global__ void probe(const v8i* a, const v8i* b, const int* sa, const int* sb, v4f* d) {
  const int l = threadIdx.x;
  v4f c = {0.f, 0.f, 0.f, 0.f};
  c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a[l], b[l], c, 0, 0, OSA, sa[l], OSB, sb[l]);
  d[l] = c;
}

// fp32 -> e4m3 by the hardware conversion the quantizer uses (v_cvt_pk_fp8_f32, RNE): two values per call
__global__ void cvt(const float* x, uint16_t* q, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (2 * i + 1 < n) q[i] = (uint16_t)__builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
}

static uint32_t rng = 12345u;
static uint32_t nxt() { rng ^= rng << 13; rng ^= rng >> 17; rng ^= rng << 5; return rng; }

int main(int argc, char** argv) {
  const char* out = argc > 1 ? argv[1] : "mx_probe.bin";
  FILE* f = fopen(out, "wb");
  if (!f) return 1;
  for (int trial = 0; trial < 4; ++trial) {
    std::vector<uint8_t> A(64 * 32), B(64 * 32);
    std::vector<int> SA(64), SB(64);
    for (auto& x : A) x = (uint8_t)(((nxt() & 1) << 7) | ((4 + nxt() % 7) << 3) | (nxt() & 7));  // |x| in [2^-3, 2^3)
    for (auto& x : B) x = (uint8_t)(((nxt() & 1) << 7) | ((4 + nxt() % 7) << 3) | (nxt() & 7));
    // scale registers: 4 random bytes each (op_sel picks one), exponents 124..130
    for (auto& s : SA) s = (int)((124 + nxt() % 7) | ((124 + nxt() % 7) << 8) | ((124 + nxt() % 7) << 16) | ((124 + nxt() % 7) << 24));
    for (auto& s : SB) s = (int)((124 + nxt() % 7) | ((124 + nxt() % 7) << 8) | ((124 + nxt() % 7) << 16) | ((124 + nxt() % 7) << 24));
    v8i *da, *db; int *dsa, *dsb; v4f* dd;
    hipMalloc(&da, 64 * 32); hipMalloc(&db, 64 * 32); hipMalloc(&dsa, 256); hipMalloc(&dsb, 256); hipMalloc(&dd, 64 * 16);
    hipMemcpy(da, A.data(), 64 * 32, hipMemcpyHostToDevice);
    hipMemcpy(db, B.data(), 64 * 32, hipMemcpyHostToDevice);
    hipMemcpy(dsa, SA.data(), 256, hipMemcpyHostToDevice);
    hipMemcpy(dsb, SB.data(), 256, hipMemcpyHostToDevice);
    std::vector<float> D(256);
    const int osa = trial & 1 ? 1 : 0, osb = trial & 2 ? 2 : 0;
    if (trial == 0) hipLaunchKernelGGL((probe<0, 0>), dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
    if (trial == 1) hipLaunchKernelGGL((probe<1, 0>), dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
    if (trial == 2) hipLaunchKernelGGL((probe<0, 2>), dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
    if (trial == 3) hipLaunchKernelGGL((probe<1, 2>), dim3(1), dim3(64), 0, 0, da, db, dsa, dsb, dd);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    hipMemcpy(D.data(), dd, 1024, hipMemcpyDeviceToHost);
    int hdr[2] = {osa, osb};
    fwrite(hdr, 4, 2, f);
    fwrite(A.data(), 1, 2048, f); fwrite(B.data(), 1, 2048, f);
    fwrite(SA.data(), 4, 64, f); fwrite(SB.data(), 4, 64, f);
    fwrite(D.data(), 4, 256, f);
    hipFree(da); hipFree(db); hipFree(dsa); hipFree(dsb); hipFree(dd);
  }
  {  // conversion check: 8192 values over the e4m3 range incl. subnormals, exact ties and halfway points
    const int n = 8192;
    std::vector<float> X(n);
    for (int i = 0; i < n; ++i) {
      const float mag = ldexpf(1.0f + (float)(nxt() % 4096) / 4096.f, (int)(nxt() % 19) - 12);  // 2^-12 .. 2^7
      X[i] = (nxt() & 1) ? -mag : mag;
      if (i % 7 == 0) X[i] = ldexpf((float)(2 * (nxt() % 16) + 1) / 16.f, (int)(nxt() % 14) - 9);  // ties at every scale
      if (X[i] > 448.f) X[i] = 448.f;
      if (X[i] < -448.f) X[i] = -448.f;
    }
    float* dx; uint16_t* dq;
    (void)hipMalloc(&dx, n * 4); (void)hipMalloc(&dq, n);
    (void)hipMemcpy(dx, X.data(), n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(cvt, dim3(n / 2 / 256), dim3(256), 0, 0, dx, dq, n);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    std::vector<uint8_t> Q(n);
    (void)hipMemcpy(Q.data(), dq, n, hipMemcpyDeviceToHost);
    fwrite(X.data(), 4, n, f);
    fwrite(Q.data(), 1, n, f);
  }
  fclose(f);
  printf("mx_probe: wrote %s\n", out);
  return 0;
}

// Debug harness for topp_sample_kernel: includes the library source with ICAP_TOPP_DEBUG (kernel printf) and
// runs one tie-heavy row: 10 logits of 30 at 100..109, the rest 0, V = 50257, temperature 1, top_p 0.5 / 0.9.
#define ICAP_TOPP_DEBUG 1
#include "../../gpt2-image-captioning_amd/csrc/elementwise.hip"
#include <vector>
#include <cstdio>
int main() {
  const int64_t V = 50257;
  std::vector<float> h(V, 0.f);
  for (int j = 100; j < 110; ++j) h[j] = 30.f;
  float* d; int64_t* o;
  hipMalloc(&d, V * 4); hipMalloc(&o, 8);
  hipMemcpy(d, h.data(), V * 4, hipMemcpyHostToDevice);
  for (float tp : {0.5f, 0.9f, 0.95f}) {
    int rc = icap_topp_sample(ICAP_F32, 1, V, d, V, 1.0f, tp, nullptr, 1234567, nullptr, 0, 50256, o, nullptr);
    int64_t r = -1;
    hipDeviceSynchronize();
    hipMemcpy(&r, o, 8, hipMemcpyDeviceToHost);
    printf("top_p %.2f rc %d -> %lld\n", tp, rc, (long long)r);
  }
  return 0;
}

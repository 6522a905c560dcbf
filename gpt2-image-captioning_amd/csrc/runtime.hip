// Error reporting and library identity for the C-ABI (include/icap.h).
#include "common.h"

namespace icap {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_last_error = std::string(what) + ": " + hipGetErrorString(e);
    return ICAP_ERR_LAUNCH;
  }
  return ICAP_OK;
}

__global__ void probe_kernel(int* out) {
  if (threadIdx.x == 0) *out = 950;
}

}  // namespace icap

extern "C" const char* icap_last_error(void) { return icap::g_last_error.c_str(); }

extern "C" int icap_version(void) { return 1; }

// Resolves a device kernel of this library without launching it: succeeds only
// when the gfx950 code object of this .so was accepted by the HIP runtime.
extern "C" int icap_device_arch_ok(void) {
  hipFuncAttributes attr;
  hipError_t e = hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&icap::probe_kernel));
  if (e != hipSuccess) {
    icap::set_error(std::string("icap_device_arch_ok: ") + hipGetErrorString(e));
    return 0;
  }
  return 1;
}

// ABI bookkeeping: version, thread-local error text, launch checking.
#include "pcfm_common.hpp"

#include <mutex>
#include <unordered_set>

namespace pcfm {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: kernel launch failed: %s", what, hipGetErrorString(e));
    return (int)e;
  }
  return PCFM_OK;
}

int allow_big_lds(const void* kernel) {
  static std::mutex mu;
  static std::unordered_set<const void*> done;
  std::lock_guard<std::mutex> lock(mu);
  if (done.count(kernel)) return PCFM_OK;
  // leave 1 KiB for the kernels' small static __shared__ arrays: the cap
  // counts dynamic bytes, the hardware limit counts both
  hipError_t e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     kLdsBytesMax - 1024);
  if (e != hipSuccess) {
    set_error("hipFuncSetAttribute(MaxDynamicSharedMemorySize): %s", hipGetErrorString(e));
    return (int)e;
  }
  done.insert(kernel);
  return PCFM_OK;
}

}  // namespace pcfm

extern "C" int pcfm_abi_version(void) { return 20; }
extern "C" const char* pcfm_last_error(void) { return pcfm::g_err; }

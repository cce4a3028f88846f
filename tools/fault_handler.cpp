// Diagnosis shim: an HSA system event handler that writes a
// GPU memory fault's virtual address and reason bits to stderr and to the file
// named by $FAULT_LOG, before the runtime tears the process down.  Loaded by
// tools/fault_probe.py through ctypes after torch has initialised HIP.
//
// Build (CPU): g++ -O2 -shared -fPIC -I/opt/rocm/include tools/fault_handler.cpp
//              -L/opt/rocm/lib -lhsa-runtime64 -o tools/libfault_handler.so
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <cstdio>
#include <cstdlib>

namespace {

void emit(const char* text) {
  std::fputs(text, stderr);
  std::fflush(stderr);
  if (const char* path = std::getenv("FAULT_LOG")) {
    if (FILE* f = std::fopen(path, "a")) {
      std::fputs(text, f);
      std::fclose(f);
    }
  }
}

hsa_status_t on_event(const hsa_amd_event_t* ev, void*) {
  char buf[256];
  if (ev->event_type == HSA_AMD_GPU_MEMORY_FAULT_EVENT) {
    std::snprintf(buf, sizeof buf, "[fault_handler] memory fault at 0x%llx reason 0x%x\n",
                  (unsigned long long)ev->memory_fault.virtual_address,
                  ev->memory_fault.fault_reason_mask);
  } else if (ev->event_type == HSA_AMD_GPU_HW_EXCEPTION_EVENT) {
    std::snprintf(buf, sizeof buf, "[fault_handler] hw exception reset %d cause %d\n",
                  (int)ev->hw_exception.reset_type, (int)ev->hw_exception.reset_cause);
  } else {
    std::snprintf(buf, sizeof buf, "[fault_handler] event %d\n", (int)ev->event_type);
  }
  emit(buf);
  return HSA_STATUS_SUCCESS;
}

}  // namespace

extern "C" int fault_handler_install() {
  return (int)hsa_amd_register_system_event_handler(on_event, nullptr);
}

// Error state, version and device checks of libaz_hip.so.
#include <stdarg.h>
#include <string.h>

#include "az_common.h"

namespace az {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

int check_launch(const char* what) {
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s: %s", what, hipGetErrorString(e));
    return AZ_ELAUNCH;
  }
  return AZ_OK;
}

}  // namespace az

extern "C" int az_abi_version(void) { return AZ_ABI_VERSION; }

extern "C" const char* az_last_error(void) { return az::g_err; }

extern "C" int az_check_device(void) {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess) {
    az::set_error("az_check_device: no HIP device");
    return AZ_EDEVICE;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) != hipSuccess) {
    az::set_error("az_check_device: hipGetDeviceProperties failed");
    return AZ_EDEVICE;
  }
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    az::set_error("az_check_device: device %d is %s, this library is built for gfx950", dev,
                  prop.gcnArchName);
    return AZ_EDEVICE;
  }
  return AZ_OK;
}

// Host staging the device reads and writes in place (zero-copy): fine-grained (coherent) pinned
// memory mapped into the device's address space, so a kernel's loads see the host's latest
// stores and its stores are visible to the host once the stream has synchronised -- with no
// copy launch on either side.  Used by the batch-1 evaluation graph (one board in, one row of
// policy/value out per MCTS leaf).
extern "C" void* az_host_alloc(size_t bytes) {
  void* p = nullptr;
  if (bytes == 0) bytes = 1;
  if (hipHostMalloc(&p, bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
    az::set_error("az_host_alloc: hipHostMalloc(%zu) failed", bytes);
    return nullptr;
  }
  void* dp = nullptr;
  if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess || dp != p) {
    az::set_error("az_host_alloc: host buffer is not mapped at the same device address");
    (void)hipHostFree(p);
    return nullptr;
  }
  memset(p, 0, bytes);
  return p;
}

extern "C" int az_host_free(void* p) {
  if (p && hipHostFree(p) != hipSuccess) {
    az::set_error("az_host_free: hipHostFree failed");
    return AZ_EDEVICE;
  }
  return AZ_OK;
}

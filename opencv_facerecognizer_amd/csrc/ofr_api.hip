// Library-level entry points of libocvf_hip.so: version, errors, device check.
#include <string.h>

#include "ofr_common.h"

namespace ofr {

static thread_local std::string g_last_error;

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

int hip_status(hipError_t e, const char* where) {
  g_last_error = std::string(where) + ": " + hipGetErrorString(e);
  return (int)e > 0 ? (int)e : OFR_E_DEVICE;
}

}  // namespace ofr

extern "C" int ofr_version(void) { return (0 << 16) | (1 << 8) | 0; }

extern "C" const char* ofr_last_error(void) { return ofr::g_last_error.c_str(); }

extern "C" int ofr_device_check(int device) {
  hipDeviceProp_t prop;
  hipError_t e = hipGetDeviceProperties(&prop, device);
  if (e != hipSuccess) return ofr::hip_status(e, "hipGetDeviceProperties");
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return ofr::fail(OFR_E_DEVICE, std::string("ofr: device is ") + prop.gcnArchName + ", this library targets gfx950");
  return OFR_OK;
}

// Shared helpers of libocvf_hip.so (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <algorithm>
#include <string>

#include "../../include/ofr.h"

namespace ofr {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

#define OFR_GLOBAL __attribute__((address_space(1)))
#define OFR_LDS __attribute__((address_space(3)))

// thread-local error message (ofr_last_error)
void set_error(const std::string& msg);
int fail(int code, const std::string& msg);
int hip_status(hipError_t e, const char* where);

#define OFR_CHECK_ARG(cond, msg) \
  do {                           \
    if (!(cond)) return ::ofr::fail(OFR_E_INVALID, msg); \
  } while (0)

#define OFR_LAUNCH_CHECK(where) \
  do {                          \
    hipError_t _e = hipGetLastError(); \
    if (_e != hipSuccess) return ::ofr::hip_status(_e, where); \
  } while (0)

// Makes `device` current for the guard's scope and restores the caller's device on every exit path
// (an entry point bound to a context's device must not allocate on, or sync, whatever device the
// calling thread happened to have current).
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int device) {
    err = hipGetDevice(&prev);
    if (err == hipSuccess && prev != device) err = hipSetDevice(device);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// Synchronises `stream` when the scope ends while armed: an early error return after an
// asynchronous copy from host memory owned by the caller's frame (std::vector) must not free that
// memory while the copy may still read it.  disarm() once the frame has synchronised itself.
struct StreamSyncGuard {
  hipStream_t stream;
  bool armed = true;
  explicit StreamSyncGuard(hipStream_t s) : stream(s) {}
  ~StreamSyncGuard() {
    if (armed) (void)hipStreamSynchronize(stream);
  }
  void disarm() { armed = false; }
  StreamSyncGuard(const StreamSyncGuard&) = delete;
  StreamSyncGuard& operator=(const StreamSyncGuard&) = delete;
};

#define OFR_DEVICE_GUARD(dev, where)                                          \
  ::ofr::DeviceGuard _ofr_dev_guard(dev);                                     \
  if (_ofr_dev_guard.err != hipSuccess) return ::ofr::hip_status(_ofr_dev_guard.err, where)

__host__ __device__ constexpr int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }
__host__ __device__ constexpr int64_t round_up(int64_t a, int64_t b) { return cdiv(a, b) * b; }

// (distance, index) ordering used everywhere: ascending distance, ties -> lower index.
// NaN never compares better than anything, so NaN candidates sink to the end.
__device__ __forceinline__ bool better_f(float a, int ia, float b, int ib) {
  return a < b || (a == b && ia < ib);
}
__device__ __forceinline__ bool better_d(double a, int64_t ia, double b, int64_t ib) {
  return a < b || (a == b && ia < ib);
}

}  // namespace ofr

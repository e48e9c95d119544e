// Error plumbing shared by the C-ABI translation units (engine.cpp, vf.cpp, rollout.cpp):
// every exported entry runs its body under guarded(), which maps the exception
// type to the TRPO_ERR_* code and keeps the message for trpo_last_error().
#pragma once
#include "../../include/trpo_engine.h"

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <stdexcept>
#include <string>

namespace trpo_abi {

inline thread_local std::string g_last_error;

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct ArgError : std::runtime_error {
  using std::runtime_error::runtime_error;
};
struct RcclError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

#define HIPCHECK(x)                                                                       \
  do {                                                                                    \
    hipError_t e_ = (x);                                                                  \
    if (e_ != hipSuccess)                                                                 \
      throw ::trpo_abi::HipError(std::string(#x) + " failed: " + hipGetErrorString(e_));  \
  } while (0)
#define NCCLCHECK(x)                                                                      \
  do {                                                                                    \
    ncclResult_t r_ = (x);                                                                \
    if (r_ != ncclSuccess)                                                                \
      throw ::trpo_abi::RcclError(std::string(#x) + " failed: " + ncclGetErrorString(r_)); \
  } while (0)
#define REQUIRE(c, msg)                          \
  do {                                           \
    if (!(c)) throw ::trpo_abi::ArgError(msg);   \
  } while (0)

template <class F>
int guarded(F&& f) {
  try {
    f();
    return TRPO_OK;
  } catch (const ArgError& e) {
    g_last_error = e.what();
    return TRPO_ERR_ARG;
  } catch (const RcclError& e) {
    g_last_error = e.what();
    return TRPO_ERR_RCCL;
  } catch (const HipError& e) {
    g_last_error = e.what();
    return TRPO_ERR_HIP;
  } catch (const std::exception& e) {
    g_last_error = e.what();
    return TRPO_ERR_STATE;
  }
}

inline int pad4(int x) { return (x + 3) & ~3; }

inline void check_launch() { HIPCHECK(hipGetLastError()); }

// caller pointer (host or device, TRPO_MEM_*) -> device buffer on `s`; host copies are
// synchronous so the caller may free its buffer on return
inline void copy_in(void* dst, const void* src, size_t bytes, int mem, hipStream_t s) {
  if (bytes == 0) return;
  HIPCHECK(hipMemcpyAsync(dst, src, bytes, mem == TRPO_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice,
                          s));
  if (mem != TRPO_MEM_DEVICE) HIPCHECK(hipStreamSynchronize(s));
}
inline void copy_out(void* dst, const void* src, size_t bytes, int mem, hipStream_t s) {
  if (bytes == 0) return;
  HIPCHECK(hipMemcpyAsync(dst, src, bytes, mem == TRPO_MEM_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost,
                          s));
  HIPCHECK(hipStreamSynchronize(s));
}

}  // namespace trpo_abi

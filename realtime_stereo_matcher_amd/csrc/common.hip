// Host-side plumbing of the C ABI: thread-local error string, argument checks.
#include "common.h"

#include <cstdio>

namespace smcv {

std::string& last_error() {
  static thread_local std::string msg;
  return msg;
}

int fail(int code, const std::string& msg) {
  last_error() = msg;
  return code;
}

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    return fail(SM_ELAUNCH, std::string(what) + ": " + hipGetErrorString(e));
  }
  return SM_OK;
}

int read_strides(const int64_t* s, int64_t C, int64_t H, int64_t W, Strides4* out,
                 const char* name) {
  if (s == nullptr) {
    out->h = W;
    out->c = H * W;
    out->n = C * H * W;
    return SM_OK;
  }
  if (s[3] != 1) {
    return fail(SM_EINVAL, std::string(name) + ": W stride must be 1 (rows contiguous)");
  }
  if (s[0] < 0 || s[1] < 0 || s[2] < 0) {
    return fail(SM_EINVAL, std::string(name) + ": negative strides are not supported");
  }
  out->n = s[0];
  out->c = s[1];
  out->h = s[2];
  return SM_OK;
}

}  // namespace smcv

extern "C" int sm_version(void) { return 100; }  // 0.1.0

extern "C" const char* sm_last_error(void) { return smcv::last_error().c_str(); }

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

int stream_device(hipStream_t st) {
  int dev = 0;
  if (st == nullptr || hipStreamGetDevice(st, &dev) != hipSuccess) {
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  }
  return dev;
}

namespace {
std::atomic<int> g_cus[64];
}

int device_cus(int dev) {
  if (dev < 0 || dev >= 64) return 256;
  int n = g_cus[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
    n = 256;
  g_cus[dev].store(n, std::memory_order_relaxed);
  return n;
}

int ensure_lds_limit(const void* kern, int shm, int dev, std::atomic<unsigned long long>& done) {
  const unsigned long long bit = 1ull << (dev & 63);
  if (done.load(std::memory_order_acquire) & bit) return SM_OK;
  int cur = dev;
  if (hipGetDevice(&cur) != hipSuccess) cur = dev;
  if (cur != dev && hipSetDevice(dev) != hipSuccess) return fail(SM_ELAUNCH, "hipSetDevice failed");
  const hipError_t e = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, shm);
  if (cur != dev) (void)hipSetDevice(cur);
  if (e != hipSuccess)
    return fail(SM_ELAUNCH, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  done.fetch_or(bit, std::memory_order_acq_rel);
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

extern "C" int sm_version(void) { return 201; }  // 0.2.1: enum values 3, 4, 6, 7, 9, 10 retired; 12 added; SM_FUSED_DISP_F32 rounds the
                                                   // cells (SM_FUSED_EXACT_ACC: the old form)

extern "C" const char* sm_last_error(void) { return smcv::last_error().c_str(); }

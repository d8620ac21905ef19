// Shared helpers for the gfx950 stereo cost-volume kernels: dtype traits, feature-map
// views, argument validation and the thread-local error string of the C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include <atomic>
#include <string>

#include "../../include/stereocv.h"

namespace smcv {

// ------------------------------------------------------------------------------- errors
std::string& last_error();
int fail(int code, const std::string& msg);
int check_launch(const char* what);

// ------------------------------------------------------------------------------- dtypes
// Storage scalars.  bf16 is handled as raw 16-bit patterns with explicit RNE rounding so
// the conversion is identical to torch's (round-to-nearest-even, NaN stays NaN).
struct bf16_t { uint16_t bits; };

template <typename T> struct io;
template <> struct io<float> {
  static __device__ __forceinline__ float to_f(float v) { return v; }
  static __device__ __forceinline__ float from_f(float v) { return v; }
};
template <> struct io<__half> {
  static __device__ __forceinline__ float to_f(__half v) { return __half2float(v); }
  static __device__ __forceinline__ __half from_f(float v) { return __float2half_rn(v); }
};
template <> struct io<bf16_t> {
  static __device__ __forceinline__ float to_f(bf16_t v) {
    return __uint_as_float(static_cast<uint32_t>(v.bits) << 16);
  }
  static __device__ __forceinline__ bf16_t from_f(float v) {
    uint32_t u = __float_as_uint(v);
    bf16_t r;
    if ((u & 0x7fffffffu) > 0x7f800000u) {
      r.bits = static_cast<uint16_t>((u >> 16) | 0x0040u);  // quiet NaN, sign kept
    } else {
      r.bits = static_cast<uint16_t>((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
    }
    return r;
  }
};

template <typename T> __device__ __forceinline__ float to_f(T v) { return io<T>::to_f(v); }
template <typename T> __device__ __forceinline__ T from_f(float v) { return io<T>::from_f(v); }

inline int elem_size(int dtype) { return dtype == SM_F64 ? 8 : dtype == SM_F32 ? 4 : 2; }
inline bool valid_dtype(int dtype) { return dtype == SM_F32 || dtype == SM_F16 || dtype == SM_BF16; }

// float64 (f64.hip; the copies in cv_copy.hip)
int f64_dot_entry(const void* left, const void* right, void* out, int64_t N, int64_t C, int64_t H,
                  int64_t W, int64_t D, int64_t G, const int64_t* l_strides,
                  const int64_t* r_strides, int mode, void* stream);
int f64_softargmin_entry(const void* volume, void* out, int64_t N, int64_t D, int64_t H, int64_t W,
                         int flags, const int64_t* vol_strides, void* stream);
int f64_argext_entry(const void* volume, int64_t* out, int64_t N, int64_t D, int64_t H, int64_t W,
                     int mode, const int64_t* vol_strides, void* stream);

// ------------------------------------------------------------------------------- views
// Element strides of an (N, C, H, W) feature map; W stride is 1 by contract.
struct Strides4 {
  int64_t n, c, h;
};

int read_strides(const int64_t* s, int64_t C, int64_t H, int64_t W, Strides4* out,
                 const char* name);

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// ------------------------------------------------------------------------------- launches
// The device a stream belongs to (the current device for the null stream or on error).
int stream_device(hipStream_t st);
// Compute units of a device, cached per device (atomics: concurrent callers are safe).
int device_cus(int dev);
// Raise `kern`'s dynamic-LDS limit to `shm` bytes on `dev`, once per (kernel, device): `done`
// is the kernel's own bitmask of devices already raised.  The attribute applies to the
// current device, so it is switched to `dev` for the call and restored.
int ensure_lds_limit(const void* kern, int shm, int dev, std::atomic<unsigned long long>& done);


// Diagnostic phase stamps (scripts/ip_stamps.hip builds this file with -DSMCV_STAMPS; the
// library never does).  Each wave accumulates s_memtime deltas per phase.
#ifdef SMCV_STAMPS
constexpr int kStampPhases = 12;
extern __device__ unsigned long long g_stamps[4096][kStampPhases];
#define SM_STAMP_IN(ph) SM_STAMP(ph)
#define SM_STAMP_DECL                              \
  unsigned long long st_acc[kStampPhases] = {0};   \
  unsigned long long st_t = __builtin_amdgcn_s_memtime();
#define SM_STAMP(ph)                                           \
  do {                                                         \
    __builtin_amdgcn_sched_barrier(0);                         \
    const unsigned long long st_n = __builtin_amdgcn_s_memtime(); \
    st_acc[ph] += st_n - st_t;                                 \
    st_t = st_n;                                               \
    __builtin_amdgcn_sched_barrier(0);                         \
  } while (0)
#define SM_STAMP_FLUSH                                                         \
  if ((threadIdx.x & 63) == 0) {                                               \
    const int gw = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);        \
    if (gw < 4096)                                                             \
      for (int ph = 0; ph < kStampPhases; ++ph) g_stamps[gw][ph] = st_acc[ph]; \
  }
#else
#define SM_STAMP_DECL
#define SM_STAMP(ph) \
  do {               \
  } while (0)
#define SM_STAMP_FLUSH
#define SM_STAMP_IN(ph) \
  do {                  \
  } while (0)
#endif

}  // namespace smcv

// Dispatch a templated body on the runtime dtype code.
#define SM_DISPATCH_DTYPE(dtype, T, ...)                                   \
  switch (dtype) {                                                         \
    case SM_F32: { using T = float; __VA_ARGS__; } break;                  \
    case SM_F16: { using T = __half; __VA_ARGS__; } break;                 \
    case SM_BF16: { using T = ::smcv::bf16_t; __VA_ARGS__; } break;        \
    default: return ::smcv::fail(SM_EDTYPE, "unsupported dtype code");     \
  }

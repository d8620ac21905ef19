// Disparity regression over D of an (N, D, H, W) volume.
//
//   soft-argmin  disp = sum_d d * softmax_d(v)   model/mobile_disp_net_c.py:208-220,
//                                                inline model/mobile_stereo_net.py:144-147
//   presoftmax   disp = sum_d d * v              model/mobile_stereo_net_v4.py:10-14
//   hard argext  first index of min/max over D   build-defined
//
// One lane owns one pixel; the wave sweeps 64 (x4 with float4 loads) consecutive pixels of a
// row, so every load of a disparity plane is a coalesced 256 B / 1 KiB wave access.  The
// softmax is a single streaming pass (online max with a rescale per 8-plane chunk) with
// fp64 accumulators for sum(e) and sum(d*e): the result is within a few fp32 ulp of the
// exact value, i.e. the parity error budget is torch's own fp32 noise.
#include "common.h"

#include <math.h>

namespace smcv {
namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 8;

struct VolView {
  int64_t n, d, h;  // element strides; W stride is 1
};

template <typename T, int PX, bool PRESOFT>
__global__ __launch_bounds__(kThreads) void softargmin_kernel(const T* __restrict__ vol,
                                                              T* __restrict__ out, int D, int H,
                                                              int W, VolView vs) {
  const int y = blockIdx.y;
  const int n = blockIdx.z;
  const int x0 = (blockIdx.x * kThreads + threadIdx.x) * PX;
  if (x0 >= W) return;
  const T* base = vol + n * vs.n + (int64_t)y * vs.h + x0;
  const bool full = (x0 + PX) <= W;

  float m[PX];
  double s[PX], t[PX];
  bool has_nan[PX];
#pragma unroll
  for (int p = 0; p < PX; ++p) {
    has_nan[p] = false;
    m[p] = -INFINITY;
    s[p] = 0.0;
    t[p] = 0.0;
  }
  for (int d0 = 0; d0 < D; d0 += kChunk) {
    const int nd = min(kChunk, D - d0);
    float v[kChunk][PX];
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      if (k < nd) {
        const T* q = base + (int64_t)(d0 + k) * vs.d;
        if (PX == 4 && full && sizeof(T) == 4) {
          const float4 f = *reinterpret_cast<const float4*>(q);
          v[k][0] = f.x;
          v[k][1 % PX] = f.y;
          v[k][2 % PX] = f.z;
          v[k][3 % PX] = f.w;
        } else {
#pragma unroll
          for (int p = 0; p < PX; ++p) v[k][p] = (x0 + p < W) ? to_f(q[p]) : 0.f;
        }
      } else {
#pragma unroll
        for (int p = 0; p < PX; ++p) v[k][p] = -INFINITY;
      }
    }
    if (PRESOFT) {
#pragma unroll
      for (int k = 0; k < kChunk; ++k)
        if (k < nd)
#pragma unroll
          for (int p = 0; p < PX; ++p) t[p] += (double)(d0 + k) * (double)v[k][p];
    } else {
#pragma unroll
      for (int p = 0; p < PX; ++p) {
        float cm = v[0][p];
        bool nan = v[0][p] != v[0][p];
#pragma unroll
        for (int k = 1; k < kChunk; ++k) {
          cm = fmaxf(cm, v[k][p]);
          nan |= v[k][p] != v[k][p];
        }
        has_nan[p] |= nan;
        if (cm == -INFINITY) continue;  // nothing finite yet in this chunk (or column)
        if (cm > m[p]) {  // new running max: rescale the accumulators once per chunk
          const double f = (m[p] == -INFINITY) ? 0.0 : (double)expf(m[p] - cm);
          s[p] *= f;
          t[p] *= f;
          m[p] = cm;
        }
#pragma unroll
        for (int k = 0; k < kChunk; ++k) {
          if (k < nd) {
            const float e = expf(v[k][p] - m[p]);
            s[p] += (double)e;
            t[p] += (double)(d0 + k) * (double)e;
          }
        }
      }
    }
  }
  T* o = out + ((int64_t)n * H + y) * W + x0;
#pragma unroll
  for (int p = 0; p < PX; ++p) {
    if (x0 + p < W) {
      float r;
      if (PRESOFT) {
        r = (float)t[p];
      } else if (D == 0) {
        r = 0.f;  // empty softmax axis: the weighted sum is empty -> 0
      } else {
        // NaN anywhere in the column, or an all -inf / any +inf column, gives NaN as in torch
        r = (has_nan[p] || m[p] == INFINITY || m[p] == -INFINITY) ? NAN : (float)(t[p] / s[p]);
      }
      o[p] = from_f<T>(r);
    }
  }
}

template <typename T, bool MAXMODE>
__global__ __launch_bounds__(kThreads) void argext_kernel(const T* __restrict__ vol,
                                                          int64_t* __restrict__ out, int D, int H,
                                                          int W, VolView vs) {
  const int y = blockIdx.y;
  const int n = blockIdx.z;
  const int x = blockIdx.x * kThreads + threadIdx.x;
  if (x >= W) return;
  const T* base = vol + n * vs.n + (int64_t)y * vs.h + x;
  float best = to_f(base[0]);
  int idx = 0;
  bool isnan_best = best != best;
  for (int d0 = 1; d0 < D; d0 += kChunk) {
    float v[kChunk];
#pragma unroll
    for (int k = 0; k < kChunk; ++k)
      v[k] = (d0 + k < D) ? to_f(base[(int64_t)(d0 + k) * vs.d]) : (MAXMODE ? -INFINITY : INFINITY);
#pragma unroll
    for (int k = 0; k < kChunk; ++k) {
      if (d0 + k < D && !isnan_best) {
        const bool vnan = v[k] != v[k];
        const bool better = MAXMODE ? (v[k] > best) : (v[k] < best);  // strict: first index wins
        if (vnan || better) {
          best = v[k];
          idx = d0 + k;
          isnan_best = vnan;
        }
      }
    }
  }
  out[((int64_t)n * H + y) * W + x] = idx;
}

int check_vol(const void* volume, const void* out, int dtype, int64_t N, int64_t D, int64_t H,
              int64_t W, const int64_t* s, VolView* vs) {
  if (!valid_dtype(dtype)) return fail(SM_EDTYPE, "unsupported dtype code");
  if (N < 0 || D < 0 || H < 0 || W < 0) return fail(SM_EINVAL, "negative size");
  if (H > 65535 || N > 65535) return fail(SM_EINVAL, "N or H > 65535 not supported");
  if (N * H * W > 0 && (volume == nullptr || out == nullptr))
    return fail(SM_EINVAL, "null pointer");
  if (s == nullptr) {
    vs->h = W;
    vs->d = H * W;
    vs->n = D * H * W;
  } else {
    if (s[3] != 1) return fail(SM_EINVAL, "volume: W stride must be 1");
    vs->n = s[0];
    vs->d = s[1];
    vs->h = s[2];
  }
  return SM_OK;
}

}  // namespace

int softargmin_entry(const void* volume, void* out, int dtype, int64_t N, int64_t D, int64_t H,
                     int64_t W, int flags, const int64_t* vol_strides, void* stream) {
  VolView vs;
  int rc = check_vol(volume, out, dtype, N, D, H, W, vol_strides, &vs);
  if (rc) return rc;
  if (flags != SM_REGRESS_SOFTMAX && flags != SM_REGRESS_PRESOFTMAXED)
    return fail(SM_EINVAL, "unknown regression flags");
  if (N * H * W == 0) return SM_OK;
  hipStream_t st = as_stream(stream);
  const bool presoft = flags == SM_REGRESS_PRESOFTMAXED;
  const bool v4 = dtype == SM_F32 && (W % 4 == 0) && (vs.h % 4 == 0) && (vs.d % 4 == 0) &&
                  (vs.n % 4 == 0) && ((reinterpret_cast<uintptr_t>(volume) & 15u) == 0);
  SM_DISPATCH_DTYPE(dtype, T, {
    const T* v = static_cast<const T*>(volume);
    T* o = static_cast<T*>(out);
    if (v4) {
      dim3 grid((unsigned)ceil_div(W, kThreads * 4), (unsigned)H, (unsigned)N);
      if (presoft)
        hipLaunchKernelGGL((softargmin_kernel<T, 4, true>), grid, dim3(kThreads), 0, st, v, o,
                           (int)D, (int)H, (int)W, vs);
      else
        hipLaunchKernelGGL((softargmin_kernel<T, 4, false>), grid, dim3(kThreads), 0, st, v, o,
                           (int)D, (int)H, (int)W, vs);
    } else {
      dim3 grid((unsigned)ceil_div(W, kThreads), (unsigned)H, (unsigned)N);
      if (presoft)
        hipLaunchKernelGGL((softargmin_kernel<T, 1, true>), grid, dim3(kThreads), 0, st, v, o,
                           (int)D, (int)H, (int)W, vs);
      else
        hipLaunchKernelGGL((softargmin_kernel<T, 1, false>), grid, dim3(kThreads), 0, st, v, o,
                           (int)D, (int)H, (int)W, vs);
    }
  });
  return check_launch("softargmin_kernel");
}

int argext_entry(const void* volume, int64_t* out, int dtype, int64_t N, int64_t D, int64_t H,
                 int64_t W, int mode, const int64_t* vol_strides, void* stream) {
  VolView vs;
  int rc = check_vol(volume, out, dtype, N, D, H, W, vol_strides, &vs);
  if (rc) return rc;
  if (mode != SM_ARGMIN && mode != SM_ARGMAX) return fail(SM_EINVAL, "unknown argext mode");
  if (N * H * W == 0) return SM_OK;
  if (D <= 0) return fail(SM_EINVAL, "argext over an empty D axis");
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)ceil_div(W, kThreads), (unsigned)H, (unsigned)N);
  SM_DISPATCH_DTYPE(dtype, T, {
    const T* v = static_cast<const T*>(volume);
    if (mode == SM_ARGMAX)
      hipLaunchKernelGGL((argext_kernel<T, true>), grid, dim3(kThreads), 0, st, v, out, (int)D,
                         (int)H, (int)W, vs);
    else
      hipLaunchKernelGGL((argext_kernel<T, false>), grid, dim3(kThreads), 0, st, v, out, (int)D,
                         (int)H, (int)W, vs);
  });
  return check_launch("argext_kernel");
}

}  // namespace smcv

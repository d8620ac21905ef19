// Disparity regression over D of an (N, D, H, W) volume.
//
//   soft-argmin  disp = sum_d d * softmax_d(v)   model/mobile_disp_net_c.py:208-220,
//                                                inline model/mobile_stereo_net.py:144-147
//   presoftmax   disp = sum_d d * v              model/mobile_stereo_net_v4.py:10-14
//   hard argext  first index of min/max over D   build-defined
//
// One lane owns one pixel (four with float4 loads) of a 64-lane row segment, so every load of
// a disparity plane is a coalesced 256 B / 1 KiB wave access; the four waves of a block split
// D.  The softmax is a single streaming pass (online max with a rescale per 8-plane chunk)
// with fp64 accumulators for sum(e) and sum(d*e): the result is within a few fp32 ulp of the
// exact value, i.e. the parity error budget is torch's own fp32 noise.  A plane whose rows are
// contiguous is addressed as one flat pixel axis (no block straddles a row end), and fp32
// soft-argmin there takes softargmin_wave_kernel (fp32 per chunk, fp64 across chunks).
#include "common.h"

#include <math.h>

namespace smcv {
namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 8;

struct VolView {
  int64_t n, d, h;    // element strides; W stride is 1
  bool flat = false;  // rows contiguous: (H, W) is addressed as one axis of H*W pixels
};

// Block = 4 waves over the SAME 64*PX pixels of a row; wave w owns the disparity quarter
// [w*Dq, (w+1)*Dq).  Each lane keeps an online softmax (running max m, fp64 sums s = sum e,
// t = sum d*e) per pixel; the four partial states are merged through LDS by wave 0.  Splitting
// D across waves gives 4x the loads in flight of a one-wave-per-pixel sweep.
// TO: the output dtype -- T, or float for an fp16 / bf16 volume regressed to fp32 (the
// reference's autocast eval: F.softmax and torch.sum run in fp32 on an fp16 volume,
// mobile_stereo_net.py:144-147 under evaluate_stereo.py:48).
template <typename T, typename TO, int PX, bool PRESOFT>
__global__ __launch_bounds__(kThreads) void softargmin_kernel(const T* __restrict__ vol,
                                                              TO* __restrict__ out, int D, int H,
                                                              int W, VolView vs) {
  __shared__ float sm_m[4][PX][64];
  __shared__ double sm_s[4][PX][64];
  __shared__ double sm_t[4][PX][64];
  __shared__ int sm_nan[4][PX][64];
  const int y = blockIdx.y;
  const int n = blockIdx.z;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int x0 = (blockIdx.x * 64 + lane) * PX;
  const bool any = x0 < W;
  const bool full = (x0 + PX) <= W;
  const int Dq = (D + 3) >> 2;
  const int dbeg = min(D, wave * Dq);
  const int dend = min(D, dbeg + Dq);
  const T* base = vol + n * vs.n + (int64_t)y * vs.h + (any ? x0 : 0);

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
  if (any) {
    for (int d0 = dbeg; d0 < dend; d0 += kChunk) {
      const int nd = min(kChunk, dend - d0);
      float v[kChunk][PX];
#pragma unroll
      for (int k = 0; k < kChunk; ++k) {
        const T* qp = base + (int64_t)min(d0 + k, dend - 1) * vs.d;  // clamped: loads stay unconditional
        if (PX == 4 && sizeof(T) == 4) {
          float4 f;
          if (full) {
            f = *reinterpret_cast<const float4*>(qp);
          } else {
            f.x = to_f(qp[0]);
            f.y = (x0 + 1 < W) ? to_f(qp[1]) : 0.f;
            f.z = (x0 + 2 < W) ? to_f(qp[2]) : 0.f;
            f.w = (x0 + 3 < W) ? to_f(qp[3]) : 0.f;
          }
          v[k][0] = f.x;
          v[k][1 % PX] = f.y;
          v[k][2 % PX] = f.z;
          v[k][3 % PX] = f.w;
        } else {
#pragma unroll
          for (int p = 0; p < PX; ++p) v[k][p] = (x0 + p < W) ? to_f(qp[p]) : 0.f;
        }
        if (k >= nd) {
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
          if (cm == -INFINITY) continue;  // nothing finite yet in this chunk
          if (cm > m[p]) {                 // new running max: rescale once per chunk
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
  }
  // ---- merge the four disparity quarters
#pragma unroll
  for (int p = 0; p < PX; ++p) {
    sm_m[wave][p][lane] = m[p];
    sm_s[wave][p][lane] = s[p];
    sm_t[wave][p][lane] = t[p];
    sm_nan[wave][p][lane] = has_nan[p];
  }
  __syncthreads();
  if (wave != 0 || !any) return;
  TO* o = out + ((int64_t)n * H + y) * W + x0;
#pragma unroll
  for (int p = 0; p < PX; ++p) {
    if (x0 + p >= W) continue;
    float r;
    if (PRESOFT) {
      double tt = 0.0;
      for (int w = 0; w < 4; ++w) tt += sm_t[w][p][lane];
      r = (float)tt;
    } else if (D == 0) {
      r = 0.f;  // empty softmax axis: the weighted sum is empty -> 0
    } else {
      float M = -INFINITY;
      bool nan = false;
      for (int w = 0; w < 4; ++w) {
        M = fmaxf(M, sm_m[w][p][lane]);
        nan |= sm_nan[w][p][lane] != 0;
      }
      double S = 0.0, Tt = 0.0;
      if (M != -INFINITY && M != INFINITY) {
        for (int w = 0; w < 4; ++w) {
          const float mw = sm_m[w][p][lane];
          if (mw == -INFINITY) continue;
          const double f = (double)expf(mw - M);
          S += sm_s[w][p][lane] * f;
          Tt += sm_t[w][p][lane] * f;
        }
      }
      // NaN anywhere in the column, or an all -inf / any +inf column, gives NaN as in torch
      r = (nan || M == INFINITY || M == -INFINITY) ? NAN : (float)(Tt / S);
    }
    o[p] = from_f<TO>(r);
  }
}

// One KC-plane chunk of a lane's pixel p into its online-softmax state (m, S, T).  FULL: all KC
// planes are real (no per-element masking).  NaN handling: a NaN in a chunk that has a finite
// value makes e, hence S, NaN; a chunk with nothing but -inf and NaN poisons the pixel with
// m = +inf, which the merge turns into NaN like a +inf column (torch gives NaN for both).
template <int KC, bool FULL>
__device__ __forceinline__ void fold_chunk(const float (&v)[KC], int nd, int d0, float& m,
                                           double& S, double& T) {
  constexpr float kL2E = 1.4426950408889634f;
  float cm = FULL || 0 < nd ? v[0] : -INFINITY;
#pragma unroll
  for (int k = 1; k < KC; ++k) cm = fmaxf(cm, (FULL || k < nd) ? v[k] : -INFINITY);
  if (cm == -INFINITY) {  // nothing finite: only a NaN matters
    bool nan = false;
#pragma unroll
    for (int k = 0; k < KC; ++k) nan |= (FULL || k < nd) && v[k] != v[k];
    if (nan) m = INFINITY;
    return;
  }
  if (cm > m) {  // new running max: rescale once per chunk
    const double f = (m == -INFINITY) ? 0.0 : (double)expf(m - cm);
    S *= f;
    T *= f;
    m = cm;
  }
  float sc = 0.f, tc = 0.f;
#pragma unroll
  for (int k = 0; k < KC; ++k) {
    if (FULL || k < nd) {
      const float e = __builtin_amdgcn_exp2f((v[k] - m) * kL2E);
      sc += e;
      tc = fmaf((float)k, e, tc);
    }
  }
  S += (double)sc;
  T += (double)d0 * (double)sc + (double)tc;
}

// fp32 soft-argmin over a volume whose (H, W) plane is contiguous, addressed as a flat pixel
// axis (the host passes H = 1, W = H*W): one wave per unit = (n, 256-pixel group), 4 pixels per
// lane, over ALL of D with KC float4 plane loads in flight.  Per chunk each lane folds its
// pixels in fp32 (sum e and sum k*e relative to the chunk start, e = 2^((v-m) log2 e) on
// v_exp_f32) and carries them into fp64 sums once per chunk: 0.6 fp64 ops per element instead
// of 4.  No LDS merge and no barrier: a one-wave block retires as soon as its wave ends (r01,
// cfg2: 74 us vs 79 us for 4 waves splitting D with an LDS merge, and vs 105 us for the first
// fp64-per-element kernel).  WPB waves per block work on consecutive units.
template <int KC, int WPB, bool PRESOFT = false>
__global__ __launch_bounds__(64 * WPB) void softargmin_wave_kernel(const float* __restrict__ vol,
                                                                   float* __restrict__ out, int D,
                                                                   int W, int64_t vsn, int64_t vsd,
                                                                   int nunits) {
  const int P = (W + 255) >> 8;
  const int unit = blockIdx.x * WPB + (threadIdx.x >> 6);
  if (unit >= nunits) return;
  const int n = unit / P;
  const int lane = threadIdx.x & 63;
  const int x0 = ((unit - n * P) * 64 + lane) * 4;
  if (x0 >= W) return;
  const float* base = vol + n * vsn + x0;
  float m[4];
  double S[4], T[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    m[p] = -INFINITY;
    S[p] = 0.0;
    T[p] = 0.0;
  }
  for (int d0 = 0; d0 < D; d0 += KC) {
    const int nd = min(KC, D - d0);
    float4 v4[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k)
      v4[k] = *reinterpret_cast<const float4*>(base + (int64_t)min(d0 + k, D - 1) * vsd);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float v[KC];
#pragma unroll
      for (int k = 0; k < KC; ++k) v[k] = p == 0 ? v4[k].x : p == 1 ? v4[k].y : p == 2 ? v4[k].z : v4[k].w;
      if (PRESOFT) {  // sum_d d * v, fp64 per element as the generic kernel
#pragma unroll
        for (int k = 0; k < KC; ++k)
          if (k < nd) T[p] += (double)(d0 + k) * (double)v[k];
      } else if (nd == KC) {
        fold_chunk<KC, true>(v, nd, d0, m[p], S[p], T[p]);
      } else {
        fold_chunk<KC, false>(v, nd, d0, m[p], S[p], T[p]);
      }
    }
  }
  float res[4];
#pragma unroll
  for (int p = 0; p < 4; ++p)
    res[p] = PRESOFT ? (float)T[p]
             : (D == 0) ? 0.f : (m[p] == INFINITY || m[p] == -INFINITY) ? NAN : (float)(T[p] / S[p]);
  *reinterpret_cast<float4*>(out + (int64_t)n * W + x0) = make_float4(res[0], res[1], res[2], res[3]);
}

// Hard argmin/argmax with the same 4-wave disparity split; the quarters are merged in
// disparity order with the same strict comparison, so the FIRST extreme index wins.
template <typename T, bool MAXMODE>
__global__ __launch_bounds__(kThreads) void argext_kernel(const T* __restrict__ vol,
                                                          int64_t* __restrict__ out, int D, int H,
                                                          int W, VolView vs) {
  __shared__ float sm_b[4][64];
  __shared__ int sm_i[4][64];
  const int y = blockIdx.y;
  const int n = blockIdx.z;
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int x = blockIdx.x * 64 + lane;
  const bool ok = x < W;
  const int Dq = (D + 3) >> 2;
  const int dbeg = min(D, wave * Dq);
  const int dend = min(D, dbeg + Dq);
  const T* base = vol + n * vs.n + (int64_t)y * vs.h + (ok ? x : 0);
  float best = MAXMODE ? -INFINITY : INFINITY;
  int idx = -1;  // -1: this quarter is empty
  bool isnan_best = false;
  if (ok) {
    for (int d0 = dbeg; d0 < dend; d0 += kChunk) {
      float v[kChunk];
#pragma unroll
      for (int k = 0; k < kChunk; ++k) v[k] = to_f(base[(int64_t)min(d0 + k, dend - 1) * vs.d]);
#pragma unroll
      for (int k = 0; k < kChunk; ++k) {
        if (d0 + k < dend && !isnan_best) {
          const bool vnan = v[k] != v[k];
          const bool better = idx < 0 || (MAXMODE ? (v[k] > best) : (v[k] < best));
          if (vnan || better) {
            best = v[k];
            idx = d0 + k;
            isnan_best = vnan;
          }
        }
      }
    }
  }
  sm_b[wave][lane] = best;
  sm_i[wave][lane] = idx;
  __syncthreads();
  if (wave != 0 || !ok) return;
  float B = 0.f;
  int I = -1;
  for (int w = 0; w < 4; ++w) {
    const int iw = sm_i[w][lane];
    if (iw < 0) continue;
    const float bw = sm_b[w][lane];
    if (I < 0) {
      B = bw;
      I = iw;
      continue;
    }
    if (B != B) break;  // a NaN already won
    const bool better = (bw != bw) || (MAXMODE ? (bw > B) : (bw < B));
    if (better) {
      B = bw;
      I = iw;
    }
  }
  out[((int64_t)n * H + y) * W + x] = I < 0 ? 0 : I;
}

// fp32 argext over a flat contiguous plane: one wave per 256-pixel unit, 4 pixels per lane,
// over ALL of D with KC float4 plane loads in flight (no LDS merge, as softargmin_wave_kernel);
// first index on ties, NaN wins (torch.argmax / argmin), as argext_kernel.
template <bool MAXMODE, int KC>
__global__ __launch_bounds__(64) void argext_wave_kernel(const float* __restrict__ vol,
                                                         int64_t* __restrict__ out, int D, int W,
                                                         int64_t vsn, int64_t vsd, int nunits) {
  const int P = (W + 255) >> 8;
  const int unit = blockIdx.x;
  if (unit >= nunits) return;
  const int n = unit / P;
  const int lane = threadIdx.x & 63;
  const int x0 = ((unit - n * P) * 64 + lane) * 4;
  if (x0 >= W) return;
  const float* base = vol + n * vsn + x0;
  float best[4];
  int idx[4];
  bool nanb[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    best[p] = MAXMODE ? -INFINITY : INFINITY;
    idx[p] = -1;
    nanb[p] = false;
  }
  for (int d0 = 0; d0 < D; d0 += KC) {
    float4 v4[KC];
#pragma unroll
    for (int k = 0; k < KC; ++k)
      v4[k] = *reinterpret_cast<const float4*>(base + (int64_t)min(d0 + k, D - 1) * vsd);
#pragma unroll
    for (int k = 0; k < KC; ++k) {
      if (d0 + k < D) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const float v = p == 0 ? v4[k].x : p == 1 ? v4[k].y : p == 2 ? v4[k].z : v4[k].w;
          const bool vnan = v != v;
          const bool better = idx[p] < 0 || (MAXMODE ? (v > best[p]) : (v < best[p]));
          if (!nanb[p] && (vnan || better)) {
            best[p] = v;
            idx[p] = d0 + k;
            nanb[p] = vnan;
          }
        }
      }
    }
  }
  int64_t* o = out + (int64_t)n * W + x0;
  reinterpret_cast<longlong2*>(o)[0] = make_longlong2(idx[0] < 0 ? 0 : idx[0], idx[1] < 0 ? 0 : idx[1]);
  reinterpret_cast<longlong2*>(o)[1] = make_longlong2(idx[2] < 0 ? 0 : idx[2], idx[3] < 0 ? 0 : idx[3]);
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
  // A plane whose rows are contiguous is one flat pixel axis: no block straddles a row end.
  if (vs->h == W && H > 1 && H * W < ((int64_t)1 << 30)) {
    vs->h = H * W;
    vs->flat = true;
  }
  return SM_OK;
}

// (H, W) -> (1, H*W) when check_vol flattened the plane (vs.h == H*W).
inline void flatten_plane(const VolView& vs, int64_t* H, int64_t* W) {
  if (vs.flat) {
    *W = *H * *W;
    *H = 1;
  }
}

}  // namespace

int softargmin_entry(const void* volume, void* out, int dtype, int64_t N, int64_t D, int64_t H,
                     int64_t W, int flags, const int64_t* vol_strides, void* stream) {
  if (dtype == SM_F64) return f64_softargmin_entry(volume, out, N, D, H, W, flags, vol_strides, stream);
  VolView vs;
  int rc = check_vol(volume, out, dtype, N, D, H, W, vol_strides, &vs);
  if (rc) return rc;
  if ((flags & ~(SM_REGRESS_PRESOFTMAXED | SM_REGRESS_OUT_F32)) != 0)
    return fail(SM_EINVAL, "unknown regression flags");
  if (N * H * W == 0) return SM_OK;
  hipStream_t st = as_stream(stream);
  const bool presoft = (flags & SM_REGRESS_PRESOFTMAXED) != 0;
  // fp32 output from an fp16 / bf16 volume (for an fp32 volume the flag changes nothing)
  const bool out32 = (flags & SM_REGRESS_OUT_F32) != 0 && dtype != SM_F32;
  flatten_plane(vs, &H, &W);
  const bool flat4 = dtype == SM_F32 && (H == 1) && (W % 4 == 0) &&
                     (vs.d % 4 == 0) && (vs.n % 4 == 0) && (H * W < (int64_t)1 << 30) &&
                     ((reinterpret_cast<uintptr_t>(volume) & 15u) == 0) &&
                     ((reinterpret_cast<uintptr_t>(out) & 15u) == 0);  // float4 stores
  if (flat4) {
    const int Wf = (int)W;
    const int64_t nunits = ceil_div(Wf, 64 * 4) * N;
    if (nunits > INT32_MAX) return fail(SM_EINVAL, "soft-argmin: too many pixels for one launch");
    // one 64-lane wave per block (measured r01: 16-plane chunks or 4 waves per block no faster)
    if (presoft)
      hipLaunchKernelGGL((softargmin_wave_kernel<8, 1, true>), dim3((unsigned)nunits), dim3(64), 0,
                         st, static_cast<const float*>(volume), static_cast<float*>(out), (int)D,
                         Wf, vs.n, vs.d, (int)nunits);
    else
      hipLaunchKernelGGL((softargmin_wave_kernel<8, 1>), dim3((unsigned)nunits), dim3(64), 0, st,
                         static_cast<const float*>(volume), static_cast<float*>(out), (int)D, Wf,
                         vs.n, vs.d, (int)nunits);
    return check_launch("softargmin_wave_kernel");
  }
  const bool v4 = dtype == SM_F32 && (W % 4 == 0) && (vs.h % 4 == 0) && (vs.d % 4 == 0) &&
                  (vs.n % 4 == 0) && ((reinterpret_cast<uintptr_t>(volume) & 15u) == 0);
  auto go = [&](auto tin, auto tout) {
    using T = decltype(tin);
    using TO = decltype(tout);
    const T* v = static_cast<const T*>(volume);
    TO* o = static_cast<TO*>(out);
    if (v4) {
      dim3 grid((unsigned)ceil_div(W, 64 * 4), (unsigned)H, (unsigned)N);
      if (presoft)
        hipLaunchKernelGGL((softargmin_kernel<T, TO, 4, true>), grid, dim3(kThreads), 0, st, v, o,
                           (int)D, (int)H, (int)W, vs);
      else
        hipLaunchKernelGGL((softargmin_kernel<T, TO, 4, false>), grid, dim3(kThreads), 0, st, v, o,
                           (int)D, (int)H, (int)W, vs);
    } else {
      dim3 grid((unsigned)ceil_div(W, 64), (unsigned)H, (unsigned)N);
      if (presoft)
        hipLaunchKernelGGL((softargmin_kernel<T, TO, 1, true>), grid, dim3(kThreads), 0, st, v, o,
                           (int)D, (int)H, (int)W, vs);
      else
        hipLaunchKernelGGL((softargmin_kernel<T, TO, 1, false>), grid, dim3(kThreads), 0, st, v, o,
                           (int)D, (int)H, (int)W, vs);
    }
  };
  SM_DISPATCH_DTYPE(dtype, T, {
    if (out32)
      go(T{}, float{});
    else
      go(T{}, T{});
  });
  return check_launch("softargmin_kernel");
}

int argext_entry(const void* volume, int64_t* out, int dtype, int64_t N, int64_t D, int64_t H,
                 int64_t W, int mode, const int64_t* vol_strides, void* stream) {
  if (dtype == SM_F64) return f64_argext_entry(volume, out, N, D, H, W, mode, vol_strides, stream);
  VolView vs;
  int rc = check_vol(volume, out, dtype, N, D, H, W, vol_strides, &vs);
  if (rc) return rc;
  if (mode != SM_ARGMIN && mode != SM_ARGMAX) return fail(SM_EINVAL, "unknown argext mode");
  if (N * H * W == 0) return SM_OK;
  if (D <= 0) return fail(SM_EINVAL, "argext over an empty D axis");
  hipStream_t st = as_stream(stream);
  flatten_plane(vs, &H, &W);
  if (dtype == SM_F32 && H == 1 && W % 4 == 0 && vs.d % 4 == 0 && vs.n % 4 == 0 &&
      W < ((int64_t)1 << 30) && ((reinterpret_cast<uintptr_t>(volume) & 15u) == 0) &&
      ((reinterpret_cast<uintptr_t>(out) & 15u) == 0)) {
    const int64_t nunits = ceil_div(W, 64 * 4) * N;
    if (nunits > INT32_MAX) return fail(SM_EINVAL, "argext: too many pixels for one launch");
    const float* v = static_cast<const float*>(volume);
    if (mode == SM_ARGMAX)
      hipLaunchKernelGGL((argext_wave_kernel<true, 8>), dim3((unsigned)nunits), dim3(64), 0, st, v,
                         out, (int)D, (int)W, vs.n, vs.d, (int)nunits);
    else
      hipLaunchKernelGGL((argext_wave_kernel<false, 8>), dim3((unsigned)nunits), dim3(64), 0, st, v,
                         out, (int)D, (int)W, vs.n, vs.d, (int)nunits);
    return check_launch("argext_wave_kernel");
  }
  dim3 grid((unsigned)ceil_div(W, 64), (unsigned)H, (unsigned)N);
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

// Dot-product cost volumes on the gfx950 VALU: inner product (sum over C), correlation
// (mean over C) and groupwise (mean over contiguous C/G channel blocks, D innermost).
//
// Reference semantics (babiking/realtime_stereo_matcher):
//   inner product  cost_volume/inner_product.py:11-42      out (N,D,H,W), sum, 0 for x<d
//   correlation    model/mobile_disp_net_c.py:188-205      out (N,D,H,W), mean, 0 for x<d
//   groupwise      cost_volume/groupwise.py:24-56          out (N,G,H,W,D) fp32, mean/group
//
// Design (one workgroup = one (n, group, y) row segment of TX=64 left pixels):
//   * the left tile L[c][x0..x0+64) and the right WINDOW R[c][x0-DCH .. x0+64) are staged
//     in LDS per 16-channel slab, converted to fp32 once;
//   * the right window is re-used across the whole disparity sweep: thread (xg, dg) owns
//     4 contiguous pixels x and TD contiguous disparities d, so for every channel it reads
//     one float4 of L and (TD+4)/4 float4 of R and issues 4*TD FMAs (register tile
//     sliding along the anti-diagonal j = x - d);
//   * fp32 accumulation, one rounding to the output dtype at the store;
//   * output rows are written with 16-B stores along x (NDHW) or along d (NGHWD).
#include "common.h"

namespace smcv {
namespace {

constexpr int kTX = 64;       // left pixels per workgroup
constexpr int kCC = 16;       // channels per LDS slab
constexpr int kThreads = 256; // 16 x-groups * 16 d-groups

enum Layout { kNDHW = 0, kNGHWD = 1 };

template <typename T, typename TO, int TD, int LAYOUT>
__global__ __launch_bounds__(kThreads) void dot_volume_valu(
    const T* __restrict__ L, const T* __restrict__ R, TO* __restrict__ out, int C, int H,
    int W, int D, int G, Strides4 ls, Strides4 rs, int divisor) {
  constexpr int DCH = 16 * TD;    // disparities per pass
  constexpr int RW = kTX + DCH;   // right-window width
  __shared__ __attribute__((aligned(16))) float Ls[kCC][kTX];
  __shared__ __attribute__((aligned(16))) float Rs[kCC][RW];

  const int tid = threadIdx.x;
  const int xg = tid & 15;
  const int dg = tid >> 4;
  const int x0 = blockIdx.x * kTX;
  const int y = blockIdx.y;
  const int ng = blockIdx.z;  // n * G + g
  const int n = ng / G;
  const int g = ng - n * G;
  const int cpg = C / G;
  const int cbase = g * cpg;

  const T* Lrow = L + n * ls.n + (int64_t)cbase * ls.c + (int64_t)y * ls.h;
  const T* Rrow = R + n * rs.n + (int64_t)cbase * rs.c + (int64_t)y * rs.h;
  // divisor < 0: plain sum; otherwise the mean's element count (0 -> 0/0 = NaN, as torch)
  const float scale_div = (float)divisor;

  for (int d0 = 0; d0 < D; d0 += DCH) {
    float acc[TD][4];
#pragma unroll
    for (int b = 0; b < TD; ++b)
#pragma unroll
      for (int a = 0; a < 4; ++a) acc[b][a] = 0.f;

    const int js = x0 - d0 - DCH;  // right column held in Rs[.][0]
    const bool active = (d0 + dg * TD) < D && (x0 + 4 * xg) < W;

    for (int c0 = 0; c0 < cpg; c0 += kCC) {
      const int cc = min(kCC, cpg - c0);
      __syncthreads();
      for (int e = tid; e < kCC * kTX; e += kThreads) {
        const int c = e / kTX, i = e - c * kTX, x = x0 + i;
        float v = 0.f;
        if (c < cc && x < W) v = to_f(Lrow[(int64_t)(c0 + c) * ls.c + x]);
        Ls[c][i] = v;
      }
      for (int e = tid; e < kCC * RW; e += kThreads) {
        const int c = e / RW, i = e - c * RW, j = js + i;
        float v = 0.f;
        if (c < cc && j >= 0 && j < W) v = to_f(Rrow[(int64_t)(c0 + c) * rs.c + j]);
        Rs[c][i] = v;
      }
      __syncthreads();
      if (active) {
        const int base = 4 * xg + (15 - dg) * TD;
        for (int c = 0; c < cc; ++c) {
          const float4 l4 = *reinterpret_cast<const float4*>(&Ls[c][4 * xg]);
          const float lv[4] = {l4.x, l4.y, l4.z, l4.w};
          float r[TD + 4];
#pragma unroll
          for (int m = 0; m < (TD + 4) / 4; ++m) {
            const float4 q = *reinterpret_cast<const float4*>(&Rs[c][base + 4 * m]);
            r[4 * m + 0] = q.x;
            r[4 * m + 1] = q.y;
            r[4 * m + 2] = q.z;
            r[4 * m + 3] = q.w;
          }
#pragma unroll
          for (int b = 0; b < TD; ++b)
#pragma unroll
            for (int a = 0; a < 4; ++a) acc[b][a] = fmaf(lv[a], r[TD + a - b], acc[b][a]);
        }
      }
    }

    if (active) {
#pragma unroll
      for (int b = 0; b < TD; ++b) {
        const int d = d0 + dg * TD + b;
        if (d >= D) break;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
          const int x = x0 + 4 * xg + a;
          if (x >= W) break;
          float v = (x >= d) ? acc[b][a] : 0.f;
          if (divisor >= 0 && x >= d) v = v / scale_div;
          size_t o;
          if (LAYOUT == kNDHW) {
            o = (((size_t)n * D + d) * H + y) * (size_t)W + x;
          } else {
            o = ((((size_t)n * G + g) * H + y) * (size_t)W + x) * (size_t)D + d;
          }
          out[o] = from_f<TO>(v);
        }
      }
    }
  }
}

template <typename T, typename TO, int LAYOUT>
int launch_dot(const void* l, const void* r, void* o, int64_t N, int64_t C, int64_t H,
               int64_t W, int64_t D, int64_t G, Strides4 ls, Strides4 rs, int divisor,
               hipStream_t st) {
  dim3 grid((unsigned)ceil_div(W, kTX), (unsigned)H, (unsigned)(N * G));
  const T* L = static_cast<const T*>(l);
  const T* R = static_cast<const T*>(r);
  TO* out = static_cast<TO*>(o);
  const int iC = (int)C, iH = (int)H, iW = (int)W, iD = (int)D, iG = (int)G;
  if (D <= 64) {
    hipLaunchKernelGGL((dot_volume_valu<T, TO, 4, LAYOUT>), grid, dim3(kThreads), 0, st, L, R,
                       out, iC, iH, iW, iD, iG, ls, rs, divisor);
  } else if (D <= 128) {
    hipLaunchKernelGGL((dot_volume_valu<T, TO, 8, LAYOUT>), grid, dim3(kThreads), 0, st, L, R,
                       out, iC, iH, iW, iD, iG, ls, rs, divisor);
  } else if (D <= 192) {
    hipLaunchKernelGGL((dot_volume_valu<T, TO, 12, LAYOUT>), grid, dim3(kThreads), 0, st, L, R,
                       out, iC, iH, iW, iD, iG, ls, rs, divisor);
  } else {
    hipLaunchKernelGGL((dot_volume_valu<T, TO, 16, LAYOUT>), grid, dim3(kThreads), 0, st, L, R,
                       out, iC, iH, iW, iD, iG, ls, rs, divisor);
  }
  return check_launch("dot_volume_valu");
}

}  // namespace

// Shared validation for the (N,C,H,W) x2 -> volume entry points.
int check_dot_args(const void* left, const void* right, const void* out, int dtype, int64_t N,
                   int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                   const int64_t* r_strides, Strides4* ls, Strides4* rs) {
  if (!valid_dtype(dtype) && dtype != SM_F64) return fail(SM_EDTYPE, "unsupported dtype code");
  if (N < 0 || C < 0 || H < 0 || W < 0 || D < 0) return fail(SM_EINVAL, "negative size");
  if (H > 65535 || W > (1 << 30) || D > (1 << 20) || C > (1 << 24))
    return fail(SM_EINVAL, "size out of supported range (H <= 65535)");
  const int64_t total = N * C * H * W;
  if (total > 0 && (left == nullptr || right == nullptr))
    return fail(SM_EINVAL, "null feature pointer");
  if (N * D * H * W > 0 && out == nullptr) return fail(SM_EINVAL, "null output pointer");
  int rc = read_strides(l_strides, C, H, W, ls, "left");
  if (rc) return rc;
  return read_strides(r_strides, C, H, W, rs, "right");
}

int dot_volume_valu_entry(const void* left, const void* right, void* out, int dtype,
                          int64_t N, int64_t C, int64_t H, int64_t W, int64_t D, int64_t G,
                          const int64_t* l_strides, const int64_t* r_strides, int mode,
                          void* stream) {
  // mode 0: inner product (sum, NDHW, out dtype = in dtype)
  // mode 1: correlation mean (NDHW, out dtype = in dtype)
  // mode 2: groupwise mean (NGHWD, fp32 out)
  if (dtype == SM_F64)  // fp64 products and sums (f64.hip)
    return f64_dot_entry(left, right, out, N, C, H, W, D, G, l_strides, r_strides, mode, stream);
  Strides4 ls, rs;
  int rc = check_dot_args(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &ls, &rs);
  if (rc) return rc;
  if (mode == 2) {
    if (G <= 0 || C % G != 0) return fail(SM_EINVAL, "groupwise: C % G != 0");
  } else {
    G = 1;
  }
  if (N == 0 || H == 0 || W == 0 || D == 0 || G == 0) return SM_OK;
  if (N * G > 65535) return fail(SM_EINVAL, "N*G > 65535 not supported");
  hipStream_t st = as_stream(stream);
  // sum over an empty channel axis is 0; a mean over it is 0/0 = NaN, as in torch
  const int divisor = mode == 0 ? -1 : (mode == 1 ? (int)C : (int)(C / G));
  if (mode == 2) {
    SM_DISPATCH_DTYPE(dtype, T,
                      return launch_dot<T, float, kNGHWD>(left, right, out, N, C, H, W, D, G, ls,
                                                          rs, divisor, st));
  } else {
    SM_DISPATCH_DTYPE(dtype, T,
                      return launch_dot<T, T, kNDHW>(left, right, out, N, C, H, W, D, 1, ls, rs,
                                                     divisor, st));
  }
  return SM_OK;
}

}  // namespace smcv

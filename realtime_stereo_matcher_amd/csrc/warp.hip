// Disparity / flow warp of an image or feature map.
//
//   warp_by_flow_map(image, flow)   tools/warp.py:5-42, model/mobile_stereo_net_v2.py:59-96
//                                   (= _v3.py:60-97), called by RefineNet (_v3.py:136, _v2.py:127)
//
// The reference builds a sampling grid from the flow and calls F.grid_sample (bilinear, zero
// padding, align_corners=False).  Its normalisation divides by (w - 1) and (h - 1) while
// grid_sample un-normalises with align_corners=False, so the sampled position is
//   ix = ((2 (x - fx) / (w - 1) - 1) + 1) * (Wi / 2) - 0.5,   and likewise iy with fy = 0 for a
// one-channel flow: the warp also resamples vertically by h / (h - 1).  This kernel evaluates
// exactly that fp32 operation sequence (the CPU grid_sample's form of the un-normalisation,
// GridSamplerKernel.cpp: (g + 1) * size / 2 - 0.5) and the same bilinear weights
// (nw = (1 - dy)(1 - dx), ...; out-of-image corners contribute 0, as zero padding).
//
// One lane owns one output pixel: it derives the four corner offsets and weights once, then
// walks the channels, so each channel costs four gathers (neighbouring lanes read neighbouring
// image pixels of at most two rows: L1/L2 hits) and one coalesced store.  The image is read
// about once and the output written once: HBM-bound.
#include "common.h"

#include <math.h>

#include <algorithm>

namespace smcv {
namespace {

constexpr int kWarpThreads = 256;
constexpr int kWarpCU = 4;  // channels in flight per lane

struct WarpArgs {
  const float* img;
  const float* flow;
  float* out;
  int C, H, W, Hi, Wi, fch;
  int64_t isn, isc, ish;  // image strides (W stride 1)
  int64_t fsn, fsc, fsh;  // flow strides (W stride 1)
  float sx, sy;           // Wi / 2, Hi / 2
  float dw, dh;           // (float)(w - 1.0), (float)(h - 1.0)
};

// Output pixel (n, y, x): the four bilinear weights (nw, ne, sw, se), the top-left corner
// (x0, y0) and which corners lie inside the image.  The reference's fp32 operation sequence.
struct Corners {
  float w[4];
  bool ok[4];
  int x0, y0;
};
__device__ __forceinline__ Corners corners_of(const WarpArgs& a, int n, int y, int x) {
#pragma clang fp contract(off)  // separate roundings, as the reference's grid math and blend
  const float* fl = a.flow + n * a.fsn + (int64_t)y * a.fsh + x;
  // grid, exactly as the reference: (x - f) -> 2 * . / (w - 1) - 1   (tools/warp.py:19-36)
  float gx = (float)x - fl[0];
  float gy = (float)y;
  if (a.fch == 2) gy = gy - fl[a.fsc];
  gx = 2.0f * gx / a.dw - 1.0f;
  gy = 2.0f * gy / a.dh - 1.0f;
  // grid_sample, align_corners=False: un-normalise, bilinear corners
  const float ix = (gx + 1.0f) * a.sx - 0.5f;
  const float iy = (gy + 1.0f) * a.sy - 0.5f;
  const float fx0 = floorf(ix), fy0 = floorf(iy);
  const float dx = ix - fx0, dy = iy - fy0;
  const float ex = 1.0f - dx, sy = 1.0f - dy;
  Corners q;
  q.w[0] = sy * ex;  // nw
  q.w[1] = sy * dx;  // ne
  q.w[2] = dy * ex;  // sw
  q.w[3] = dy * dx;  // se
  const bool finite = fabsf(ix) < 2.0e9f && fabsf(iy) < 2.0e9f;  // int conversion in range
  q.x0 = finite ? (int)fx0 : -2;
  q.y0 = finite ? (int)fy0 : -2;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int xx = q.x0 + (k & 1), yy = q.y0 + (k >> 1);
    q.ok[k] = finite && xx >= 0 && xx < a.Wi && yy >= 0 && yy < a.Hi;
  }
  return q;
}

__global__ __launch_bounds__(kWarpThreads) void warp_kernel(WarpArgs a, int cpb) {
#pragma clang fp contract(off)  // separate roundings, as the reference's blend
  // block (pixel chunk, channel chunk, n): the waves in flight share a few channel planes
  const int n = blockIdx.z;
  const int cbeg = blockIdx.y * cpb, cend = min(a.C, cbeg + cpb);
  const int64_t p = (int64_t)blockIdx.x * kWarpThreads + threadIdx.x;
  const int64_t HW = (int64_t)a.H * a.W;
  if (p >= HW) return;
  const int y = (int)(p / a.W);
  const int x = (int)(p - (int64_t)y * a.W);
  const Corners q = corners_of(a, n, y, x);
  const float* w = q.w;
  const bool* ok = q.ok;
  const int x0 = q.x0, y0 = q.y0;
  int64_t off[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) off[k] = ok[k] ? (int64_t)(y0 + (k >> 1)) * a.ish + x0 + (k & 1) : 0;
  const float* ib = a.img + n * a.isn;
  float* ob = a.out + ((int64_t)n * a.C) * HW + p;
  int c = cbeg;
  if (a.Wi >= 2) {
    // The two x-corners of a row are neighbours: one 8-byte (dword-aligned) load per row and
    // channel, at x0 clamped into [0, Wi-2]; each corner picks its half, or 0 outside the image.
    // Rows outside the image read row 0 and contribute 0.  Same values, same blend as below.
    typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
    const int xc = min(max(x0, 0), a.Wi - 2);
    const bool r0 = ok[0] || ok[1], r1 = ok[2] || ok[3];  // row y0 / y0+1 inside (x aside)
    const int64_t o0 = (int64_t)(r0 ? y0 : 0) * a.ish + xc;
    const int64_t o1 = (int64_t)(r1 ? y0 + 1 : 0) * a.ish + xc;
    const bool lw = x0 == xc;      // the west corner is the low half (else the high half)
    const bool le = x0 + 1 == xc;  // the east corner is the low half (x0 = -1)
    for (; c + kWarpCU <= cend; c += kWarpCU) {
      f2u t[kWarpCU], b[kWarpCU];
#pragma unroll
      for (int u = 0; u < kWarpCU; ++u) {
        t[u] = *reinterpret_cast<const f2u*>(ib + (int64_t)(c + u) * a.isc + o0);
        b[u] = *reinterpret_cast<const f2u*>(ib + (int64_t)(c + u) * a.isc + o1);
      }
#pragma unroll
      for (int u = 0; u < kWarpCU; ++u) {
        const float v0 = ok[0] ? (lw ? t[u].x : t[u].y) : 0.f;
        const float v1 = ok[1] ? (le ? t[u].x : t[u].y) : 0.f;
        const float v2 = ok[2] ? (lw ? b[u].x : b[u].y) : 0.f;
        const float v3 = ok[3] ? (le ? b[u].x : b[u].y) : 0.f;
        ob[(int64_t)(c + u) * HW] = v0 * w[0] + v1 * w[1] + v2 * w[2] + v3 * w[3];
      }
    }
  }
  for (; c + kWarpCU <= cend; c += kWarpCU) {
    float v[kWarpCU][4];
#pragma unroll
    for (int u = 0; u < kWarpCU; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) v[u][k] = ok[k] ? ib[(int64_t)(c + u) * a.isc + off[k]] : 0.f;
#pragma unroll
    for (int u = 0; u < kWarpCU; ++u)
      ob[(int64_t)(c + u) * HW] = v[u][0] * w[0] + v[u][1] * w[1] + v[u][2] * w[2] + v[u][3] * w[3];
  }
  for (; c < cend; ++c) {
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = ok[k] ? ib[(int64_t)c * a.isc + off[k]] : 0.f;
    ob[(int64_t)c * HW] = v[0] * w[0] + v[1] * w[1] + v[2] * w[2] + v[3] * w[3];
  }
}

// Two-channel flows, channel-last: a flow scatters the rows a wave samples, so in the (N, C, H, W)
// image every corner of every channel is its own 128-B line (warp_kernel: 0.18 of HBM at a
// sigma-4 flow).  warp_to_nhwc first copies the image to (N, Hi, Wi, Cp) (Cp = C rounded up to 4,
// zero padded; coalesced reads per channel row, contiguous 16-B writes per pixel), then
// warp_gather_nhwc gives a pixel's 4-channel groups to consecutive lanes: one corner of a pixel
// is Cp * 4 contiguous bytes (one line at C = 32), the blend is warp_kernel's, and the block's
// 64 x C outputs leave through LDS as coalesced channel rows.
constexpr int kNhwcPx = 64;     // pixels per transpose block
constexpr int kGatherPx = 128;  // pixels per gather block (<= kWarpThreads: one corner lane each)

__global__ __launch_bounds__(kWarpThreads) void warp_to_nhwc(WarpArgs a, float* ws, int Cp) {
  extern __shared__ float tile[];  // [64 px][Cp + 1]
  const int n = blockIdx.z, yy = blockIdx.y, x0 = blockIdx.x * kNhwcPx;
  const int np = min(kNhwcPx, a.Wi - x0);
  const int S = Cp + 1;
  const float* src = a.img + n * a.isn + (int64_t)yy * a.ish + x0;
  for (int i = threadIdx.x; i < Cp * kNhwcPx; i += kWarpThreads) {
    const int c = i / kNhwcPx, px = i % kNhwcPx;
    tile[px * S + c] = (c < a.C && px < np) ? src[(int64_t)c * a.isc + px] : 0.f;
  }
  __syncthreads();
  const int G = Cp >> 2;
  float4* dst = reinterpret_cast<float4*>(ws + (((int64_t)n * a.Hi + yy) * a.Wi + x0) * Cp);
  for (int i = threadIdx.x; i < np * G; i += kWarpThreads) {
    const int px = i / G, g = i - px * G;
    const float* s = tile + px * S + 4 * g;
    dst[i] = make_float4(s[0], s[1], s[2], s[3]);
  }
}

__global__ __launch_bounds__(kWarpThreads) void warp_gather_nhwc(WarpArgs a, const float* ws, int Cp) {
#pragma clang fp contract(off)  // separate roundings, as the reference's blend
  // LDS: the block's 128 pixels' corners (4 image-pixel indices, -1 outside; 4 weights), then
  // the outputs [C][128 + 1]
  __shared__ int cidx[kGatherPx][4];
  __shared__ float cw[kGatherPx][4];
  extern __shared__ float otile[];
  const int n = blockIdx.y;
  const int64_t HW = (int64_t)a.H * a.W;
  const int64_t p0 = (int64_t)blockIdx.x * kGatherPx;
  const int np = (int)min<int64_t>(kGatherPx, HW - p0);
  if (threadIdx.x < np) {  // corners once per pixel (flow reads coalesced)
    const int64_t p = p0 + threadIdx.x;
    const int y = (int)(p / a.W), x = (int)(p - (int64_t)y * a.W);
    const Corners q = corners_of(a, n, y, x);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      cidx[threadIdx.x][k] = q.ok[k] ? (q.y0 + (k >> 1)) * a.Wi + q.x0 + (k & 1) : -1;
      cw[threadIdx.x][k] = q.w[k];
    }
  }
  __syncthreads();
  const int G = Cp >> 2;
  const float4* img = reinterpret_cast<const float4*>(ws + (int64_t)n * a.Hi * a.Wi * Cp);
  constexpr int U = 4;  // items per lane in flight: 16 gathers issued before the first blend
  for (int i0 = threadIdx.x; i0 < np * G; i0 += U * kWarpThreads) {
    float4 v[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * kWarpThreads;
      const int px = min(i / G, np - 1), g = i - (i / G) * G;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ci = i < np * G ? cidx[px][k] : -1;
        v[u][k] = ci >= 0 ? img[(int64_t)ci * G + g] : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * kWarpThreads;
      if (i >= np * G) break;
      const int px = i / G, g = i - px * G;
      const float* w = cw[px];
      const float4* vv = v[u];
      const float r[4] = {vv[0].x * w[0] + vv[1].x * w[1] + vv[2].x * w[2] + vv[3].x * w[3],
                          vv[0].y * w[0] + vv[1].y * w[1] + vv[2].y * w[2] + vv[3].y * w[3],
                          vv[0].z * w[0] + vv[1].z * w[1] + vv[2].z * w[2] + vv[3].z * w[3],
                          vv[0].w * w[0] + vv[1].w * w[1] + vv[2].w * w[2] + vv[3].w * w[3]};
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (4 * g + j < a.C) otile[(4 * g + j) * (kGatherPx + 1) + px] = r[j];
    }
  }
  __syncthreads();
  float* ob = a.out + (int64_t)n * a.C * HW + p0;
  for (int i = threadIdx.x; i < a.C * kGatherPx; i += kWarpThreads) {
    const int c = i / kGatherPx, px = i % kGatherPx;
    if (px < np) ob[(int64_t)c * HW + px] = otile[c * (kGatherPx + 1) + px];
  }
}

// Disparity (one-channel flow) warps: iy does not depend on x, so output row y reads only
// image rows y0 = floor(iy) and y0 + 1.  A block owns (n, y, a chunk of CC channels): it copies
// those two rows of its channels into LDS with coalesced 16-B loads (column 0 is a zero pad
// that out-of-image corners read), then every lane blends its pixels from LDS: the random
// per-lane x of a disparity map costs LDS bank conflicts instead of one L1 request per lane.
// Same operation sequence (and results) as warp_kernel.
template <bool V4>
__global__ __launch_bounds__(kWarpThreads) void warp_rows_kernel(WarpArgs a, int CC) {
#pragma clang fp contract(off)
  extern __shared__ float srow[];  // [CC][2][Wi + 4]: element 3 of each row is the zero pad
  const int c0 = blockIdx.x * CC;
  const int y = blockIdx.y;
  const int n = blockIdx.z;
  const int nc = min(CC, a.C - c0);
  const int RS = a.Wi + 4;  // row stride in LDS (16-B aligned rows, data from element 4)
  const float gy = 2.0f * (float)y / a.dh - 1.0f;
  const float iy = (gy + 1.0f) * a.sy - 0.5f;
  const float fy0 = floorf(iy);
  const float dy = iy - fy0, sy = 1.0f - dy;
  const bool finite = fabsf(iy) < 2.0e9f;
  const int y0 = finite ? (int)fy0 : -2;
  // the flow values of this lane's first kPre pixels are loaded before the staging loads, so
  // their latency overlaps the rows' instead of following the barrier
  const float* fl = a.flow + n * a.fsn + (int64_t)y * a.fsh;
  constexpr int kPre = 4;
  float fv[kPre];
#pragma unroll
  for (int k = 0; k < kPre; ++k) {
    const int x = threadIdx.x + k * kWarpThreads;
    fv[k] = x < a.W ? fl[x] : 0.f;
  }
  // ---- stage rows y0, y0 + 1 of channels c0 .. c0 + nc (all loads of a lane issued first)
  const float* ib = a.img + n * a.isn + (int64_t)c0 * a.isc;
  const bool r0ok = y0 >= 0 && y0 < a.Hi, r1ok = y0 + 1 >= 0 && y0 + 1 < a.Hi;
  const int64_t roff0 = (int64_t)(r0ok ? y0 : 0) * a.ish, roff1 = (int64_t)(r1ok ? y0 + 1 : 0) * a.ish;
  if (threadIdx.x < 2 * nc) srow[threadIdx.x * RS + 3] = 0.f;
  if (V4) {
    const int Q = a.Wi >> 2, total = 2 * nc * Q;
    constexpr int U = 8;
    for (int i0 = threadIdx.x; i0 < total; i0 += U * kWarpThreads) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * kWarpThreads;
        const int r = i / Q, q = i - r * Q;
        const bool ok = i < total && ((r & 1) ? r1ok : r0ok);
        v[u] = ok ? reinterpret_cast<const float4*>(ib + (int64_t)(r >> 1) * a.isc + ((r & 1) ? roff1 : roff0))[q]
                  : make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + u * kWarpThreads;
        const int r = i / Q, q = i - r * Q;
        if (i < total) reinterpret_cast<float4*>(srow + r * RS + 4)[q] = v[u];
      }
    }
  } else {
    const int total = 2 * nc * a.Wi;
    for (int i = threadIdx.x; i < total; i += kWarpThreads) {
      const int r = i / a.Wi, q = i - r * a.Wi;
      const bool ok = (r & 1) ? r1ok : r0ok;
      srow[r * RS + 4 + q] = ok ? ib[(int64_t)(r >> 1) * a.isc + ((r & 1) ? roff1 : roff0) + q] : 0.f;
    }
  }
  const int64_t HW = (int64_t)a.H * a.W;
  float* ob = a.out + ((int64_t)n * a.C + c0) * HW + (int64_t)y * a.W;
  // pixel x with flow f: LDS columns of its two corners and the four bilinear weights
  auto corners = [&](int x, float f, int& ia, int& ib2, float (&w)[4]) {
    float gx = (float)x - f;
    gx = 2.0f * gx / a.dw - 1.0f;
    const float ix = (gx + 1.0f) * a.sx - 0.5f;
    const float fx0 = floorf(ix);
    const float dx = ix - fx0, ex = 1.0f - dx;
    w[0] = sy * ex, w[1] = sy * dx, w[2] = dy * ex, w[3] = dy * dx;  // nw, ne, sw, se
    const bool ok = finite && fabsf(ix) < 2.0e9f;
    const int x0 = ok ? (int)fx0 : -2;
    ia = (ok && x0 >= 0 && x0 < a.Wi) ? x0 + 4 : 3;
    ib2 = (ok && x0 + 1 >= 0 && x0 + 1 < a.Wi) ? x0 + 5 : 3;
  };
  auto blend = [&](int x, int ia, int ib2, const float (&w)[4]) {
    for (int c = 0; c < nc; ++c) {
      const float* s0 = srow + (2 * c) * RS;
      const float* s1 = s0 + RS;
      ob[(int64_t)c * HW + x] = s0[ia] * w[0] + s0[ib2] * w[1] + s1[ia] * w[2] + s1[ib2] * w[3];
    }
  };
  int pa[kPre], pb[kPre];
  float pw[kPre][4];
#pragma unroll
  for (int k = 0; k < kPre; ++k) corners(threadIdx.x + k * kWarpThreads, fv[k], pa[k], pb[k], pw[k]);
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kPre; ++k) {
    const int x = threadIdx.x + k * kWarpThreads;
    if (x < a.W) blend(x, pa[k], pb[k], pw[k]);
  }
  for (int x = threadIdx.x + kPre * kWarpThreads; x < a.W; x += kWarpThreads) {  // W > 1024
    int ia, ib2;
    float w[4];
    corners(x, fl[x], ia, ib2, w);
    blend(x, ia, ib2, w);
  }
}

}  // namespace

// Bytes of the channel-last image copy the two-channel path uses (0: the shape takes the other
// kernels).
int64_t warp_workspace_bytes(int64_t N, int64_t C, int64_t Hi, int64_t Wi, int64_t flow_channels) {
  if (flow_channels != 2 || N <= 0 || C <= 0 || C > 64 || Hi <= 0 || Wi <= 0) return 0;
  const int64_t Cp = (C + 3) / 4 * 4;
  if (Hi * Wi >= ((int64_t)1 << 31) || N * Hi * Wi * Cp >= ((int64_t)1 << 40)) return 0;
  return N * Hi * Wi * Cp * 4;
}

int warp_entry(const void* image, const void* flow, void* out, int dtype, int64_t N, int64_t C,
               int64_t Hi, int64_t Wi, int64_t H, int64_t W, int64_t flow_channels,
               const int64_t* image_strides, const int64_t* flow_strides, void* stream,
               void* workspace, int64_t workspace_bytes) {
  if (dtype != SM_F32) return fail(SM_EDTYPE, "warp_by_flow_map: float32 image and flow only");
  if (N < 0 || C < 0 || Hi < 0 || Wi < 0 || H < 0 || W < 0) return fail(SM_EINVAL, "negative size");
  if (flow_channels != 1 && flow_channels != 2)
    return fail(SM_EINVAL, "invalid flow map dimension (1 or 2)");
  if (N > 65535) return fail(SM_EINVAL, "N > 65535 not supported");
  if (H * W >= ((int64_t)1 << 31) || Hi >= INT32_MAX || Wi >= INT32_MAX || C >= INT32_MAX)
    return fail(SM_EINVAL, "warp_by_flow_map: plane too large");
  if (N * C * H * W == 0) return SM_OK;
  if (image == nullptr || flow == nullptr || out == nullptr) return fail(SM_EINVAL, "null pointer");
  WarpArgs a;
  a.img = static_cast<const float*>(image);
  a.flow = static_cast<const float*>(flow);
  a.out = static_cast<float*>(out);
  a.C = (int)C, a.H = (int)H, a.W = (int)W, a.Hi = (int)Hi, a.Wi = (int)Wi;
  a.fch = (int)flow_channels;
  if (image_strides) {
    if (image_strides[3] != 1 && Wi > 1) return fail(SM_EINVAL, "image: W stride must be 1");
    a.isn = image_strides[0], a.isc = image_strides[1], a.ish = image_strides[2];
  } else {
    a.ish = Wi, a.isc = Hi * Wi, a.isn = C * Hi * Wi;
  }
  if (flow_strides) {
    if (flow_strides[3] != 1 && W > 1) return fail(SM_EINVAL, "flow: W stride must be 1");
    a.fsn = flow_strides[0], a.fsc = flow_strides[1], a.fsh = flow_strides[2];
  } else {
    a.fsh = W, a.fsc = H * W, a.fsn = flow_channels * H * W;
  }
  // the reference's scalars: (w - 1.0), (h - 1.0) rounded to the grid dtype; Wi / 2, Hi / 2
  a.dw = (float)((double)W - 1.0);
  a.dh = (float)((double)H - 1.0);
  a.sx = (float)Wi / 2.0f;
  a.sy = (float)Hi / 2.0f;
  hipStream_t st = as_stream(stream);
  // disparity warps with rows that fit: the LDS row kernel, CC channels per block (<= 32 KB)
  const int64_t row_bytes = 2 * (Wi + 4) * 4;
  if (flow_channels == 1 && row_bytes <= 32768 && H <= 65535) {
    // CC = 4 at Wi = 960 (measured r01: CC 1/2/4/8 -> 70/48/42/58 us on 1x32x540x960)
    const int CC = (int)std::max<int64_t>(1, std::min<int64_t>(8, 32768 / row_bytes));
    const bool v4 = (Wi % 4 == 0) && (a.ish % 4 == 0) && (a.isc % 4 == 0) && (a.isn % 4 == 0) &&
                    ((reinterpret_cast<uintptr_t>(image) & 15u) == 0);
    dim3 grid((unsigned)ceil_div(C, CC), (unsigned)H, (unsigned)N);
    const size_t shm = (size_t)CC * row_bytes;
    if (v4)
      hipLaunchKernelGGL(warp_rows_kernel<true>, grid, dim3(kWarpThreads), shm, st, a, CC);
    else
      hipLaunchKernelGGL(warp_rows_kernel<false>, grid, dim3(kWarpThreads), shm, st, a, CC);
    return check_launch("warp_rows_kernel");
  }
  const int64_t need = warp_workspace_bytes(N, C, Hi, Wi, flow_channels);
  if (need > 0 && workspace != nullptr && workspace_bytes >= need &&
      (reinterpret_cast<uintptr_t>(workspace) & 15u) == 0 && Hi <= 65535) {
    const int Cp = (int)((C + 3) / 4 * 4);
    float* ws = static_cast<float*>(workspace);
    hipLaunchKernelGGL(warp_to_nhwc, dim3((unsigned)ceil_div(Wi, kNhwcPx), (unsigned)Hi, (unsigned)N),
                       dim3(kWarpThreads), (size_t)kNhwcPx * (Cp + 1) * 4, st, a, ws, Cp);
    if (int rc = check_launch("warp_to_nhwc")) return rc;
    hipLaunchKernelGGL(warp_gather_nhwc, dim3((unsigned)ceil_div(H * W, kGatherPx), (unsigned)N),
                       dim3(kWarpThreads), (size_t)C * (kGatherPx + 1) * 4, st, a,
                       static_cast<const float*>(ws), Cp);
    return check_launch("warp_gather_nhwc");
  }
  // channels per block: the waves in flight share a few channel planes (1x32x540x960, sigma-4
  // flow: 94-96 us with 8 channels per block against 100 us with all 32; r03 A/B).  An LDS
  // window of the tile's source rows (8 x 32 tile, 8-pixel halo) measured slower (133 us).
  const int cpb = 8;
  dim3 grid((unsigned)ceil_div(H * W, kWarpThreads), (unsigned)ceil_div(C, cpb), (unsigned)N);
  hipLaunchKernelGGL(warp_kernel, grid, dim3(kWarpThreads), 0, st, a, cpb);
  return check_launch("warp_kernel");
}

}  // namespace smcv

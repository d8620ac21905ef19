// Copy-type cost volumes (pure HBM-write kernels): concatenate, interweave, shifted
// interweave and the difference volume.
//
// Reference semantics (babiking/realtime_stereo_matcher):
//   concatenate        cost_volume/concatenate.py:11-41     (N,2C,H,W,D), 0 for x<d
//   interweave         cost_volume/interweave.py:10-22      (N,2C,H,W), even=L, odd=R
//                      = interweave_tensors model/mobile_stereo_net_v4.py:17-23
//   shifted interweave model/mobile_stereo_net_v4.py:443-461 (N,2C,D,H,W), 0 for x<d
//   difference volume  model/mobile_stereo_net.py:8-27        (N,C,D,H,W), 1.0 for x<d
//
// One workgroup owns one (n, c, y) feature row: the left and right rows are staged once
// in LDS (raw bits, so copies are bit-exact), then every output row that depends on them
// (D shifted copies) is streamed out with 16-byte stores.  Inputs are read once from HBM;
// the kernels are bound by the HBM write stream.
#include "common.h"

namespace smcv {
namespace {

constexpr int kThreads = 256;
constexpr int kRowMax = 8192;  // elements of one staged row (fp32: 32 KiB per row)

template <int BYTES> struct raw;
template <> struct raw<2> { using type = uint16_t; };
template <> struct raw<4> { using type = uint32_t; };
template <> struct raw<8> { using type = uint64_t; };

// 16-byte vector of raw elements.
template <typename U> struct vec16 {
  static constexpr int N = 16 / sizeof(U);
  U v[N];
};

// Plain 16-B stores: streaming whole 128-B lines they write at 5.8-6.2 TB/s, where the
// non-temporal form reached 5.1 TB/s (store microbenchmark, r01).
template <typename U>
__device__ __forceinline__ void store16(U* dst, const vec16<U>& s) {
  *reinterpret_cast<uint4*>(dst) = *reinterpret_cast<const uint4*>(s.v);
}

// Stage left/right rows (n, c, y) into LDS as raw bits.
template <typename U>
__device__ __forceinline__ void stage_rows(U* Ls, U* Rs, const U* Lrow, const U* Rrow, int W) {
  for (int x = threadIdx.x; x < W; x += kThreads) {
    Ls[x] = Lrow[x];
    Rs[x] = Rrow[x];
  }
  __syncthreads();
}

// ------------------------------------------------------------------ concatenate (N,2C,H,W,D)
template <typename U, bool VEC, bool DV>
__global__ __launch_bounds__(kThreads) void concat_kernel(const U* __restrict__ L,
                                                          const U* __restrict__ R,
                                                          U* __restrict__ out, int C, int H,
                                                          int W, int D, Strides4 ls, Strides4 rs,
                                                          int lgdv) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_c[];
  U* Ls = reinterpret_cast<U*>(smem_c);
  U* Rs = Ls + W;
  const int row = blockIdx.x;  // (n*C + c)*H + y
  const int y = row % H;
  const int nc = row / H;
  const int c = nc % C;
  const int n = nc / C;
  stage_rows(Ls, Rs, L + n * ls.n + (int64_t)c * ls.c + (int64_t)y * ls.h,
             R + n * rs.n + (int64_t)c * rs.c + (int64_t)y * rs.h, W);
  const size_t span = (size_t)W * D;
  U* outL = out + (((size_t)n * 2 * C + c) * H + y) * span;
  U* outR = out + (((size_t)n * 2 * C + C + c) * H + y) * span;
  const unsigned uD = (unsigned)D;
  if (VEC) {
    constexpr int NV = vec16<U>::N;
    const unsigned nvec = (unsigned)(span / NV);
    for (unsigned v = threadIdx.x; v < nvec; v += kThreads) {
      const unsigned e0 = v * NV;
      vec16<U> a, b;
      if (DV) {  // whole vector shares one x
        // D / NV a power of two (lgdv >= 0, uniform): a shift instead of an integer division
        const unsigned x = lgdv >= 0 ? v >> lgdv : e0 / uD;
        const unsigned d0 = lgdv >= 0 ? (v & ((1u << lgdv) - 1)) * NV : e0 - x * uD;
        const U lx = Ls[x];
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const unsigned d = d0 + k;
          const bool ok = d <= x;
          a.v[k] = ok ? lx : U(0);
          b.v[k] = ok ? Rs[ok ? x - d : 0] : U(0);
        }
      } else {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const unsigned e = e0 + k;
          const unsigned x = e / uD;
          const unsigned d = e - x * uD;
          const bool ok = d <= x;
          a.v[k] = ok ? Ls[x] : U(0);
          b.v[k] = ok ? Rs[ok ? x - d : 0] : U(0);
        }
      }
      store16(outL + e0, a);
      store16(outR + e0, b);
    }
  } else {
    for (unsigned e = threadIdx.x; e < span; e += kThreads) {
      const unsigned x = e / uD;
      const unsigned d = e - x * uD;
      const bool ok = d <= x;
      outL[e] = ok ? Ls[x] : U(0);
      outR[e] = ok ? Rs[ok ? x - d : 0] : U(0);
    }
  }
}

// ------------------------------------------------------------------ interweave (N,2C,H,W)
template <typename U, bool VEC>
__global__ __launch_bounds__(kThreads) void interweave_kernel(const U* __restrict__ L,
                                                              const U* __restrict__ R,
                                                              U* __restrict__ out, int C, int H,
                                                              int W, Strides4 ls, Strides4 rs) {
  const int row = blockIdx.x;
  const int y = row % H;
  const int nc = row / H;
  const int c = nc % C;
  const int n = nc / C;
  const U* Lrow = L + n * ls.n + (int64_t)c * ls.c + (int64_t)y * ls.h;
  const U* Rrow = R + n * rs.n + (int64_t)c * rs.c + (int64_t)y * rs.h;
  U* oL = out + (((size_t)n * 2 * C + 2 * c) * H + y) * (size_t)W;
  U* oR = out + (((size_t)n * 2 * C + 2 * c + 1) * H + y) * (size_t)W;
  if (VEC) {
    constexpr int NV = vec16<U>::N;
    const int nvec = W / NV;
    for (int v = threadIdx.x; v < nvec; v += kThreads) {
      const uint4 a = reinterpret_cast<const uint4*>(Lrow)[v];
      const uint4 b = reinterpret_cast<const uint4*>(Rrow)[v];
      reinterpret_cast<uint4*>(oL)[v] = a;
      reinterpret_cast<uint4*>(oR)[v] = b;
    }
  } else {
    for (int x = threadIdx.x; x < W; x += kThreads) {
      oL[x] = Lrow[x];
      oR[x] = Rrow[x];
    }
  }
}

// one subtraction in the input dtype (fp64 natively; the 16-bit types through fp32, exact
// before the one rounding), and the difference volume's 1.0 fill
template <typename T> __device__ __forceinline__ T diff(T a, T b) { return from_f<T>(to_f(a) - to_f(b)); }
template <> __device__ __forceinline__ double diff<double>(double a, double b) { return a - b; }
template <typename T> __device__ __forceinline__ T one() { return from_f<T>(1.f); }
template <> __device__ __forceinline__ double one<double>() { return 1.0; }
template <typename T> __device__ __forceinline__ T zero() { return from_f<T>(0.f); }
template <> __device__ __forceinline__ double zero<double>() { return 0.0; }

// ------------------------------------------- shifted interweave (N,2C,D,H,W) / diff (N,C,D,H,W)
// MODE 0: shifted interweave (raw copy, 0 fill); MODE 1: L - R(x-d) with 1.0 fill.
template <typename T, int MODE, bool VEC, bool STAGED>
__global__ __launch_bounds__(kThreads) void shifted_rows_kernel(const T* __restrict__ L,
                                                                const T* __restrict__ R,
                                                                T* __restrict__ out, int C, int H,
                                                                int W, int D, Strides4 ls,
                                                                Strides4 rs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_s[];
  T* Ls = reinterpret_cast<T*>(smem_s);
  T* Rs = Ls + (STAGED ? W : 0);
  const int row = blockIdx.x;
  const int y = row % H;
  const int nc = row / H;
  const int c = nc % C;
  const int n = nc / C;
  const T* Lrow = L + n * ls.n + (int64_t)c * ls.c + (int64_t)y * ls.h;
  const T* Rrow = R + n * rs.n + (int64_t)c * rs.c + (int64_t)y * rs.h;
  const T* Lsrc = Lrow;
  const T* Rsrc = Rrow;
  if (STAGED) {
    for (int x = threadIdx.x; x < W; x += kThreads) {
      Ls[x] = Lrow[x];
      Rs[x] = Rrow[x];
    }
    __syncthreads();
    Lsrc = Ls;
    Rsrc = Rs;
  }
  const size_t plane = (size_t)H * W;
  T* base0;
  T* base1;
  T zero_or_one;
  if (MODE == 0) {
    base0 = out + ((size_t)n * 2 * C + 2 * c) * D * plane + (size_t)y * W;
    base1 = out + ((size_t)n * 2 * C + 2 * c + 1) * D * plane + (size_t)y * W;
    zero_or_one = zero<T>();
  } else {
    base0 = out + ((size_t)n * C + c) * D * plane + (size_t)y * W;
    base1 = base0;
    zero_or_one = one<T>();
  }
  constexpr int NV = 16 / sizeof(T);
  for (int d = 0; d < D; ++d) {
    T* o0 = base0 + (size_t)d * plane;
    T* o1 = base1 + (size_t)d * plane;
    if (VEC) {
      const int nvec = W / NV;
      for (int v = threadIdx.x; v < nvec; v += kThreads) {
        const int x0 = v * NV;
        T a[NV], b[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          const int x = x0 + k;
          const bool ok = x >= d;
          const T lv = Lsrc[x];
          const T rv = Rsrc[ok ? x - d : 0];
          if (MODE == 0) {
            a[k] = ok ? lv : zero_or_one;
            b[k] = ok ? rv : zero_or_one;
          } else {
            a[k] = ok ? diff(lv, rv) : zero_or_one;
          }
        }
        using V = typename raw<sizeof(T)>::type;
        store16(reinterpret_cast<V*>(o0 + x0), *reinterpret_cast<const vec16<V>*>(a));
        if (MODE == 0) store16(reinterpret_cast<V*>(o1 + x0), *reinterpret_cast<const vec16<V>*>(b));
      }
    } else {
      for (int x = threadIdx.x; x < W; x += kThreads) {
        const bool ok = x >= d;
        const T lv = Lsrc[x];
        const T rv = Rsrc[ok ? x - d : 0];
        if (MODE == 0) {
          o0[x] = ok ? lv : zero_or_one;
          o1[x] = ok ? rv : zero_or_one;
        } else {
          o0[x] = ok ? diff(lv, rv) : zero_or_one;
        }
      }
    }
  }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

int check_dot_args(const void* left, const void* right, const void* out, int dtype, int64_t N,
                   int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                   const int64_t* r_strides, Strides4* ls, Strides4* rs);

int concat_entry(const void* left, const void* right, void* out, int dtype, int64_t N,
                 int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                 const int64_t* r_strides, void* stream) {
  Strides4 ls, rs;
  int rc = check_dot_args(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &ls, &rs);
  if (rc) return rc;
  if (N * C * H * W * D == 0) return SM_OK;
  if (W > kRowMax) return fail(SM_EINVAL, "concat: W > 8192 not supported");
  if (N * C * H > (int64_t)INT32_MAX || W * D > (int64_t)UINT32_MAX)
    return fail(SM_EINVAL, "concat: volume too large");
  const int es = elem_size(dtype);
  const int nv = 16 / es;
  const bool vec = ((W * D) % nv == 0) && aligned16(out);
  const bool dv = (D % nv == 0);
  const int64_t dvec = D / nv;  // vectors per pixel on the DV path
  const int lgdv = dv && (dvec & (dvec - 1)) == 0 ? __builtin_ctzll((unsigned long long)dvec) : -1;
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)(N * C * H));
  const size_t shm = 2 * (size_t)W * es;
#define SM_CONCAT_LAUNCH(U)                                                                     \
  do {                                                                                         \
    const U* l = static_cast<const U*>(left);                                                  \
    const U* r = static_cast<const U*>(right);                                                 \
    U* o = static_cast<U*>(out);                                                               \
    if (vec && dv)                                                                             \
      hipLaunchKernelGGL((concat_kernel<U, true, true>), grid, dim3(kThreads), shm, st, l, r, o, \
                         (int)C, (int)H, (int)W, (int)D, ls, rs, lgdv);                        \
    else if (vec)                                                                              \
      hipLaunchKernelGGL((concat_kernel<U, true, false>), grid, dim3(kThreads), shm, st, l, r, \
                         o, (int)C, (int)H, (int)W, (int)D, ls, rs, -1);                       \
    else                                                                                       \
      hipLaunchKernelGGL((concat_kernel<U, false, false>), grid, dim3(kThreads), shm, st, l, r, \
                         o, (int)C, (int)H, (int)W, (int)D, ls, rs, -1);                       \
  } while (0)
  if (es == 8) SM_CONCAT_LAUNCH(uint64_t); else if (es == 4) SM_CONCAT_LAUNCH(uint32_t); else SM_CONCAT_LAUNCH(uint16_t);
#undef SM_CONCAT_LAUNCH
  return check_launch("concat_kernel");
}

int interweave_entry(const void* left, const void* right, void* out, int dtype, int64_t N,
                     int64_t C, int64_t H, int64_t W, const int64_t* l_strides,
                     const int64_t* r_strides, void* stream) {
  Strides4 ls, rs;
  int rc = check_dot_args(left, right, out, dtype, N, C, H, W, 1, l_strides, r_strides, &ls, &rs);
  if (rc) return rc;
  if (N * C * H * W == 0) return SM_OK;
  if (N * C * H > (int64_t)INT32_MAX) return fail(SM_EINVAL, "interweave: too many rows");
  const int es = elem_size(dtype);
  const int nv = 16 / es;
  // vector path needs every row start 16-B aligned on both sides
  const bool vec = (W % nv == 0) && aligned16(out) && aligned16(left) && aligned16(right) &&
                   ls.n % nv == 0 && ls.c % nv == 0 && ls.h % nv == 0 && rs.n % nv == 0 &&
                   rs.c % nv == 0 && rs.h % nv == 0;
  hipStream_t st = as_stream(stream);
  dim3 grid((unsigned)(N * C * H));
#define SM_IW_LAUNCH(U)                                                                         \
  do {                                                                                         \
    const U* l = static_cast<const U*>(left);                                                  \
    const U* r = static_cast<const U*>(right);                                                 \
    U* o = static_cast<U*>(out);                                                               \
    if (vec)                                                                                   \
      hipLaunchKernelGGL((interweave_kernel<U, true>), grid, dim3(kThreads), 0, st, l, r, o,   \
                         (int)C, (int)H, (int)W, ls, rs);                                      \
    else                                                                                       \
      hipLaunchKernelGGL((interweave_kernel<U, false>), grid, dim3(kThreads), 0, st, l, r, o,  \
                         (int)C, (int)H, (int)W, ls, rs);                                      \
  } while (0)
  if (es == 8) SM_IW_LAUNCH(uint64_t); else if (es == 4) SM_IW_LAUNCH(uint32_t); else SM_IW_LAUNCH(uint16_t);
#undef SM_IW_LAUNCH
  return check_launch("interweave_kernel");
}

template <typename T, int MODE>
static int launch_shifted(const void* left, const void* right, void* out, int64_t N, int64_t C,
                          int64_t H, int64_t W, int64_t D, Strides4 ls, Strides4 rs,
                          hipStream_t st) {
  const int nv = 16 / (int)sizeof(T);
  const bool vec = (W % nv == 0) && aligned16(out);
  const bool staged = W <= kRowMax;
  const size_t shm = staged ? 2 * (size_t)W * sizeof(T) : 0;
  dim3 grid((unsigned)(N * C * H));
  const T* l = static_cast<const T*>(left);
  const T* r = static_cast<const T*>(right);
  T* o = static_cast<T*>(out);
  const int iC = (int)C, iH = (int)H, iW = (int)W, iD = (int)D;
  if (vec && staged)
    hipLaunchKernelGGL((shifted_rows_kernel<T, MODE, true, true>), grid, dim3(kThreads), shm, st,
                       l, r, o, iC, iH, iW, iD, ls, rs);
  else if (staged)
    hipLaunchKernelGGL((shifted_rows_kernel<T, MODE, false, true>), grid, dim3(kThreads), shm, st,
                       l, r, o, iC, iH, iW, iD, ls, rs);
  else if (vec)
    hipLaunchKernelGGL((shifted_rows_kernel<T, MODE, true, false>), grid, dim3(kThreads), shm, st,
                       l, r, o, iC, iH, iW, iD, ls, rs);
  else
    hipLaunchKernelGGL((shifted_rows_kernel<T, MODE, false, false>), grid, dim3(kThreads), shm,
                       st, l, r, o, iC, iH, iW, iD, ls, rs);
  return check_launch("shifted_rows_kernel");
}

int shifted_entry(const void* left, const void* right, void* out, int dtype, int64_t N,
                  int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                  const int64_t* r_strides, int mode, void* stream) {
  Strides4 ls, rs;
  int rc = check_dot_args(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &ls, &rs);
  if (rc) return rc;
  if (N * C * H * W * D == 0) return SM_OK;
  if (N * C * H > (int64_t)INT32_MAX) return fail(SM_EINVAL, "too many feature rows");
  hipStream_t st = as_stream(stream);
  if (mode == 0) {
    // raw-bit copy: fp16 and bf16 share one 16-bit instantiation
    if (dtype == SM_F64) return launch_shifted<double, 0>(left, right, out, N, C, H, W, D, ls, rs, st);
    if (dtype == SM_F32) return launch_shifted<float, 0>(left, right, out, N, C, H, W, D, ls, rs, st);
    return launch_shifted<__half, 0>(left, right, out, N, C, H, W, D, ls, rs, st);
  }
  if (dtype == SM_F64) return launch_shifted<double, 1>(left, right, out, N, C, H, W, D, ls, rs, st);
  SM_DISPATCH_DTYPE(dtype, T,
                    return launch_shifted<T, 1>(left, right, out, N, C, H, W, D, ls, rs, st));
  return SM_OK;
}

}  // namespace smcv

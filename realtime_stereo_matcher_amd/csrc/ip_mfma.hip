// Inner-product / correlation cost volume on the gfx950 matrix cores.
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// Per image row the volume is a BAND of the C-contraction S[j][x] = sum_c R[c][j] L[c][x]
// (d = x - j in [0, D)).  One workgroup owns a row segment of 64 left pixels; each of its four
// waves owns a 16-pixel x-block and accumulates the T = 1 + ceil((D-1)/16) 16x16 S-blocks of its
// band (8 % over-compute at D = 192) with v_mfma_f32_16x16x32_bf16, K = 32 channels per step.
//
// fp32 features are split EXACTLY into three bf16 planes (x = h + m + l, 8+8+8 significand
// bits); the six partial products h*h, h*m, m*h, h*l, m*m, l*h are accumulated in fp32 by the
// MFMA.  The three dropped terms are O(2^-24) relative, so the result is fp32-accurate
// (|err| ~ 1e-6 at C = 64, bar 1e-4) and EXACT for small-integer features (argmin bit-exact).
// fp16 features need two planes (11 bits) and 4 products (exact products); bf16 needs one.
// The matrix cores run at 16x the fp32 rate, so even 6 products leave the kernel HBM-bound.
//
// Data path per 32-channel step: the right WINDOW R[j0 .. j0+64+16(T-1)) and the left tile are
// loaded (coalesced along the row), split, and written to LDS pixel-major ([pixel][32 ch], 64 B
// per row and plane) with an XOR chunk swizzle that makes every ds_read_b128 fragment read
// bank-conflict free; the window is re-used by all T blocks of all four waves (the disparity
// sweep never re-reads HBM).  Epilogue: the accumulators are sheared (d = x - j) into an LDS
// [D][64] fp32 tile and streamed out as 256-B row segments (out rows are x-contiguous).
// Workgroups are remapped so that the x-tiles of one image row run on one XCD (shared L2 for
// the overlapping right windows).
#include "common.h"

#include <cstdlib>

namespace smcv {
namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kXT = 64;        // left pixels per workgroup (4 waves x 16)
constexpr int kKC = 32;        // channels per MFMA k-step
constexpr int kRowBytes = 64;  // one LDS pixel row of one plane: 32 bf16

// byte offset of (pixel row r, 16-B channel chunk ch) inside one plane: conflict-free for the
// 16x16x32 fragment read pattern (lane l -> row l&15, chunk l>>4) under the four ds_read_b128
// lane groups of gfx950 (MI355X_MICROARCH.md §LDS).
__device__ __forceinline__ int swz(int r, int ch) { return r * kRowBytes + 16 * (ch ^ ((r >> 2) & 2)); }

// 8 consecutive channels [cb, cb+8) of pixel j of one feature row; zero outside the image or
// past C.  Addresses are clamped and masked with selects (no branch around the loads, so the
// eight loads stay in flight together).
template <typename T>
__device__ __forceinline__ void load8(const T* __restrict__ rowp, int64_t cstride, int cb, int C,
                                      int j, int W, float (&v)[8]) {
  const bool okj = (j >= 0) && (j < W);
  const int jc = min(max(j, 0), W - 1);
  if (C <= 0) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
    return;
  }
  if (cb + 8 <= C) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = to_f(rowp[(int64_t)(cb + i) * cstride + jc]);
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = to_f(rowp[(int64_t)min(cb + i, C - 1) * cstride + jc]);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (cb + i < C) ? v[i] : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = okj ? v[i] : 0.f;
}

template <int P>
__device__ __forceinline__ void split8(const float (&v)[8], uint4 (&q)[P]) {
  // exact split x = h + m + l into bf16 planes (non-finite values keep everything in h)
  union U {
    __bf16 b[8];
    uint4 u;
  };
  U h, m, l;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float x = v[i];
    const __bf16 bh = (__bf16)x;
    h.b[i] = bh;
    if (P > 1) {
      const bool fin = __builtin_isfinite(x);
      const float r1 = fin ? x - (float)bh : 0.f;
      const __bf16 bm = (__bf16)r1;
      m.b[i] = bm;
      if (P > 2) l.b[i] = (__bf16)(r1 - (float)bm);
    }
  }
  q[0] = h.u;
  if (P > 1) q[1] = m.u;
  if (P > 2) q[2] = l.u;
}

// 4 consecutive outputs (16-B aligned for fp32, 8-B for 16-bit types) in one store.
template <typename T>
__device__ __forceinline__ void store4(T* o, float4 v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(o) = v;
  } else {
    union {
      T e[4];
      uint2 u;
    } pk;
    pk.e[0] = from_f<T>(v.x);
    pk.e[1] = from_f<T>(v.y);
    pk.e[2] = from_f<T>(v.z);
    pk.e[3] = from_f<T>(v.w);
    *reinterpret_cast<uint2*>(o) = pk.u;
  }
}

// One unit of work: a 64-pixel segment of one image row and one pass of at most DMAX
// disparities.  Consecutive work ids are the x-tiles of one row (they share right columns).
struct BandWork {
  int n, y, x0, dp, Dp, Tn, rwin, js;
};

__device__ __forceinline__ BandWork band_decode(int w, int tiles, int npass, int H, int D, int dmax) {
  BandWork k;
  const int pass = w % npass;
  const int rest = w / npass;
  const int tile = rest % tiles;
  const int row = rest / tiles;
  k.y = row % H;
  k.n = row / H;
  k.x0 = tile * kXT;
  k.dp = pass * dmax;
  k.Dp = min(dmax, D - k.dp);
  k.Tn = 1 + (k.Dp - 1 + 15) / 16;       // 16x16 band blocks per x-block
  k.rwin = kXT + 16 * (k.Tn - 1);        // right-window rows
  k.js = k.x0 - k.dp - 16 * (k.Tn - 1);  // right column held in window row 0
  return k;
}

// Persistent, software-pipelined band kernel.  Each workgroup walks a contiguous range of
// work ids owned by its XCD group; the global loads of the NEXT (work, 32-channel step) are
// issued into registers before the MFMAs and the epilogue of the current one, so HBM latency
// hides behind compute and the output stream.
template <typename T, int P, int TMAX>
__global__ __launch_bounds__(kThreads, 2) void ip_band_mfma(
    const T* __restrict__ L, const T* __restrict__ R, T* __restrict__ out, int C, int H, int W,
    int D, Strides4 ls, Strides4 rs, int divisor, int tiles, int npass, int nwork, int ablate) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int DMAX = 16 * (TMAX - 1);
  constexpr int NR = (3 + TMAX) / 4;  // window staging items per thread = RWIN*4/256 at Tn=TMAX

  // work range of this workgroup's XCD group (blocks b and b+8 share an XCD)
  const int grp = blockIdx.x & 7;
  const int gi = blockIdx.x >> 3;
  const int gsz = gridDim.x >> 3;
  const int q = nwork >> 3, rr = nwork & 7;
  const int wbeg = grp < rr ? grp * (q + 1) : rr * (q + 1) + (grp - rr) * q;
  const int wend = wbeg + q + (grp < rr ? 1 : 0);
  int w = wbeg + gi;
  if (w >= wend) return;  // whole workgroup leaves together

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int fr = lane & 15;  // fragment row / column
  const int fk = lane >> 4;  // fragment k-chunk (8 channels)
  const float fdiv = (float)divisor;

  float rv[NR][8];  // in-flight right-window chunk (8 channels of one pixel per item)
  float lv[8];      // in-flight left-tile chunk

  auto issue = [&](const BandWork& k, int c0) {
    const T* Rrow = R + k.n * rs.n + (int64_t)k.y * rs.h;
    const T* Lrow = L + k.n * ls.n + (int64_t)k.y * ls.h;
#pragma unroll
    for (int it = 0; it < NR; ++it) {
      const int e = tid + it * kThreads;
      if (e < k.rwin * 4) {  // wave-uniform (rwin*4 is a multiple of 64)
        const int ch = e / k.rwin;
        const int r = e - ch * k.rwin;
        load8(Rrow, rs.c, c0 + ch * 8, C, k.js + r, W, rv[it]);
      }
    }
    load8(Lrow, ls.c, c0 + (tid >> 6) * 8, C, k.x0 + (tid & 63), W, lv);
  };

  auto stage = [&](const BandWork& k) {
    unsigned char* Rt = smem;
    unsigned char* Lt = smem + P * k.rwin * kRowBytes;
#pragma unroll
    for (int it = 0; it < NR; ++it) {
      const int e = tid + it * kThreads;
      if (e < k.rwin * 4) {
        const int ch = e / k.rwin;
        const int r = e - ch * k.rwin;
        uint4 pk[P];
        split8<P>(rv[it], pk);
#pragma unroll
        for (int p = 0; p < P; ++p)
          *reinterpret_cast<uint4*>(Rt + p * k.rwin * kRowBytes + swz(r, ch)) = pk[p];
      }
    }
    uint4 pk[P];
    split8<P>(lv, pk);
#pragma unroll
    for (int p = 0; p < P; ++p)
      *reinterpret_cast<uint4*>(Lt + p * kXT * kRowBytes + swz(tid & 63, tid >> 6)) = pk[p];
  };

  f32x4 acc[TMAX];
  BandWork cur = band_decode(w, tiles, npass, H, D, DMAX);
  int c0 = 0;
  issue(cur, 0);

  while (true) {
    __syncthreads();  // previous fragment reads / out-tile reads are done
    stage(cur);
    __syncthreads();

    // prefetch the next (work, channel step) before this step's MFMAs and epilogue
    const bool last_step = c0 + kKC >= C;
    const int nw = last_step ? w + gsz : w;
    const int nc0 = last_step ? 0 : c0 + kKC;
    const bool has_next = nw < wend;
    const BandWork nxt = last_step ? band_decode(has_next ? nw : w, tiles, npass, H, D, DMAX) : cur;
    if (has_next && !(ablate & 2)) issue(nxt, nc0);

    if (c0 == 0) {
#pragma unroll
      for (int t = 0; t < TMAX; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // ---- band MMA: B = left x-block (cols x), A = right j-block (rows j)
    {
      const unsigned char* Rt = smem;
      const unsigned char* Lt = smem + P * cur.rwin * kRowBytes;
      bf16x8 bq[P];
#pragma unroll
      for (int p = 0; p < P; ++p)
        bq[p] = *reinterpret_cast<const bf16x8*>(Lt + p * kXT * kRowBytes + swz(16 * wave + fr, fk));
#pragma unroll
      for (int t = 0; t < TMAX; ++t) {
        if (t < cur.Tn && !(ablate & 1)) {
          bf16x8 aq[P];
#pragma unroll
          for (int p = 0; p < P; ++p)
            aq[p] = *reinterpret_cast<const bf16x8*>(Rt + p * cur.rwin * kRowBytes +
                                                     swz(16 * (wave + t) + fr, fk));
          if (P == 3) {
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[2], bq[0], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[1], bq[1], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[0], bq[2], acc[t], 0, 0, 0);
          }
          if (P >= 2) {
            if (P == 2)
              acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[1], bq[1], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[1], bq[0], acc[t], 0, 0, 0);
            acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[0], bq[1], acc[t], 0, 0, 0);
          }
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aq[0], bq[0], acc[t], 0, 0, 0);
        }
      }
    }

    if (last_step) {
      // ---- epilogue: shear S[j][x] -> out[d = x - j][x] through an LDS [Dp][64] fp32 tile
      __syncthreads();
      float* ot = reinterpret_cast<float*>(smem);
      const int xl = 16 * wave + fr;
#pragma unroll
      for (int t = 0; t < TMAX; ++t) {
        if (t < cur.Tn) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int wr = 16 * (wave + t) + 4 * fk + r;  // window row of this element
            const int dl = xl + 16 * (cur.Tn - 1) - wr;   // its local disparity
            if (dl >= 0 && dl < cur.Dp) {
              const bool inside = cur.js + wr >= 0;  // j < 0 <=> x < d: exact zero
              float v = inside ? acc[t][r] : 0.f;
              if (divisor >= 0 && inside) v = v / fdiv;
              ot[dl * kXT + xl] = v;
            }
          }
        }
      }
      __syncthreads();
      const int c4 = tid & 15;
      const int x = cur.x0 + 4 * c4;
      const bool fullrow = (cur.x0 + kXT <= W) && ((W & 3) == 0);
      if (ablate & 4) {
        // diagnostic build path: no output stream
      } else if (fullrow) {  // 16-B aligned row segments: one wide store per lane per row
        for (int dl = tid >> 4; dl < cur.Dp; dl += kThreads / 16) {
          const float4 v = *reinterpret_cast<const float4*>(ot + dl * kXT + 4 * c4);
          T* o = out + (((size_t)cur.n * D + cur.dp + dl) * H + cur.y) * (size_t)W + x;
          store4(o, v);
        }
      } else {
        for (int dl = tid >> 4; dl < cur.Dp; dl += kThreads / 16) {
          const float4 v = *reinterpret_cast<const float4*>(ot + dl * kXT + 4 * c4);
          T* o = out + (((size_t)cur.n * D + cur.dp + dl) * H + cur.y) * (size_t)W + x;
          const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (x + k < W) o[k] = from_f<T>(vv[k]);
        }
      }
    }
    if (!has_next) break;
    w = nw;
    c0 = nc0;
    cur = nxt;
  }
}

// Diagnostic ablation bits (STEREOCV_ABLATE, timing studies only; outputs become garbage):
// 1 = skip MFMAs, 2 = skip the global loads of the pipelined steps, 4 = skip output stores.
int ablate_bits() {
  const char* e = getenv("STEREOCV_ABLATE");
  return e ? atoi(e) : 0;
}

int device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

template <typename T, int P, int TMAX>
int launch_band(const void* l, const void* r, void* o, int64_t N, int64_t C, int64_t H, int64_t W,
                int64_t D, Strides4 ls, Strides4 rs, int divisor, hipStream_t st) {
  constexpr int DMAX = 16 * (TMAX - 1);
  const int tiles = (int)ceil_div(W, kXT);
  const int npass = (int)ceil_div(D, DMAX);
  const int64_t nwork = (int64_t)tiles * H * N * npass;
  if (nwork > INT32_MAX) return fail(SM_EINVAL, "inner product: too much work for one launch");
  const int Dp = (int)std::min<int64_t>(D, DMAX);
  const int Tn = 1 + (Dp - 1 + 15) / 16;
  const int rwin = kXT + 16 * (Tn - 1);
  const size_t in_bytes = (size_t)P * (rwin + kXT) * kRowBytes;
  const size_t out_bytes = (size_t)Dp * kXT * 4;
  const size_t shm = std::max(in_bytes, out_bytes);
  auto kern = ip_band_mfma<T, P, TMAX>;
  if (shm > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess)
      return fail(SM_ELAUNCH, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  }
  // persistent grid: two workgroups per CU (LDS- and register-limited), a multiple of 8
  int64_t nwg = std::min<int64_t>(nwork, 2 * (int64_t)device_cus());
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(kThreads), shm, st, static_cast<const T*>(l),
                     static_cast<const T*>(r), static_cast<T*>(o), (int)C, (int)H, (int)W, (int)D,
                     ls, rs, divisor, tiles, npass, (int)nwork, ablate_bits());
  return check_launch("ip_band_mfma");
}

template <typename T, int P>
int launch_band_d(const void* l, const void* r, void* o, int64_t N, int64_t C, int64_t H, int64_t W,
                  int64_t D, Strides4 ls, Strides4 rs, int divisor, hipStream_t st) {
  if (D <= 64) return launch_band<T, P, 5>(l, r, o, N, C, H, W, D, ls, rs, divisor, st);
  if (D <= 128) return launch_band<T, P, 9>(l, r, o, N, C, H, W, D, ls, rs, divisor, st);
  if (D <= 192) return launch_band<T, P, 13>(l, r, o, N, C, H, W, D, ls, rs, divisor, st);
  return launch_band<T, P, 17>(l, r, o, N, C, H, W, D, ls, rs, divisor, st);
}

}  // namespace

int check_dot_args(const void* left, const void* right, const void* out, int dtype, int64_t N,
                   int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                   const int64_t* r_strides, Strides4* ls, Strides4* rs);

// mode 0: inner product (sum); mode 1: correlation (mean over C).
int band_mfma_entry(const void* left, const void* right, void* out, int dtype, int64_t N, int64_t C,
                    int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                    const int64_t* r_strides, int mode, void* stream) {
  Strides4 ls, rs;
  int rc = check_dot_args(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &ls, &rs);
  if (rc) return rc;
  if (N == 0 || H == 0 || W == 0 || D == 0) return SM_OK;
  const int divisor = mode == 0 ? -1 : (int)C;
  hipStream_t st = as_stream(stream);
  switch (dtype) {
    case SM_F32: return launch_band_d<float, 3>(left, right, out, N, C, H, W, D, ls, rs, divisor, st);
    case SM_F16: return launch_band_d<__half, 2>(left, right, out, N, C, H, W, D, ls, rs, divisor, st);
    case SM_BF16: return launch_band_d<bf16_t, 1>(left, right, out, N, C, H, W, D, ls, rs, divisor, st);
    default: return fail(SM_EDTYPE, "unsupported dtype code");
  }
}

int ip_mfma_entry(const void* left, const void* right, void* out, int dtype, int64_t N, int64_t C,
                  int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                  const int64_t* r_strides, void* stream, bool* handled) {
  *handled = true;
  return band_mfma_entry(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, 0, stream);
}

}  // namespace smcv

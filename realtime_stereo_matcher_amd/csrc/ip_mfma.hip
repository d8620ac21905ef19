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

template <typename T, int P, int TMAX>
__global__ __launch_bounds__(kThreads, 2) void ip_band_mfma(
    const T* __restrict__ L, const T* __restrict__ R, T* __restrict__ out, int C, int H, int W,
    int D, Strides4 ls, Strides4 rs, int divisor, int tiles, int nblocks) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int DMAX = 16 * (TMAX - 1);

  // XCD-aware bijective remap: consecutive work ids (x-tiles of one row) share an XCD.
  const int b = blockIdx.x;
  const int q = nblocks >> 3, rr = nblocks & 7, xcd = b & 7, idx = b >> 3;
  const int wid = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + idx;
  const int tile = wid % tiles;
  const int row = wid / tiles;  // n * H + y
  const int y = row % H;
  const int n = row / H;
  const int x0 = tile * kXT;

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int fr = lane & 15;  // fragment row / column
  const int fk = lane >> 4;  // fragment k-chunk (8 channels)

  const T* Lrow = L + n * ls.n + (int64_t)y * ls.h;
  const T* Rrow = R + n * rs.n + (int64_t)y * rs.h;

  for (int dp = 0; dp < D; dp += DMAX) {
    const int Dp = min(DMAX, D - dp);
    const int Tn = 1 + (Dp - 1 + 15) / 16;  // band blocks per x-block
    const int RWIN = kXT + 16 * (Tn - 1);
    const int js = x0 - dp - 16 * (Tn - 1);  // right column held in window row 0
    unsigned char* Rt = smem;                           // P planes x RWIN rows
    unsigned char* Lt = smem + P * RWIN * kRowBytes;    // P planes x 64 rows

    f32x4 acc[TMAX];
#pragma unroll
    for (int t = 0; t < TMAX; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};

    for (int c0 = 0; c0 < C; c0 += kKC) {
      __syncthreads();  // previous step's fragment reads (and the out tile) are done
      // ---- stage the right window: thread -> (pixel row, 8-channel chunk), rows fastest
      for (int e = tid; e < RWIN * 4; e += kThreads) {
        const int ch = e / RWIN;
        const int r = e - ch * RWIN;
        const int j = js + r;
        float v[8];
        load8(Rrow, rs.c, c0 + ch * 8, C, j, W, v);
        uint4 pk[P];
        split8<P>(v, pk);
#pragma unroll
        for (int p = 0; p < P; ++p)
          *reinterpret_cast<uint4*>(Rt + p * RWIN * kRowBytes + swz(r, ch)) = pk[p];
      }
      // ---- stage the left tile (64 pixel rows x 4 chunks = one element per thread)
      {
        const int ch = tid >> 6;
        const int r = tid & 63;
        const int x = x0 + r;
        float v[8];
        load8(Lrow, ls.c, c0 + ch * 8, C, x, W, v);
        uint4 pk[P];
        split8<P>(v, pk);
#pragma unroll
        for (int p = 0; p < P; ++p)
          *reinterpret_cast<uint4*>(Lt + p * kXT * kRowBytes + swz(r, ch)) = pk[p];
      }
      __syncthreads();

      // ---- band MMA: B = left x-block (cols x), A = right j-block (rows j)
      bf16x8 bq[P];
#pragma unroll
      for (int p = 0; p < P; ++p)
        bq[p] = *reinterpret_cast<const bf16x8*>(Lt + p * kXT * kRowBytes + swz(16 * wave + fr, fk));
#pragma unroll
      for (int t = 0; t < TMAX; ++t) {
        if (t < Tn) {
          bf16x8 aq[P];
#pragma unroll
          for (int p = 0; p < P; ++p)
            aq[p] = *reinterpret_cast<const bf16x8*>(Rt + p * RWIN * kRowBytes +
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

    // ---- epilogue: shear S[j][x] -> out[d = x - j][x] through an LDS [Dp][64] fp32 tile
    __syncthreads();
    float* ot = reinterpret_cast<float*>(smem);
    const int xl = 16 * wave + fr;  // this lane's pixel within the tile
    const float fdiv = (float)divisor;
#pragma unroll
    for (int t = 0; t < TMAX; ++t) {
      if (t < Tn) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          // window row of this accumulator element and its local disparity
          const int wr = 16 * (wave + t) + 4 * fk + r;
          const int dl = xl + 16 * (Tn - 1) - wr;
          if (dl >= 0 && dl < Dp) {
            const int j = js + wr;
            float v = j >= 0 ? acc[t][r] : 0.f;  // x < d: exact zero, like torch.zeros
            if (divisor >= 0 && j >= 0) v = v / fdiv;
            ot[dl * kXT + xl] = v;
          }
        }
      }
    }
    __syncthreads();
    const int c4 = tid & 15;
    const int x = x0 + 4 * c4;
    const bool fullrow = (x0 + kXT <= W) && ((W & 3) == 0);
    for (int dl = tid >> 4; dl < Dp; dl += kThreads / 16) {
      const float4 v = *reinterpret_cast<const float4*>(ot + dl * kXT + 4 * c4);
      T* o = out + (((size_t)n * D + dp + dl) * H + y) * (size_t)W + x;
      if (fullrow) {
        if (sizeof(T) == 4) {
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
      } else {
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k)
          if (x + k < W) o[k] = from_f<T>(vv[k]);
      }
    }
  }
}

template <typename T, int P, int TMAX>
int launch_band(const void* l, const void* r, void* o, int64_t N, int64_t C, int64_t H, int64_t W,
                int64_t D, Strides4 ls, Strides4 rs, int divisor, hipStream_t st) {
  const int tiles = (int)ceil_div(W, kXT);
  const int64_t nb = (int64_t)tiles * H * N;
  if (nb > INT32_MAX) return fail(SM_EINVAL, "inner product: grid too large");
  const int Dp = (int)std::min<int64_t>(D, 16 * (TMAX - 1));
  const int Tn = 1 + (Dp - 1 + 15) / 16;
  const int rwin = kXT + 16 * (Tn - 1);
  const size_t in_bytes = (size_t)P * (rwin + kXT) * kRowBytes;
  const size_t out_bytes = (size_t)Dp * kXT * 4;
  const size_t shm = std::max(in_bytes, out_bytes);
  auto kern = ip_band_mfma<T, P, TMAX>;
  if (shm > 64 * 1024) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    if (e != hipSuccess) return fail(SM_ELAUNCH, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nb), dim3(kThreads), shm, st, static_cast<const T*>(l),
                     static_cast<const T*>(r), static_cast<T*>(o), (int)C, (int)H, (int)W, (int)D,
                     ls, rs, divisor, tiles, (int)nb);
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

// Inner-product / correlation cost volume for fp32 features on the gfx950 fp32 matrix core
// (v_mfma_f32_16x16x4_f32: an exact fp32 fma chain, 64 FLOP/clk/SIMD).
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// Same band decomposition as ip_mfma.hip (S[j][x] = sum_c R[c][j] L[c][x], d = x - j; one
// 8-wave workgroup per 128-pixel row segment, wave w owns x-block w and its T = 1 +
// ceil((D-1)/16) 16x16 band blocks) but with no operand conversion at all: the features arrive
// in LDS by LDS-DMA (global_load_lds_dwordx4, issued by inline asm) exactly as they sit in
// memory -- channel rows of pixels -- and the MFMA reads its A (right window) and B (left
// tile) fragments straight from those rows with ds_read_b32.  16 channels per step,
// double-buffered: the DMA of step s+1 flies while step s computes, one barrier per step.
// Rows are padded by 16 floats so the two 16-lane row groups of a fragment read sit 16 banks
// apart (conflict-free).  Out-of-image pixels read clamped (valid) addresses: they only feed
// outputs that the epilogue zeroes (x < d) or never stores (x >= W).  Channels past C are
// masked on the B fragment.
//
// Epilogue: accumulators are sheared (d = x - j) into a dedicated LDS [D][128] fp32 tile
// (not aliased with the stage buffers, so the next segment's DMA is already in flight) and
// streamed out as 512-B row segments; the next step retires its DMA with a hand-counted
// vmcnt that leaves those stores in flight.
#include "common.h"

#include <cstdlib>
#include <type_traits>

namespace smcv {
namespace fband {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kXT = 16 * kWaves;  // left pixels per row segment
constexpr int kKC = 16;           // channels per pipeline step (4 MFMA k-steps of 4)
constexpr int kPad = 16;          // floats of padding per LDS row (16-bank offset between rows)
constexpr int kLRow = kXT + kPad;

typedef __attribute__((address_space(3))) unsigned char lds_u8;
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const lds_u8*)p;
}
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_byte) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_byte)
      : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

struct Work {
  int n, y, x0, dp, Dp, Tn, js;
};

__device__ __forceinline__ Work decode(int w, int tiles, int npass, int H, int D, int dmax) {
  Work k;
  const int pass = w % npass;
  const int rest = w / npass;
  const int tile = rest % tiles;
  const int row = rest / tiles;
  k.y = row % H;
  k.n = row / H;
  k.x0 = tile * kXT;
  k.dp = pass * dmax;
  k.Dp = min(dmax, D - k.dp);
  k.Tn = 1 + (k.Dp - 1 + 15) / 16;
  k.js = k.x0 - k.dp - 16 * (k.Tn - 1);
  return k;
}

// Layout of one stage buffer (floats): R rows [kKC][RROW] then L rows [kKC][kLRow].
template <int TMAX>
struct Geo {
  static constexpr int DMAX = 16 * (TMAX - 1);
  static constexpr int RW = kXT + DMAX;            // right-window pixels
  static constexpr int RROW = RW + kPad;
  static constexpr int RGROUPS = kKC * RROW / 4;   // 16-B DMA groups of the R rows
  static constexpr int LGROUPS = kKC * kLRow / 4;
  static constexpr int GROUPS = RGROUPS + LGROUPS;
  static constexpr int PIECES = (GROUPS + 63) / 64;  // wave instructions per step
  static constexpr int PPW = (PIECES + kWaves - 1) / kWaves;
  static constexpr int BUF_FLOATS = PIECES * 64 * 4;  // rounded up to whole pieces
  static constexpr int OUT_FLOATS = (DMAX + 1) * kXT;  // + trash row
  static constexpr size_t SHM = (size_t)(2 * BUF_FLOATS + OUT_FLOATS) * 4;
};

template <int TMAX, bool MEAN>
__global__ __launch_bounds__(kThreads, 1) void ip_band_f32(
    const float* __restrict__ L, const float* __restrict__ R, float* __restrict__ out, int C,
    int H, int W, int D, Strides4 ls, Strides4 rs, int tiles, int npass, int nwork) {
  using G = Geo<TMAX>;
  constexpr int DMAX = G::DMAX;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* const ot = smem + 2 * G::BUF_FLOATS;

  const int grp = blockIdx.x & 7;
  const int gi = blockIdx.x >> 3;
  const int gsz = gridDim.x >> 3;
  const int q = nwork >> 3, rr = nwork & 7;
  const int wbeg = grp < rr ? grp * (q + 1) : rr * (q + 1) + (grp - rr) * q;
  const int wend = wbeg + q + (grp < rr ? 1 : 0);
  int w = wbeg + gi;
  if (w >= wend) return;

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int fr = lane & 15;
  const int fk = lane >> 4;
  const unsigned smem_lds = __builtin_amdgcn_readfirstlane(lds_addr(smem));
  const int uwave = __builtin_amdgcn_readfirstlane(wave);
  SM_STAMP_DECL

  // issue this wave's DMA pieces of (work k, channel step c0) into stage buffer b
  // Kernel-argument strides are copied to plain (SGPR) scalars first: selecting a struct
  // member per lane made hipcc fetch it with a VMEM load + vmcnt(0), draining every DMA piece
  // and output store in flight.
  const int64_t rsn = rs.n, rsc = rs.c, rsh = rs.h, lsn = ls.n, lsc = ls.c, lsh = ls.h;
  auto issue = [&](const Work& k, int c0, int b) {
    const float* Rrow = R + k.n * rsn + (int64_t)k.y * rsh;
    const float* Lrow = L + k.n * lsn + (int64_t)k.y * lsh;
#pragma unroll
    for (int pp = 0; pp < G::PPW; ++pp) {
      const int piece = uwave + kWaves * pp;
      if (piece < G::PIECES) {  // wave-uniform
        const int g = piece * 64 + lane;
        const bool isR = g < G::RGROUPS;
        // right window: row of RROW/4 groups; pad positions fetch valid junk
        const int rrow = g / (G::RROW / 4);
        const int rpx = 4 * (g - rrow * (G::RROW / 4));
        const int j = min(max(k.js + rpx, 0), W - 4);
        // left tile
        const int gl = min(max(g - G::RGROUPS, 0), G::LGROUPS - 1);
        const int lrow = gl / (kLRow / 4);
        const int lpx = 4 * (gl - lrow * (kLRow / 4));
        const int x = min(k.x0 + lpx, W - 4);
        const int64_t roff = (int64_t)min(c0 + rrow, C - 1) * rsc + j;
        const int64_t loff = (int64_t)min(c0 + lrow, C - 1) * lsc + x;
        const float* src = isR ? Rrow + roff : Lrow + loff;
        glds16(src, smem_lds + (unsigned)(b * G::BUF_FLOATS + piece * 256) * 4);
      }
    }
  };

  f32x4 acc[TMAX];
  Work cur = decode(w, tiles, npass, H, D, DMAX);
  int c0 = 0, buf = 0;
  bool counted_epi = false;
  issue(cur, 0, 0);

  while (true) {
    // retire this wave's DMA of the current step (only the epilogue's stores may stay in
    // flight), then make every wave's pieces visible
    if (counted_epi)
      vm_wait<DMAX / 16>();
    else
      vm_wait<0>();
    SM_STAMP(8);
    __syncthreads();
    SM_STAMP(0);

    const bool last_step = c0 + kKC >= C;
    const int nw = last_step ? w + gsz : w;
    const int nc0 = last_step ? 0 : c0 + kKC;
    const bool has_next = nw < wend;
    const Work nxt = last_step ? decode(has_next ? nw : w, tiles, npass, H, D, DMAX) : cur;
    if (has_next) issue(nxt, nc0, buf ^ 1);  // the other buffer: free since the barrier
    SM_STAMP(9);

    if (c0 == 0) {
#pragma unroll
      for (int t = 0; t < TMAX; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // ---- band MMA over 16 channels: 4 k-steps x T blocks, 13 independent accumulators
    const float* Rb = smem + buf * G::BUF_FLOATS;
    const float* Lb = Rb + G::RGROUPS * 4;
    const float* aL = Rb + fk * G::RROW + 16 * wave + fr;  // + s*4*RROW + 16 t
    const float* bL = Lb + fk * kLRow + 16 * wave + fr;    // + s*4*kLRow
    // full band: all 13 A values (+ B) of k-step s+1 are read into registers before the 13
    // MFMAs of k-step s issue (sched_barrier keeps the order), so the LDS latency of a read
    // hides behind a whole k-step instead of being waited for per MFMA
    auto kread = [&](int s, float (&av)[TMAX], float& bv) {
      bv = bL[s * 4 * kLRow];
      bv = (c0 + 4 * s + fk < C) ? bv : 0.f;  // channels past C contribute nothing
#pragma unroll
      for (int t = 0; t < TMAX; ++t) av[t] = aL[s * 4 * G::RROW + 16 * t];
    };
    if (cur.Tn == TMAX) {
      float a0[TMAX], a1[TMAX], b0, b1;
      kread(0, a0, b0);
#pragma unroll
      for (int s = 0; s < kKC / 4; s += 2) {
        kread(s + 1, a1, b1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < TMAX; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[t], b0, acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (s + 2 < kKC / 4) kread(s + 2, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int t = 0; t < TMAX; ++t)
          acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[t], b1, acc[t], 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
#pragma unroll
      for (int s = 0; s < kKC / 4; ++s) {
        float av[TMAX], bv;
        kread(s, av, bv);
#pragma unroll
        for (int t = 0; t < TMAX; ++t)
          if (t < cur.Tn) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t], bv, acc[t], 0, 0, 0);
      }
    }

    SM_STAMP(3);
    if (last_step) {
      // ---- epilogue: shear S[j][x] -> out[d = x - j][x] through the LDS [Dp][128] tile
      const int xl = 16 * wave + fr;
      const int b0 = fr - 4 * fk + 16 * (cur.Tn - 1);
      const int j_b = cur.js + 16 * wave + 4 * fk;
      const float fdiv = (float)C;
      float* const olane = ot + b0 * kXT + xl;
      if (cur.Tn == TMAX && cur.Dp == DMAX && cur.js >= 0) {
#pragma unroll
        for (int t = 0; t < TMAX; ++t) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float val = acc[t][r];
            if (MEAN) val = val / fdiv;
            if (t == 0 || t == TMAX - 1) {
              const int dl = b0 - 16 * t - r;
              const bool keep = (unsigned)dl < (unsigned)DMAX;
              ot[(keep ? dl : DMAX) * kXT + xl] = val;
            } else {
              olane[-(16 * t + r) * kXT] = val;
            }
          }
        }
      } else {
#pragma unroll
        for (int t = 0; t < TMAX; ++t) {
          if (t < cur.Tn) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int dl = b0 - 16 * t - r;
              const bool keep = (unsigned)dl < (unsigned)cur.Dp;
              const bool inside = j_b + 16 * t + r >= 0;  // j < 0 <=> x < d: exact zero
              float val = acc[t][r];
              if (MEAN) val = val / fdiv;
              ot[(keep ? dl : DMAX) * kXT + xl] = inside ? val : 0.f;
            }
          }
        }
      }
      SM_STAMP(5);
      __syncthreads();
      SM_STAMP(6);
      const int c4 = tid & 31;
      const int x = cur.x0 + 4 * c4;
      const bool fullrow = (cur.x0 + kXT <= W) && ((W & 3) == 0);
      if (fullrow && cur.Dp == DMAX) {  // the counted case: DMAX/16 stores per lane
#pragma unroll
        for (int it16 = 0; it16 < DMAX / 16; ++it16) {
          const int dl = (tid >> 5) + 16 * it16;
          const float4 val = *reinterpret_cast<const float4*>(ot + dl * kXT + 4 * c4);
          *reinterpret_cast<float4*>(out + (((size_t)cur.n * D + cur.dp + dl) * H + cur.y) *
                                               (size_t)W + x) = val;
        }
      } else {
        for (int dl = tid >> 5; dl < cur.Dp; dl += kThreads / 32) {
          const float4 val = *reinterpret_cast<const float4*>(ot + dl * kXT + 4 * c4);
          float* o = out + (((size_t)cur.n * D + cur.dp + dl) * H + cur.y) * (size_t)W + x;
          const float vv[4] = {val.x, val.y, val.z, val.w};
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (x + k < W) o[k] = vv[k];
        }
      }
      // the out tile is rewritten only after the next segment's steps (>= 1 barrier away)
    }
    if (last_step) SM_STAMP(7);
    counted_epi = last_step && cur.Dp == DMAX && (cur.x0 + kXT <= W) && ((W & 3) == 0);
    if (!has_next) break;
    w = nw;
    c0 = nc0;
    cur = nxt;
    buf ^= 1;
  }
  SM_STAMP_FLUSH
}

template <int TMAX>
int launch(const float* l, const float* r, float* o, int64_t N, int64_t C, int64_t H, int64_t W,
           int64_t D, Strides4 ls, Strides4 rs, bool mean, hipStream_t st) {
  using G = Geo<TMAX>;
  const int tiles = (int)ceil_div(W, kXT);
  const int npass = (int)ceil_div(D, G::DMAX);
  const int64_t nwork = (int64_t)tiles * H * N * npass;
  if (nwork > INT32_MAX) return fail(SM_EINVAL, "inner product: too much work for one launch");
  auto kern = mean ? ip_band_f32<TMAX, true> : ip_band_f32<TMAX, false>;
  static std::atomic<unsigned long long> lds_done[2];
  const int dev = stream_device(st);
  if (int rc = ensure_lds_limit(reinterpret_cast<const void*>(kern), (int)G::SHM, dev, lds_done[mean]))
    return rc;
  int64_t nwg = std::min<int64_t>(nwork, (int64_t)device_cus(dev));
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(kThreads), G::SHM, st, l, r, o, (int)C,
                     (int)H, (int)W, (int)D, ls, rs, tiles, npass, (int)nwork);
  return check_launch("ip_band_f32");
}

}  // namespace fband

int check_dot_args(const void* left, const void* right, const void* out, int dtype, int64_t N,
                   int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                   const int64_t* r_strides, Strides4* ls, Strides4* rs);

// fp32 band kernel; *handled = false when the shape needs the generic path (the DMA reads
// 16-B pixel groups: W % 4 == 0, W >= 4, 4-float-aligned rows).
int band_f32_entry(const void* left, const void* right, void* out, int dtype, int64_t N,
                   int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                   const int64_t* r_strides, int mode, void* stream, bool* handled) {
  *handled = false;
  if (dtype != SM_F32) return SM_OK;
  Strides4 ls, rs;
  int rc = check_dot_args(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &ls, &rs);
  if (rc) return rc;
  const bool vec = (W % 4 == 0) && W >= 4 && C > 0 && ls.n % 4 == 0 && ls.c % 4 == 0 &&
                   ls.h % 4 == 0 && rs.n % 4 == 0 && rs.c % 4 == 0 && rs.h % 4 == 0 &&
                   ((reinterpret_cast<uintptr_t>(left) | reinterpret_cast<uintptr_t>(right)) % 16 == 0);
  if (!vec) return SM_OK;
  *handled = true;
  if (N == 0 || H == 0 || D == 0) return SM_OK;
  const bool mean = mode == 1;
  hipStream_t st = as_stream(stream);
  const float* l = static_cast<const float*>(left);
  const float* r = static_cast<const float*>(right);
  float* o = static_cast<float*>(out);
  using namespace fband;
  if (D <= 64) return launch<5>(l, r, o, N, C, H, W, D, ls, rs, mean, st);
  if (D <= 128) return launch<9>(l, r, o, N, C, H, W, D, ls, rs, mean, st);
  // D > 192: passes of 192 disparities (a 256-wide tile would not fit LDS)
  return launch<13>(l, r, o, N, C, H, W, D, ls, rs, mean, st);
}

}  // namespace smcv

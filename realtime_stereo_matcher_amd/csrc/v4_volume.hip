// MobileStereoNetV4's interweave + Conv3d cost volume on gfx950.
//
// Reference (model/mobile_stereo_net_v4.py:443-461, stacks :317-335): for every disparity
// i < D, X = interweave(L[..., i:], R[..., :-i]) -- even channels L, odd channels R -- is read as
// a depth-64 volume of width W - i; Conv3d(1->16, (8,3,3), stride 8), (16->32, (4,3,3), stride 4),
// (32->16, (2,3,3), stride 2), each + BatchNorm + ReLU, zero padding 1 at the CROP's borders;
// then a 1x1 conv 16->1 + BatchNorm + ReLU; the result lands at x >= i of a zero (N, D, H, W)
// volume.  Eval-mode BatchNorm is folded into the weights by the caller.
//
// Decomposition.  Stride == kernel depth, so the depth axis is block-diagonal:
//   a1[b][o1](y,x)  = relu(b1 + PL[b][o1](y,x) + PR[b][o1](y,x-i))     b = depth block 0..7
//   a2[b2][o2](y,x) = relu(b2 + sum_{kd<4, o1, 3x3} W2 a1[4 b2 + kd][o1])  b2 = 0, 1
//   a3[o3](y,x)     = relu(b3 + sum_{b2, o2, 3x3} W3 a2[b2][o2])
//   out(y,x)        = relu(b4 + sum_{o3} w4 a3[o3])
// Layer 1 is linear before its ReLU and every one of its input channels is either L or R, so it
// splits into a left part PL(y,x) and a right part PR(y,x-i) that do NOT depend on i: the
// "tables" kernel computes them once per pixel (fp32 FMA), plus the single-column pieces that
// the crop removes (dx = -1 of L at x = i, dx = +1 of R at x = W - 1).  Layers 2 and 3 (92 k of
// the ~110 k flops per cell) run on v_mfma_f32_32x32x16_f16 / 16x16x32_f16 with every fp32
// operand scaled by a per-layer power of two and split into fp16 hi + lo (round to nearest) and
// three products (hh + hl + lh: exact in fp32; the dropped lo*lo' and the lo roundings leave
// ~3 * 2^-22 relative per product; fp32 accumulation).  The scales come from bounds computed on
// the device before the main kernel, so the scaled values stay below 2^15 (no fp16 overflow):
// max|W2|, max|W3| directly; |a1| <= max|b1| + max|PL| + max|PR| (v4_tmax reduces the
// tables); |a2| <= max|b2| + max_o2 sum|W2[o2]| * bound(a1).  Values far below their layer's
// bound lose only absolute precision (the fp16 subnormal step, ~2^-39 of the bound).
//
// Main kernel.  A workgroup owns (n, i, a 30-pixel column strip, a band of rows) and streams down
// the rows with three-row LDS rings of a1 (34 px halo, 8 x 16 channels) and a2 (34 px, 64
// channels).  Each of the 8 waves keeps ITS weights in VGPRs for the whole kernel: wave b holds
// the layer-2 fragments of depth block b (9 taps x 16 x 32, kd = b & 3) and a quarter of the
// layer-3 K range of one 16-pixel half; partial sums meet in LDS.  Per row: a1 row (tables ->
// relu -> split, prefetched one row ahead) | layer 2 | reduce + bias + relu -> a2 row | layer 3 |
// reduce + bias + relu + 1x1 + relu -> output row.
#include "common.h"

#include <atomic>

namespace smcv {
namespace v4vol {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int kC = 32;       // feature channels per side (V4's preconv11 output)
constexpr int kCh = 128;     // layer-1 channels: 8 depth blocks x 16
constexpr int kTX = 28;      // output pixels per strip
constexpr int kA2 = 34;      // a2 ring pixels: 32 computed (x0-1 .. x0+30; 30 used) + 2 readable pad
constexpr int kA1 = 34;      // a1 ring pixels: 32 computed (x0-2 .. x0+29) + 2 zero pad
constexpr int kThreads = 512;

// LDS layout (bytes)
constexpr int kA1Slot = 8 * kA1 * 16 * 2;      // one row: [b 8][p 34][16 ch] fp16
constexpr int kA1Plane = 3 * kA1Slot;          // three rows
constexpr int kA2Slot = kA2 * 64 * 2;          // one row: [p 34][64 ch] fp16
constexpr int kA2Plane = 3 * kA2Slot;
constexpr int kOffA1 = 0;                                  // hi plane, then lo plane
constexpr int kOffA2 = kOffA1 + 2 * kA1Plane;
constexpr int kOffP2 = kOffA2 + 2 * kA2Plane;              // [8 waves][32 px][32 o2] fp32
constexpr int kOffP3 = kOffP2 + 8 * 32 * 32 * 4;           // [8 waves][16 px][16 o3] fp32
constexpr int kShm = kOffP3 + 8 * 16 * 16 * 4;
static_assert(kShm <= 160 * 1024, "one workgroup per CU");

// layer-3 K steps (18 = 9 taps x 2 halves of 64 a2 channels) per K group of 4
__device__ __forceinline__ int ks_begin(int g) { return g == 0 ? 0 : g == 1 ? 5 : g == 2 ? 10 : 14; }
__device__ __forceinline__ int ks_end(int g) { return g == 0 ? 5 : g == 1 ? 10 : g == 2 ? 14 : 18; }

// the scale block in the workspace (after the packed weights): the four exponents v4_scales
// derives
struct Scales {
  int k_a1, k_w2, k_a2, k_w3;
};
// followed by the table maxima: one (max |PL|, max |PR|) pair per v4_tables workgroup

struct Args {
  const float* T;        // tables [n][y][x][4][128]: PL, PL without dx=-1, PR, PR without dx=+1
  const f16x8* P2;       // layer-2 B fragments [kd 4][tap 9][lane 64] hi, then the same lo
  const f16x8* P3;       // layer-3 B fragments [step 18][lane 64] hi, then lo
  const Scales* S;
  const float* b1;       // (16)
  const float* b2;       // (32)
  const float* b3;       // (16)
  const float* w4;       // (16)
  const float* b4;       // (1)
  float* out;            // (N, D, H, W) contiguous
  int N, H, W, D, strips, bands, BH;
};

// Workgroup barrier for LDS hand-offs only: this wave's LDS accesses are complete, then
// s_barrier.  The prefetched table loads and the output stores stay in flight (__syncthreads()
// would drain them with vmcnt(0) at every one of the four barriers of a row).
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// x 2^k -> fp16 hi = rn16(x 2^k), lo = rn16(x 2^k - hi) (the scaled value is below 2^15)
__device__ __forceinline__ void split16(float x, int k, _Float16& hi, _Float16& lo) {
  const float v = __builtin_ldexpf(x, k);
  hi = (_Float16)v;
  lo = (_Float16)(v - (float)hi);
}
// The same split for two values at once on v_fma_mix (band_common.h's split_pair): sc = 2^k,
// h = rn16(x sc), m = rn16(x sc - h) evaluated exactly in the mix unit and packed as (lo, hi)
// fp16 pairs -- two VALU per value instead of the convert / subtract / convert / pack sequence.
__device__ __forceinline__ void split_pair16(float a, float b, float sc, unsigned& h, unsigned& m) {
  asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h), "=&v"(m)
      : "v"(a), "v"(b), "v"(sc));
}
__device__ __forceinline__ void split8(const float (&v)[8], float sc, f16x8& hi, f16x8& lo) {
  unsigned h[4], m[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) split_pair16(v[2 * j], v[2 * j + 1], sc, h[j], m[j]);
  hi = __builtin_bit_cast(f16x8, (uint4){h[0], h[1], h[2], h[3]});
  lo = __builtin_bit_cast(f16x8, (uint4){m[0], m[1], m[2], m[3]});
}
// exponent k with b 2^k <= 2^15 (b > 0 finite), 0 for b == 0, clamped to fp32's reach
__device__ __forceinline__ int scale_exp(float b) {
  if (!(b > 0.f) || !(b < 3.4e38f)) return 0;
  return min(100, max(-100, 15 - __builtin_amdgcn_frexp_expf(b)));
}

// ------------------------------------------------------------------------------ tables
// One thread per (pixel, depth block b): the 16 layer-1 channels c = 16 b + o1 of the left and
// right halves (3x3, zero padding at the image borders), each also without the column the crop
// removes: L without its dx = -1 taps (used at x == i), R without its dx = +1 taps (used at
// x == W - 1).  Adjacent threads take adjacent pixels (coalesced feature loads); w1 sits in LDS.
__global__ __launch_bounds__(256) void v4_tables(const float* __restrict__ L,
                                                 const float* __restrict__ R, Strides4 ls,
                                                 Strides4 rs, const float* __restrict__ w1,
                                                 float* __restrict__ T, int N, int H, int W) {
  __shared__ float ws[16 * 8 * 9];
  for (int e = threadIdx.x; e < 16 * 8 * 9; e += 256) ws[e] = w1[e];
  __syncthreads();
  const int64_t px = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int b = blockIdx.y;
  if (px >= (int64_t)N * H * W) return;
  const int x = (int)(px % W);
  const int y = (int)((px / W) % H);
  const int n = (int)(px / ((int64_t)W * H));
  float lv[4][9], rv[4][9];
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) {
    const float* lp = L + n * ls.n + (int64_t)(4 * b + kk) * ls.c;
    const float* rp = R + n * rs.n + (int64_t)(4 * b + kk) * rs.c;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
      const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
      lv[kk][t] = ok ? lp[(int64_t)yy * ls.h + xx] : 0.f;
      rv[kk][t] = ok ? rp[(int64_t)yy * rs.h + xx] : 0.f;
    }
  }
  float* o = T + px * (4 * kCh) + 16 * b;
#pragma unroll 4
  for (int o1 = 0; o1 < 16; ++o1) {
    float pl = 0.f, plm = 0.f, pr = 0.f, prp = 0.f;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const float l = lv[kk][t] * ws[(o1 * 8 + 2 * kk) * 9 + t];
        const float r = rv[kk][t] * ws[(o1 * 8 + 2 * kk + 1) * 9 + t];
        pl += l;
        pr += r;
        if (t % 3 == 0) plm += l;
        if (t % 3 == 2) prp += r;
      }
    }
    o[o1] = pl;
    o[kCh + o1] = pl - plm;
    o[2 * kCh + o1] = pr;
    o[3 * kCh + o1] = pr - prp;
  }
}

// max |PL| and max |PR| over the tables (all four variants), one pair per workgroup (no
// atomics: v4_scales reduces the pairs).  A pixel's 512 table words: 256 of L, then 256 of R.
constexpr int kTmaxBlocks = 512;
__global__ __launch_bounds__(256) void v4_tmax(const float* __restrict__ T, int64_t nquads,
                                               float2* __restrict__ tmax) {
  float ml = 0.f, mr = 0.f;
  for (int64_t q = (int64_t)blockIdx.x * 256 + threadIdx.x; q < nquads; q += (int64_t)256 * gridDim.x) {
    const f32x4v v = reinterpret_cast<const f32x4v*>(T)[q];
    const float m = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
    if ((q & 127) < 64) ml = fmaxf(ml, m); else mr = fmaxf(mr, m);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    ml = fmaxf(ml, __shfl_xor(ml, o));
    mr = fmaxf(mr, __shfl_xor(mr, o));
  }
  __shared__ float2 wm[4];
  if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = make_float2(ml, mr);
  __syncthreads();
  if (threadIdx.x == 0) {
    float2 m = wm[0];
    for (int w = 1; w < 4; ++w) m = make_float2(fmaxf(m.x, wm[w].x), fmaxf(m.y, wm[w].y));
    tmax[blockIdx.x] = m;
  }
}

// ------------------------------------------------------------------------------ scales, packing
// v4_scales: the four exponents from the weights, the biases and the table maxima (v4_tmax).
// v4_pack: the MFMA B fragments, scaled and split into fp16 hi / lo.  Layer 2
// (32x32x16): lane l holds B[k = 8 (l>>5) + j][col l&31] = W2[o2 = l&31][o1 = 8 (l>>5) + j][kd]
// [dy][dx].  Layer 3 (16x16x32): step s = 2 tap + half, lane l holds B[k = 8 (l>>4) + j]
// [col l&15] = W3[o3 = l&15][o2 = k][kd = half][dy][dx].
constexpr int kN2 = 4 * 9 * 64 * 8, kN3 = 18 * 64 * 8;  // = the sizes of W2, W3

template <int NT>
__device__ __forceinline__ void v4_scales(const float* __restrict__ w2, const float* __restrict__ w3,
                                          const float* __restrict__ b1, const float* __restrict__ b2,
                                          const float2* __restrict__ tmax, int ntmax, Scales& S) {
  constexpr int NW = NT / 64;
  __shared__ float red[6][NW];
  __shared__ float rows[32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float m2 = 0.f, m3 = 0.f, mb1 = 0.f, mb2 = 0.f, ml = 0.f, mr = 0.f;
  for (int e = tid; e < kN2; e += NT) m2 = fmaxf(m2, fabsf(w2[e]));
  for (int e = tid; e < kN3; e += NT) m3 = fmaxf(m3, fabsf(w3[e]));
  for (int e = tid; e < ntmax; e += NT) {
    ml = fmaxf(ml, tmax[e].x);
    mr = fmaxf(mr, tmax[e].y);
  }
  if (tid < 16) mb1 = fabsf(b1[tid]);
  if (tid < 32) mb2 = fabsf(b2[tid]);
  // row sums of |W2| (576 terms per output channel o2)
  for (int o2 = wave; o2 < 32; o2 += NW) {
    float r = 0.f;
    for (int e = lane; e < 576; e += 64) r += fabsf(w2[o2 * 576 + e]);
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) r += __shfl_xor(r, o);
    if (lane == 0) rows[o2] = r;
  }
  float v[6] = {m2, m3, mb1, mb2, ml, mr};
#pragma unroll
  for (int q = 0; q < 6; ++q) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v[q] = fmaxf(v[q], __shfl_xor(v[q], o));
    if (lane == 0) red[q][wave] = v[q];
  }
  __syncthreads();
  __shared__ Scales ks;
  if (tid == 0) {
    float m[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, rmax = 0.f;
    for (int w = 0; w < NW; ++w)
      for (int q = 0; q < 6; ++q) m[q] = fmaxf(m[q], red[q][w]);
    for (int o2 = 0; o2 < 32; ++o2) rmax = fmaxf(rmax, rows[o2]);
    const float ba1 = m[2] + m[4] + m[5];  // |a1| <= max|b1| + max|PL| + max|PR|
    const float ba2 = m[3] + rmax * ba1;   // |a2| <= max|b2| + max_o2 sum|W2[o2]| |a1|
    ks.k_a1 = scale_exp(ba1);
    ks.k_w2 = scale_exp(m[0]);
    ks.k_a2 = scale_exp(ba2);
    ks.k_w3 = scale_exp(m[1]);
  }
  __syncthreads();
  S = ks;
}

__global__ __launch_bounds__(1024) void v4_scales_kernel(const float* __restrict__ w2,
                                                         const float* __restrict__ w3,
                                                         const float* __restrict__ b1,
                                                         const float* __restrict__ b2,
                                                         const float2* __restrict__ tmax, int ntmax,
                                                         Scales* __restrict__ S) {
  Scales sc;
  v4_scales<1024>(w2, w3, b1, b2, tmax, ntmax, sc);
  if (threadIdx.x == 0) *S = sc;
}

__global__ __launch_bounds__(256) void v4_pack(const float* __restrict__ w2,
                                               const float* __restrict__ w3,
                                               const Scales* __restrict__ S,
                                               _Float16* __restrict__ P2, _Float16* __restrict__ P3) {
  const int kw2 = S->k_w2, kw3 = S->k_w3;
  for (int e = threadIdx.x + blockIdx.x * 256; e < kN2 + kN3; e += 256 * gridDim.x) {
    if (e < kN2) {
      const int j = e & 7, ln = (e >> 3) & 63, tap = (e >> 9) % 9, kd = (e >> 9) / 9;
      const int o2 = ln & 31, o1 = 8 * (ln >> 5) + j;
      split16(w2[(((o2 * 16 + o1) * 4 + kd) * 3 + tap / 3) * 3 + tap % 3], kw2, P2[e], P2[kN2 + e]);
    } else {
      const int f = e - kN2;
      const int j = f & 7, ln = (f >> 3) & 63, st = f >> 9;
      const int tap = st >> 1, half = st & 1;
      const int o3 = ln & 15, o2 = 8 * (ln >> 4) + j;
      split16(w3[(((o3 * 32 + o2) * 2 + half) * 3 + tap / 3) * 3 + tap % 3], kw3, P3[f], P3[kN3 + f]);
    }
  }
}

// ------------------------------------------------------------------------------ main kernel
__global__ __launch_bounds__(kThreads, 1) void v4_main(Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // work: (n, i, strip, band), the band fastest so a CU's neighbours share table rows in L2
  int w = blockIdx.x;
  const int band = w % a.bands;
  w /= a.bands;
  const int strip = w % a.strips;
  w /= a.strips;
  const int i = w % a.D;
  const int n = w / a.D;
  const int H = a.H, W = a.W;
  const int x0 = strip * kTX;
  const int y0 = band * a.BH, y1 = min(H, y0 + a.BH);
  float* outp = a.out + ((int64_t)n * a.D + i) * H * W;
  if (x0 + kTX <= i || i >= W) {  // every output of the strip lies at x < i: zeros
    for (int e = tid; e < (y1 - y0) * kTX; e += kThreads) {
      const int r = y0 + e / kTX, x = x0 + e % kTX;
      if (x < W) outp[(int64_t)r * W + x] = 0.f;
    }
    return;
  }

  // ---- the layers' scale exponents (v4_pack) and the resident weights
  const int ka1 = a.S->k_a1, ka2 = a.S->k_a2;
  const float sa1 = __builtin_ldexpf(1.0f, ka1), sa2 = __builtin_ldexpf(1.0f, ka2);
  const int kout2 = -(ka1 + a.S->k_w2), kout3 = -(ka2 + a.S->k_w3);
  f16x8 w2h[9], w2l[9];
  {
    const int kd = wave & 3;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      w2h[t] = a.P2[(kd * 9 + t) * 64 + lane];
      w2l[t] = a.P2[4 * 9 * 64 + (kd * 9 + t) * 64 + lane];
    }
  }
  const int mb = wave & 1, kg = wave >> 1;  // layer 3: 16-pixel half, K group
  const int s0 = ks_begin(kg), s1 = ks_end(kg);
  f16x8 w3h[5], w3l[5];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    const int s = min(s0 + q, 17);
    w3h[q] = a.P3[s * 64 + lane];
    w3l[q] = a.P3[18 * 64 + s * 64 + lane];
  }

  unsigned char* a1h = smem + kOffA1;
  unsigned char* a1l = a1h + kA1Plane;
  unsigned char* a2h = smem + kOffA2;
  unsigned char* a2l = a2h + kA2Plane;
  float* part2 = reinterpret_cast<float*>(smem + kOffP2);
  float* part3 = reinterpret_cast<float*>(smem + kOffP3);

  // ---- a1 row prefetch: lane = (pixel p = lane >> 1, channel half hh) of depth block `wave`
  struct Pre {
    f32x4v pl[2], pr[2];
  };
  const int pp = lane >> 1, hh = lane & 1;
  const int xa = x0 - 2 + pp;   // this lane's a1 pixel
  auto fetch = [&](int s, Pre& pf) {
    const bool ok = s >= 0 && s < H && xa >= i && xa < W;
    const f32x4v z = {0.f, 0.f, 0.f, 0.f};
    pf.pl[0] = pf.pl[1] = pf.pr[0] = pf.pr[1] = z;
    if (ok) {
      const int c = wave * 16 + hh * 8;
      // the crop's borders: no L at x - 1 when x == i, no R at x + 1 when x == W - 1
      const float* tl = a.T + (((int64_t)n * H + s) * W + xa) * (4 * kCh) + (xa == i ? kCh : 0) + c;
      const float* tr = a.T + (((int64_t)n * H + s) * W + (xa - i)) * (4 * kCh) +
                        (xa == W - 1 ? 3 * kCh : 2 * kCh) + c;
      pf.pl[0] = *reinterpret_cast<const f32x4v*>(tl);
      pf.pl[1] = *reinterpret_cast<const f32x4v*>(tl + 4);
      pf.pr[0] = *reinterpret_cast<const f32x4v*>(tr);
      pf.pr[1] = *reinterpret_cast<const f32x4v*>(tr + 4);
    }
  };
  float bias1[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bias1[j] = a.b1[hh * 8 + j];
  // a1 = relu(b1 + PL + PR) for valid cells, 0 elsewhere (the crop's zero padding)
  auto put_a1 = [&](int s, const Pre& pf) {
    const int slot = ((s % 3) + 3) % 3;
    const bool ok = s >= 0 && s < H && xa >= i && xa < W;
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j)
      v[j] = ok ? fmaxf(bias1[j] + (pf.pl[j >> 2][j & 3] + pf.pr[j >> 2][j & 3]), 0.f) : 0.f;
    f16x8 h, l;
    split8(v, sa1, h, l);
    const int off = slot * kA1Slot + ((wave * kA1 + pp) * 16 + hh * 8) * 2;
    *reinterpret_cast<f16x8*>(a1h + off) = h;
    *reinterpret_cast<f16x8*>(a1l + off) = l;
  };
  // the a1 ring's two pad pixels stay zero
  for (int e = tid; e < 2 * 3 * 8 * 2 * 2; e += kThreads) {
    const int pl = e & 1, pad = (e >> 1) & 1, hv = (e >> 2) & 1, b = (e >> 3) % 8, sl = (e >> 3) / 8;
    const f16x8 z = {};
    *reinterpret_cast<f16x8*>((pl ? a1l : a1h) + sl * kA1Slot + ((b * kA1 + 32 + pad) * 16 + hv * 8) * 2) = z;
  }

  // one output-row step; the a1 table rows are prefetched two steps ahead, alternating between
  // two register sets (the loop below is unrolled by two so each set keeps its registers)
  auto step = [&](int s, Pre& pf) {
    // ---- a1 row s
    put_a1(s, pf);
    if (s + 2 <= y1 + 1) fetch(s + 2, pf);
    lds_barrier();
    const int q = s - 1;  // a2 row
    if (s >= y0) {
      // ---- layer 2, depth block `wave`: 9 taps x 3 products, K = 16 channels each
      f32x16 acc = {};
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int dy = t / 3, dx = t % 3;
        const int slot = ((q + dy - 1) % 3 + 3) % 3;
        const int m = lane & 31, h = lane >> 5;
        const int off = slot * kA1Slot + ((wave * kA1 + m + dx) * 16 + 8 * h) * 2;
        const f16x8 ah = *reinterpret_cast<const f16x8*>(a1h + off);
        const f16x8 al = *reinterpret_cast<const f16x8*>(a1l + off);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, w2h[t], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah, w2l[t], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al, w2h[t], acc, 0, 0, 0);
      }
      // partial [wave][px][o2]: lane holds col o2 = lane & 31, rows (r&3) + 8 (r>>2) + 4 (lane>>5)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        part2[(wave * 32 + m) * 32 + (lane & 31)] = acc[r];  // (scaled: 2^-kout2)
      }
    }
    lds_barrier();
    if (s >= y0) {
      // ---- a2 row q = relu(b2 + sum of the 4 depth blocks of its half), masked
      const int m = tid >> 4, g = tid & 15;  // pixel, group of 4 channels (ch = 32 b2 + o2)
      const int b2 = g >> 3, o2 = (4 * g) & 31;
      const int x = x0 - 1 + m;
      const bool ok = q >= 0 && q < H && x >= i && x < W;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int kd = 0; kd < 4; ++kd) {
        const f32x4v pv = *reinterpret_cast<const f32x4v*>(part2 + ((4 * b2 + kd) * 32 + m) * 32 + o2);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] += pv[j];
      }
      // back to the unscaled sum (exact: a power of two), then the bias
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = a.b2[o2 + j] + __builtin_ldexpf(v[j], kout2);
      float r4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) r4[j] = ok ? fmaxf(v[j], 0.f) : 0.f;
      unsigned hp[2], lp[2];
      split_pair16(r4[0], r4[1], sa2, hp[0], lp[0]);
      split_pair16(r4[2], r4[3], sa2, hp[1], lp[1]);
      const f16x4 h = __builtin_bit_cast(f16x4, (uint2){hp[0], hp[1]});
      const f16x4 l = __builtin_bit_cast(f16x4, (uint2){lp[0], lp[1]});
      const int slot = ((q % 3) + 3) % 3;
      const int off = slot * kA2Slot + (m * 64 + 4 * g) * 2;
      *reinterpret_cast<f16x4*>(a2h + off) = h;
      *reinterpret_cast<f16x4*>(a2l + off) = l;
      if (m < 2) {  // the ring's 2 readable pad pixels (32, 33): zeros
        const int off2 = slot * kA2Slot + ((32 + m) * 64 + 4 * g) * 2;
        const f16x4 z = {};
        *reinterpret_cast<f16x4*>(a2h + off2) = z;
        *reinterpret_cast<f16x4*>(a2l + off2) = z;
      }
    }
    lds_barrier();
    const int r = s - 2;  // output row
    if (s >= y0 + 2) {
      // ---- layer 3: this wave's K steps for its 16-pixel half
      f32x4v acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int qq = 0; qq < 5; ++qq) {
        const int st = s0 + qq;
        if (st < s1) {
          const int tap = st >> 1, half = st & 1, dy = tap / 3, dx = tap % 3;
          const int slot = ((r + dy - 1) % 3 + 3) % 3;
          const int px = 16 * mb + (lane & 15) + dx;
          const int off = slot * kA2Slot + (px * 64 + half * 32 + 8 * (lane >> 4)) * 2;
          const f16x8 ah = *reinterpret_cast<const f16x8*>(a2h + off);
          const f16x8 al = *reinterpret_cast<const f16x8*>(a2l + off);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, w3h[qq], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, w3l[qq], acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, w3h[qq], acc, 0, 0, 0);
        }
      }
      // partial [wave][px 16][o3 16]: col o3 = lane & 15, rows (lane >> 4) * 4 + reg
#pragma unroll
      for (int rr = 0; rr < 4; ++rr)
        part3[(wave * 16 + (lane >> 4) * 4 + rr) * 16 + (lane & 15)] = acc[rr];  // (2^-kout3)
    }
    lds_barrier();
    if (s >= y0 + 2 && tid < 512) {
      // ---- a3 = relu(b3 + sum over the 4 K groups), out = relu(b4 + w4 . a3), masked
      const int o = tid >> 4, o3 = tid & 15;  // output pixel 0..31, channel
      const int half = o >> 4, ol = o & 15;
      float v = 0.f;
#pragma unroll
      for (int g = 0; g < 4; ++g) v += part3[((2 * g + half) * 16 + ol) * 16 + o3];
      v = a.b3[o3] + __builtin_ldexpf(v, kout3);
      v = fmaxf(v, 0.f) * a.w4[o3];
      // sum over the 16 lanes of this pixel (aligned 16-lane groups of the wave)
#pragma unroll
      for (int sh = 8; sh >= 1; sh >>= 1) v += __shfl_xor(v, sh, 16);
      const int x = x0 + o;
      if (o3 == 0 && o < kTX && x < W) outp[(int64_t)r * W + x] = x >= i ? fmaxf(v + a.b4[0], 0.f) : 0.f;
    }
  };
  Pre pa, pb;
  fetch(y0 - 2, pa);
  fetch(y0 - 1, pb);
  for (int s = y0 - 2; s <= y1 + 1; s += 2) {
    step(s, pa);
    if (s + 1 <= y1 + 1) step(s + 1, pb);
  }
}

}  // namespace v4vol

size_t v4_workspace_bytes(int64_t N, int64_t H, int64_t W) {
  const size_t tables = (size_t)N * H * W * 4 * v4vol::kCh * sizeof(float);
  const size_t packed = (size_t)2 * (4 * 9 * 64 * 8 + 18 * 64 * 8) * 2;
  // + the scale block and the per-workgroup table maxima (v4_tmax)
  return ((tables + 255) / 256) * 256 + packed + 64 + (size_t)v4vol::kTmaxBlocks * 8;
}

int v4_volume_entry(const float* L, const float* R, float* out, int64_t N, int64_t C, int64_t H,
                    int64_t W, int64_t D, const int64_t* l_strides, const int64_t* r_strides,
                    const float* w1, const float* b1, const float* w2, const float* b2,
                    const float* w3, const float* b3, const float* w4, const float* b4,
                    void* workspace, size_t workspace_bytes, hipStream_t st) {
  using namespace v4vol;
  if (N < 0 || H < 0 || W < 0 || D < 0) return fail(SM_EINVAL, "v4_volume: negative size");
  if (C != kC) return fail(SM_EUNSUPPORTED, "v4_volume: the V4 stack needs C = 32 feature channels");
  if (N * D * H * W == 0) return SM_OK;
  if (!L || !R || !out || !w1 || !b1 || !w2 || !b2 || !w3 || !b3 || !w4 || !b4 || !workspace)
    return fail(SM_EINVAL, "v4_volume: null pointer");
  if (workspace_bytes < v4_workspace_bytes(N, H, W))
    return fail(SM_EINVAL, "v4_volume: workspace too small (sm_v4_volume_workspace_bytes)");
  if (H * W >= ((int64_t)1 << 31) / (4 * kCh) / std::max<int64_t>(N, 1) || W >= (1 << 24))
    return fail(SM_EINVAL, "v4_volume: planes too large");
  Strides4 ls, rs;
  int rc = read_strides(l_strides, C, H, W, &ls, "left");
  if (rc != SM_OK) return rc;
  rc = read_strides(r_strides, C, H, W, &rs, "right");
  if (rc != SM_OK) return rc;
  float* T = static_cast<float*>(workspace);
  const size_t tables = (size_t)N * H * W * 4 * kCh * sizeof(float);
  _Float16* P2 = reinterpret_cast<_Float16*>(static_cast<unsigned char*>(workspace) + ((tables + 255) / 256) * 256);
  _Float16* P3 = P2 + 2 * kN2;
  Scales* S = reinterpret_cast<Scales*>(P3 + 2 * kN3);
  float2* tmax = reinterpret_cast<float2*>(reinterpret_cast<unsigned char*>(S) + 64);
  hipLaunchKernelGGL(v4_tables, dim3((unsigned)ceil_div(N * H * W, 256), 8), dim3(256), 0, st, L, R,
                     ls, rs, w1, T, (int)N, (int)H, (int)W);
  rc = check_launch("v4_tables");
  if (rc != SM_OK) return rc;
  hipLaunchKernelGGL(v4_tmax, dim3(kTmaxBlocks), dim3(256), 0, st, T, N * H * W * kCh, tmax);
  rc = check_launch("v4_tmax");
  if (rc != SM_OK) return rc;
  hipLaunchKernelGGL(v4_scales_kernel, dim3(1), dim3(1024), 0, st, w2, w3, b1, b2, tmax, kTmaxBlocks, S);
  rc = check_launch("v4_scales_kernel");
  if (rc != SM_OK) return rc;
  hipLaunchKernelGGL(v4_pack, dim3(16), dim3(256), 0, st, w2, w3, S, P2, P3);
  rc = check_launch("v4_pack");
  if (rc != SM_OK) return rc;
  Args a;
  a.T = T;
  a.P2 = reinterpret_cast<const f16x8*>(P2);
  a.P3 = reinterpret_cast<const f16x8*>(P3);
  a.S = S;
  a.b1 = b1;
  a.b2 = b2;
  a.b3 = b3;
  a.w4 = w4;
  a.b4 = b4;
  a.out = out;
  a.N = (int)N;
  a.H = (int)H;
  a.W = (int)W;
  a.D = (int)D;
  a.strips = (int)ceil_div(W, kTX);
  // row bands: enough workgroups to fill the chip twice, at most ~8 % halo rows
  const int64_t base = N * D * a.strips;
  int bands = (int)std::min<int64_t>(std::max<int64_t>(1, ceil_div(2048, std::max<int64_t>(base, 1))),
                                     std::max<int64_t>(1, H / 24));
  a.BH = (int)ceil_div(H, bands);
  a.bands = (int)ceil_div(H, a.BH);
  const int64_t nwg = base * a.bands;
  if (nwg >= INT32_MAX) return fail(SM_EINVAL, "v4_volume: too much work for one launch");
  static std::atomic<unsigned long long> lds_done{0};
  const int dev = stream_device(st);
  rc = ensure_lds_limit(reinterpret_cast<const void*>(v4_main), kShm, dev, lds_done);
  if (rc != SM_OK) return rc;
  hipLaunchKernelGGL(v4_main, dim3((unsigned)nwg), dim3(kThreads), kShm, st, a);
  return check_launch("v4_main");
}

}  // namespace smcv

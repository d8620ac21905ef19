// Inner-product / correlation cost volume (N, D, H, W) from fp32 features: the sliding-window
// role-split band kernel ("sl"), one workgroup of eight waves per CU, per SIMD a compute wave and
// a memory wave (as band_rs, ip_rs.hip).
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// The contraction, the operands (per-segment power-of-two scale, round-to-nearest two-plane fp16
// split, h*h' + h*m' + m*h' on v_mfma_f32_32x32x16_f16), the 32 x 32 blocks of a compute wave and
// the scale control are band_rs's.  What changes is the feature path:
//   * a workgroup owns whole image rows and walks their 128-pixel segments left to right, so the
//     right window of segment s, R columns [x0 - DMAX, x0 + 128), is the previous segment's window
//     slid by 128 columns.  The window stays in LDS for all C channels as a ring of 32-column
//     blocks (block b in slot b mod NB), and a segment loads and splits only its own 128 left and
//     128 new right columns: 256 staged columns per segment instead of band_rs's 448
//     (128 + DMAX + 128), i.e. 43 % fewer feature loads and splits at D = 192;
//   * the slots of the window's oldest 128 columns are free for a channel step as soon as the
//     current segment has multiplied that step, so with C = 64 (four steps) the next segment's
//     columns are staged into them one step later (NB = 4 + DMAX/32); with one step (C = 16) the
//     ring has four slack blocks;
//   * a memory wave stages 4 pixels x 4 channels per lane (one 16-channel step of 128 columns is
//     two waves' work), L and R by different wave pairs, every step;
//   * the compute wave shears its accumulators into a 3-slot ring of 32 x 32 chunks during the
//     next pass's first step, block by block between that step's MFMAs (block T-1 first), and
//     reads each chunk out as soon as it is complete and before its slot is reused; the last two
//     chunks drain over the next steps.  (band_rs wrote all T-1 chunks at once: 96 KB of ring.)
//     LDS at C = 64, D = 192: 80 KB window + 16 KB left tiles + 48 KB shear rings.
//   * segments are counted per workgroup (sigma), and the window block of segment sigma, pass p,
//     relative block j is ring block 4 sigma - (dp + DMAX)/32 + j: a row change keeps the ring's
//     slot sequence, and the columns left of x = 0 (previous row's data) reach only cells x < d,
//     which the kernel forces to 0 (the same select band_rs uses for its zero pad).
// D > 192 (two passes of pw = 32 m <= DMAX disparities, C = 16: the correlation at D = 256) keeps
// both passes' windows resident; the passes of a segment are consecutive steps, and the fused
// volume-free pass carries each pixel's soft-argmin state from pass 0 to pass 1 in registers.
#include "band_common.h"

#ifndef SMCV_SL_DIAG_ROLE
#define SMCV_SL_DIAG_ROLE 0
#endif
#ifndef SMCV_SL_ABLATE
#define SMCV_SL_ABLATE 0  // diagnostics only (var_so builds): 1 no ring writes, 2 no chunk reads or
#endif                    // stores, 4 no feature loads, 8 no MFMA, 16 no staging (no LDS writes),
                          // 32 no per-step barrier, 64 chunk stores without the ring reads
#ifndef SMCV_SL_NTLOAD
#define SMCV_SL_NTLOAD 0  // feature loads non-temporal (each feature byte is read once)
#endif
#ifndef SMCV_SL_NTSTORE
#define SMCV_SL_NTSTORE SMCV_NT_STORE  // volume stores non-temporal
#endif
#ifndef SMCV_SL_SETS
#define SMCV_SL_SETS 4  // feature-load register sets (loads issued SETS - 1 steps ahead)
#endif
#ifndef SMCV_SL_MAP
#define SMCV_SL_MAP 1  // rows of a workgroup: 1 XCD-contiguous ranges, 0 strided over the grid
#endif
#ifndef SMCV_SL_FOLD_IL
#define SMCV_SL_FOLD_IL 0  // 1: fold block t right before its MFMAs (measured 4-7 % slower, r6q); 0: all first
#endif

namespace smcv {
namespace h2band {

namespace slide {
constexpr int kCW = 4;                 // compute waves (one per SIMD), as many memory waves
constexpr int kThreads = 2 * 64 * kCW;
constexpr int kKC = 16;                // channels per step (one 32x32x16 k-step)
constexpr int kSlot = 32 * 32 * 4;     // one shear chunk: 32 d x 32 x fp32
constexpr int kBlk = 32 * 32;          // one 32-row block of one fp16 plane (16 channels)

template <int TMAX, int NKS, int NP, int FUSE>
struct Geo {
  static constexpr int DMAX = 32 * (TMAX - 1);
  // R ring blocks per channel step: the window (4 + NP DMAX/32 blocks at most), plus four slack
  // blocks when one step must stage the next segment's columns while its own window is in use
  static constexpr int NB = NKS >= 2 ? (TMAX - 1) + 4 : NP * (TMAX - 1) + 8;
  static constexpr int RPL = NB * kBlk;          // one plane (h or m) of one channel step
  static constexpr int RSTEP = 2 * RPL;
  static constexpr int L0 = NKS * RSTEP;         // two left tiles (128 rows, h + m planes)
  static constexpr int LPL = 128 * 32;
  static constexpr int LBUF = 2 * LPL;
  static constexpr int SH0 = L0 + 2 * LBUF;      // the compute waves' shear rings
  static constexpr int SHW = FUSE == 2 ? 0 : 3 * kSlot;
  static constexpr int MAXW = SH0 + kCW * SHW;   // maxima: max|L| of 8 segments, max|R| of the
  static constexpr size_t SHM = (size_t)MAXW + 24 * 4;  // two 64-column halves of 8 pieces
  static_assert(SHM <= 160 * 1024, "one workgroup per CU");
  static_assert(NKS == 1 || NKS % 2 == 0, "channel steps");
  static_assert(NP == 1 || NKS == 1, "two D passes keep one channel step's windows");
};

// The staging tasks of step q of a segment (0 <= q < NP NKS): the segment offset (0 or 1) and
// channel step of the left tile (L) and of the right columns (R) staged in it; has = false: none.
struct Task {
  bool has;
  int del, kc;
};
template <int NKS, int NP>
constexpr Task l_task(int q) {
  if (NP == 2) return q == 0 ? Task{true, 1, 0} : Task{false, 0, 0};
  if (NKS == 1) return Task{true, 1, 0};
  return Task{true, (q + 1) / NKS, (q + 1) % NKS};  // the next step's tile
}
template <int NKS, int NP>
constexpr Task r_task(int q) {
  if (NP == 2) return q == 1 ? Task{true, 1, 0} : Task{false, 0, 0};
  if (NKS == 1) return Task{true, 1, 0};
  // step q frees the window's oldest columns of channel step q - 1: the next segment's go there;
  // step 0 stages this segment's last channel step (its slots were freed by the previous segment)
  return q == 0 ? Task{true, 0, NKS - 1} : Task{true, 1, q - 1};
}
constexpr int pmod(int a, int m) { return ((a % m) + m) % m; }
}  // namespace slide

template <bool CW, bool MEAN, int TMAX, int NKS, int NP, int NSETS, int FUSE>
__device__ __forceinline__ void sl_role(const Args& args, unsigned char* smem) {
  using namespace slide;
  using G = Geo<TMAX, NKS, NP, FUSE>;
  constexpr bool VOL = FUSE != 2;
  constexpr int T = TMAX;
  constexpr int DMAX = G::DMAX;
  constexpr int NB = G::NB;
  constexpr int NSTEP = NP * NKS;
  // the range check on a segment's maxima: after its steps (C = 64: its last right columns are
  // staged in its own first step), or before them (one channel step: everything it reads was
  // staged, and its maxima published, one step earlier)
  constexpr bool CHECK_FIRST = NKS == 1;
  static_assert(T >= 5, "the 3-slot shear ring needs blocks T-1 .. 0 to reach chunk T-4 >= 1");
  constexpr bool isC = CW;
  const float* __restrict__ L = static_cast<const float*>(args.L);
  const float* __restrict__ R = static_cast<const float*>(args.R);
  const int H = args.H, W = args.W, D = args.D;
  const Strides4 ls = args.ls, rs = args.rs;

  // The (n, y) rows a workgroup walks: segment sigma is row rbeg + (sigma / tiles) rstep, tile
  // sigma % tiles.  SMCV_SL_MAP 1 (with a grid of whole XCD groups): XCD group b & 7 (workgroups
  // b and b + 8 share an XCD, as Sched assumes) owns a contiguous eighth of the rows and its
  // workgroups take rows gi, gi + 32, ... of it, so an XCD works on ~32 neighbouring rows at a
  // time; else rows b, b + nwg, ... (round 5).  The write stream of the first map measured 6 %
  // faster in the memory-pattern micro (profiles/r06/memory/).
  const int bwg = blockIdx.x, nwg = gridDim.x;
  const int rows = args.nwork;
  if (bwg >= rows) return;  // the whole workgroup leaves together
  int rbeg = bwg, rstep = nwg, rcnt = (rows - bwg + nwg - 1) / nwg;
  if (SMCV_SL_MAP && nwg % 8 == 0 && rows >= nwg) {  // then every group has >= nwg / 8 rows
    const int grp = bwg & 7, gi = bwg >> 3, gsz = nwg >> 3;
    const int q = rows / 8, r = rows % 8;
    const int gb = grp * q + min(grp, r), gc = q + (grp < r ? 1 : 0);
    rbeg = gb + gi;
    rstep = gsz;
    rcnt = (gc - gi + gsz - 1) / gsz;
  }
  const int nitems = rcnt * args.tiles;
  auto witem = [&](int i) -> Work {
    const unsigned ii = (unsigned)min(i, nitems - 1);
    const unsigned ri = fdiv(ii, args.fd_tiles);
    const int s = (int)(ii - ri * (unsigned)args.tiles);
    const unsigned row = (unsigned)rbeg + ri * (unsigned)rstep;
    const unsigned nn = fdiv(row, args.fd_h);
    Work k;
    k.n = (int)nn;
    k.y = (int)(row - nn * (unsigned)H);
    k.g = 0;
    k.x0 = s * kXT;
    k.dp = 0;
    k.Dp = min(args.pw, D);
    k.js = k.x0 - DMAX;
    k.pass = 0;
    return k;
  };
  auto pass_of = [&](Work k, int p) -> Work {
    k.pass = p;
    k.dp = p * args.pw;
    k.Dp = min(args.pw, D - k.dp);
    k.js = k.x0 - k.dp - DMAX;
    return k;
  };

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rw = wave & (kCW - 1);  // the 32-pixel slice (and shear ring) of a compute wave
  const int lane = tid & 63;
  const int lr = lane & 31;
  const int hh = lane >> 5;
  const unsigned sbase = lds_addr(smem);
  const unsigned maxw = sbase + (unsigned)G::MAXW;  // Lmax[8], then Rmax[8][2]

  // ------------------------------------------------------- staging role of a memory-wave lane
  // waves 4, 5 stage left tiles, 6, 7 right columns; wave parity wp: channels 8 wp .. 8 wp + 7 of
  // the step; lane: pixel group g (4 pixels), channels 8 wp + 4 c4 .. + 3.  Over 16 consecutive
  // lanes (one ds_write_b64 lane group) (g & 7, c4) take 16 distinct values: conflict-free.
  const int mw = max(wave - kCW, 0);
  const bool isR = mw >= 2;  // wave-uniform
  const int wp = mw & 1;
  const int gq = (lane & 7) | (((lane >> 4) & 3) << 3);
  const int c4 = (lane >> 3) & 1;
  const int chl = 8 * wp + 4 * c4;
  const int64_t cs = isR ? rs.c : ls.c;
  // this lane's byte offset within a 32-row block / within the 128-row left tile (pixel 0 of its
  // group; pixel p at ^ 32 p)
  const unsigned o_blk = (unsigned)swz(4 * (gq & 7), wp) + 8u * (unsigned)c4;
  const unsigned o_l = (unsigned)swz(4 * gq, wp) + 8u * (unsigned)c4;

  f32x4v sv[NSETS][4];
  bool okp[NSETS];
  auto load = [&](int set, const Work& k, int kc) __attribute__((always_inline)) {
    const int px = k.x0 + 4 * gq;
    okp[set] = px < W;
    const int pxc = min(px, W - 4);  // pad groups (x >= W): a valid group, staged as zeros
    const float* p = (isR ? R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h
                          : L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h) +
                     pxc + (int64_t)(kc * kKC + chl) * cs;
    int64_t csl = cs;
    asm volatile("" : "+v"(csl));
    if constexpr (SMCV_SL_ABLATE & 4) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sv[set][j] = f32x4v{1.f, -1.f, 0.5f, 2.f};
        asm volatile("" : "+v"(sv[set][j]));
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      // compiler-tracked: it places the vmcnt waits itself
      if constexpr (SMCV_SL_NTLOAD) {
        typedef __attribute__((address_space(1))) const void gcvoid;
        sv[set][j] = __builtin_nontemporal_load(
            reinterpret_cast<__attribute__((address_space(1))) const f32x4v*>((gcvoid*)p));
      } else {
        gload<false>(sv[set][j], p);
      }
      p += csl;
    }
  };
  int kL = 0, kR = 0;  // scale exponents of the staging side (workgroup-uniform)
  float mx = 0.f;      // this lane's max|x| over the segment tile / right piece being staged
  // stage set `set` to LDS byte address dst (this lane's pixel-0 word of the h plane; the m plane
  // at + poff); keep = false: compute nothing but the loads' consumption (a half-piece's other
  // half, which must not be written)
  auto stage = [&](int set, unsigned dst, unsigned poff, bool keep) __attribute__((always_inline)) {
    f32x4v(&x)[4] = sv[set];
    float m0 = 0.f, m1 = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m0) : "v"(x[j].x), "v"(x[j].y));
      asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m1) : "v"(x[j].z), "v"(x[j].w));
    }
    mx = okp[set] && keep ? fmaxf(mx, fmaxf(m0, m1)) : mx;
    const float sc = okp[set] ? __builtin_ldexpf(1.0f, isR ? kR : kL) : 0.f;
    unsigned o0 = dst;
    asm volatile("" : "+v"(o0));
#pragma unroll
    for (int pp = 0; pp < 4; pp += 2) {
      uint4 wh, wm;
      const float xs[8] = {x[0][pp], x[1][pp], x[2][pp], x[3][pp],
                           x[0][pp + 1], x[1][pp + 1], x[2][pp + 1], x[3][pp + 1]};
      split_quad(xs, sc, wh, wm);
      if (keep && !(SMCV_SL_ABLATE & 16)) {
        const unsigned a0 = o0 ^ (32u * pp), a1 = o0 ^ (32u * (pp + 1));
        *reinterpret_cast<__attribute__((address_space(3))) u32x2*>(a0) = u32x2{wh.x, wh.y};
        *reinterpret_cast<__attribute__((address_space(3))) u32x2*>(a0 + poff) = u32x2{wm.x, wm.y};
        *reinterpret_cast<__attribute__((address_space(3))) u32x2*>(a1) = u32x2{wh.z, wh.w};
        *reinterpret_cast<__attribute__((address_space(3))) u32x2*>(a1 + poff) = u32x2{wm.z, wm.w};
      }
    }
  };
  // LDS destination of a right-column task: piece sigma (blocks 4 sigma .. 4 sigma + 3), channel
  // step kc; this lane's block is gq / 8
  auto r_dst = [&](int sigma, int kc) -> unsigned {
    int sl = pmod(4 * sigma, NB) + (gq >> 3);
    sl = sl >= NB ? sl - NB : sl;
    return sbase + (unsigned)(kc * G::RSTEP + sl * kBlk) + o_blk;
  };
  auto l_dst = [&](int lp) -> unsigned { return sbase + (unsigned)(G::L0 + lp * G::LBUF) + o_l; };
  // publish this lane set's maxima: a left tile (one word) or a right piece (its two 64-column
  // halves: lanes 0-31 hold pixel groups 0-15, lanes 32-63 groups 16-31)
  auto publish = [&](int sigma) __attribute__((always_inline)) {
    float v = mx;
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
    if (isR) {
      if (lr == 0)
        asm volatile("ds_max_u32 %0, %1" : : "v"(maxw + 32u + 8u * (unsigned)(sigma & 7) + 4u * (unsigned)hh),
                     "v"(__float_as_uint(v)) : "memory");
    } else {
      v = fmaxf(v, __shfl_xor(v, 32));
      if (lane == 0)
        asm volatile("ds_max_u32 %0, %1" : : "v"(maxw + 4u * (unsigned)(sigma & 7)), "v"(__float_as_uint(v))
                     : "memory");
    }
  };

  // --------------------------------------------------------------- compute role of a wave
  f32x16 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = f32x16{};
  auto mma = [](f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  };

  // the pass whose accumulators go into the ring next (workgroup-uniform)
  Work pw = witem(0);
  int p_kk = 0;
  bool p_special = false;  // scaled (kk != 0) or holding cells x < d (js < 0)
  int p_bytes = 0;         // 0x80000000 (valid) or 0 (every store dropped)
  bool p_full = false;     // the whole 128-pixel segment and all DMAX disparities are stored
  float* p_ob = static_cast<float*>(args.out);
  const int64_t plane_stride = (int64_t)H * W;
  const bool nt_rows = __builtin_amdgcn_readfirstlane(W % 16 == 0 ? 1 : 0) != 0;
  // volume-free fused pass with two D passes: pass 0's soft-argmin state of the lane pair's pixel
  [[maybe_unused]] float f_m = 0.f;
  [[maybe_unused]] double f_s = 0.0, f_t = 0.0;

  // ---------------------------------------------------------------------- the shear ring
  // Lane (lr, hh), element i of block t: R row c_i + 4 hh (c_i = (i & 3) + 8 (i >> 2)), pixel
  // x0 + 32 rw + lr, local disparity 32 (a + 1) + u - c_i with a = T-2-t, u = lr - 4 hh: chunk
  // a + 1 row u - c_i (u >= c_i) or chunk a row 32 + u - c_i.  Chunk c lives in slot c mod 3
  // (ring + 4096 slot, [32 d][32 x] fp32).  When slot(a + 1) = slot(a) + 1 the element's address
  // is wb + 4096 slot(a + 1) - 128 c_i - 512 with wb = ring + 512 + 128 u + 4 lr (an immediate
  // offset per element); the blocks with a = 2 mod 3 (slots 2 and 0, among them a = -1, whose
  // chunk -1 half lands in slot 2 and is overwritten later) use per-lane addresses wrap[i].
  // ds_write_b32: bank = (32 row + lr) mod 32, conflict free.
  const int u = lr - 4 * hh;
  const unsigned ring = sbase + (unsigned)(G::SH0 + rw * G::SHW);
  const unsigned wb = ring + (unsigned)(512 + 128 * u + 4 * lr);
  unsigned wrap[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int ci = (i & 3) + 8 * (i >> 2);
    wrap[i] = u >= ci ? ring + (unsigned)(128 * (u - ci) + 4 * lr)
                      : ring + (unsigned)(2 * kSlot + 128 * (32 + u - ci) + 4 * lr);
  }
  auto write_block = [&]<int t, bool SPEC>() __attribute__((always_inline)) {
    if constexpr (SMCV_SL_ABLATE & 1) return;
    constexpr int a = T - 2 - t;
    constexpr bool WR = pmod(a, 3) == 2;
    constexpr int sa1 = pmod(a + 1, 3);
    const int jl = pw.js + 32 * rw + 4 * hh;
    const unsigned wbl = wb;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ci = (i & 3) + 8 * (i >> 2);
      float val = acc[t][i];
      if constexpr (MEAN) val *= args.mul;
      if constexpr (SPEC) {
        val = __builtin_ldexpf(val, p_kk);
        val = jl + 32 * t + ci >= 0 ? val : 0.f;  // R rows left of x = 0: cells x < d
      }
      if constexpr (WR) {
        const unsigned wa = wrap[i];
        asm volatile("ds_write_b32 %0, %1" : : "v"(wa), "v"(val) : "memory");
      } else {
        // (>= 0: a non-wrapping block has chunk a + 1 in slot 1 or 2)
        const int imm = sa1 * kSlot - 128 * ci - 512;
        asm volatile("ds_write_b32 %0, %1 offset:%2" : : "v"(wbl), "v"(val), "n"(imm) : "memory");
      }
    }
  };
  const int rl = lane >> 3, cl = lane & 7;
  // chunk c (slot c mod 3): rows 8 qq + rl, pixels 4 cl .. 4 cl + 3 -> out[n, dp + 32 c + row, y,
  // x0 + 32 rw + 4 cl ..]
  auto drain_read = [&]<int c>(f32x4v(&vp)[4]) __attribute__((always_inline)) {
    if constexpr (!VOL || (SMCV_SL_ABLATE & 2)) return;
    if constexpr (SMCV_SL_ABLATE & 64) {
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        vp[qq] = f32x4v{0.f, 0.f, 0.f, 0.f};
        asm volatile("" : "+v"(vp[qq]));
      }
      return;
    }
    int rr = rl, cc = cl;
    asm volatile("" : "+v"(rr), "+v"(cc));
    const unsigned rb = ring + (unsigned)(rr * 128 + 16 * cc);
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) vp[qq] = lds_load4(rb + (unsigned)(pmod(c, 3) * kSlot + qq * 1024));
  };
  auto drain_store = [&]<int c>(const f32x4v(&vp)[4]) __attribute__((always_inline)) {
    if constexpr (!VOL || (SMCV_SL_ABLATE & 2)) return;
    int rr = rl, cc = cl;
    asm volatile("" : "+v"(rr), "+v"(cc));
    float* cb = p_ob + (int64_t)(32 * c) * plane_stride;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(cb, (short)0, p_bytes, 0x00020000);
    const unsigned q8 = (unsigned)(8 * plane_stride * 4);
    const unsigned lo = (unsigned)(rr * plane_stride * 4 + 16 * cc);
    // non-temporal stores when the volume rows are 64-B aligned (W % 16 == 0: every 128-B
    // piece of a store fills whole 64-B halves of lines); otherwise a piece straddles two lines
    // that a neighbouring wave completes, and plain stores let L2 merge the halves before the
    // write-back (W = 952 / 956: 1,517 / 1,557 against 1,903 / 2,209 us per 8-pair launch,
    // profiles/r06/stale/r6r_*; W = 928 / 944 / 960 as fast or faster non-temporal)
    auto st = [&](const f32x4v& v, unsigned off) __attribute__((always_inline)) {
      const auto u = __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, v);
      if (SMCV_SL_NTSTORE && nt_rows)
        __builtin_amdgcn_raw_buffer_store_b128(u, rsrc, off, 0, 2);
      else
        __builtin_amdgcn_raw_buffer_store_b128(u, rsrc, off, 0, 0);
    };
    if (p_full) {  // every cell of the chunk is inside the volume
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) st(vp[qq], lo + (unsigned)qq * q8);
    } else {
      // masked lanes: the offset's top bit set (out of range, dropped)
      const unsigned xbad = (unsigned)(pw.x0 + 32 * rw + 4 * cc >= W) << 31;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const unsigned bad = xbad | ((unsigned)(32 * c + 8 * qq + rr >= pw.Dp) << 31);
        st(vp[qq], (lo + (unsigned)qq * q8) | bad);
      }
    }
  };
  auto drain = [&]<int c>() __attribute__((always_inline)) {
    f32x4v vp[4];
    drain_read.template operator()<c>(vp);
    drain_store.template operator()<c>(vp);
  };
  auto set_prev = [&](const Work& k, bool valid) __attribute__((always_inline)) {
    pw = k;
    p_kk = -(kL + kR);
    p_special = p_kk != 0 || k.js < 0;
    p_bytes = valid ? (int)0x80000000 : 0;
    p_full = k.Dp == DMAX && k.x0 + kXT <= W;
    p_ob = static_cast<float*>(args.out) +
           (((int64_t)k.n * D + k.dp) * plane_stride + (int64_t)k.y * W + k.x0 + 32 * rw);
  };
  // the previous pass's fold finished: the lane pair merged, then the disparity stored (one D
  // pass) or pass 0's state kept in registers for pass 1 (two passes)
  [[maybe_unused]] float fm = -INFINITY;
  [[maybe_unused]] double fs = 0.0, ft = 0.0;
  auto fold_finish = [&]() __attribute__((always_inline)) {
    float M;
    fold_pair_merge(fm, fs, ft, M);
    if constexpr (NP == 1) {
      const int x = pw.x0 + 32 * rw + lr;
      if (hh == 0 && x < W)
        store_one<float>(args.disp + ((size_t)pw.n * H + pw.y) * W + x, (float)(ft / fs));
    } else {
      const double to = ft + (double)pw.dp * fs;
      if (pw.pass == 0) {
        f_m = M;
        f_s = fs;
        f_t = to;
      } else {
        fused_two_pass_store(args, pw, rw, lr, hh, f_m, f_s, f_t, M, fs, to);
      }
    }
  };
  // one block of that fold (the SPEC flags workgroup-uniform: one branch per block)
  auto fold_one = [&]<int t>() __attribute__((always_inline)) {
    const bool sc = p_kk != 0, xl = pw.js < 0;
    if (!sc && !xl)
      fold_block<T, MEAN, false, false, FoldF32, t>(acc[t], args, pw, -p_kk, 0, rw, lr, hh, fm, fs, ft);
    else if (sc && !xl)
      fold_block<T, MEAN, true, false, FoldF32, t>(acc[t], args, pw, -p_kk, 0, rw, lr, hh, fm, fs, ft);
    else if (!sc)
      fold_block<T, MEAN, false, true, FoldF32, t>(acc[t], args, pw, -p_kk, 0, rw, lr, hh, fm, fs, ft);
    else
      fold_block<T, MEAN, true, true, FoldF32, t>(acc[t], args, pw, -p_kk, 0, rw, lr, hh, fm, fs, ft);
  };
  // FUSE: the previous pass's soft-argmin straight from the accumulators (band_common.h), before
  // the next pass's first MFMAs overwrite them; nothing for an invalid segment.  Two D passes
  // without the volume: pass 0's state waits in registers for pass 1.
  auto fuse_regs = [&]() __attribute__((always_inline)) {
    if constexpr (FUSE != 0) {
      if (p_bytes == 0) return;
      auto go = [&](auto scale, auto xlt) __attribute__((always_inline)) {
        constexpr bool SC = decltype(scale)::value, XL = decltype(xlt)::value;
        if constexpr (NP == 1) {
          fused_softargmin<T, MEAN, SC, XL, false, FoldF32>(acc, args, pw, -p_kk, 0, rw, lr, hh);
        } else {
          float m;
          double s, t;
          fused_softargmin_state<T, MEAN, SC, XL, FoldF32>(acc, args, pw, -p_kk, 0, rw, lr, hh, m, s, t);
          if (pw.pass == 0) {
            f_m = m;
            f_s = s;
            f_t = t;
          } else {
            fused_two_pass_store(args, pw, rw, lr, hh, f_m, f_s, f_t, m, s, t);
          }
        }
      };
      const bool sc = p_kk != 0, xl = pw.js < 0;
      if (!sc && !xl)
        go(std::false_type{}, std::false_type{});
      else if (sc && !xl)
        go(std::true_type{}, std::false_type{});
      else if (!sc)
        go(std::false_type{}, std::true_type{});
      else
        go(std::true_type{}, std::true_type{});
    }
  };

  auto barrier = []() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };

  // --------------------------------------------------------------------------- the steps
  // The loop body runs U segments (U NSTEP a multiple of NSETS: the load sets), so every step's
  // load set and tasks are fixed at compile time.  Step GS of the body is step q = GS % NSTEP of
  // body segment GS / NSTEP; wq[k] is the work item of segment it + k.
  constexpr int U = [] {
    int uu = 1;
    while ((uu * NSTEP) % NSETS != 0) ++uu;
    return uu;
  }();
  constexpr int LOOK = NSETS - 1;
  constexpr int LA = 2 + (LOOK + NSTEP - 1) / NSTEP;
  int it = 0;     // the segment multiplied
  int lpar = 0;   // the left tile buffer the current step reads
  int s_rel = 0;  // the current segment's tile index within its row
  Work wq[LA];
#pragma unroll
  for (int k = 0; k < LA; ++k) wq[k] = witem(k);
  // the current pass's window: the slot of block rw of the pass's window, times the block size
  int sw = 0;
  auto set_window = [&](int p) __attribute__((always_inline)) {
    int s0 = pmod(4 * it - (p * args.pw + DMAX) / 32 + rw, NB);
    sw = __builtin_amdgcn_readfirstlane(s0);
  };
  auto rslot = [&](int t) -> unsigned {  // block t of the compute wave's band (t < T <= NB)
    const int s = sw + t;
    return (unsigned)((s >= NB ? s - NB : s) * kBlk);
  };

  // MFMAs of one channel step: block t = T-1 .. 0 (the shear order), with the ring writes of the
  // previous pass's block t first when SHEAR, and the chunk readouts between them
  // (SPEC: a workgroup-uniform branch around each block's ring writes only; a whole second copy
  // of the step, MFMAs included, made the register allocator spill at the join)
  // FOLD (the fused passes' first step, SMCV_SL_FOLD_IL): block t is folded into the previous
  // pass's soft-argmin right before its MFMAs overwrite it, so the fold's VALU work of block t - 1
  // issues while block t's MFMAs run (the fold order T-1 .. 0: the same in the volume-kept and the
  // volume-free pass, which stay bit-identical)
  auto matrix = [&]<int KS, bool SHEAR, bool FOLD = false>(unsigned lb) __attribute__((always_inline)) {
    const unsigned char* bb = smem + lb + 32 * rw * 32 + swz(lr, hh);
    const f16x8 bh = *reinterpret_cast<const f16x8*>(bb);
    const f16x8 bmv = *reinterpret_cast<const f16x8*>(bb + G::LPL);
    const unsigned char* rk = smem + KS * G::RSTEP + swz(lr, hh);
    [[maybe_unused]] f32x4v cv[4];
    [&]<int... K_>(std::integer_sequence<int, K_...>) __attribute__((always_inline)) {
      (
          [&]() __attribute__((always_inline)) {
            constexpr int t = T - 1 - K_;
            constexpr int cr = T - 4 - t;  // the chunk read before this block's ring writes
            // the block's fragments first (their latency hides behind the ring writes); the
            // address is opaque so the reads are not hoisted over earlier blocks
            unsigned ao = rslot(t);
            asm volatile("" : "+v"(ao));
            const unsigned char* ab = rk + ao;
            const f16x8 ah = *reinterpret_cast<const f16x8*>(ab);
            const f16x8 am = *reinterpret_cast<const f16x8*>(ab + G::RPL);
            if constexpr (FOLD) {
              if (p_bytes != 0) fold_one.template operator()<t>();
            }
            if constexpr (SHEAR && VOL) {
              if constexpr (cr >= 0) drain_read.template operator()<cr>(cv);
              if (__builtin_expect(p_special, 0))
                write_block.template operator()<t, true>();
              else
                write_block.template operator()<t, false>();
            }
            if constexpr (SMCV_SL_ABLATE & 8) {  // accumulators opaque: the fold stays whole
              asm volatile("" : "+v"(acc[t]) : "v"(ah), "v"(am), "v"(bh), "v"(bmv));
            } else {
              f32x16 c;
              if constexpr (KS == 0)
                c = mma(am, bh, f32x16{});
              else
                c = mma(am, bh, acc[t]);
              c = mma(ah, bmv, c);
              acc[t] = mma(ah, bh, c);
            }
            if constexpr (SHEAR && VOL && cr >= 0) drain_store.template operator()<cr>(cv);
            if constexpr (SHEAR && VOL) __builtin_amdgcn_sched_barrier(0);
          }(),
          ...);
    }(std::make_integer_sequence<int, T>{});
  };
  auto first_step = [&]<int KS>(unsigned lb) __attribute__((always_inline)) {
    // (not at C = 16 with 7 blocks: its compute wave would spill)
    constexpr bool FIL = FUSE != 0 && SMCV_SL_FOLD_IL && !(NKS == 1 && T == 7);
    if constexpr (FIL) {
      fm = -INFINITY;
      fs = 0.0;
      ft = 0.0;
    } else {
      fuse_regs();
    }
    if constexpr (VOL) {
      matrix.template operator()<KS, true, FIL>(lb);
      if constexpr (FIL) {
        if (p_bytes != 0) fold_finish();
      }
      if constexpr (NKS == 1) {  // the last two chunks now (the next step shears again)
        drain.template operator()<T - 3>();
        drain.template operator()<T - 2>();
      }
    } else {
      matrix.template operator()<KS, false, FIL>(lb);
      if constexpr (FIL) {
        if (p_bytes != 0) fold_finish();
      }
    }
  };

  auto step = [&]<int GS>() __attribute__((always_inline)) {
    constexpr int q = GS % NSTEP;
    constexpr int KS = q % NKS;
    constexpr int SI = GS / NSTEP;
    const unsigned lb = (unsigned)(G::L0 + lpar * G::LBUF);
    if constexpr (isC) {
      if constexpr (KS == 0) {
        set_window(q / NKS);
        first_step.template operator()<KS>(lb);
      } else {
        // the previous pass's chunks T-3 (step 1) and T-2 (step 2; with two steps, both in step 1):
        // read before the MFMAs, stored after them
        constexpr int c0 = KS == 1 ? T - 3 : T - 2;
        constexpr int c1 = (KS == 1 && NKS == 2) ? T - 2 : -1;
        [[maybe_unused]] f32x4v pv[2][4];
        if constexpr (VOL && KS <= 2) drain_read.template operator()<c0>(pv[0]);
        if constexpr (VOL && c1 >= 0) drain_read.template operator()<c1 < 0 ? 0 : c1>(pv[1]);
        matrix.template operator()<KS, false>(lb);
        if constexpr (VOL && KS <= 2) drain_store.template operator()<c0>(pv[0]);
        if constexpr (VOL && c1 >= 0) drain_store.template operator()<c1 < 0 ? 0 : c1>(pv[1]);
      }
    } else {
      // loads for the step LOOK ahead (set (GS + LOOK) % NSETS)
      constexpr int GL = GS + LOOK;
      constexpr int ql = GL % NSTEP, segl = GL / NSTEP - SI;
      // (isR is wave-uniform at run time: both tasks are compiled, the branch picks one)
      constexpr Task tlL = l_task<NKS, NP>(ql), tlR = r_task<NKS, NP>(ql);
      if (isR) {
        if constexpr (tlR.has) load(GL % NSETS, wq[segl + tlR.del], tlR.kc);
      } else {
        if constexpr (tlL.has) load(GL % NSETS, wq[segl + tlL.del], tlL.kc);
      }
      // this step's tasks
      constexpr Task sL = l_task<NKS, NP>(q), sR = r_task<NKS, NP>(q);
      if (isR) {
        if constexpr (sR.has) {
          if constexpr (sR.kc == 0) mx = 0.f;
          stage(GS % NSETS, r_dst(it + sR.del, sR.kc), (unsigned)G::RPL, true);
          if constexpr (sR.kc == NKS - 1) publish(it + sR.del);
        }
      } else {
        if constexpr (sL.has) {
          if constexpr (sL.kc == 0) mx = 0.f;
          // the next step's (NP = 2: the next segment's) tile: the other buffer
          stage(GS % NSETS, l_dst(lpar ^ 1), (unsigned)G::LPL, true);
          if constexpr (sL.kc == NKS - 1) publish(it + sL.del);
        }
      }
    }
    if constexpr (!(SMCV_SL_ABLATE & 32)) barrier();
    if constexpr (NP == 1) lpar ^= 1;
  };

  // exact fp32 FMA path for a segment holding a non-finite value or out of the scale range
  auto slow_segment = [&](const Work& k0) __attribute__((always_inline)) {
    if constexpr (FUSE != 0) {  // every disparity of the segment (both passes at once)
      Work kd = k0;
      kd.dp = 0;
      kd.Dp = D;
      slow_softargmin_f32<MEAN>(args, kd, tid, kThreads);
    }
    for (int p = 0; p < NP; ++p) {
      const Work k = pass_of(k0, p);
      if constexpr (VOL) {
        const float mul = MEAN ? args.mul : 1.0f;
        float* out = static_cast<float*>(args.out);
        const float* lrow = L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;
        const float* rrow = R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h;
        for (int idx = tid; idx < k.Dp * kXT; idx += kThreads) {
          const int dl = idx / kXT, x = k.x0 + idx % kXT, d = k.dp + dl;
          if (x >= W) continue;
          float s = 0.f;
          if (x >= d) {
            for (int c = 0; c < args.cpg; ++c)
              s = __builtin_fmaf(lrow[(int64_t)c * ls.c + x], rrow[(int64_t)c * rs.c + x - d], s);
            s *= mul;
          }
          store_one<float>(out + (((int64_t)k.n * D + d) * H + k.y) * W + x, s);
        }
      }
    }
  };

  // ----------------------------------------------------------------------------- main loop
  if (tid < 24) *lds_word(maxw + 4 * tid) = 0u;
  barrier();  // cleared before any wave publishes

  // (Re)start the pipeline at segment `it` (its step 0, body step GS0): the memory waves stage
  // the left tile of step 0 and the whole right window of the segment (every channel step; the
  // pieces of the same row only), then issue the loads of the LOOK steps after it.  A (re)start
  // keeps the published maxima (they are of the raw features); with one channel step it
  // publishes what it stages (nothing before it did).
  auto prologue = [&]<int GS0>() __attribute__((always_inline)) {
    if constexpr (!isC) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const Work k0 = wq[0];
      if (!isR) {
        load(0, k0, 0);
        mx = 0.f;
        stage(0, l_dst(lpar), (unsigned)G::LPL, true);
        if constexpr (NKS == 1) publish(it);
      } else {
        // pieces it - j, j = 0 .. JW (the window's leftmost piece: half 1 only when its first
        // half is outside the window), of this row only
        constexpr int WB = (NP == 1 ? DMAX : 2 * DMAX) / 32;  // window blocks left of x0 (max)
        const int wbl = NP == 1 ? DMAX / 32 : (args.pw + DMAX) / 32;
        const int jw = min((wbl + 3) / 4, s_rel);
        static_assert(WB <= 12, "window");
        // oldest piece first: piece it's max stays in mx for the regular flow, which publishes
        // it (C = 64) after staging the piece's last channel step in the segment's first step
        for (int j = jw; j >= 0; --j) {
          // the piece's first half is in the window iff its blocks 0-1 are: 4 j <= wbl
          const bool h0 = j == 0 || 4 * j <= wbl;
          const bool keep = hh == 1 || h0;
          const Work kj = witem(it - j);
          mx = 0.f;
          for (int kc = 0; kc < NKS; ++kc) {
            load(0, kj, kc);
            stage(0, r_dst(it - j, kc), (unsigned)G::RPL, keep);
          }
          if (NKS == 1 || j > 0) publish(it - j);
        }
        if constexpr (NKS == 1) mx = 0.f;
      }
      // the loads in flight at a step-0 boundary: those of steps 0 .. LOOK - 1
      [&]<int... K_>(std::integer_sequence<int, K_...>) __attribute__((always_inline)) {
        (
            [&]() __attribute__((always_inline)) {
              constexpr int ql = K_ % NSTEP, segl = K_ / NSTEP;
              constexpr Task tL = l_task<NKS, NP>(ql), tR = r_task<NKS, NP>(ql);
              if (isR) {
                if constexpr (tR.has) load((GS0 + K_) % NSETS, wq[segl + tR.del], tR.kc);
              } else {
                if constexpr (tL.has) load((GS0 + K_) % NSETS, wq[segl + tL.del], tL.kc);
              }
            }(),
            ...);
      }(std::make_integer_sequence<int, LOOK>{});
      // (as band_rs: a (re)start may land its loads in other registers than the steady loop,
      // which copies them over at the join, and the compiler's wait placement merges both paths;
      // a compiler-visible vmcnt(0) here leaves nothing pending on this rare path)
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    barrier();
  };
  prologue.template operator()<0>();
  set_prev(pass_of(wq[0], NP - 1), false);
  bool redone = false;

  // the range check of segment `it` on its maxima: 0 valid, 1 exact slow path, 2 restart (with
  // new scale exponents already set)
  auto check = [&]() __attribute__((always_inline)) -> int {
    const float ml = __uint_as_float(*lds_word(maxw + 4u * (unsigned)(it & 7)));
    // the window's right-piece halves: pieces it - j of this row, half 1 of the leftmost when its
    // half 0 is outside
    const int wbl = NP == 1 ? DMAX / 32 : (args.pw + DMAX) / 32;
    float mr = 0.f;
    const int jw = min((wbl + 3) / 4, s_rel);
    for (int j = 0; j <= jw; ++j) {
      const unsigned w2 = maxw + 32u + 8u * (unsigned)((it - j) & 7);
      const bool h0 = j == 0 || 4 * j <= wbl;
      if (h0) mr = fmaxf(mr, __uint_as_float(*lds_word(w2)));
      mr = fmaxf(mr, __uint_as_float(*lds_word(w2 + 4)));
    }
    const bool fin = ml <= 3.4e38f && mr <= 3.4e38f;
    const int el = ml > 0.f ? exp_of(ml) : 0, er = mr > 0.f ? exp_of(mr) : 0;
    const bool okl = ml == 0.f || (el + kL <= 15 && el + kL >= -1);
    const bool okr = mr == 0.f || (er + kR <= 15 && er + kR >= -1);
    if (fin && okl && okr) return 0;
    const int nkl = ml > 0.f ? 13 - el : kL, nkr = mr > 0.f ? 13 - er : kR;
    if (!fin || redone || nkl < -100 || nkl > 100 || nkr < -100 || nkr > 100) return 1;
    kL = nkl;
    kR = nkr;
    return 2;
  };
  auto restart = [&]<int GS0>() __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();  // every wave has read the maxima and the staged planes
    prologue.template operator()<GS0>();
  };

  // Body segment SI: its steps, then its range check; returns true when the workgroup's last
  // segment is done.
  auto segment = [&]<int SI>() __attribute__((always_inline)) -> bool {
    const int lpar0 = lpar;
    bool valid = true;
    if constexpr (CHECK_FIRST) {
      const int r = check();
      if (r == 2) {
        redone = true;
        restart.template operator()<SI * NSTEP>();
      }
      valid = r == 0 || r == 2;
      if (r == 1) slow_segment(wq[0]);
      redone = false;
    }
    for (;;) {
      [&]<int... K_>(std::integer_sequence<int, K_...>) __attribute__((always_inline)) {
        (
            [&]() __attribute__((always_inline)) {
              constexpr int q = K_;
              // a pass ends: its accumulators go into the ring at the next step (set_prev)
              if constexpr (q > 0 && q % NKS == 0) set_prev(pass_of(wq[0], q / NKS - 1), valid);
              step.template operator()<SI * NSTEP + K_>();
            }(),
            ...);
      }(std::make_integer_sequence<int, NSTEP>{});
      if constexpr (!CHECK_FIRST) {
        const int r = check();
        if (r == 2) {
          lpar = lpar0;
          redone = true;
          // the re-run's first step shears this run's accumulators: drop them
          set_prev(pass_of(wq[0], NP - 1), false);
          restart.template operator()<SI * NSTEP>();
          continue;
        }
        valid = r == 0;
        if (r == 1) slow_segment(wq[0]);
        redone = false;
      }
      break;
    }
    set_prev(pass_of(wq[0], NP - 1), valid);
    // clear the maxima sets segment it + 4 will use (their last reader was segment it - 1)
    if (tid < 3) *lds_word(maxw + (tid == 0 ? 4u * (unsigned)((it + 4) & 7)
                                            : 32u + 8u * (unsigned)((it + 4) & 7) + 4u * (unsigned)(tid - 1))) = 0u;
    if constexpr (NP == 2) lpar ^= 1;
    ++it;
    s_rel = s_rel + 1 == args.tiles ? 0 : s_rel + 1;
#pragma unroll
    for (int k = 0; k + 1 < LA; ++k) wq[k] = wq[k + 1];
    wq[LA - 1] = witem(it + LA - 1);
    return it >= nitems;
  };
  [&]() __attribute__((always_inline)) {
    for (;;) {
      bool done = false;
      [&]<int... S_>(std::integer_sequence<int, S_...>) __attribute__((always_inline)) {
        ((done = done || segment.template operator()<S_>()), ...);
      }(std::make_integer_sequence<int, U>{});
      if (done) return;
    }
  }();
  // the last pass: into the ring, then out
  if constexpr (isC) {
    fuse_regs();
    if constexpr (VOL) {
      auto shear_out = [&]<bool SPEC>() __attribute__((always_inline)) {
        f32x4v cv[4];
        [&]<int... K_>(std::integer_sequence<int, K_...>) __attribute__((always_inline)) {
          (
              [&]() __attribute__((always_inline)) {
                constexpr int t = T - 1 - K_;
                constexpr int cr = T - 4 - t;
                if constexpr (cr >= 0) drain_read.template operator()<cr>(cv);
                write_block.template operator()<t, SPEC>();
                if constexpr (cr >= 0) drain_store.template operator()<cr>(cv);
              }(),
              ...);
        }(std::make_integer_sequence<int, T>{});
        drain.template operator()<T - 3>();
        drain.template operator()<T - 2>();
      };
      if (p_special)
        shear_out.template operator()<true>();
      else
        shear_out.template operator()<false>();
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing in flight when the registers die
}

// FUSE 0: the volume; 1: the volume and its soft-argmin; 2: the soft-argmin only
template <bool MEAN, int TMAX, int NKS, int NP, int NSETS, int FUSE>
__global__ __launch_bounds__(slide::kThreads, 1) void band_sl(Args args) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) < slide::kCW) {
#if SMCV_SL_DIAG_ROLE != 2  // (register-usage diagnostics only: 1 compute role alone, 2 memory)
    sl_role<true, MEAN, TMAX, NKS, NP, NSETS, FUSE>(args, smem);
#endif
  } else {
#if SMCV_SL_DIAG_ROLE != 1
    sl_role<false, MEAN, TMAX, NKS, NP, NSETS, FUSE>(args, smem);
#endif
  }
}

template <bool MEAN, int TMAX, int NKS, int NP, int NSETS, int FUSE>
int launch_sl(Args a, int64_t N, hipStream_t st) {
  using G = slide::Geo<TMAX, NKS, NP, FUSE>;
  a.tiles = (int)ceil_div(a.W, kXT);
  const int64_t rows = (int64_t)a.H * N;
  if (rows * a.tiles > INT32_MAX / 64) return fail(SM_EINVAL, "band kernel: too much work for one launch");
  a.nwork = (int)rows;
  a.fd_tiles = make_fastdiv((unsigned)a.tiles);
  a.fd_h = make_fastdiv((unsigned)a.H);
  auto kern = band_sl<MEAN, TMAX, NKS, NP, NSETS, FUSE>;
  static std::atomic<unsigned long long> lds_done{0};
  const int dev = stream_device(st);
  if (int rc = ensure_lds_limit(reinterpret_cast<const void*>(kern), (int)G::SHM, dev, lds_done))
    return rc;
  const int64_t nwg = std::min<int64_t>(rows, (int64_t)device_cus(dev));
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(slide::kThreads), G::SHM, st, a);
  return check_launch("band_sl");
}

// fp32 inner product / correlation volume on the sliding-window kernel; *handled = false when the
// shape is not one it takes: 4-element aligned rows of W >= 4, one channel group, C = 16 NKS with
// NKS in {1, 4}; one D pass of 65..192 disparities, or (C = 16) two passes of pw = 32 m <= 128
// disparities (D = 256: pw = 128) -- the fused pass with the volume kept only for one pass; 32
// disparity planes spanning < 2 GB (the store offsets).
int band_sl_run(const Args& a0, int64_t N, bool mean, bool aligned4, hipStream_t st, bool* handled,
                int fuse) {
  *handled = false;
  Args a = a0;
  const int nks = a.cpg / 16;
  if (!aligned4 || a.G != 1 || a.W < 4 || a.cpg % 16 != 0 || (nks != 1 && nks != 4) ||
      (int64_t)a.H * a.W * 4 * 32 >= ((int64_t)1 << 31))
    return SM_OK;
  int np = 1;
  if (a.npass == 1) {
    if (a.pw <= 64 || a.pw > 192) return SM_OK;
  } else {
    // two passes of a 32-multiple width <= 128 (C = 16, no volume + disparity)
    const int pw2 = (int)((ceil_div(a.D, 2) + 31) / 32 * 32);
    if (nks != 1 || a.D > 256 || a.D <= 192 || pw2 > 128 || fuse == 1) return SM_OK;
    a.npass = 2;
    a.pw = pw2;
    np = 2;
  }
  // the mean with the volume kept, one channel step, D > 128: its compute wave would spill.  Its
  // volume-free call stays off band_sl too: that pair (band_h2db with the volume, band_rs without)
  // folds the scaled cells and returns one disparity bit for bit (band_sl folds with FoldF32)
  if (mean && nks == 1 && a.pw > 128 && np == 1) return SM_OK;
  *handled = true;
  auto go = [&](auto tm, auto nk, auto npc) {
    constexpr int TM = decltype(tm)::value, NK = decltype(nk)::value, NPC = decltype(npc)::value;
    constexpr int NS = NK == 1 ? 2 : SMCV_SL_SETS;
    auto f = [&](auto fc) {
      constexpr int FU = decltype(fc)::value;
      if constexpr (FU == 1 && NPC == 2) {
        return (int)SM_EUNSUPPORTED;  // (excluded above)
      } else if constexpr (NK == 1 && TM == 7 && NPC == 1) {
        // the mean at C = 16 with one pass of > 128 disparities is excluded above (its volume-kept
        // compute wave would spill; its volume-free call pairs with band_h2db's): not compiled
        if (mean) return fail(SM_EINVAL, "band_sl: unhandled mean shape");
        return launch_sl<false, TM, NK, NPC, NS, FU>(a, N, st);
      } else {
        return mean ? launch_sl<true, TM, NK, NPC, NS, FU>(a, N, st)
                    : launch_sl<false, TM, NK, NPC, NS, FU>(a, N, st);
      }
    };
    return fuse == 2   ? f(std::integral_constant<int, 2>{})
           : fuse == 1 ? f(std::integral_constant<int, 1>{})
                       : f(std::integral_constant<int, 0>{});
  };
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I4 = std::integral_constant<int, 4>;
  using T5 = std::integral_constant<int, 5>;
  using T7 = std::integral_constant<int, 7>;
  if (np == 2) return go(T5{}, I1{}, I2{});
  if (a.pw <= 128) return nks == 1 ? go(T5{}, I1{}, I1{}) : go(T5{}, I4{}, I1{});
  return nks == 1 ? go(T7{}, I1{}, I1{}) : go(T7{}, I4{}, I1{});
}

}  // namespace h2band
}  // namespace smcv

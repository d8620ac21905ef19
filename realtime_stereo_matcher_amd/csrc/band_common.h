// Helpers shared by the band cost-volume kernels (ip_h2.hip: band_h2; ip_h2db.hip: band_h2db;
// ip_rs.hip: band_rs; ip_sl.hip: band_sl):
// operand typedefs, the plane swizzle, the work decomposition, LDS accessors, the hand-counted
// feature loads and their vmcnt wait, the output stores and the fp32 two-plane split.
#pragma once

#include "common.h"

#include <math.h>

#include <type_traits>

#ifndef SMCV_NT_STORE
#define SMCV_NT_STORE 1  // volume stores non-temporal (0: plain, for A/B)
#endif

#ifndef SMCV_ABLATE
#define SMCV_ABLATE 0  // diagnostics only (scripts/ip_stamps.hip): 1 no MFMA, 2 all feature
#endif                 // loads from one line, 4 no stores, 8 no epilogue, 16 no staging
                       // (planes not written), 32 no shear (accumulators stored unsheared)
#ifndef SMCV_PREFETCH
#define SMCV_PREFETCH 0  // L2 touches two steps ahead (1: on; measured slower on cfg2, r01)
#endif

namespace smcv {
namespace h2band {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 hp2 __attribute__((ext_vector_type(2)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int kXT = 128;  // left pixels per row segment (both band kernels)
constexpr int kPF = SMCV_PREFETCH ? 1 : 0;  // touch instructions issued after each step's loads

// byte offset of (plane row r, 8-channel chunk h).  Fragment reads: lane l -> row base + (l & 31),
// chunk l >> 5; plane writes: 8 consecutive lanes -> rows 4i + p of one 32-row block.  Both are
// conflict-free under the gfx950 ds_read_b128 / ds_write_b128 lane groups (scripts/check_swizzle.py).
__device__ __forceinline__ int swz(int r, int h) {
  return ((r ^ ((r >> 2) & 3)) << 5) + ((h ^ ((r >> 4) & 1)) << 4);
}

// n / d for 32-bit n by one 64-bit high multiply: m = floor(2^64 / d) + 1 is exact for every
// n < 2^32 (the error n e / 2^64 < 2^-32 stays below 1 / d); m = 0 marks d = 1.
struct FastDiv {
  unsigned long long m;
  unsigned d;
};
inline FastDiv make_fastdiv(unsigned d) { return {d == 1 ? 0ull : ~0ull / d + 1, d}; }
__device__ __forceinline__ unsigned fdiv(unsigned n, const FastDiv& f) {
  return f.m ? (unsigned)__umul64hi((unsigned long long)n, f.m) : n;
}

struct Args {
  const void* L;
  const void* R;
  void* out;    // volume; nullptr: not stored (fused kernel only)
  float* disp;  // fused kernel: (N, H, W) disparities
  int C, cpg, G, H, W, D;
  Strides4 ls, rs;
  int tiles, npass, pw, nwork;
  float mul;  // MEAN: 1 / (channels averaged)
  int round;  // fused pass of fp16 / bf16 features: regress the cells rounded to the feature dtype
  // volume-free fused kernel with npass > 1: each pass's partial soft-argmin state per pixel
  // (max, sum e, sum d e relative to that max), merged by fused_merge_kernel
  double* ws_s;
  double* ws_t;
  float* ws_m;
  int64_t nhw;  // N H W: the workspace's per-pass stride
  // the decode's divisors (npass, tiles, G, H) as multiplies (band_rs, set by its launcher)
  FastDiv fd_np, fd_tiles, fd_g, fd_h;
};

struct Work {
  int n, y, g, x0, dp, Dp, js, pass;
};

// decode() with the divisions as multiplies (Args::fd_*)
__device__ __forceinline__ Work decode_fd(unsigned w, const Args& a, int dmax) {
  Work k;
  const unsigned r1 = fdiv(w, a.fd_np);
  k.pass = (int)(w - r1 * (unsigned)a.npass);
  const unsigned r2 = fdiv(r1, a.fd_tiles);
  const int tile = (int)(r1 - r2 * (unsigned)a.tiles);
  const unsigned row = fdiv(r2, a.fd_g);
  k.g = (int)(r2 - row * (unsigned)a.G);
  const unsigned nn = fdiv(row, a.fd_h);
  k.y = (int)(row - nn * (unsigned)a.H);
  k.n = (int)nn;
  k.x0 = tile * kXT;
  k.dp = k.pass * a.pw;
  k.Dp = min(a.pw, a.D - k.dp);
  k.js = k.x0 - k.dp - dmax;
  return k;
}

// work index w = (((n H + y) G + g) tiles + tile) npass + pass: consecutive items are
// neighbouring segments of one row (and group), which share right-window columns in L2
__device__ __forceinline__ Work decode(int w, const Args& a, int dmax) {
  Work k;
  const int pass = w % a.npass;
  const int r1 = w / a.npass;
  const int tile = r1 % a.tiles;
  const int r2 = r1 / a.tiles;
  k.g = r2 % a.G;
  const int row = r2 / a.G;
  k.y = row % a.H;
  k.n = row / a.H;
  k.x0 = tile * kXT;
  k.dp = pass * a.pw;
  k.pass = pass;
  k.Dp = min(a.pw, a.D - k.dp);
  k.js = k.x0 - k.dp - dmax;
  return k;
}

typedef __attribute__((address_space(3))) unsigned char lds_u8;
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const lds_u8*)p;
}
__device__ __forceinline__ void lds_store1(unsigned addr, float v) {
  *reinterpret_cast<__attribute__((address_space(3))) float*>(addr) = v;
}
__device__ __forceinline__ float lds_load1(unsigned addr) {
  return *reinterpret_cast<__attribute__((address_space(3))) float*>(addr);
}
__device__ __forceinline__ f32x4v lds_load4(unsigned addr) {
  return *reinterpret_cast<__attribute__((address_space(3))) f32x4v*>(addr);
}
__device__ __forceinline__ __attribute__((address_space(3))) unsigned* lds_word(unsigned addr) {
  return reinterpret_cast<__attribute__((address_space(3))) unsigned*>(addr);
}

// a 4-pixel group of one channel row in registers: 16 B (fp32) or 8 B (fp16 / bf16)
template <typename T> struct Quad { using type = u32x2; };
template <> struct Quad<float> { using type = f32x4v; };

// Feature loads are issued by inline asm so that the compiler neither waits for them itself
// (its control-flow merges would put vmcnt(0) -- a wait for every output store in flight --
// in front of every step) nor knows them: the kernel counts vmcnt by hand (vm_wait).
template <bool ASM, typename QT>
__device__ __forceinline__ void gload(QT& v, const void* p) {
  if constexpr (!ASM) {  // compiler-tracked (the fused kernels: see band_h2)
    typedef __attribute__((address_space(1))) const void gcvoid;
    v = *reinterpret_cast<__attribute__((address_space(1))) const QT*>((gcvoid*)p);
  } else if constexpr (sizeof(QT) == 16) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  } else {
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  }
}

// Wait for the feature loads: vmcnt(N + NPF) when N output stores were issued after them (they
// may stay in flight, as may the NPF touches issued right after the loads), else vmcnt(NPF).
// One asm statement with the scalar branch inside, and the loaded registers (and the touch
// destination) as tied operands: no use of them is scheduled before the wait, and the register
// allocator has a single place (the load's destination) to keep them.
template <int N, int NPF, bool ASM = true, typename QT>
__device__ __forceinline__ void vm_wait(QT (&v)[8], unsigned& pf, int after_stores) {
  if constexpr (!ASM) return;  // compiler-tracked loads: the compiler places the waits
  asm volatile(
      "s_cmp_eq_u32 %9, 0\n\t"
      "s_cbranch_scc1 .Lvm_all%=\n\t"
      "s_waitcnt vmcnt(%10)\n\t"
      "s_branch .Lvm_done%=\n"
      ".Lvm_all%=:\n\t"
      "s_waitcnt vmcnt(%11)\n"
      ".Lvm_done%=:"
      : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
        "+v"(v[7]), "+v"(pf)
      : "s"(after_stores), "n"(N + NPF), "n"(NPF)
      : "memory", "scc");
}

// 4 fp32 results -> storage type (round to nearest even; NaN stays NaN, overflow gives inf).
// Global address space explicitly: a flat store would count in vmcnt out of order.
// NT (compile time, so each instantiation holds ONE kind of store: an if / else of a
// non-temporal and a plain store to one address is merged by the compiler into a plain store,
// dropping the non-temporal hint -- that silently happened to every fp32 volume store in r02):
//   true: non-temporal -- the volume is written once and never re-read by this kernel; plain
//         stores allocate its lines in L2 and evict the feature lines the loads reuse
//         (scripts/micro/mlp_patterns.hip: cfg2 reads + writes 140 us plain vs 106 us nt);
//   false: plain -- fp32 rows with W % 4 != 0, whose 128-B row pieces straddle two lines: L2
//         merges the two halves of a line before it writes the line back.
template <bool NT, typename T>
__device__ __forceinline__ void store_quad(T* p, f32x4v v) {
  typedef __attribute__((address_space(1))) void gvoid;
  gvoid* g = (gvoid*)p;
  if constexpr (sizeof(T) == 4) {
    if constexpr (SMCV_NT_STORE && NT)
      __builtin_nontemporal_store(v, reinterpret_cast<__attribute__((address_space(1))) f32x4v*>(g));
    else
      *reinterpret_cast<__attribute__((address_space(1))) f32x4v*>(g) = v;
  } else if constexpr (std::is_same<T, __half>::value) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const h4 r = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
    if constexpr (SMCV_NT_STORE && NT)
      __builtin_nontemporal_store(r, reinterpret_cast<__attribute__((address_space(1))) h4*>(g));
    else
      *reinterpret_cast<__attribute__((address_space(1))) h4*>(g) = r;
  } else {
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    const b4 r = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    if constexpr (SMCV_NT_STORE && NT)
      __builtin_nontemporal_store(r, reinterpret_cast<__attribute__((address_space(1))) b4*>(g));
    else
      *reinterpret_cast<__attribute__((address_space(1))) b4*>(g) = r;
  }
}
template <typename T>
__device__ __forceinline__ void store_one(T* p, float v) {
  typedef __attribute__((address_space(1))) void gvoid;
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<__attribute__((address_space(1))) float*>((gvoid*)p) = v;
  } else {
    const T h = (T)v;
    *reinterpret_cast<__attribute__((address_space(1))) unsigned short*>((gvoid*)p) =
        __builtin_bit_cast(unsigned short, h);
  }
}

template <typename T>
__device__ __forceinline__ float ld1(const T* p) { return (float)*p; }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// The fp32 split of two values x (channels 2q, 2q+1 of one pixel), scaled by sc = 2^k (exact):
// h = rn16(x sc) and m = rn16(x sc - h), packed as (lo, hi) fp16 pairs.  Four v_fma_mix*, i.e.
// two VALU per value (the compiler's cvt / cvt-back / subtract / pack sequence took four): the
// mix forms evaluate x * sc - h exactly (x sc is exact, and h is its rounding, so the difference
// is an fp32 number) and round it to fp16 once -- bit-identical to that sequence.
__device__ __forceinline__ void split_pair(float a, float b, float sc, unsigned& h, unsigned& m) {
  asm("v_fma_mixlo_f16 %0, %2, %4, 0\n\t"
      "v_fma_mixhi_f16 %0, %3, %4, 0\n\t"
      "v_fma_mixlo_f16 %1, %2, %4, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %1, %3, %4, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h), "=&v"(m)
      : "v"(a), "v"(b), "v"(sc));
}

// split_pair for four pairs at once (one pixel's 8 channels -> 16 B of h, 16 B of m), ordered
// for instruction-level parallelism: each write depends on one issued four instructions earlier
// (split_pair's four are one dependent chain, which a lone wave on its SIMD waits out).
__device__ __forceinline__ void split_quad(const float (&x)[8], float sc, uint4& h, uint4& m) {
  asm("v_fma_mixlo_f16 %0, %8, %16, 0\n\t"
      "v_fma_mixlo_f16 %1, %10, %16, 0\n\t"
      "v_fma_mixlo_f16 %2, %12, %16, 0\n\t"
      "v_fma_mixlo_f16 %3, %14, %16, 0\n\t"
      "v_fma_mixhi_f16 %0, %9, %16, 0\n\t"
      "v_fma_mixhi_f16 %1, %11, %16, 0\n\t"
      "v_fma_mixhi_f16 %2, %13, %16, 0\n\t"
      "v_fma_mixhi_f16 %3, %15, %16, 0\n\t"
      "v_fma_mixlo_f16 %4, %8, %16, -%0 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %5, %10, %16, -%1 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %6, %12, %16, -%2 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixlo_f16 %7, %14, %16, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %4, %9, %16, -%0 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %5, %11, %16, -%1 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %6, %13, %16, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %7, %15, %16, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(h.x), "=&v"(h.y), "=&v"(h.z), "=&v"(h.w), "=&v"(m.x), "=&v"(m.y), "=&v"(m.z),
        "=&v"(m.w)
      : "v"(x[0]), "v"(x[1]), "v"(x[2]), "v"(x[3]), "v"(x[4]), "v"(x[5]), "v"(x[6]), "v"(x[7]),
        "v"(sc));
}

// exponent e with x = f 2^e, f in [0.5, 1) (x > 0 finite)
__device__ __forceinline__ int exp_of(float x) { return __builtin_amdgcn_frexp_expf(x); }

// The persistent grid's schedule (band_h2, band_h2db, band_rs).  Workgroups b and b+8 share an
// XCD, and each XCD group walks a contiguous range of row segments, so neighbouring segments of
// a row run on one XCD at the same time and share its L2 for the right window.  Item i of a
// workgroup is segment j = gi + (i / npass) gsz of its group's range, pass i % npass: the D
// passes of a segment are consecutive items of one workgroup, so the second pass's feature
// loads find the lines the first one fetched in L2 (concurrent passes on different workgroups
// drift apart and miss: cfg4 fetched its features 1.95x in round 2).  With gsz % 8 == 0 every
// workgroup would keep one tile index (j % 8) for the whole launch, so the workgroups of the
// 64-pixel last tile of a 960-pixel row would idle half the time; rotating each complete
// aligned 8-segment block by the round spreads the short tiles over all workgroups (the set
// of segments in flight per round, and so the L2 sharing, is unchanged).
#ifndef SMCV_SCHED_PHASE
#define SMCV_SCHED_PHASE 0
#endif
#ifndef SMCV_FOLD_FMA
#define SMCV_FOLD_FMA 1  // band_sl's fused fold: 1/C and 2^kk folded into the exponent's FMA (0:
#endif                   // the cells scaled one by one; cfg4 volume-free 5 % slower, r05)
#ifndef SMCV_FOLD_PK
#define SMCV_FOLD_PK 1  // FoldFma's (band_sl's) per-cell exponent, sum and weighted sum as packed
#endif                  // fp32 pairs (v_pk_fma_f32 / v_pk_mul_f32 / v_pk_add_f32): cfg4 volume-free
                        // -9 %, cfg2 -4 %, volume kept flat (profiles/r06/ab/r6w_*, round 6)
#ifndef SMCV_SCHED_IL
#define SMCV_SCHED_IL 0  // diagnostic: chunks of IL segments dealt round-robin to the XCD groups
#endif                   // instead of one contiguous range each (IL a multiple of 8)
struct Sched {
  int gi, gsz, sbeg, scnt, nitems, npass, phase;
  bool rot, none;
  __device__ __forceinline__ Sched(int nwork, int np) {
    const int grp = blockIdx.x & 7;
    gi = blockIdx.x >> 3;
    gsz = gridDim.x >> 3;
    npass = np;
    const int nseg = nwork / np;
    const int q = nseg >> 3, rr = nseg & 7;
    sbeg = grp < rr ? grp * (q + 1) : rr * (q + 1) + (grp - rr) * q;
    scnt = q + (grp < rr ? 1 : 0);
    if constexpr (SMCV_SCHED_IL > 0) {
      const int nch = (nseg + SMCV_SCHED_IL - 1) / SMCV_SCHED_IL;
      const int mine = nch > grp ? (nch - grp + 7) / 8 : 0;
      const int last = nseg - (nch - 1) * SMCV_SCHED_IL;  // the last chunk's segments
      sbeg = grp;
      scnt = mine * SMCV_SCHED_IL - (((nch - 1) & 7) == grp ? SMCV_SCHED_IL - last : 0);
    }
    none = gi >= scnt;  // the whole workgroup leaves together
    nitems = none ? 0 : ((scnt - gi + gsz - 1) / gsz) * np;
    rot = (gsz & 7) == 0;
    // diagnostic: start each XCD's walk at a different point of its range (a rotation, so every
    // segment is still taken once), so the eight XCDs' streams are not a fixed stride apart
    phase = SMCV_SCHED_PHASE == 0 ? 0 : (int)(((long long)scnt * grp / (8 * SMCV_SCHED_PHASE)) & ~7);
  }
  __device__ __forceinline__ int seg_of(int local) const {
    if constexpr (SMCV_SCHED_IL > 0)  // sbeg = the group: chunk local / IL is global chunk grp + 8 (local / IL)
      return (sbeg + 8 * (local / SMCV_SCHED_IL)) * SMCV_SCHED_IL + local % SMCV_SCHED_IL;
    return sbeg + local;
  }
  __device__ __forceinline__ int rotate(int local) const {
    if (SMCV_SCHED_PHASE == 0) return local;
    local += phase;
    return local >= scnt ? local - scnt : local;
  }
  __device__ __forceinline__ int item_fd(int i, const FastDiv& fnp) const {
    const int si = (int)fdiv((unsigned)i, fnp);
    const int p = i - si * npass;
    const int j = gi + si * gsz;
    const int b = j & ~7;
    const int seg = seg_of(rotate((rot && b + 8 <= scnt) ? (b | ((j + si) & 7)) : j));
    return seg * npass + p;
  }
  __device__ __forceinline__ int item(int i) const {
    const int si = npass == 1 ? i : i / npass;
    const int p = i - si * npass;
    const int j = gi + si * gsz;
    const int b = j & ~7;
    const int seg = seg_of(rotate((rot && b + 8 <= scnt) ? (b | ((j + si) & 7)) : j));
    return seg * npass + p;
  }
};

// The fused pass's exact fp32 path for a segment the band cannot take (a non-finite value, a
// scale fp32 cannot reach): each pixel's cells by fp32 FMA over the channels, folded online into
// the soft-argmin in fp64 (band_rs; band_h2 keeps its own copy).  Several D passes
// (args.ws_m): the pass's partial state, d global; a NaN cell or a +inf maximum is carried as
// s = NaN, which fused_merge_kernel propagates; an all -inf pass contributes nothing.
template <bool MEAN>
__device__ __forceinline__ void slow_softargmin_f32(const Args& args, const Work& k, int tid,
                                                    int nthreads) {
  const float mul = MEAN ? args.mul : 1.0f;
  const float* lrow = static_cast<const float*>(args.L) + (int64_t)k.n * args.ls.n +
                      (int64_t)k.y * args.ls.h;
  const float* rrow = static_cast<const float*>(args.R) + (int64_t)k.n * args.rs.n +
                      (int64_t)k.y * args.rs.h;
  for (int xx = tid; xx < kXT; xx += nthreads) {
    const int x = k.x0 + xx;
    if (x >= args.W) continue;
    float m = -INFINITY;
    double s = 0.0, t = 0.0;  // relative to m; t over the pass-local d
    bool nan = false;
    for (int d = 0; d < k.Dp; ++d) {
      const int dg = k.dp + d;
      float v = 0.f;
      if (x >= dg) {
        for (int c = 0; c < args.cpg; ++c)
          v = __builtin_fmaf(lrow[(int64_t)c * args.ls.c + x], rrow[(int64_t)c * args.rs.c + x - dg], v);
        v *= mul;
      }
      nan |= v != v;
      if (v > m) {
        const double f = m == -INFINITY ? 0.0 : (double)expf(m - v);
        s *= f;
        t *= f;
        m = v;
      }
      if (m != INFINITY && m != -INFINITY) {
        const double e = (double)expf(v - m);
        s += e;
        t += (double)d * e;
      }
    }
    const size_t px = ((size_t)k.n * args.H + k.y) * args.W + x;
    if (args.ws_m != nullptr) {
      typedef __attribute__((address_space(1))) void gvoid;
      const size_t o = (size_t)k.pass * ((size_t)args.nhw) + px;
      const double sv = (nan || m == INFINITY) ? (double)NAN : s;
      *reinterpret_cast<__attribute__((address_space(1))) double*>((gvoid*)(args.ws_s + o)) = sv;
      *reinterpret_cast<__attribute__((address_space(1))) double*>((gvoid*)(args.ws_t + o)) =
          t + (double)k.dp * sv;
      store_one<float>(args.ws_m + o, m);
    } else {
      store_one<float>(args.disp + px, (nan || m == INFINITY || m == -INFINITY) ? NAN : (float)(t / s));
    }
  }
}

// One block of the fused soft-argmin fold (shared by every fused path, so a fold split between
// waves performs the same arithmetic in the same order as one wave's): lane (lr, hh) holds, for
// pixel x0 + 32 wave + lr, the cells of local disparity dl = 32 (T-1-t) + u - c_i (block t,
// element i, u = lr - 4 hh).  The block's maximum, the running sums (m, s = sum e, tt = sum dl e,
// relative to m) rescaled when it grows, the block's exps summed in fp32 and carried into fp64.
// Cells outside 0 <= dl < Dp enter as -inf (e = 0): the first and the last block always, the
// middle ones when Dp < DMAX.  No NaN / inf flags: a NaN cell makes its e NaN, a +inf maximum
// makes (inf - inf) NaN, an all -inf pixel gives 0 / 0 -- torch's NaN each time.  The shift
// max(m, -FLT_MAX) keeps exp2 finite-argument when no cell is finite yet.  SCALE multiplies back
// by 2^-(kL+kR); XLT forces the cells x < d (R pad rows) to 0, as the volume has them; RT (not
// float): the cell rounded to RT first.
// RT = FoldFma: the fp32 cells with 1/C and 2^kk folded into the exponent's FMA (the cells stay
// raw; their block maximum is scaled once, K > 0 keeps it the maximum): e = 2^(fma(x, K, -sh)
// log2 e), two operations per cell instead of the scale, subtract and multiply.  A kernel pair
// whose volume-kept and volume-free calls must agree bit for bit uses the same RT.  SMCV_FOLD_PK:
// FoldFma folds the cells in packed fp32 pairs (even / odd partial sums).
struct FoldFma {};
using FoldF32 = std::conditional<SMCV_FOLD_FMA != 0, FoldFma, float>::type;

template <int TMAX, bool MEAN, bool SCALE, bool XLT, typename RT, int t>
__device__ __forceinline__ void fold_block(const f32x16& blk, const Args& args, const Work& k,
                                           int kL, int kR, int wave, int lr, int hh, float& m,
                                           double& s, double& tt) {
  constexpr int DMAX = 32 * (TMAX - 1);
  constexpr float kL2E = 1.4426950408889634f;
  const float mul = args.mul;
  const int kk = -(kL + kR);
  const int jlane = k.js + 32 * wave + 4 * hh;
  auto body = [&](auto maskc) __attribute__((always_inline)) {
    int ub = lr - 4 * hh + 32 * (TMAX - 1 - t);  // dl = ub - c_i; opaque per block (not hoisted)
    asm volatile("" : "+v"(ub));
    float v[16];
    float bm = -INFINITY;
    if constexpr (std::is_same<RT, FoldFma>::value) {
      // the mean's 1/C and the scale 2^kk folded into the exponent's FMA: the cells stay raw,
      // their maximum is scaled once (K > 0: monotonic), e = 2^((x K - max) log2 e)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ci = (i & 3) + 8 * (i >> 2);
        float x = blk[i];
        if constexpr (XLT) x = jlane + 32 * t + ci >= 0 ? x : 0.f;
        if constexpr (decltype(maskc)::value) x = (unsigned)(ub - ci) < (unsigned)k.Dp ? x : -INFINITY;
        v[i] = x;
        bm = fmaxf(bm, x);
      }
      float K = MEAN ? mul : 1.f;
      if constexpr (SCALE) K = __builtin_ldexpf(K, kk);
      const float nm = fmaxf(m, bm * K);
      const float sh = fmaxf(nm, -3.402823466e38f);
      const float f = __builtin_amdgcn_exp2f((m - sh) * kL2E);
      // e = 2^((x K - sh) log2 e) with x K - sh formed by one FMA (exact product, one rounding),
      // then scaled: the exponent's error is relative to x K - sh, not to |x K|.  (Round 5's
      // one-FMA form x (K log2 e) - sh log2 e carried an error of 2^-24 |sh| log2 e: fine for
      // cells of O(10), but cells of 1e30 lost the maximum's own weight, NaN, and the shift
      // needed a clamp at 2e38)  No clamp: x K - sh <= 0 when K is a power of two
      // (the sum, the mean over 2^k channels, the 2^kk scales: bm K exact), and a result below
      // -FLT_MAX rounds to -inf, e = 0.  For other K, sh = bm K rounded can sit half an ulp below
      // the maximum cell's product, whose exponent is then that residual (<= 2^-25 |sh|): it
      // overflows exp2 only for |sh| > 2^32.
      const float nsh = -sh;
#if SMCV_FOLD_PK
      // cells (2j, 2j+1) as one packed pair: the same per-cell arithmetic, two partial sums per
      // lane (even and odd cells) added at the end
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      const f32x2 K2 = {K, K}, N2 = {nsh, nsh}, L2 = {kL2E, kL2E};
      f32x2 ps2 = {0.f, 0.f}, pc2 = {0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        const f32x2 x2 = {v[i], v[i + 1]};
        const f32x2 y2 = __builtin_elementwise_fma(x2, K2, N2) * L2;
        const f32x2 e2 = {__builtin_amdgcn_exp2f(y2.x), __builtin_amdgcn_exp2f(y2.y)};
        const f32x2 c2 = {(float)((i & 3) + 8 * (i >> 2)), (float)(((i + 1) & 3) + 8 * (i >> 2))};
        ps2 += e2;
        pc2 = __builtin_elementwise_fma(c2, e2, pc2);
      }
      const float ps = ps2.x + ps2.y, pc = pc2.x + pc2.y;
#else
      float ps = 0.f, pc = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float e = __builtin_amdgcn_exp2f(fmaf(v[i], K, nsh) * kL2E);
        ps += e;
        pc = fmaf((float)((i & 3) + 8 * (i >> 2)), e, pc);
      }
#endif
      s = s * (double)f + (double)ps;
      tt = tt * (double)f + (double)ub * (double)ps - (double)pc;
      m = nm;
      __builtin_amdgcn_sched_barrier(0);
    } else {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ci = (i & 3) + 8 * (i >> 2);
      float x = blk[i];
      if (MEAN) x *= mul;
      if constexpr (SCALE) x = __builtin_ldexpf(x, kk);
      if constexpr (XLT) x = jlane + 32 * t + ci >= 0 ? x : 0.f;
      if constexpr (!std::is_same<RT, float>::value) x = (float)(RT)x;
      if constexpr (decltype(maskc)::value) x = (unsigned)(ub - ci) < (unsigned)k.Dp ? x : -INFINITY;
      v[i] = x;
      bm = fmaxf(bm, x);
    }
    const float nm = fmaxf(m, bm);
    const float sh = fmaxf(nm, -3.402823466e38f);
    const float f = __builtin_amdgcn_exp2f((m - sh) * kL2E);
    // (scalar also under SMCV_FOLD_PK: packed, band_h2's fp16 volume-free pass measured 0.7 %
    // slower, profiles/r06/ab/r6w_*, and band_rs / band_h2db FUSE 1 spill with the pairs)
    float ps = 0.f, pc = 0.f;  // sum e, sum c_i e
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float e = __builtin_amdgcn_exp2f((v[i] - sh) * kL2E);
      ps += e;
      pc = fmaf((float)((i & 3) + 8 * (i >> 2)), e, pc);
    }
    s = s * (double)f + (double)ps;
    tt = tt * (double)f + (double)ub * (double)ps - (double)pc;  // sum (ub - c_i) e
    m = nm;
    __builtin_amdgcn_sched_barrier(0);
    }
  };
  // the first and the last block always straddle the band's ends; the middle ones only when
  // Dp < DMAX (a uniform branch: the common full-D item runs them unmasked)
  if constexpr (t == 0 || t == TMAX - 1)
    body(std::true_type{});
  else if (k.Dp == DMAX)
    body(std::false_type{});
  else
    body(std::true_type{});
}

// Blocks [B0, B1) of a wave's accumulators folded into (m, s, tt).
template <int TMAX, bool MEAN, bool SCALE, bool XLT, typename RT, int B0, int B1>
__device__ __forceinline__ void fold_blocks(const f32x16* blk, const Args& args, const Work& k,
                                            int kL, int kR, int wave, int lr, int hh, float& m,
                                            double& s, double& tt) {
  [&]<int... T_>(std::integer_sequence<int, T_...>) __attribute__((always_inline)) {
    (fold_block<TMAX, MEAN, SCALE, XLT, RT, B0 + T_>(blk[T_], args, k, kL, kR, wave, lr, hh, m, s, tt), ...);
  }(std::make_integer_sequence<int, B1 - B0>{});
}

// The lane pair's merge: (lr, 0) and (lr, 1) hold the two row halves of the pixel; after it both
// hold M and the sums relative to M.
__device__ __forceinline__ void fold_pair_merge(float m, double& s, double& tt, float& M) {
  constexpr float kL2E = 1.4426950408889634f;
  M = fmaxf(m, __shfl_xor(m, 32));
  const double g = (double)__builtin_amdgcn_exp2f((m - fmaxf(M, -3.402823466e38f)) * kL2E);
  s *= g;
  tt *= g;
  s += __shfl_xor(s, 32);
  tt += __shfl_xor(tt, 32);
}

// Soft-argmin straight from a wave's band accumulators (the fused pass, f-1): every block folded
// (fold_block), the pair merged by one shuffle; lane hh = 0 stores the disparity (one pass) or the
// pass's partial state (several D passes, args.ws_m).  WS: the partial-state form exists (several
// D passes); without it only the disparity store is compiled.
template <int TMAX, bool MEAN, bool SCALE, bool XLT, bool WS = true, typename RT = float>
__device__ __forceinline__ void fused_softargmin(const f32x16 (&acc)[TMAX], const Args& args,
                                                 const Work& k, int kL, int kR, int wave, int lr,
                                                 int hh) {
  float m = -INFINITY;
  double s = 0.0, tt = 0.0;
  fold_blocks<TMAX, MEAN, SCALE, XLT, RT, 0, TMAX>(acc, args, k, kL, kR, wave, lr, hh, m, s, tt);
  float M;
  fold_pair_merge(m, s, tt, M);
  const int x = k.x0 + 32 * wave + lr;
  if (hh == 0 && x < args.W) {
    const size_t px = ((size_t)k.n * args.H + k.y) * args.W + x;
    if (WS && args.ws_m != nullptr) {  // one of several D passes: its partial state, d global
      typedef __attribute__((address_space(1))) void gvoid;
      const size_t o = (size_t)k.pass * ((size_t)args.nhw) + px;
      *reinterpret_cast<__attribute__((address_space(1))) double*>((gvoid*)(args.ws_s + o)) = s;
      *reinterpret_cast<__attribute__((address_space(1))) double*>((gvoid*)(args.ws_t + o)) =
          tt + (double)k.dp * s;
      store_one<float>(args.ws_m + o, M);
    } else {
      store_one<float>(args.disp + px, (float)(tt / s));
    }
  }
}

// fused_softargmin's fold without the store: the lane pair's merged state of one D pass -- the
// maximum M, s = sum e and t = sum d e relative to M with d GLOBAL (t + dp s) -- in both lanes of
// the pair (band_sl: the two passes of a segment run back to back on one wave, so pass 0's state
// waits in registers for pass 1 instead of going through a workspace).
template <int TMAX, bool MEAN, bool SCALE, bool XLT, typename RT = float>
__device__ __forceinline__ void fused_softargmin_state(const f32x16 (&acc)[TMAX], const Args& args,
                                                       const Work& k, int kL, int kR, int wave,
                                                       int lr, int hh, float& Mo, double& so,
                                                       double& to) {
  float m = -INFINITY;
  double s = 0.0, tt = 0.0;
  fold_blocks<TMAX, MEAN, SCALE, XLT, RT, 0, TMAX>(acc, args, k, kL, kR, wave, lr, hh, m, s, tt);
  fold_pair_merge(m, s, tt, Mo);
  so = s;
  to = tt + (double)k.dp * s;
}

// The two passes' states merged (fused_merge_kernel's arithmetic) and the disparity stored by
// lane hh = 0 of the pair.
__device__ __forceinline__ void fused_two_pass_store(const Args& args, const Work& k, int wave,
                                                     int lr, int hh, float m0, double s0,
                                                     double t0, float m1, double s1, double t1) {
  constexpr float kL2E = 1.4426950408889634f;
  const float M = fmaxf(m0, m1);
  const float sh = fmaxf(M, -3.402823466e38f);
  const double g0 = (double)__builtin_amdgcn_exp2f((m0 - sh) * kL2E);
  const double g1 = (double)__builtin_amdgcn_exp2f((m1 - sh) * kL2E);
  const double s = s0 * g0 + s1 * g1;
  const double t = t0 * g0 + t1 * g1;
  const int x = k.x0 + 32 * wave + lr;
  if (hh == 0 && x < args.W) {
    const size_t px = ((size_t)k.n * args.H + k.y) * args.W + x;
    store_one<float>(args.disp + px, (float)(t / s));
  }
}

}  // namespace h2band
}  // namespace smcv

// Band cost volumes on gfx950 matrix cores, warp-specialised ("ws" kernels): inner product /
// correlation (N, D, H, W), groupwise (N, G, H, W, D), and the inner product / correlation fused
// with soft-argmin.
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//            TorchGroupwiseCost.forward      cost_volume/groupwise.py:24-56 (mean per group, D last)
//            disparity_regression            model/mobile_disp_net_c.py:208-220 (fused variant)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// Per image row the volume is a band of the contraction S[j][x] = sum_c R[c][j] L[c][x]
// (d = x - j).  One workgroup per CU (persistent grid) owns a sequence of 128-pixel row
// segments ("items") of one channel group and splits its 8 waves into two roles:
//   * 4 staging waves keep the next two 16-channel stages of features in flight in registers
//     (compiler-tracked loads: these waves issue no stores, so the compiler's vmcnt is exact),
//     convert a landed stage into the operand plane(s) of an LDS stage slot and publish the
//     slot's header (item, stage, scales, maxima).
//   * 4 MFMA waves: wave w owns x-block w (32 pixels) of the item and its T = 1 + DMAX/32
//     32x32 band blocks, accumulated on v_mfma_f32_32x32x16_{f16,bf16}.  After an item's last
//     stage a wave shears its blocks (d = x - j) into its full-item LDS ring; the volume rows of
//     that item leave the ring a few chunks per stage DURING THE NEXT ITEM's stages, in the
//     shadow of its matrix work, so the output stream overlaps the loads instead of following
//     them.  Fused, the wave folds the ring's columns into an online softmax instead.
// Two stage slots alternate; ONE workgroup barrier per stage separates "staging writes slot s+1"
// from "MFMA reads slot s".
//
// Operands.  fp16 / bf16 features are staged as they are (one plane; their products are exact
// in fp32: one MFMA per block and 16-channel step).  fp32 features are scaled by a per-item
// power of two 2^k (exact) and split into two fp16 planes by round-to-nearest:
// h = rn16(x 2^k), m = rn16(x 2^k - h), so x 2^k = h + m + e with |e| <= 2^-22 |x 2^k|
// (+ 2^-25 absolute below the fp16 normal range); the products h*h' + h*m' + m*h' (exact in
// fp32; the dropped m*m', h*e', e*h' are each at most 2^-22 relative) accumulate in fp32, and the
// result is multiplied back by 2^-(kL+kR) (ldexp, exact).  Integer features are exact.
//
// Scale control (fp32).  The staging lanes track max|x| of everything they stage for an item
// and publish the per-wave maxima with the item's last stage.  The MFMA waves accept the item
// when both scaled maxima lie in [2^-2, 2^15) (or are 0); otherwise they ask the staging waves
// (control words, generation-numbered) to restage the item with k = 13 - exponent(max) (scaled
// maximum in [2^12, 2^13)), which then carries to later items, so smoothly varying feature
// scales cost nothing.  Items holding +-inf (or a scale fp32 cannot reach, or failing twice)
// take an exact fp32 FMA path.  NaN needs no special case: it propagates through the split and
// the products like through the reference sum.  Cells x < d are forced to 0 as in the reference
// (an R pad row can meet a NaN or an inf).
#include "common.h"

#include <math.h>

#include <atomic>
#include <type_traits>

#ifndef SMCV_NT_STORE
#define SMCV_NT_STORE 1  // volume stores non-temporal (0: plain, for A/B)
#endif

#ifndef SMCV_ABLATE
#define SMCV_ABLATE 0  // diagnostics only (scripts/ws_ablate.hip): 1 no MFMA, 2 no fragment reads
#endif                 // or MFMA, 4 no volume stores, 8 no shear/epilogue, 16 no staging split /
                       // plane writes, 32 no feature loads (staging converts stale registers)

namespace smcv {
namespace wsband {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int kMW = 4;                      // MFMA waves: one 32-pixel x-block each
constexpr int kPW = 4;                      // staging waves
constexpr int kThreads = 64 * (kMW + kPW);  // one workgroup per CU
constexpr int kXT = 32 * kMW;               // left pixels per row segment (item)
constexpr int kKC = 16;                     // channels per stage (one 32x32x16 k-step)
constexpr int kRowB = 32;                   // bytes per plane row: 16 x 16-bit
constexpr int kChunk = 32 * 32 * 4;         // one ring chunk: 32 disparities x 32 pixels, fp32
constexpr int kLoads = 8;                   // feature loads per staging lane and stage
constexpr int kHdr = 64;                    // bytes per stage-slot header
constexpr int kLdsMax = 160 * 1024;
enum { kNDHW = 0, kNGHWD = 1 };
// stage-slot header words
enum { hIt = 0, hKs = 1, hKL = 2, hKR = 3, hMaxL = 4, hMaxR = 8 };

// byte offset of (plane row r, 8-channel chunk h).  Fragment reads: lane l -> row base + (l & 31),
// chunk l >> 5; plane writes: 8 consecutive lanes -> rows 4i + p of one 32-row block.  Both are
// conflict-free under the gfx950 ds_read_b128 / ds_write_b128 lane groups (scripts/check_swizzle.py).
__device__ __forceinline__ int swz(int r, int h) {
  return ((r ^ ((r >> 2) & 3)) << 5) + ((h ^ ((r >> 4) & 1)) << 4);
}

// LDS image: [2 stage slots: operand plane(s)] [4 full-item shear rings] [2 slot headers]
//            [2 control records] [dump words]
template <typename T, int TMAX>
struct Geo {
  static constexpr int NP = sizeof(T) == 4 ? 2 : 1;  // operand planes
  static constexpr int DMAX = 32 * (TMAX - 1);
  static constexpr int RW = kXT + DMAX;   // right-window rows
  static constexpr int ROWS = RW + kXT;   // + left-tile rows
  static constexpr int PLANE = ROWS * kRowB;
  static constexpr int STAGE = NP * PLANE;  // one stage slot
  static constexpr int NCH = TMAX - 1;      // volume chunks (32 disparities) per MFMA wave
  static constexpr int RINGW = NCH * kChunk;
  static constexpr int RING = 2 * STAGE;
  static constexpr int HDR = RING + kMW * RINGW;  // two slot headers
  static constexpr int CTRL = HDR + 2 * kHdr;     // two control records (iteration parity)
  static constexpr int DUMP = CTRL + 32;           // one word per MFMA lane (partial blocks)
  static constexpr size_t SHM = (size_t)DUMP + 4 * 64 * kMW;
  static_assert(RW % 32 == 0 && kXT % 32 == 0, "8-lane write groups stay inside one chunk");
  static_assert(SHM <= (size_t)kLdsMax, "one workgroup per CU");
};

struct Args {
  const void* L;
  const void* R;
  void* out;    // volume; nullptr: not stored (fused kernel only)
  float* disp;  // fused kernel: (N, H, W) disparities
  int C, cpg, G, H, W, D;
  Strides4 ls, rs;
  int tiles, npass, pw, nwork;
  float mul;  // MEAN: 1 / (channels averaged)
};

struct Work {
  int n, y, g, x0, dp, Dp, js;
};

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
__device__ __forceinline__ __attribute__((address_space(3))) int* lds_int(unsigned addr) {
  return reinterpret_cast<__attribute__((address_space(3))) int*>(addr);
}
__device__ __forceinline__ int rfl(int v) { return __builtin_amdgcn_readfirstlane(v); }

// The one workgroup barrier per stage: every LDS access of this wave is complete, then s_barrier.
// Output stores and feature loads stay in flight (no vmcnt wait).
__device__ __forceinline__ void stage_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// a 4-pixel group of one channel row in registers: 16 B (fp32) or 8 B (fp16 / bf16)
template <typename T> struct Quad { using type = u32x2; };
template <> struct Quad<float> { using type = f32x4v; };

// Feature loads of the staging waves: inline asm, so that the compiler neither waits for them
// itself (its waitcnt pass loses track of which of the two register sets is older across the
// stage loop and drains both) nor knows them; the waves count vmcnt by hand (vm_wait: the older
// set = all but the newer set's kLoads loads).  scripts/check_ws_asm.py replays the compiled
// code's vector-memory queue and checks that no instruction touches a load's registers before
// its wait.
template <typename QT>
__device__ __forceinline__ void gload(QT& v, const void* p) {
  if constexpr (sizeof(QT) == 16) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  } else {
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  }
}
// Wait until at most N loads of this wave are in flight; the set about to be consumed is tied.
template <int N, typename QT>
__device__ __forceinline__ void vm_wait(QT (&v)[kLoads]) {
  asm volatile("s_waitcnt vmcnt(%8)"
               : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]),
                 "+v"(v[6]), "+v"(v[7])
               : "n"(N)
               : "memory");
}

// 4 fp32 results -> storage type (round to nearest even; NaN stays NaN, overflow gives inf).
template <typename T>
__device__ __forceinline__ void store_quad(T* p, f32x4v v) {
  typedef __attribute__((address_space(1))) void gvoid;
  gvoid* g = (gvoid*)p;
  // non-temporal: the volume is written once and never re-read by this kernel; plain stores
  // would allocate its lines in L2 and evict the feature lines the loads reuse
  // (scripts/micro/mlp_patterns.hip: cfg2 reads + writes 140 us plain vs 106 us nt)
  if constexpr (sizeof(T) == 4) {
    if (SMCV_NT_STORE)
      __builtin_nontemporal_store(v, reinterpret_cast<__attribute__((address_space(1))) f32x4v*>(g));
    else
      *reinterpret_cast<__attribute__((address_space(1))) f32x4v*>(g) = v;
  } else if constexpr (std::is_same<T, __half>::value) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const h4 r = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
    if (SMCV_NT_STORE)
      __builtin_nontemporal_store(r, reinterpret_cast<__attribute__((address_space(1))) h4*>(g));
    else
      *reinterpret_cast<__attribute__((address_space(1))) h4*>(g) = r;
  } else {
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    const b4 r = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    if (SMCV_NT_STORE)
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

// exponent e with x = f 2^e, f in [0.5, 1) (x > 0 finite)
__device__ __forceinline__ int exp_of(float x) { return __builtin_amdgcn_frexp_expf(x); }

template <int I> using IC = std::integral_constant<int, I>;

template <typename T, typename TO, int TMAX, bool MEAN, int LAYOUT, bool FUSE>
__global__ __launch_bounds__(kThreads, 2) void band_ws(Args args) {
  using G = Geo<T, TMAX>;
  constexpr int DMAX = G::DMAX;
  constexpr int NP = G::NP;
  constexpr int NCH = G::NCH;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const T* __restrict__ L = static_cast<const T*>(args.L);
  const T* __restrict__ R = static_cast<const T*>(args.R);
  TO* __restrict__ out = static_cast<TO*>(args.out);
  const int cpg = args.cpg, H = args.H, W = args.W, D = args.D;
  const Strides4 ls = args.ls, rs = args.rs;

  // work range of this workgroup's XCD group (blocks b and b+8 share an XCD): consecutive
  // segments of a row run on one XCD at the same time and share its L2 for the right window
  const int grp = blockIdx.x & 7;
  const int gi = blockIdx.x >> 3;
  const int gsz = gridDim.x >> 3;
  const int q8 = args.nwork >> 3, r8 = args.nwork & 7;
  const int wbeg = grp < r8 ? grp * (q8 + 1) : r8 * (q8 + 1) + (grp - r8) * q8;
  const int wend = wbeg + q8 + (grp < r8 ? 1 : 0);
  if (wbeg + gi >= wend) return;  // the whole workgroup leaves together, before any barrier
  const int nitems = (wend - (wbeg + gi) + gsz - 1) / gsz;
  // item i of this workgroup is group-local index j = gi + i gsz.  With gsz % 8 == 0 every
  // workgroup would keep one tile index (j % 8) for the whole launch, so the workgroups of the
  // 64-pixel last tile of a 960-pixel row would idle half the time; rotating each complete
  // aligned 8-item block by the round i = j / gsz spreads the short tiles over all workgroups.
  const int wcnt = wend - wbeg;
  const bool rot = (gsz & 7) == 0;
  auto witem = [&](int i) -> int {
    const int j = gi + i * gsz;
    const int b = j & ~7;
    return wbeg + ((rot && b + 8 <= wcnt) ? (b | ((j + i) & 7)) : j);
  };
  const int nks = (cpg + kKC - 1) / kKC;

  const int tid = threadIdx.x;
  const int wave = rfl(tid >> 6);
  const int lane = tid & 63;
  const unsigned hdr0 = lds_addr(smem + G::HDR);
  const unsigned ctrl0 = lds_addr(smem + G::CTRL);
  SM_STAMP_DECL

  if (wave >= kMW) {
    // =========================================================================== staging role
    // Every staging wave serves one tensor: waves 0 .. PR-1 the right window (rows 0 .. RW-1 of
    // the planes), wave PR the left tile (rows RW ..).  Lane (ch, g) of a part owns pixel group g
    // (4 pixels, plane rows prow .. prow+3) of 8-channel chunk ch.  A wave's loads are one
    // uniform (scalar) row base + a 32-bit lane offset; the item's decode runs once per item.
    // Stage q's 8 channel rows sit in register set q % 2; they were loaded two stages earlier.
    constexpr int GR = G::RW / 4, GL = kXT / 4;  // pixel groups of the window / the tile
    constexpr int PR = (2 * GR + 63) / 64;       // right-window waves
    static_assert(PR + 1 <= kPW, "the left tile needs a staging wave of its own");
    const int pw = wave - kMW;
    const bool isR = pw < PR;  // uniform
    const int tr = isR ? 64 * pw + lane : lane;
    const int gcnt = isR ? GR : GL;
    const bool active = (isR || pw == PR) && tr < 2 * gcnt;
    const int ch = min(tr / gcnt, 1);                  // 8-channel chunk
    const int g = min(tr - ch * gcnt, gcnt - 1);       // pixel group
    const int prow = (isR ? 0 : G::RW) + 4 * g;        // plane row of the group's first pixel
    const Strides4 ts = isR ? rs : ls;                 // uniform
    const T* tbase = isR ? R : L;
    const bool cfull = rfl(cpg % kKC) == 0;  // uniform: a scalar branch

    using QT = typename Quad<T>::type;
    struct Set {
      QT v[kLoads];
      int nv;      // valid channels of v (0: pixels outside the image, an idle lane)
      int it, ks;  // the stage held (item -1: past the last item)
    };
    Set st[1];
    int cit = 0, cks = 0;  // cursor: the next stage to load
    // the cursor item's row: uniform base (elements) and this lane's pixel offset
    const T* ibase = tbase;
    int ipx = 0;
    bool iok = false;
    // the cursor's stage into set s: exactly kLoads loads per wave and stage, on every path (past
    // the last item and in a wave with no lanes to stage: reloads of a row start) -- the count
    // vm_wait relies on
    auto load = [&](Set& s) {
      cit = rfl(cit);  // wave-uniform control (scalar branches only, no exec-masked paths)
      cks = rfl(cks);
      s.it = cit;
      s.ks = cks;
      s.nv = 0;
      const T* q = tbase;
      int lim = 0;
      if (cit >= 0) {
        if (cks == 0) {  // a new item: its row base and this lane's pixels
          const Work k = decode(witem(cit), args, DMAX);
          ibase = tbase + (int64_t)k.n * ts.n + (int64_t)k.y * ts.h + (int64_t)k.g * cpg * ts.c;
          const int px = (isR ? k.js : k.x0) + 4 * g;
          iok = active && px >= 0 && px < W;
          ipx = iok ? px : 0;
        }
        const int cl = cks * kKC + 8 * ch;  // channel within the group
        s.nv = iok ? min(max(cpg - cl, 0), 8) : 0;
        // channel tail: clamp to the group's last channel (put() zeroes the tail)
        lim = cfull ? 7 : min(max(cpg - 1 - cl, 0), 7);
        q = ibase + (int64_t)min(cl, cpg - 1) * ts.c + ipx;
        if (++cks == nks) {
          cks = 0;
          if (++cit >= nitems) cit = -1;
        }
      }
      if constexpr (!(SMCV_ABLATE & 32)) {
        // the channel stride, opaque here: the 8 addresses are stepped, not 8 hoisted offsets
        int64_t csl = ts.c;
        asm volatile("" : "+v"(csl));
#pragma unroll
        for (int kk = 0; kk < kLoads; ++kk) {
          gload(s.v[kk], q);
          if (kk < lim) q += csl;
        }
      }
    };

    int kcL = 0, kcR = 0;  // carried scale exponents (fp32): used by the next item staged
    int kiL = 0, kiR = 0;  // scale exponents of the item being staged
    float mx = 0.f;        // this lane's max|x| over the item being staged (fp32 only)
    // register set s -> operand plane(s) of stage slot sp + its header
    auto put = [&](Set& s, int sp) {
      const unsigned hb = hdr0 + (unsigned)(sp * kHdr);
      if (rfl(s.it) < 0) {
        if (pw == 0 && lane == 0) *lds_int(hb + 4 * hIt) = -1;
        return;
      }
      if (rfl(s.ks) == 0) {
        kiL = kcL;
        kiR = kcR;
        mx = 0.f;
      }
      unsigned char* base = smem + sp * G::STAGE;
      if (active && !(SMCV_ABLATE & 16)) {
        if constexpr (NP == 2) {
          f32x4v v[kLoads];
#pragma unroll
          for (int kk = 0; kk < kLoads; ++kk) v[kk] = s.v[kk];
          if (__any(s.nv != kLoads)) {  // row edges / channel tail only
#pragma unroll
            for (int kk = 0; kk < kLoads; ++kk)
              if (kk >= s.nv) v[kk] = f32x4v{0.f, 0.f, 0.f, 0.f};
          }
#pragma unroll
          for (int kk = 0; kk < kLoads; ++kk)
            mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[kk].x), fabsf(v[kk].y)),
                                 fmaxf(fabsf(v[kk].z), fabsf(v[kk].w))));
          // h = rn16(x sc), m = rn16(x sc - h) (v_cvt_pk_f16_f32 rounds to nearest even)
          auto split = [&](float sc, auto scaled) {
#pragma unroll
            for (int p = 0; p < 4; ++p) {
              uint4 wh, wm;
              unsigned* ph = reinterpret_cast<unsigned*>(&wh);
              unsigned* pm = reinterpret_cast<unsigned*>(&wm);
#pragma unroll
              for (int qq = 0; qq < 4; ++qq) {
                const float a = v[2 * qq][p], b = v[2 * qq + 1][p];
                const float as = decltype(scaled)::value ? a * sc : a;
                const float bs = decltype(scaled)::value ? b * sc : b;
                const h16x2 hv = {(_Float16)as, (_Float16)bs};
                const float ra = decltype(scaled)::value ? __builtin_fmaf(a, sc, -(float)hv[0])
                                                         : a - (float)hv[0];
                const float rb = decltype(scaled)::value ? __builtin_fmaf(b, sc, -(float)hv[1])
                                                         : b - (float)hv[1];
                const h16x2 mv = {(_Float16)ra, (_Float16)rb};
                ph[qq] = __builtin_bit_cast(unsigned, hv);
                pm[qq] = __builtin_bit_cast(unsigned, mv);
              }
              const int off = swz(prow + p, ch);
              *reinterpret_cast<uint4*>(base + off) = wh;
              *reinterpret_cast<uint4*>(base + G::PLANE + off) = wm;
            }
          };
          if (rfl(kiL | kiR) == 0) {  // uniform: a scalar branch
            split(1.0f, std::false_type{});
          } else {
            split(__builtin_ldexpf(1.0f, isR ? kiR : kiL), std::true_type{});
          }
        } else {
          // 16-bit features as they are: 8 channels x 4 pixels -> 4 rows of 8 channels
          u32x2 qv[kLoads];
#pragma unroll
          for (int kk = 0; kk < kLoads; ++kk) qv[kk] = s.v[kk];
          if (__any(s.nv != kLoads)) {
#pragma unroll
            for (int kk = 0; kk < kLoads; ++kk)
              if (kk >= s.nv) qv[kk] = u32x2{0u, 0u};
          }
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            uint4 w;
            unsigned* pwd = reinterpret_cast<unsigned*>(&w);
#pragma unroll
            for (int j = 0; j < 4; ++j) {  // channels 2j (low half), 2j+1 (high half) of pixel p
              const unsigned lo = p < 2 ? qv[2 * j].x : qv[2 * j].y;
              const unsigned hi = p < 2 ? qv[2 * j + 1].x : qv[2 * j + 1].y;
              pwd[j] = __builtin_amdgcn_perm(hi, lo, (p & 1) ? 0x07060302u : 0x05040100u);
            }
            *reinterpret_cast<uint4*>(base + swz(prow + p, ch)) = w;
          }
        }
      }
      if (pw == 0 && lane == 0) {
        *lds_int(hb + 4 * hIt) = s.it;
        *lds_int(hb + 4 * hKs) = s.ks;
        *lds_int(hb + 4 * hKL) = kiL;
        *lds_int(hb + 4 * hKR) = kiR;
      }
      if constexpr (NP == 2) {
        if (rfl(s.ks) == nks - 1) {  // the item's maxima, per staging wave
          const float m = wave_max(mx);  // a wave stages one tensor
          if (lane == 0) {
            *lds_int(hb + 4 * (hMaxL + pw)) = __float_as_int(isR ? 0.f : m);
            *lds_int(hb + 4 * (hMaxR + pw)) = __float_as_int(isR ? m : 0.f);
          }
        }
      }
    };

    // One register set: stage q's loads are issued right after stage q-1 was staged, so they
    // have a whole stage iteration (the MFMA waves' matrix work and stores) to land.  The loop
    // has ONE load site (a second one, e.g. for a restage, makes the register allocator move the
    // set between load sites, i.e. copy registers whose loads have not landed).
    Set& cs_ = st[0];
    // prologue: stage 0 into slot 0 (landed before the loop: no load in flight at its entry)
    load(cs_);
    vm_wait<0>(cs_.v);
    put(cs_, 0);
    bool ended = rfl(cs_.it) < 0;
    int gseen = 0;  // control generation seen
    int par = 0;    // iteration parity (control record read this iteration)
    int sp = 1;     // slot written this iteration
    // iteration s writes stage s+1 into slot (s+1) % 2.  A restage request: the stage in flight
    // is dropped (nothing is staged this iteration; the MFMA waves skip two iterations) and the
    // cursor restarts at the item's first stage.
    for (;;) {
      load(cs_);  // the next stage (after a restage: the wrong one, dropped below)
      SM_STAMP(6);
      stage_barrier();
      SM_STAMP(3);
      const unsigned cb = ctrl0 + (unsigned)(16 * par);
      par ^= 1;
      const int gen = rfl(*lds_int(cb));
      const bool restage = gen > gseen;
      if (restage) {
        gseen = gen;
        kcL = rfl(*lds_int(cb + 8));
        kcR = rfl(*lds_int(cb + 12));
        cit = rfl(*lds_int(cb + 4));
        cks = 0;
      }
      // every path from the load reaches this wait: the set is live (not reusable) in between
      vm_wait<0>(cs_.v);  // this wave's only vector-memory operations are these loads
      if (!restage && ended) break;
      ended = ended && !restage;
      SM_STAMP(4);
      if (!restage) {
        put(cs_, sp);
        ended = rfl(cs_.it) < 0;
      }
      SM_STAMP(5);
      sp ^= 1;
    }
    SM_STAMP_FLUSH
    return;
  }

  // ============================================================================== MFMA role
  const bool store_vol = rfl(args.out != nullptr ? 1 : 0) != 0 && !(SMCV_ABLATE & 4);
  // NGHWD quads are 16-B aligned only when D % 4 == 0
  const bool dq = LAYOUT == kNDHW || rfl(D & 3) == 0;
  const int lr = lane & 31;
  const int hh = lane >> 5;
  using FV = typename std::conditional<std::is_same<T, __bf16>::value, bf16x8, f16x8>::type;
  constexpr int NB = NP == 2 ? 2 : 4;  // fragment buffers: blocks read ahead of the MFMAs
  f32x16 acc[TMAX];
  auto mma = [](FV a, FV b, f32x16 c) {
    if constexpr (std::is_same<T, __bf16>::value) {
      return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
    } else {
      return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    }
  };
  const int aoff = 32 * wave * kRowB + swz(lr, hh);            // + 1024 t
  const int boff = (G::RW + 32 * wave) * kRowB + swz(lr, hh);
  auto band = [&](const unsigned char* sb, auto first) {
    if (SMCV_ABLATE & 2) return;
    const unsigned char* abase = sb + aoff;
    const unsigned char* bbase = sb + boff;
    const FV bh = *reinterpret_cast<const FV*>(bbase);
    FV bm = bh;
    if constexpr (NP == 2) bm = *reinterpret_cast<const FV*>(bbase + G::PLANE);
    FV ah[NB], am[NB];
    auto rd = [&](int t) {
      ah[t % NB] = *reinterpret_cast<const FV*>(abase + 1024 * t);
      if constexpr (NP == 2) am[t % NB] = *reinterpret_cast<const FV*>(abase + G::PLANE + 1024 * t);
    };
#pragma unroll
    for (int t = 0; t < NB - 1 && t < TMAX; ++t) rd(t);
#pragma unroll
    for (int t = 0; t < TMAX; ++t) {
      if (t + NB - 1 < TMAX) rd(t + NB - 1);
      __builtin_amdgcn_sched_barrier(0);
      f32x16 c;
      if constexpr (decltype(first)::value) {
        c = f32x16{};
      } else {
        c = acc[t];
      }
      if (SMCV_ABLATE & 1) {  // keep the fragments live, no matrix work
        c[0] += (float)ah[t % NB][0] + (float)bh[0];
        if constexpr (NP == 2) c[1] += (float)am[t % NB][0] + (float)bm[0];
        acc[t] = c;
      } else {
        if constexpr (NP == 2) {
          c = mma(am[t % NB], bh, c);
          c = mma(ah[t % NB], bm, c);
        }
        acc[t] = mma(ah[t % NB], bh, c);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ------------------------------------------------------------------------- shear + ring
  // Lane (lr, hh) holds, in block t, element i at R row jj = c_i + 4 hh (c_i = (i & 3) +
  // 8 (i >> 2)) and L column lr: local disparity dl = 32 (a + 1) + u - c_i with a = T-2-t and
  // u = lr - 4 hh, i.e. chunk a+1 (row u - c_i) when u >= c_i, else chunk a (row 32 + u - c_i).
  // Chunks 0 .. T-2 are the wave's volume rows; block T-1's rows below chunk 0 (d < 0) and
  // block 0's rows past chunk T-2 (d >= DMAX) are not written.  The full-item ring of a wave:
  //   NDHW:  [chunk][32 d][32 x] fp32 (a readout row = 128 B of x);
  //   NGHWD: [32 x][32 NCH d] fp32, the d-quad index XOR-ed with (x >> 1) & 1 when the row is a
  //          multiple of 64 words (a readout row = 128 B of d).
  // The shear writes (ds_write_b32, 32-lane halves: distinct u -> distinct banks) and the
  // 16-B readouts (4 x 16-lane groups) are conflict-free in both layouts.
  constexpr int NGROW = 32 * NCH;                          // NGHWD ring row, words
  constexpr int NGX = (NGROW % 64 == 0) ? 32 : 0;          // NGHWD d-quad swizzle (words)
  const unsigned ringw = lds_addr(smem + G::RING) + (unsigned)(wave * G::RINGW);
  const int u = lr - 4 * hh;
  const unsigned wbase = LAYOUT == kNDHW ? ringw + (unsigned)(4 * lr + 128 * u)
                                         : ringw + (unsigned)(4 * NGROW * lr);
  const int ngsw = LAYOUT == kNDHW ? 0 : NGX * ((lr >> 1) & 1);
  const int rl = lane >> 3, cl = lane & 7;  // readout: rows (NDHW) / pixels (NGHWD) 8qq + rl
  const size_t plane_stride = (size_t)H * W;
  // lane part of the readout store addresses, in elements (32-bit: the host keeps 8 H W < 2^31)
  const int lane_st = LAYOUT == kNDHW ? rl * H * W + 4 * cl : rl * D + 4 * cl;
  // lane part of the readout LDS addresses
  auto rd_addr = [&](int a, int qq) -> unsigned {
    if constexpr (LAYOUT == kNDHW) {
      return ringw + (unsigned)(a * kChunk + (8 * qq + rl) * 128 + 16 * cl);
    } else {
      const int x = 8 * qq + rl;
      return ringw + (unsigned)(4 * (NGROW * x + ((32 * a + 4 * cl) ^ (NGX * ((x >> 1) & 1)))));
    }
  };

  // SCALE: multiply back by 2^-(kL+kR); XLT: the segment has cells x < d (R pad rows), forced
  // to 0.  Compile-time, so the common case costs no VALU.
  const unsigned dump = lds_addr(smem + G::DUMP) + (unsigned)(4 * tid);
  auto shear = [&](const Work& k, int kk, auto scale, auto xlt) {
    const float mul = args.mul;
    const int jlane = k.js + 32 * wave + 4 * hh;  // R row of element c_i of block 0, minus c_i
#pragma unroll
    for (int t = TMAX - 1; t >= 0; --t) {
      const int a = TMAX - 2 - t;
      // per block, opaque to the compiler: the per-element addresses and selects below are
      // recomputed in each block instead of being hoisted out of the block loop
      unsigned wb = wbase;
      int uu = u, jl = jlane, sw = ngsw;
      asm volatile("" : "+v"(wb), "+v"(uu), "+v"(jl), "+v"(sw));
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ci = (i & 3) + 8 * (i >> 2);
        float val = acc[t][i];
        if (MEAN) val *= mul;
        if constexpr (decltype(scale)::value) val = __builtin_ldexpf(val, kk);
        if constexpr (decltype(xlt)::value) val = jl + 32 * t + ci >= 0 ? val : 0.f;
        unsigned addr;
        if constexpr (LAYOUT == kNDHW) {
          addr = wb + (unsigned)((a + 1) * kChunk - ci * 128);
        } else {
          addr = wb + 4u * (unsigned)((32 * (a + 1) + uu - ci) ^ sw);
        }
        // block T-1 (a = -1): only chunk 0 (u >= c_i); block 0 (a = T-2): only chunk T-2; the
        // other elements go to this lane's dump word (branch-free)
        if (t == TMAX - 1) addr = uu >= ci ? addr : dump;
        if (t == 0) addr = uu < ci ? addr : dump;
        lds_store1(addr, val);
      }
      // one block at a time (the live accumulators shrink block by block)
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto shear_item = [&](const Work& k, int kL, int kR) {
    using TT = std::true_type;
    using FF = std::false_type;
    const bool xl = rfl(k.js) < 0;
    if constexpr (NP == 2) {
      if (rfl(kL + kR) != 0) {
        if (xl)
          shear(k, -(kL + kR), TT{}, TT{});
        else
          shear(k, -(kL + kR), TT{}, FF{});
        return;
      }
    }
    if (xl)
      shear(k, 0, FF{}, TT{});
    else
      shear(k, 0, FF{}, FF{});
  };

  // ---------------------------------------------------------------------------- the output
  // The item whose rows sit in the ring: its chunks [pc, NCH) are still to be stored.
  Work pk = {0, 0, 0, 0, 0, 0, 0};
  int pc = NCH;    // next chunk to store (NCH: nothing pending)
  bool pfast = false;
  // store chunks [pc, c1) of the pending item (each: 4 x 16-B ring reads, then 4 stores per lane)
  auto store_chunks = [&](int c1) {
    for (; pc < c1; ++pc) {
      const int a = pc;
      f32x4v v[4];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) v[qq] = lds_load4(rd_addr(a, qq));
      const int x0w = pk.x0 + 32 * wave;
      if constexpr (LAYOUT == kNDHW) {
        TO* ol = out + (((size_t)pk.n * D + pk.dp + 32 * a) * plane_stride + (size_t)pk.y * W + x0w) +
                 lane_st;
        const size_t st8 = (size_t)8 * plane_stride;  // rows 8 apart
        if (pfast) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            asm volatile("" : "+v"(ol));
            store_quad<TO>(ol, v[qq]);
            ol += st8;
          }
        } else {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            asm volatile("" : "+v"(ol));
            const int dl = 32 * a + 8 * qq + rl;
            if (dl < pk.Dp && x0w + 4 * cl < W) store_quad<TO>(ol, v[qq]);
            ol += st8;
          }
        }
      } else {
        const size_t pix = (((size_t)pk.n * args.G + pk.g) * H + pk.y) * (size_t)W + x0w;
        TO* ol = out + (pix * (size_t)D + pk.dp + 32 * a) + lane_st;
        asm volatile("" : "+v"(ol));
        if (pfast) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) store_quad<TO>(ol + (size_t)(8 * qq) * D, v[qq]);
        } else {
          const int d0 = 32 * a + 4 * cl;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            if (x0w + 8 * qq + rl >= W) continue;
            if (d0 + 4 <= pk.Dp && dq) {
              store_quad<TO>(ol + (size_t)(8 * qq) * D, v[qq]);
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (d0 + e < pk.Dp) store_one<TO>(ol + (size_t)(8 * qq) * D + e, v[qq][e]);
            }
          }
        }
      }
    }
  };
  // chunks per stage: the pending item's rows leave over the next item's nks stages
  const int cps = (NCH + nks - 1) / nks;

  // fused soft-argmin of the item in the ring: pixel lr of the wave, rows 16 hh .. 16 hh + 15 of
  // every chunk (conflict-free column reads), online softmax (running max; per-chunk fp32 sums
  // relative to the chunk's first row, fp64 across chunks); the two row halves merge at the end
  auto fuse_item = [&](const Work& k) {
    float fm = -INFINITY;
    double fs = 0.0, ft = 0.0;
    bool fnan = false;
    const unsigned colb = ringw + (unsigned)(16 * hh * 128 + 4 * lr);
    for (int a = 0; a < NCH; ++a) {
      float vv[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float x = lds_load1(colb + (unsigned)(a * kChunk + r * 128));
        vv[r] = 32 * a + 16 * hh + r < k.Dp ? x : -INFINITY;  // beyond D: not in the softmax
      }
      bool nn = false;
      float cm = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        nn |= vv[r] != vv[r];
        cm = fmaxf(cm, vv[r]);
      }
      fnan |= nn;
      const float nm = fmaxf(fm, cm);
      const bool fin = nm != -INFINITY && nm != INFINITY;
      // rescale the running sums to the new maximum (factor 1 when it did not grow)
      const float f = fin && fm != -INFINITY ? expf(fm - nm) : 0.f;
      float ps = 0.f, pt = 0.f;  // this chunk, disparities relative to its row 32 a + 16 hh
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float ex = fin ? expf(vv[r] - nm) : 0.f;
        ps += ex;
        pt = fmaf((float)r, ex, pt);
      }
      fs = fs * (double)f + (double)ps;
      ft = ft * (double)f + (double)(32 * a + 16 * hh) * (double)ps + (double)pt;
      fm = nm;
    }
    const bool nn2 = __shfl_xor((int)fnan, 32) != 0;  // the other row half of the pixel
    const float M = fmaxf(fm, __shfl_xor(fm, 32));
    const double f = (fm == -INFINITY || M == INFINITY) ? 0.0 : (double)expf(fm - M);
    double s = fs * f, t = ft * f;
    s += __shfl_xor(s, 32);
    t += __shfl_xor(t, 32);
    // NaN anywhere in the column, or an all -inf / any +inf column: NaN, as torch
    const bool bad = fnan || nn2 || M == INFINITY || M == -INFINITY;
    const int x = k.x0 + 32 * wave + lr;
    if (hh == 0 && x < W)
      store_one<float>(args.disp + ((size_t)k.n * H + k.y) * W + x, bad ? NAN : (float)(t / s));
  };

  // exact fp32 path for an item holding +-inf (or a scale fp32 cannot reach); MFMA waves only
  auto slow_segment = [&](const Work& k) {
    const int mt = tid;  // 0 .. 64 kMW - 1
    constexpr int kMT = 64 * kMW;
    const float mul = MEAN ? args.mul : 1.0f;
    const T* lrow = L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h + (int64_t)k.g * cpg * ls.c;
    const T* rrow = R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h + (int64_t)k.g * cpg * rs.c;
    auto cell = [&](int x, int d) {
      float s = 0.f;
      if (x >= d) {
        for (int c = 0; c < cpg; ++c)
          s = __builtin_fmaf(ld1(lrow + (int64_t)c * ls.c + x),
                             ld1(rrow + (int64_t)c * rs.c + x - d), s);
        s *= mul;
      }
      return s;
    };
    if (store_vol) {
      for (int idx = mt; idx < k.Dp * kXT; idx += kMT) {
        const int dl = idx / kXT, x = k.x0 + idx % kXT, d = k.dp + dl;
        if (x >= W) continue;
        const float s = cell(x, d);
        if constexpr (LAYOUT == kNDHW) {
          store_one<TO>(out + (((size_t)k.n * D + d) * H + k.y) * W + x, s);
        } else {
          store_one<TO>(out + ((((size_t)k.n * args.G + k.g) * H + k.y) * W + x) * D + d, s);
        }
      }
    }
    if constexpr (FUSE) {
      for (int xx = mt; xx < kXT; xx += kMT) {
        const int x = k.x0 + xx;
        if (x >= W) continue;
        float m = -INFINITY;
        double s = 0.0, t = 0.0;
        bool nan = false;
        for (int d = 0; d < k.Dp; ++d) {
          const float v = cell(x, d);
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
        store_one<float>(args.disp + ((size_t)k.n * H + k.y) * W + x,
                         (nan || m == INFINITY || m == -INFINITY) ? NAN : (float)(t / s));
      }
    }
  };

  // ----------------------------------------------------------------------------- main loop
  // iteration s: consume stage slot s % 2 (staged during iteration s-1)
  if (tid < 8) *lds_int(ctrl0 + 4 * tid) = 0;  // both control records: generation 0
  int gseen = 0;
  int sp = 0, par = 0;
  int retried = -1;  // the item last sent back for restaging (a second failure takes the slow path)
  int mskip = 0;     // iterations still to skip after a restage request
  for (;;) {
    SM_STAMP(2);
    stage_barrier();
    SM_STAMP(0);
    const unsigned cb = ctrl0 + (unsigned)(16 * par);
    par ^= 1;
    const int gen = rfl(*lds_int(cb));
    if (gen > gseen) {  // a restage request: this slot and the next were not staged for it
      gseen = gen;
      mskip = 2;
    }
    if (mskip > 0) {
      --mskip;
      sp ^= 1;
      continue;
    }
    const unsigned hb = hdr0 + (unsigned)(sp * kHdr);
    const int it = rfl(*lds_int(hb + 4 * hIt));
    const int ks = it < 0 ? 0 : rfl(*lds_int(hb + 4 * hKs));
    const unsigned char* sb = smem + sp * G::STAGE;
    if (it >= 0) {
      if (ks == 0)
        band(sb, std::true_type{});
      else
        band(sb, std::false_type{});
    }
    SM_STAMP(1);
    // this stage's share of the previous item's volume rows, in the shadow of the MFMAs (all of
    // them once the work has ended)
    if (store_vol) store_chunks(it < 0 ? NCH : min(NCH, (ks + 1) * cps));
    if (it < 0) break;
    if (ks == nks - 1) {
      const Work k = decode(witem(it), args, DMAX);
      const int kL = rfl(*lds_int(hb + 4 * hKL)), kR = rfl(*lds_int(hb + 4 * hKR));
      bool ok = true;
      if constexpr (NP == 2) {
        float ml = 0.f, mr = 0.f;
#pragma unroll
        for (int w = 0; w < kPW; ++w) {
          ml = fmaxf(ml, __int_as_float(*lds_int(hb + 4 * (hMaxL + w))));
          mr = fmaxf(mr, __int_as_float(*lds_int(hb + 4 * (hMaxR + w))));
        }
        const bool fin = ml <= 3.4e38f && mr <= 3.4e38f;  // no +-inf staged
        const int el = ml > 0.f ? exp_of(ml) : 0, er = mr > 0.f ? exp_of(mr) : 0;
        const bool okl = ml == 0.f || (el + kL <= 15 && el + kL >= -1);
        const bool okr = mr == 0.f || (er + kR <= 15 && er + kR >= -1);
        ok = fin && okl && okr;
        if (!ok) {
          const int nkl = ml > 0.f ? 13 - el : kL, nkr = mr > 0.f ? 13 - er : kR;
          if (!fin || retried == it || nkl < -100 || nkl > 100 || nkr < -100 || nkr > 100) {
            slow_segment(k);
          } else {
            retried = it;
            // the next iteration's control record (read by everyone after the barrier)
            const unsigned nb = ctrl0 + (unsigned)(16 * par);
            if (tid == 0) {
              *lds_int(nb + 4) = it;
              *lds_int(nb + 8) = nkl;
              *lds_int(nb + 12) = nkr;
              *lds_int(nb) = gseen + 1;
            }
          }
        }
      }
      if (ok && !(SMCV_ABLATE & 8)) {
        // the ring is rewritten: the previous item's last rows leave first
        shear_item(k, kL, kR);
        if constexpr (FUSE) fuse_item(k);
        if (store_vol) {
          pk = k;
          pc = 0;
          pfast = dq && k.x0 + kXT <= W && k.Dp == DMAX;
        }
      }
    }
    sp ^= 1;
  }
  SM_STAMP_FLUSH
}

template <typename T, typename TO, int TMAX, bool MEAN, int LAYOUT, bool FUSE>
int launch(Args a, int64_t N, hipStream_t st) {
  using G = Geo<T, TMAX>;
  a.tiles = (int)ceil_div(a.W, kXT);
  const int64_t nwork = (int64_t)a.tiles * a.H * N * a.G * a.npass;
  if (nwork > INT32_MAX / 64) return fail(SM_EINVAL, "band kernel: too much work for one launch");
  a.nwork = (int)nwork;
  auto kern = band_ws<T, TO, TMAX, MEAN, LAYOUT, FUSE>;
  static std::atomic<unsigned long long> lds_done{0};  // per instantiation
  const int dev = stream_device(st);
  if (int rc = ensure_lds_limit(reinterpret_cast<const void*>(kern), (int)G::SHM, dev, lds_done))
    return rc;
  int64_t nwg = std::min<int64_t>(nwork, (int64_t)device_cus(dev));
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(kThreads), G::SHM, st, a);
  return check_launch("band_ws");
}

// the smallest band geometry that holds one D pass of pw disparities
template <typename F>
int by_tmax(int64_t pw, F f) {
  if (pw <= 32) return f(std::integral_constant<int, 2>{});
  if (pw <= 64) return f(std::integral_constant<int, 3>{});
  if (pw <= 128) return f(std::integral_constant<int, 5>{});
  return f(std::integral_constant<int, 7>{});
}

}  // namespace wsband

int check_dot_args(const void* left, const void* right, const void* out, int dtype, int64_t N,
                   int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                   const int64_t* r_strides, Strides4* ls, Strides4* rs);

namespace {
// Shared validation; *vec = the shape takes the band kernels (4-pixel groups: W % 4 == 0,
// 4-element aligned rows and feature pointers, a 16-B aligned output, channels > 0).
int ws_prepare(const void* left, const void* right, const void* out, int dtype, int64_t N,
               int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
               const int64_t* r_strides, wsband::Args* a, bool* vec) {
  Strides4 ls, rs;
  int rc = check_dot_args(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &ls, &rs);
  if (rc) return rc;
  const uintptr_t align = 4 * (uintptr_t)elem_size(dtype);
  *vec = (W % 4 == 0) && W >= 4 && C > 0 && ls.n % 4 == 0 && ls.c % 4 == 0 && ls.h % 4 == 0 &&
         rs.n % 4 == 0 && rs.c % 4 == 0 && rs.h % 4 == 0 &&
         ((reinterpret_cast<uintptr_t>(left) | reinterpret_cast<uintptr_t>(right)) % align == 0) &&
         reinterpret_cast<uintptr_t>(out) % 16 == 0 && 8 * H * W < INT32_MAX &&
         8 * W * std::max<int64_t>(D, 1) < INT32_MAX &&
         // the staging lanes' 32-bit byte offsets: pixels + up to 15 channel rows
         (16 * std::max(ls.c, rs.c) + W) * elem_size(dtype) < INT32_MAX;
  // D passes of at most 192 disparities, balanced (D = 256: two passes of 128); a pass width
  // that is a multiple of 4 keeps every right-window pixel group aligned
  const int64_t npass = ceil_div(std::max<int64_t>(D, 1), (int64_t)192);
  const int64_t pw = (ceil_div(std::max<int64_t>(D, 1), npass) + 3) / 4 * 4;
  a->L = left;
  a->R = right;
  a->out = const_cast<void*>(out);
  a->disp = nullptr;
  a->C = (int)C;
  a->cpg = (int)C;
  a->G = 1;
  a->H = (int)H;
  a->W = (int)W;
  a->D = (int)D;
  a->ls = ls;
  a->rs = rs;
  a->tiles = 0;
  a->npass = (int)npass;
  a->pw = (int)pw;
  a->nwork = 0;
  a->mul = 1.0f;
  return SM_OK;
}
}  // namespace

// Inner product (mode 0, sum) / correlation (mode 1, mean) -> (N, D, H, W) in the input dtype.
// *handled = false when the shape needs the generic path.
int band_ws_entry(const void* left, const void* right, void* out, int dtype, int64_t N, int64_t C,
                  int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                  const int64_t* r_strides, int mode, void* stream, bool* handled) {
  using namespace wsband;
  *handled = false;
  Args a;
  bool vec = false;
  int rc = ws_prepare(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &a, &vec);
  if (rc) return rc;
  if (!vec) return SM_OK;
  *handled = true;
  if (N == 0 || H == 0 || D == 0) return SM_OK;
  const bool mean = mode == 1;
  a.mul = 1.0f / (float)C;
  hipStream_t st = as_stream(stream);
  SM_DISPATCH_DTYPE(dtype, T0, {
    using T = typename std::conditional<std::is_same<T0, bf16_t>::value, __bf16, T0>::type;
    return by_tmax(a.pw, [&](auto tm) {
      constexpr int TM = decltype(tm)::value;
      return mean ? launch<T, T, TM, true, wsband::kNDHW, false>(a, N, st)
                  : launch<T, T, TM, false, wsband::kNDHW, false>(a, N, st);
    });
  });
  return SM_OK;
}

// Groupwise (mean over C/G contiguous channels) -> (N, G, H, W, D) float32.
int band_ws_groupwise_entry(const void* left, const void* right, float* out, int dtype, int64_t N,
                            int64_t C, int64_t H, int64_t W, int64_t D, int64_t G,
                            const int64_t* l_strides, const int64_t* r_strides, void* stream,
                            bool* handled) {
  using namespace wsband;
  *handled = false;
  if (G <= 0 || C % G != 0) return fail(SM_EINVAL, "groupwise: C % G != 0");
  Args a;
  bool vec = false;
  int rc = ws_prepare(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &a, &vec);
  if (rc) return rc;
  if (!vec) return SM_OK;
  *handled = true;
  if (N == 0 || H == 0 || D == 0) return SM_OK;
  a.G = (int)G;
  a.cpg = (int)(C / G);
  a.mul = 1.0f / (float)a.cpg;
  hipStream_t st = as_stream(stream);
  SM_DISPATCH_DTYPE(dtype, T0, {
    using T = typename std::conditional<std::is_same<T0, bf16_t>::value, __bf16, T0>::type;
    return by_tmax(a.pw, [&](auto tm) {
      constexpr int TM = decltype(tm)::value;
      return launch<T, float, TM, true, wsband::kNGHWD, false>(a, N, st);
    });
  });
  return SM_OK;
}

// Inner product / correlation fused with soft-argmin: disparity (N, H, W) fp32, and the volume
// when out != nullptr.  fp32 features, one D pass (D <= 192); *handled = false otherwise.
int band_ws_fused_entry(const void* left, const void* right, void* out, float* disp, int dtype,
                        int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                        const int64_t* l_strides, const int64_t* r_strides, int mode,
                        void* stream, bool* handled) {
  using namespace wsband;
  *handled = false;
  if (disp == nullptr && N * H * W > 0) return fail(SM_EINVAL, "null disparity pointer");
  Args a;
  bool vec = false;
  // (the volume check of check_dot_args needs a pointer when only the disparity is wanted)
  int rc = ws_prepare(left, right, out ? out : disp, dtype, N, C, H, W, D, l_strides, r_strides,
                      &a, &vec);
  if (rc) return rc;
  if (N * H * W == 0) {
    *handled = true;
    return SM_OK;
  }
  vec = vec && reinterpret_cast<uintptr_t>(disp) % 16 == 0;
  if (!vec || dtype != SM_F32 || a.npass != 1 || D == 0) return SM_OK;
  *handled = true;
  a.out = out;
  a.disp = disp;
  a.mul = 1.0f / (float)C;
  const bool mean = mode == 1;
  hipStream_t st = as_stream(stream);
  return by_tmax(a.pw, [&](auto tm) {
    constexpr int TM = decltype(tm)::value;
    return mean ? launch<float, float, TM, true, wsband::kNDHW, true>(a, N, st)
                : launch<float, float, TM, false, wsband::kNDHW, true>(a, N, st);
  });
}

}  // namespace smcv

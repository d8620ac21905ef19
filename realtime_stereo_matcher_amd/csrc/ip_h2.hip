// Inner-product / correlation cost volume on gfx950 matrix cores, fp16 two-plane split
// ("h2"): the fp32 default of sm_cv_inner_product / sm_cv_correlation_mean.
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// Per image row the volume is a band of the contraction S[j][x] = sum_c R[c][j] L[c][x]
// (d = x - j).  A workgroup (4 waves) owns a 128-pixel row segment; wave w owns x-block w
// (32 pixels) and its T = 1 + DMAX/32 32x32 band blocks, accumulated with
// v_mfma_f32_32x32x16_f16.  Every wave does everything (load, split, MFMA, shear, store) and
// the CU holds TWO such workgroups, so one workgroup's output stream overlaps the other's
// matrix work without any intra-workgroup role split.
//
// Arithmetic.  Each fp32 value is scaled by a per-segment power of two 2^k (exact) and split
// into two fp16 planes by round-toward-zero: h = rtz16(x 2^k), m = rtz16(x 2^k - h).  Then
// x 2^k = h + m + e with |e| < 2^-20 |x 2^k| (+ 2^-24 absolute below the fp16 normal range),
// and the products h*h' + h*m' + m*h' (exact in fp32; the dropped m*m', h*e', e*h' are each
// below 2^-20 relative) accumulate in fp32 on the matrix cores.  The result is multiplied back
// by 2^-(kL+kR) (ldexp, exact).  Integer-valued features are exact (m = 0).
//
// Scale control (range safety of fp16).  Every lane tracks max|x| of the values it stages; at
// the end of a segment the workgroup knows max|L| and max|R| over everything it staged.  The
// segment is accepted when both scaled maxima lie in [2^-2, 2^15) (or are 0); otherwise the
// segment is recomputed with k = 13 - exponent(max) (scaled maximum in [2^12, 2^13)), and that
// k carries to the next segment, so smoothly varying feature scales cost nothing.  Segments
// holding +-inf (or a scale fp32 cannot reach) take an exact fp32 FMA path.  NaN needs no
// special case: it propagates through the split and the products like through the reference
// sum, and cells x < d are forced to 0 as in the reference.
//
// Data flow per 16-channel step (one barrier pair): the step's features were loaded into
// registers one step earlier; barrier A (the previous step's fragment reads are done), split
// into the two planes in LDS (row/chunk XOR swizzle: conflict-free 16-B writes and fragment
// reads, scripts/check_swizzle.py), issue the loads of step s+1, barrier B, 3 MFMAs per band
// block.  After a segment's last step the accumulators are sheared (d = x - j) block by block
// through a 3-slot ring of 32-row x 512-B chunks; each block completes one chunk, which the
// four waves stream out as 512-B row segments (two rows per store instruction).
#include "common.h"

#include <type_traits>

#ifndef SMCV_ABLATE
#define SMCV_ABLATE 0  // diagnostics only (scripts/ip_stamps.hip): 1 no MFMA, 2 all feature
#endif                 // loads from one line, 4 no stores, 8 no epilogue

namespace smcv {
namespace h2band {

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __fp16 hp2 __attribute__((ext_vector_type(2)));
typedef float f32x4v __attribute__((ext_vector_type(4)));

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kXT = 32 * kWaves;    // left pixels per row segment
constexpr int kKC = 16;             // channels per step (one 32x32x16 k-step)
constexpr int kRowB = 32;           // bytes per plane row: 16 fp16
constexpr int kSlot = 32 * 512;     // one ring chunk: 32 output rows x 128 px fp32
constexpr int kRing = 3 * kSlot;

// byte offset of (plane row r, 8-channel chunk h).  Fragment reads: lane l -> row base + (l & 31),
// chunk l >> 5; plane writes: 8 consecutive lanes -> rows 4i + p of one 32-row block.  Both are
// conflict-free under the gfx950 ds_read_b128 / ds_write_b128 lane groups (scripts/check_swizzle.py).
__device__ __forceinline__ int swz(int r, int h) {
  return ((r ^ ((r >> 2) & 3)) << 5) + ((h ^ ((r >> 4) & 1)) << 4);
}

template <int TMAX>
struct Geo {
  static constexpr int DMAX = 32 * (TMAX - 1);
  static constexpr int RW = kXT + DMAX;   // right-window rows
  static constexpr int ROWS = RW + kXT;   // + left-tile rows
  static constexpr int PLANE = ROWS * kRowB;
  static constexpr int GROUPS = ROWS / 4; // 4-pixel groups per 8-channel chunk
  static constexpr int ITEMS = 2 * GROUPS;
  static constexpr int RING = 2 * PLANE;  // ring byte offset
  static constexpr int MAXW = RING + kRing;  // 4 words: max|L|, max|R| for segment parity 0/1
  static constexpr size_t SHM = (size_t)MAXW + 16;
  static_assert(ITEMS <= kThreads, "one staging item per lane");
  static_assert(GROUPS % 8 == 0, "8-lane write groups stay inside one chunk");
  static_assert(SHM * 2 <= 160 * 1024, "two workgroups per CU");
};

struct Work {
  int n, y, x0, dp, Dp, js;
};

__device__ __forceinline__ Work decode(int w, int tiles, int npass, int H, int D, int pw,
                                       int dmax) {
  Work k;
  const int pass = w % npass;
  const int rest = w / npass;
  const int tile = rest % tiles;
  const int row = rest / tiles;
  k.y = row % H;
  k.n = row / H;
  k.x0 = tile * kXT;
  k.dp = pass * pw;
  k.Dp = min(pw, D - k.dp);
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
__device__ __forceinline__ f32x4v lds_load4(unsigned addr) {
  return *reinterpret_cast<__attribute__((address_space(3))) f32x4v*>(addr);
}
__device__ __forceinline__ __attribute__((address_space(3))) unsigned* lds_word(unsigned addr) {
  return reinterpret_cast<__attribute__((address_space(3))) unsigned*>(addr);
}

// a 4-pixel group of one channel row in registers: 16 B (fp32) or 8 B (fp16 / bf16)
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
template <typename T> struct Quad { using type = u32x2; };
template <> struct Quad<float> { using type = f32x4v; };

// Feature loads are issued by inline asm so that the compiler neither waits for them itself
// (its control-flow merges would put vmcnt(0) -- a wait for every output store in flight --
// in front of every step) nor knows them: the kernel counts vmcnt by hand (vm_wait).
template <typename QT>
__device__ __forceinline__ void gload(QT& v, const void* p) {
  if constexpr (sizeof(QT) == 16) {
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  } else {
    asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  }
}
// Wait for the feature loads: vmcnt(N) when N output stores were issued after them (they may
// stay in flight), else vmcnt(0).  One asm statement with the scalar branch inside, and the
// loaded registers as tied operands: no use of them is scheduled before the wait, and the
// register allocator has a single place (the load's destination) to keep them.
template <int N, typename QT>
__device__ __forceinline__ void vm_wait(QT (&v)[8], int after_stores) {
  asm volatile(
      "s_cmp_eq_u32 %8, 0\n\t"
      "s_cbranch_scc1 .Lvm_all%=\n\t"
      "s_waitcnt vmcnt(%9)\n\t"
      "s_branch .Lvm_done%=\n"
      ".Lvm_all%=:\n\t"
      "s_waitcnt vmcnt(0)\n"
      ".Lvm_done%=:"
      : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
        "+v"(v[7])
      : "s"(after_stores), "n"(N)
      : "memory", "scc");
}

template <typename T>
__device__ __forceinline__ float4 quad_to_f32(typename Quad<T>::type q) {
  if constexpr (sizeof(T) == 4) {
    return make_float4(q.x, q.y, q.z, q.w);
  } else if constexpr (std::is_same<T, __half>::value) {
    // (a bit_cast of q.y to a 2 x __fp16 vector miscompiles to q.x with ROCm 7.2 clang)
    const unsigned x = q.x, y = q.y;
    auto f = [](unsigned short b) { return (float)__builtin_bit_cast(_Float16, b); };
    return make_float4(f(x & 0xffffu), f(x >> 16), f(y & 0xffffu), f(y >> 16));
  } else {  // bf16: the value is the high half of an fp32
    return make_float4(__uint_as_float(q.x << 16), __uint_as_float(q.x & 0xffff0000u),
                       __uint_as_float(q.y << 16), __uint_as_float(q.y & 0xffff0000u));
  }
}

// 4 fp32 results -> storage type (round to nearest even; NaN stays NaN, overflow gives inf).
// Global address space explicitly: a flat store would count in vmcnt out of order.
template <typename T>
__device__ __forceinline__ void store_quad(T* p, f32x4v v) {
  typedef __attribute__((address_space(1))) void gvoid;
  gvoid* g = (gvoid*)p;
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<__attribute__((address_space(1))) f32x4v*>(g) = v;
  } else if constexpr (std::is_same<T, __half>::value) {
    typedef _Float16 h4 __attribute__((ext_vector_type(4)));
    const h4 r = {(_Float16)v.x, (_Float16)v.y, (_Float16)v.z, (_Float16)v.w};
    *reinterpret_cast<__attribute__((address_space(1))) h4*>(g) = r;
  } else {
    typedef __bf16 b4 __attribute__((ext_vector_type(4)));
    const b4 r = {(__bf16)v.x, (__bf16)v.y, (__bf16)v.z, (__bf16)v.w};
    *reinterpret_cast<__attribute__((address_space(1))) b4*>(g) = r;
  }
}

template <typename T>
__device__ __forceinline__ float ld1(const T* p) { return (float)*p; }
template <typename T>
__device__ __forceinline__ void st1(T* p, float v) { *p = (T)v; }

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// exponent e with x = f 2^e, f in [0.5, 1) (x > 0 finite)
__device__ __forceinline__ int exp_of(float x) { return __builtin_amdgcn_frexp_expf(x); }

template <typename T, int TMAX, bool MEAN>
__global__ __launch_bounds__(kThreads, 2) void ip_band_h2(
    const T* __restrict__ L, const T* __restrict__ R, T* __restrict__ out, int C,
    int H, int W, int D, Strides4 ls, Strides4 rs, int tiles, int npass, int pw, int nwork,
    int stagger) {
  using G = Geo<TMAX>;
  constexpr int DMAX = G::DMAX;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  // work range of this workgroup's XCD group (blocks b and b+8 share an XCD): consecutive
  // segments of a row run on one XCD at the same time and share its L2 for the right window
  const int grp = blockIdx.x & 7;
  const int gi = blockIdx.x >> 3;
  const int gsz = gridDim.x >> 3;
  const int q = nwork >> 3, rr = nwork & 7;
  const int wbeg = grp < rr ? grp * (q + 1) : rr * (q + 1) + (grp - rr) * q;
  const int wend = wbeg + q + (grp < rr ? 1 : 0);
  if (wbeg + gi >= wend) return;  // the whole workgroup leaves together
  const int nitems = (wend - (wbeg + gi) + gsz - 1) / gsz;
  const int nks = (C + kKC - 1) / kKC;
  const int S = nitems * nks;  // pipeline steps of this workgroup
  // the second workgroup of a CU starts later, so the two are not in phase (one streams its
  // output while the other loads and multiplies)
  if (stagger > 0 && blockIdx.x >= gridDim.x / 2)
    for (int i = 0; i < stagger; ++i) __builtin_amdgcn_s_sleep(64);

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  SM_STAMP_DECL

  // ---------------------------------------------------------------- staging role of a lane
  const bool active = tid < G::ITEMS;
  const int ch = min(tid / G::GROUPS, 1);                  // 8-channel chunk
  const int g = min(tid - ch * G::GROUPS, G::GROUPS - 1);  // rows 4g .. 4g+3
  const bool isR = 4 * g < G::RW;
  const int64_t cs = isR ? rs.c : ls.c;
  const bool cfull = __builtin_amdgcn_readfirstlane(C % kKC) == 0;  // uniform: a scalar branch

  using QT = typename Quad<T>::type;
  struct Set {
    QT v[8];
    int nv;  // valid channels of v (0: pixels outside the image or an idle lane)
  };
  Set st;  // one set: the loads of step s+1 fly during step s's matrix work
  auto load = [&](Set& st, int s) {
    s = min(s, S - 1);  // past the end: reload the last step (nobody consumes it)
    const int it = s / nks;
    const int c0 = (s - it * nks) * kKC + 8 * ch;
    const Work k = decode(wbeg + gi + it * gsz, tiles, npass, H, D, pw, DMAX);
    const int px = isR ? k.js + 4 * g : k.x0 + 4 * g - G::RW;
    const bool okp = active && px >= 0 && px < W;
    const T* row = isR ? R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h
                       : L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;
    const T* p = row + (okp ? px : 0) + (int64_t)min(c0, C - 1) * cs;
    if (SMCV_ABLATE & 2) p = L + 4 * (lane & 7);
    st.nv = okp ? min(max(C - c0, 0), 8) : 0;
    // channel tail: clamp to the last channel (one code path; put() zeroes the tail)
    const int lim = cfull ? 7 : min(max(C - 1 - c0, 0), 7);
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) gload(st.v[kk], p + min(kk, lim) * cs);
  };

  int kL = 0, kR = 0;  // per-segment scale exponents (workgroup-uniform)
  float mx = 0.f;      // this lane's max|x| over the current segment
  // split one step into the h / m planes (scaled by 2^k when k != 0)
  auto put = [&](Set& st) {
    if (!active) return;
    float4 v[8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) v[kk] = quad_to_f32<T>(st.v[kk]);
    if (__any(st.nv != 8)) {  // row edges / channel tail only
#pragma unroll
      for (int kk = 0; kk < 8; ++kk)
        if (kk >= st.nv) v[kk] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
      mx = fmaxf(mx, fmaxf(fmaxf(fabsf(v[kk].x), fabsf(v[kk].y)),
                           fmaxf(fabsf(v[kk].z), fabsf(v[kk].w))));
    float col[4][8];
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      col[0][kk] = v[kk].x;
      col[1][kk] = v[kk].y;
      col[2][kk] = v[kk].z;
      col[3][kk] = v[kk].w;
    }
    unsigned char* base = smem;
    auto split = [&](float sc, auto scaled) {
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint4 wh, wm;
        unsigned* ph = reinterpret_cast<unsigned*>(&wh);
        unsigned* pm = reinterpret_cast<unsigned*>(&wm);
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const float a = col[p][2 * qq], b = col[p][2 * qq + 1];
          const float as = decltype(scaled)::value ? a * sc : a;
          const float bs = decltype(scaled)::value ? b * sc : b;
          const hp2 hv = __builtin_amdgcn_cvt_pkrtz(as, bs);
          const float ra = __builtin_fmaf(a, sc, -(float)hv[0]);
          const float rb = __builtin_fmaf(b, sc, -(float)hv[1]);
          const hp2 mv = __builtin_amdgcn_cvt_pkrtz(ra, rb);
          ph[qq] = __builtin_bit_cast(unsigned, hv);
          pm[qq] = __builtin_bit_cast(unsigned, mv);
        }
        const int off = swz(4 * g + p, ch);
        *reinterpret_cast<uint4*>(base + off) = wh;
        *reinterpret_cast<uint4*>(base + G::PLANE + off) = wm;
      }
    };
    if (__builtin_amdgcn_readfirstlane(kL | kR) == 0) {  // uniform: a scalar branch
      split(1.0f, std::false_type{});
    } else {
      split(__builtin_ldexpf(1.0f, isR ? kR : kL), std::true_type{});
    }
  };

  // ------------------------------------------------------------------- MFMA role of a wave
  const int lr = lane & 31;
  const int hh = lane >> 5;
  const unsigned char* abase = smem + 32 * wave * kRowB + swz(lr, hh);            // + 1024 t
  const unsigned char* bbase = smem + (G::RW + 32 * wave) * kRowB + swz(lr, hh);
  f32x16 acc[TMAX];
  auto band = [&](auto first) {
    f16x8 bh = *reinterpret_cast<const f16x8*>(bbase);
    f16x8 bm = *reinterpret_cast<const f16x8*>(bbase + G::PLANE);
    f16x8 ah[3], am[3];
    auto rd = [&](int t) {
      ah[t % 3] = *reinterpret_cast<const f16x8*>(abase + 1024 * t);
      am[t % 3] = *reinterpret_cast<const f16x8*>(abase + G::PLANE + 1024 * t);
    };
    rd(0);
    if (TMAX > 1) rd(1);
#pragma unroll
    for (int t = 0; t < TMAX; ++t) {
      if (t + 2 < TMAX) rd(t + 2);
      __builtin_amdgcn_sched_barrier(0);
      if (!(SMCV_ABLATE & 1)) {
        f32x16 c;
        if constexpr (decltype(first)::value) {
          c = f32x16{};
        } else {
          c = acc[t];
        }
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(am[t % 3], bh, c, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t % 3], bm, c, 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t % 3], bh, c, 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ------------------------------------------------------------------------------ epilogue
  // Lane (lr, hh) holds, in block t, element i at R row jj = c_i + 4 hh (c_i = (i & 3) +
  // 8 (i >> 2)) and L column lr: local disparity dl = 32 (a + 1) + u - c_i with a = T-2-t and
  // u = lr - 4 hh.  dl lies in chunk a+1 (row u - c_i) when u >= c_i, else in chunk a (row
  // 32 + u - c_i).  Chunk m lives in ring slot (m + 3) % 3; for slot(a) != 2 the two slots are
  // adjacent and the address is one base plus a compile-time offset.  Block a completes chunk
  // a (chunk -1 and chunk T-1 hold only rows no one stores).
  const unsigned ring0 = lds_addr(smem + G::RING);
  const int u = lr - 4 * hh;
  const unsigned wbase = ring0 + 4u * (32 * wave + lr) + (unsigned)u * 512u;  // u >= -4
  const int srow = 8 * wave + hh;  // this lane's first store row in a chunk (+2 qq)
  const unsigned rbase = ring0 + (unsigned)srow * 512u + 16u * lr;
  const size_t plane_stride = (size_t)H * W;

  // SCALE: multiply back by 2^-(kL+kR); XLT: the segment has cells x < d (R pad rows), forced
  // to 0 (an R pad row can meet a NaN).  Compile-time, so the common case costs no VALU.
  auto epilogue_v = [&](const Work& k, bool fast, auto scale, auto xlt) {
    const bool fullx = k.x0 + kXT <= W;
    T* const olane = out + ((size_t)k.n * D + k.dp + srow) * plane_stride +
                         (size_t)k.y * W + k.x0 + 4 * lr;
    const bool okx = k.x0 + 4 * lr < W;
    const float mul = MEAN ? 1.0f / (float)C : 1.0f;
    const int kk = -(kL + kR);
    const int jlane = k.js + 32 * wave + 4 * hh;  // R row of element c_i of block 0, minus c_i
#pragma unroll
    for (int t = TMAX - 1; t >= 0; --t) {
      const int a = TMAX - 2 - t;
      const int sa = (a + 3) % 3, sb = (a + 4) % 3;  // slots of chunks a, a+1
      unsigned wb = wbase;
      asm volatile("" : "+v"(wb));  // per block: not hoisted (and spilled)
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ci = (i & 3) + 8 * (i >> 2);
        float val = acc[t][i];
        if (MEAN) val *= mul;
        if constexpr (decltype(scale)::value) val = __builtin_ldexpf(val, kk);
        if constexpr (decltype(xlt)::value) val = jlane + 32 * t + ci >= 0 ? val : 0.f;
        unsigned addr;
        if (sa != 2) {  // ring0 + col + slot(a+1) kSlot + (u - c_i) 512, both cases
          addr = wb + (unsigned)(sb * kSlot - ci * 512);
        } else {  // chunk a in slot 2, chunk a+1 in slot 0
          addr = wb + (unsigned)(3 * kSlot - ci * 512) - (u >= ci ? 3u * kSlot : 0u);
        }
        lds_store1(addr, val);
      }
      __syncthreads();
      if (a >= 0) {
        // chunk a is complete: this wave's quarter (8 rows, two per store instruction)
        const unsigned rb = rbase + (unsigned)sa * kSlot;
        f32x4v v[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) v[qq] = lds_load4(rb + 1024u * qq);
        T* ol = olane + (size_t)(32 * a) * plane_stride;
        asm volatile("" : "+v"(ol));
        if (fast) {  // every store valid: exactly 4 (T-1) per lane, counted by vm_wait
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) store_quad<T>(ol + (size_t)(2 * qq) * plane_stride, v[qq]);
        } else {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            const int dl = 32 * a + 2 * qq + srow;
            if (dl < k.Dp && (fullx || okx) && !(SMCV_ABLATE & 4))
              store_quad<T>(ol + (size_t)(2 * qq) * plane_stride, v[qq]);
          }
        }
      }
    }
  };

  auto epilogue = [&](const Work& k, bool fast) {
    using TT = std::true_type;
    using FF = std::false_type;
    const bool sc = __builtin_amdgcn_readfirstlane(kL + kR) != 0;
    const bool xl = __builtin_amdgcn_readfirstlane(k.js) < 0;
    if (sc) {
      if (xl) epilogue_v(k, fast, TT{}, TT{});
      else epilogue_v(k, fast, TT{}, FF{});
    } else {
      if (xl) epilogue_v(k, fast, FF{}, TT{});
      else epilogue_v(k, fast, FF{}, FF{});
    }
  };

  // exact fp32 path for a segment holding +-inf (or a scale fp32 cannot reach)
  auto slow_segment = [&](const Work& k) {
    const float mul = MEAN ? 1.0f / (float)C : 1.0f;
    const T* lrow = L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;
    const T* rrow = R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h;
    for (int idx = tid; idx < k.Dp * kXT; idx += kThreads) {
      const int dl = idx / kXT, x = k.x0 + idx % kXT, d = k.dp + dl;
      if (x >= W) continue;
      float s = 0.f;
      if (x >= d) {
        for (int c = 0; c < C; ++c) s = __builtin_fmaf(ld1(lrow + (int64_t)c * ls.c + x),
                                                       ld1(rrow + (int64_t)c * rs.c + x - d), s);
        s *= mul;
      }
      st1(out + (((size_t)k.n * D + d) * H + k.y) * W + x, s);
    }
  };

  // ----------------------------------------------------------------------------- main loop
  // maxima words: [0] max|L| parity 0, [1] max|R| parity 0, [2], [3] parity 1
  const unsigned maxw = lds_addr(smem + G::MAXW);
  if (tid < 4) *reinterpret_cast<__attribute__((address_space(3))) unsigned*>(maxw + 4 * tid) = 0u;
  bool redone = false;  // the current segment is a recomputation
  bool pend = false;    // 4 (T-1) output stores were issued after the outstanding feature loads
  // one pipeline step; returns true when the segment must be recomputed from its first step
  auto body = [&](int s) -> bool {
    const int it = s / nks;
    const int ks = s - it * nks;
    const Work k = decode(wbeg + gi + it * gsz, tiles, npass, H, D, pw, DMAX);
    if (ks == 0) mx = 0.f;
    __syncthreads();  // A: the previous step's fragment reads are done
    SM_STAMP(0);
    vm_wait<4 * (TMAX - 1)>(st.v, __builtin_amdgcn_readfirstlane((int)pend));
    pend = false;
    put(st);
    const unsigned par = (unsigned)(it & 1) * 8u;
    if (ks == nks - 1) {
      const float ml = wave_max(isR ? 0.f : mx), mr = wave_max(isR ? mx : 0.f);
      if (lane == 0) {
        __hip_atomic_fetch_max(lds_word(maxw + par), __float_as_uint(ml), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_max(lds_word(maxw + par + 4), __float_as_uint(mr), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      if (tid < 2)  // the next segment's words: last read before barrier A of this step
        *reinterpret_cast<__attribute__((address_space(3))) unsigned*>(maxw + (8u - par) + 4 * tid) = 0u;
    }
    SM_STAMP(1);
    load(st, s + 1);
    SM_STAMP(2);
    __syncthreads();  // B: the planes of step s are complete
    SM_STAMP(0);
    if (ks == 0)
      band(std::true_type{});
    else
      band(std::false_type{});
    SM_STAMP(3);
    if (ks != nks - 1) return false;
    // ---- end of a segment: range check, then the epilogue
    const float ml = __uint_as_float(*reinterpret_cast<__attribute__((address_space(3))) unsigned*>(maxw + par));
    const float mr = __uint_as_float(*reinterpret_cast<__attribute__((address_space(3))) unsigned*>(maxw + par + 4));
    const bool fin = ml <= 3.4e38f && mr <= 3.4e38f;  // no +-inf staged
    const int el = ml > 0.f ? exp_of(ml) : 0, er = mr > 0.f ? exp_of(mr) : 0;
    const bool okl = ml == 0.f || (el + kL <= 15 && el + kL >= -1);
    const bool okr = mr == 0.f || (er + kR <= 15 && er + kR >= -1);
    if (fin && okl && okr) {
      const bool fast = k.x0 + kXT <= W && k.Dp == DMAX && !(SMCV_ABLATE & 12);
      if (!(SMCV_ABLATE & 8)) epilogue(k, fast);
      pend = fast;  // exactly 4 (T-1) stores per lane were issued after the loads
      SM_STAMP(4);
      redone = false;
      return false;
    }
    const int nkl = ml > 0.f ? 13 - el : kL, nkr = mr > 0.f ? 13 - er : kR;
    if (!fin || redone || nkl < -100 || nkl > 100 || nkr < -100 || nkr > 100) {
      slow_segment(k);
      redone = false;
      return false;
    }
    kL = nkl;
    kR = nkr;
    redone = true;
    __syncthreads();  // every wave has read the maxima before they are cleared
    if (tid < 2)
      *reinterpret_cast<__attribute__((address_space(3))) unsigned*>(maxw + par + 4 * tid) = 0u;
    return true;
  };

  load(st, 0);
  for (int s = 0; s < S; ++s) {
    if (body(s)) {  // recompute the segment: restart its steps
      vm_wait<0>(st.v, 0);  // the registers must not have a load in flight when reloaded
      s = (s / nks) * nks;
      load(st, s);
      --s;
    }
  }
  vm_wait<0>(st.v, 0);  // the last (clamped) prefetch lands before its registers die
  SM_STAMP_FLUSH
}

int device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

// start offset of the second workgroup per CU, in units of 64 x 64 cycles (diagnostic override:
// STEREOCV_H2_STAGGER)
int stagger_units() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("STEREOCV_H2_STAGGER");
    v = e ? atoi(e) : 0;
  }
  return v;
}

template <typename T, int TMAX>
int launch(const T* l, const T* r, T* o, int64_t N, int64_t C, int64_t H, int64_t W,
           int64_t D, int64_t npass, int64_t pw, Strides4 ls, Strides4 rs, bool mean,
           hipStream_t st) {
  using G = Geo<TMAX>;
  const int tiles = (int)ceil_div(W, kXT);
  const int64_t nwork = (int64_t)tiles * H * N * npass;
  if (nwork > INT32_MAX / 64) return fail(SM_EINVAL, "inner product: too much work for one launch");
  auto kern = mean ? ip_band_h2<T, TMAX, true> : ip_band_h2<T, TMAX, false>;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::SHM);
  if (e != hipSuccess)
    return fail(SM_ELAUNCH, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  int64_t nwg = std::min<int64_t>(nwork, 2 * (int64_t)device_cus());
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(kThreads), G::SHM, st, l, r, o, (int)C,
                     (int)H, (int)W, (int)D, ls, rs, tiles, (int)npass, (int)pw, (int)nwork,
                     stagger_units());
  return check_launch("ip_band_h2");
}

}  // namespace h2band

int check_dot_args(const void* left, const void* right, const void* out, int dtype, int64_t N,
                   int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                   const int64_t* r_strides, Strides4* ls, Strides4* rs);

// Two-plane fp16 band kernel for fp32 / fp16 / bf16 features; *handled = false when the shape
// needs the generic path (4-pixel groups: W % 4 == 0, 4-element aligned rows and base
// pointers, C > 0).
int band_h2_entry(const void* left, const void* right, void* out, int dtype, int64_t N, int64_t C,
                  int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                  const int64_t* r_strides, int mode, void* stream, bool* handled) {
  *handled = false;
  Strides4 ls, rs;
  int rc = check_dot_args(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &ls, &rs);
  if (rc) return rc;
  const uintptr_t align = 4 * (uintptr_t)elem_size(dtype);
  const bool vec = (W % 4 == 0) && W >= 4 && C > 0 && ls.n % 4 == 0 && ls.c % 4 == 0 &&
                   ls.h % 4 == 0 && rs.n % 4 == 0 && rs.c % 4 == 0 && rs.h % 4 == 0 &&
                   ((reinterpret_cast<uintptr_t>(left) | reinterpret_cast<uintptr_t>(right)) % align == 0);
  if (!vec) return SM_OK;
  *handled = true;
  if (N == 0 || H == 0 || D == 0) return SM_OK;
  const bool mean = mode == 1;
  hipStream_t st = as_stream(stream);
  using namespace h2band;
  // D passes of at most 192 disparities, balanced (D = 256: two passes of 128); a pass width
  // that is a multiple of 4 keeps every right-window pixel group aligned
  const int64_t npass = ceil_div(D, (int64_t)192);
  const int64_t pw = (ceil_div(D, npass) + 3) / 4 * 4;
  SM_DISPATCH_DTYPE(dtype, T0, {
    using T = typename std::conditional<std::is_same<T0, bf16_t>::value, __bf16, T0>::type;
    const T* l = static_cast<const T*>(left);
    const T* r = static_cast<const T*>(right);
    T* o = static_cast<T*>(out);
    if (pw <= 32) return launch<T, 2>(l, r, o, N, C, H, W, D, npass, pw, ls, rs, mean, st);
    if (pw <= 64) return launch<T, 3>(l, r, o, N, C, H, W, D, npass, pw, ls, rs, mean, st);
    if (pw <= 128) return launch<T, 5>(l, r, o, N, C, H, W, D, npass, pw, ls, rs, mean, st);
    return launch<T, 7>(l, r, o, N, C, H, W, D, npass, pw, ls, rs, mean, st);
  });
  return SM_OK;
}

}  // namespace smcv

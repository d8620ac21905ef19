// Inner-product / correlation cost volume (N, D, H, W) from fp32 features, re-tiled for four
// waves per SIMD ("b16": 16-pixel waves on v_mfma_f32_16x16x32_f16).
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// The contraction, the operands (per-segment power-of-two scale, round-to-nearest two-plane fp16
// split, h*h' + h*m' + m*h' in fp32), the scale control, the exact fp32 path for segments the
// split cannot take and the hand-counted load pipeline are band_h2's (ip_h2.hip).  What changes
// is the tiling, so that the accumulators of a wave fit 128 registers and a SIMD holds four waves
// (band_h2's 32-pixel waves carry 7 x 16 = 112 accumulator registers and run two):
//   * a workgroup of 8 waves owns a 128-pixel row segment; wave w owns x-block w of 16 pixels
//     and its TB = 1 + DMAX/16 band blocks of 16 x 16 (13 blocks x 4 = 52 accumulator registers
//     for D = 192; the band's padding waste is 8 % instead of 17 %);
//   * a step stages 32 channels (one 16x16x32 k-step) into two 16-channel sub-planes per operand
//     plane, with band_h2's row swizzle (the 16x16x32 fragment reads -- lane l: row l & 15,
//     8-channel chunk l >> 4 -- are conflict-free on it too: scripts/check_swizzle.py);
//   * a 16 x 16 block shears through a private 2-slot ring of 16 d x 16 x fp32 chunks (1 KB):
//     two slots suffice because a wave's LDS operations execute in order, so block a+1's writes
//     into chunk a's slot follow chunk a's readout; one ds_read_b128 per lane reads a chunk and
//     one store instruction writes it, 16 volume rows x 64 B.
// LDS: 2 planes x 2 sub-planes x 448 rows x 32 B + 8 x 2 KB of rings = 72 KB per workgroup, two
// workgroups (16 waves) per CU.
#include "band_common.h"

namespace smcv {
namespace h2band {

#ifndef SMCV_B16_NT
#define SMCV_B16_NT 0  // volume stores: 0 plain (default), 1 non-temporal (A/B)
#endif
// A chunk row is 64 B, half a 128-B line whose other half the neighbouring wave writes.  Plain
// stores let L2 merge the two halves before the line goes to HBM; non-temporal 64-B pieces
// reach HBM as half-line writes (scripts/micro/store_patterns.hip: 16 rows x 64 B per store,
// 127 us non-temporal against 76 us plain for a cfg2 volume).
constexpr bool kB16NT = SMCV_B16_NT != 0;

constexpr int bWaves = 8;
constexpr int bThreads = 64 * bWaves;
constexpr int bXW = 16;             // pixels per wave
constexpr int bKC = 32;             // channels per step (one 16x16x32 k-step)
constexpr int bSlot = 16 * 16 * 4;  // one ring chunk: 16 d x 16 x fp32
static_assert(bXW * bWaves == kXT, "a segment is 8 waves of 16 pixels");

template <int TB>
struct GeoB {
  static constexpr int DMAX = 16 * (TB - 1);
  static constexpr int RW = kXT + DMAX;     // right-window rows
  static constexpr int ROWS = RW + kXT;     // + left-tile rows
  static constexpr int SUB = ROWS * 32;     // a 16-channel sub-plane (rows of 16 x fp16)
  static constexpr int PLANE = 2 * SUB;     // the step's 32 channels, h or m
  static constexpr int GROUPS = ROWS / 4;   // 4-pixel groups
  static constexpr int ITEMS = 4 * GROUPS;  // staging items: (4-pixel group, 8-channel chunk)
  static constexpr int RING = 2 * PLANE;    // the eight wave rings (2 KB each)
  static constexpr int MAXW = RING + bWaves * 2 * bSlot;  // max|L|, max|R| per segment parity
  static constexpr size_t SHM = (size_t)MAXW + 16;
  static_assert(ITEMS <= bThreads, "one staging item per lane");
  static_assert(GROUPS % 8 == 0, "8-lane write groups stay inside one chunk");
  static_assert(SUB % 1024 == 0, "sub-plane offsets leave the swizzled row bits alone");
  static_assert(SHM * 2 <= 160 * 1024, "two workgroups per CU");
};

// vm_wait (band_common.h) without the touch operand: wait for the 8 feature loads, letting the N
// output stores issued after them stay in flight when after_stores != 0
template <int N>
__device__ __forceinline__ void vm_wait_b(f32x4v (&v)[8], int after_stores) {
  asm volatile(
      "s_cmp_eq_u32 %8, 0\n\t"
      "s_cbranch_scc1 .Lvmb_all%=\n\t"
      "s_waitcnt vmcnt(%9)\n\t"
      "s_branch .Lvmb_done%=\n"
      ".Lvmb_all%=:\n\t"
      "s_waitcnt vmcnt(0)\n"
      ".Lvmb_done%=:"
      : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]),
        "+v"(v[7])
      : "s"(after_stores), "n"(N)
      : "memory", "scc");
}

template <bool MEAN, int TB>
__global__ __launch_bounds__(bThreads, 4) void band_b16(Args args) {
  using G = GeoB<TB>;
  constexpr int DMAX = G::DMAX;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const float* __restrict__ L = static_cast<const float*>(args.L);
  const float* __restrict__ R = static_cast<const float*>(args.R);
  float* __restrict__ out = static_cast<float*>(args.out);
  const int cpg = args.cpg, H = args.H, W = args.W, D = args.D;
  const Strides4 ls = args.ls, rs = args.rs;

  // the persistent schedule: XCD-grouped segment ranges, D passes consecutive (Sched)
  const Sched sched(args.nwork, args.npass);
  if (sched.none) return;  // the whole workgroup leaves together
  const int nitems = sched.nitems;
  auto witem = [&](int i) -> int { return sched.item(i); };
  const int nks = (cpg + bKC - 1) / bKC;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  SM_STAMP_DECL

  // ---------------------------------------------------------------- staging role of a lane
  const bool active = tid < G::ITEMS;
  const int ch = min(tid / G::GROUPS, 3);                  // 8-channel chunk of the step
  const int g = min(tid - ch * G::GROUPS, G::GROUPS - 1);  // rows 4g .. 4g+3
  const bool isR = 4 * g < G::RW;
  const int64_t cs = isR ? rs.c : ls.c;
  const bool cfull = __builtin_amdgcn_readfirstlane(cpg % bKC) == 0;

  struct Set {
    f32x4v v[8];
    int nv;  // valid channels of v (0: pixels outside the image or an idle lane)
  };
  Set st;
  auto row_of = [&](const Work& k) {
    return isR ? R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h
               : L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;
  };
  auto load = [&](Set& st, const Work& k, int ks) {
    const int cl = ks * bKC + 8 * ch;
    const int px = isR ? k.js + 4 * g : k.x0 + 4 * g - G::RW;
    const bool okp = active && px >= 0 && px < W;
    const float* p = row_of(k) + (okp ? px : 0) + (int64_t)min(cl, cpg - 1) * cs;
    if (SMCV_ABLATE & 2) p = L + 4 * (lane & 7);
    st.nv = okp ? min(max(cpg - cl, 0), 8) : 0;
    const int lim = cfull ? 7 : min(max(cpg - 1 - cl, 0), 7);
    int64_t csl = cs;
    asm volatile("" : "+v"(csl));
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      gload<true>(st.v[kk], p);
      if (kk < lim) p += csl;
    }
  };

  int kL = 0, kR = 0;  // per-segment scale exponents (workgroup-uniform)
  float mx = 0.f;      // this lane's max|x| over the current segment
  auto put = [&](Set& st) {
    if (!active || (SMCV_ABLATE & 16)) return;
    const float sc = __builtin_ldexpf(1.0f, isR ? kR : kL);
    auto stage = [&](const f32x4v (&v)[8]) {
      float m0 = mx, m1 = 0.f;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m0) : "v"(v[kk].x), "v"(v[kk].y));
        asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m1) : "v"(v[kk].z), "v"(v[kk].w));
      }
      mx = fmaxf(m0, m1);
      // the lane's staging offset: sub-plane ch >> 1, 16-B chunk ch & 1 of rows 4g .. 4g+3,
      // recomputed per step from an opaque thread index (registers are the scarce resource);
      // swz(4g + p, h) = swz(4g, h) ^ 32 p, and the sub-plane offset leaves bits 5-6 alone
      int ti = tid;
      asm volatile("" : "+v"(ti));
      const int tch = min(ti / G::GROUPS, 3), tg = ti - tch * G::GROUPS;
      const unsigned o0 = (unsigned)((tch >> 1) * G::SUB + swz(4 * tg, tch & 1));
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint4 wh, wm;
        split_pair(v[0][p], v[1][p], sc, wh.x, wm.x);
        split_pair(v[2][p], v[3][p], sc, wh.y, wm.y);
        split_pair(v[4][p], v[5][p], sc, wh.z, wm.z);
        split_pair(v[6][p], v[7][p], sc, wh.w, wm.w);
        const unsigned off = o0 ^ (32u * p);
        *reinterpret_cast<uint4*>(smem + off) = wh;
        *reinterpret_cast<uint4*>(smem + G::PLANE + off) = wm;
      }
    };
    if (__builtin_expect(__any(st.nv != 8), 0)) {  // row edges / channel tail only: zeroed in
#pragma unroll                                     // place (a copy would double the live set)
      for (int kk = 0; kk < 8; ++kk)
        if (kk >= st.nv) st.v[kk] = f32x4v{0.f, 0.f, 0.f, 0.f};
    }
    stage(st.v);
  };

  // ------------------------------------------------------------------- MFMA role of a wave
  // 16x16x32: lane l holds A[row l & 15][k 8 (l >> 4) .. +7] and B[k ..][col l & 15];
  // the accumulator element i of lane l is (row 4 (l >> 4) + i, col l & 15).
  f32x4v acc[TB];
  auto mma = [](f16x8 a, f16x8 b, f32x4v c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(a, b, c, 0, 0, 0);
  };
  auto band = [&](auto first) {
    // block t's A rows are 16 wave + 16 t + r16: swz flips the chunk bit with row bit 4, so even
    // and odd blocks differ in bit 4 of the address (ae, ae ^ 16), then + 512 t.  Derived per
    // step from an opaque lane index (no loop-invariant registers).
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int r16 = ln & 15, kc = ln >> 4;
    const unsigned bof = (unsigned)((kc >> 1) * G::SUB + swz(G::RW + 16 * wave + r16, kc & 1));
    const unsigned ae = (unsigned)((kc >> 1) * G::SUB + swz(16 * wave + r16, kc & 1));
    const f16x8 bh = *reinterpret_cast<const f16x8*>(smem + bof);
    const f16x8 bm = *reinterpret_cast<const f16x8*>(smem + G::PLANE + bof);
#pragma unroll
    for (int t = 0; t < TB; ++t) {
      // block t's fragments right before its MFMAs: four waves per SIMD cover the LDS latency
      const unsigned o = ((t & 1) ? (ae ^ 16u) : ae) + 512u * t;
      const f16x8 ah = *reinterpret_cast<const f16x8*>(smem + o);
      const f16x8 am = *reinterpret_cast<const f16x8*>(smem + G::PLANE + o);
      __builtin_amdgcn_sched_barrier(0);
      f32x4v c;
      if constexpr (decltype(first)::value) {
        c = f32x4v{0.f, 0.f, 0.f, 0.f};
      } else {
        c = acc[t];
      }
      if (!(SMCV_ABLATE & 1)) {
        c = mma(am, bh, c);
        c = mma(ah, bm, c);
        c = mma(ah, bh, c);
      }
      acc[t] = c;
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ------------------------------------------------------------------------------ epilogue
  // Block t (a = TB-2-t), lane (xl = l & 15, lg = l >> 4), element i: R row 4 lg + i, pixel
  // x0w + xl, local disparity 16 (a + 1) + u_i with u_i = xl - 4 lg - i: chunk a+1 row u_i when
  // u_i >= 0, else chunk a row 16 + u_i.  Ring [slot][16 d][16 x] (64-B rows), chunk m in slot
  // m & 1: the writes of a half-wave are at most 2-way on a bank (free for ds_write_b32), the
  // 16-B readouts (lane l: row l >> 2, pixels 4 (l & 3) ..) conflict-free.
  const size_t plane_stride = (size_t)H * W;

  // The lane constants of the epilogue are derived per segment from an opaque copy of the lane
  // index, so nothing of the epilogue stays live (in registers) across the steps.
  auto epilogue_v = [&](const Work& k, bool fast, auto scale, auto xlt) {
    int ln = lane;
    asm volatile("" : "+v"(ln));
    const int xl = ln & 15, lg = ln >> 4;
    const unsigned ringw = lds_addr(smem + G::RING) + (unsigned)(wave * 2 * bSlot);
    unsigned wv[4];  // ring addresses of the 4 elements for an even a (odd a: ^ 1024)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int u = xl - 4 * lg - i;
      wv[i] = ringw + (unsigned)(64 * (u & 15) + 4 * xl + (u >= 0 ? bSlot : 0));
    }
    const unsigned rdb = ringw + (unsigned)(16 * ln);
    const int x0w = k.x0 + bXW * wave;
    const float mul = args.mul;
    const int kk = -(kL + kR);
    const int jlane = k.js + 16 * wave + 4 * lg;  // R pixel of element i of block 0, minus i
    // the store pointer steps 16 planes per chunk (kept opaque: no per-chunk 64-bit offsets)
    float* ol = out + (((size_t)k.n * D + k.dp) * plane_stride + (size_t)k.y * W + x0w) +
                ((ln >> 2) * plane_stride + 4 * (ln & 3));
    const size_t st16 = (size_t)16 * plane_stride;
#pragma unroll
    for (int t = TB - 1; t >= 0; --t) {
      const int a = TB - 2 - t;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float val = acc[t][i];
        if (MEAN) val *= mul;
        if constexpr (decltype(scale)::value) val = __builtin_ldexpf(val, kk);
        if constexpr (decltype(xlt)::value) val = jlane + 16 * t + i >= 0 ? val : 0.f;
        // the ring wraps at 2 KB: chunk parity by XOR (the rings are 2-KB aligned in LDS)
        const unsigned addr = (a & 1) ? (wv[i] ^ (unsigned)bSlot) : wv[i];
        lds_store1(addr, val);
      }
      asm volatile("" ::: "memory");
      if (a >= 0) {
        const f32x4v v = lds_load4(rdb + (unsigned)((a & 1) * bSlot));
        asm volatile("" : "+v"(ol));
        if (SMCV_ABLATE & 4) {
          if (v[0] == 1.2345f) store_quad<kB16NT>(ol, v);  // keeps the readout live
        } else if (fast) {  // every store valid: exactly TB-1 per lane, counted by vm_wait_b
          store_quad<kB16NT>(ol, v);
        } else {
          const int dl = 16 * a + (ln >> 2);
          if (dl < k.Dp && x0w + 4 * (ln & 3) < W) store_quad<kB16NT>(ol, v);
        }
        ol += st16;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  auto epilogue = [&](const Work& k, bool fast) {
    using TT = std::true_type;
    using FF = std::false_type;
    const bool xl_ = __builtin_amdgcn_readfirstlane(k.js) < 0;
    if (__builtin_amdgcn_readfirstlane(kL + kR) != 0) {
      if (xl_)
        epilogue_v(k, fast, TT{}, TT{});
      else
        epilogue_v(k, fast, TT{}, FF{});
      return;
    }
    if (xl_)
      epilogue_v(k, fast, FF{}, TT{});
    else
      epilogue_v(k, fast, FF{}, FF{});
  };

  // exact fp32 path for a segment holding +-inf (or a scale the split cannot reach)
  auto slow_segment = [&](const Work& k) {
    const float mul = MEAN ? args.mul : 1.0f;
    const float* lrow = L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;
    const float* rrow = R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h;
    for (int idx = tid; idx < k.Dp * kXT; idx += bThreads) {
      const int dl = idx / kXT, x = k.x0 + idx % kXT, d = k.dp + dl;
      if (x >= W) continue;
      float s = 0.f;
      if (x >= d) {
        for (int c = 0; c < cpg; ++c)
          s = __builtin_fmaf(ld1(lrow + (int64_t)c * ls.c + x), ld1(rrow + (int64_t)c * rs.c + x - d), s);
        s *= mul;
      }
      store_one<float>(out + (((size_t)k.n * D + d) * H + k.y) * W + x, s);
    }
  };

  // ----------------------------------------------------------------------------- main loop
  const unsigned maxw = lds_addr(smem + G::MAXW);
  if (tid < 4) *lds_word(maxw + 4 * tid) = 0u;
  bool redone = false;  // the current segment is a recomputation
  bool pend = false;    // TB-1 output stores were issued after the outstanding feature loads
  auto body = [&](const Work& k, int it, int ks, const Work& nx, int ks1, bool more) -> bool {
    if (ks == 0) mx = 0.f;
    __syncthreads();  // A: the previous step's fragment reads are done
    SM_STAMP(0);
    vm_wait_b<TB - 1>(st.v, __builtin_amdgcn_readfirstlane((int)pend));
#ifdef SMCV_STAMPS
    if (ks == 0) SM_STAMP(5); else if (ks == 1) SM_STAMP(6); else SM_STAMP(7);
#endif
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
        *lds_word(maxw + (8u - par) + 4 * tid) = 0u;
    }
    SM_STAMP(1);
    if (more) load(st, nx, ks1);
    SM_STAMP(2);
    __syncthreads();  // B: the planes of step s are complete
    SM_STAMP(0);
    __builtin_amdgcn_s_setprio(1);
    if (ks == 0)
      band(std::true_type{});
    else
      band(std::false_type{});
    __builtin_amdgcn_s_setprio(0);
    SM_STAMP(3);
    if (ks != nks - 1) return false;
    // ---- end of a segment: range check, then the epilogue
    const bool fast = k.x0 + kXT <= W && k.Dp == DMAX;
    const float ml = __uint_as_float(*lds_word(maxw + par));
    const float mr = __uint_as_float(*lds_word(maxw + par + 4));
    const bool fin = ml <= 3.4e38f && mr <= 3.4e38f;  // no +-inf staged
    const int el = ml > 0.f ? exp_of(ml) : 0, er = mr > 0.f ? exp_of(mr) : 0;
    const bool okl = ml == 0.f || (el + kL <= 15 && el + kL >= -1);
    const bool okr = mr == 0.f || (er + kR <= 15 && er + kR >= -1);
    if (fin && okl && okr) {
      if (!(SMCV_ABLATE & 8)) epilogue(k, fast);
      pend = fast && !(SMCV_ABLATE & 12);  // exactly TB-1 stores per lane were issued after the loads
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
    if (tid < 2) *lds_word(maxw + par + 4 * tid) = 0u;
    return true;
  };

  Work cur = decode(witem(0), args, DMAX);
  load(st, cur, 0);
  for (int it = 0, ks = 0; it < nitems;) {
    const bool last = ks == nks - 1;
    const bool more = !last || it + 1 < nitems;
    const Work nx = last && more ? decode(witem(it + 1), args, DMAX) : cur;
    if (body(cur, it, ks, nx, last ? 0 : ks + 1, more)) {  // recompute the segment
      vm_wait_b<0>(st.v, 0);  // no load in flight when the registers are reloaded
      ks = 0;
      load(st, cur, 0);
      continue;
    }
    if (last) {
      cur = nx;
      ++it;
      ks = 0;
    } else {
      ++ks;
    }
  }
  vm_wait_b<0>(st.v, 0);  // nothing in flight when the registers die
  SM_STAMP_FLUSH
}

template <bool MEAN, int TB>
int launch_b16(Args a, int64_t N, hipStream_t st) {
  using G = GeoB<TB>;
  a.tiles = (int)ceil_div(a.W, kXT);
  const int64_t nwork = (int64_t)a.tiles * a.H * N * a.G * a.npass;
  if (nwork > INT32_MAX / 64) return fail(SM_EINVAL, "band kernel: too much work for one launch");
  a.nwork = (int)nwork;
  auto kern = band_b16<MEAN, TB>;
  static std::atomic<unsigned long long> lds_done{0};  // per instantiation
  const int dev = stream_device(st);
  if (int rc = ensure_lds_limit(reinterpret_cast<const void*>(kern), (int)G::SHM, dev, lds_done))
    return rc;
  int64_t nwg = std::min<int64_t>(nwork, 2 * (int64_t)device_cus(dev));
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(bThreads), G::SHM, st, a);
  return check_launch("band_b16");
}

// fp32 inner product / correlation volume on the b16 kernel: *handled = false when the shape is
// not one it takes (the caller then runs band_h2).  `a` comes from h2_prepare.
int band_b16_run(const Args& a, int64_t N, bool mean, bool aligned4, hipStream_t st,
                 bool* handled) {
  *handled = false;
  if (!aligned4 || a.G != 1 || (int64_t)16 * a.H * a.W >= INT32_MAX || a.pw > 192) return SM_OK;
  *handled = true;
  auto go = [&](auto tb) {
    constexpr int TB = decltype(tb)::value;
    return mean ? launch_b16<true, TB>(a, N, st) : launch_b16<false, TB>(a, N, st);
  };
  if (a.pw <= 32) return go(std::integral_constant<int, 3>{});
  if (a.pw <= 64) return go(std::integral_constant<int, 5>{});
  if (a.pw <= 128) return go(std::integral_constant<int, 9>{});
  if (mean) {  // the correlation's 1/C scaling does not fit 128 registers at TB = 13: band_h2
    *handled = false;
    return SM_OK;
  }
  return launch_b16<false, 13>(a, N, st);
}

}  // namespace h2band
}  // namespace smcv

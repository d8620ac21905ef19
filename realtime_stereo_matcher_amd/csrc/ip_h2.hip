// Band cost volumes on gfx950 matrix cores ("h2" kernels): inner product / correlation
// (N, D, H, W), groupwise (N, G, H, W, D), and the inner product fused with soft-argmin.
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//            TorchGroupwiseCost.forward      cost_volume/groupwise.py:24-56 (mean per group, D last)
//            disparity_regression            model/mobile_disp_net_c.py:208-220 (fused variant)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// Per image row the volume is a band of the contraction S[j][x] = sum_c R[c][j] L[c][x]
// (d = x - j).  A workgroup (4 waves) owns a 128-pixel row segment of one channel group; wave w
// owns x-block w (32 pixels) and its T = 1 + DMAX/32 32x32 band blocks, accumulated on the
// matrix cores.  Every wave does everything (load, stage, MFMA, shear, store) and the CU holds
// TWO such workgroups, so one workgroup's output stream overlaps the other's loads and MFMAs.
//
// Operands.  fp16 / bf16 features are staged as they are (one plane; their products are exact
// in fp32: one MFMA per block and 16-channel step).  fp32 features are scaled by a per-segment
// power of two 2^k (exact) and split into two fp16 planes by round-to-nearest:
// h = rn16(x 2^k), m = rn16(x 2^k - h), so x 2^k = h + m + e with |e| <= 2^-22 |x 2^k|
// (+ 2^-25 absolute below the fp16 normal range); the products h*h' + h*m' + m*h' (exact in
// fp32; the dropped m*m', h*e', e*h' are each at most 2^-22 relative) accumulate in fp32, and
// the result is multiplied back by 2^-(kL+kR) (ldexp, exact).  Integer features are exact.
//
// Scale control (fp32).  Every lane tracks max|x| of the values it stages; at the end of a
// segment the workgroup knows max|L| and max|R| over everything it staged.  The segment is
// accepted when both scaled maxima lie in [2^-2, 2^15) (or are 0); otherwise it is recomputed
// with k = 13 - exponent(max) (scaled maximum in [2^12, 2^13)), and that k carries to the next
// segment, so smoothly varying feature scales cost nothing.  Segments holding +-inf (or a scale
// fp32 cannot reach) take an exact fp32 FMA path.  NaN needs no special case: it propagates
// through the split and the products like through the reference sum.  Cells x < d are forced
// to 0 as in the reference (an R pad row can meet a NaN or an inf).
//
// Data flow per 16-channel step (one barrier pair): the step's features were loaded into
// registers one step earlier (inline-asm loads whose vmcnt is counted by hand, so the output
// stores stay in flight: vm_wait), and their 128-B lines were touched into L2 one step before
// that (touch); barrier A (the previous step's fragment reads are done), stage into the
// plane(s) in LDS (row/chunk XOR swizzle: conflict-free 16-B writes and fragment reads,
// scripts/check_swizzle.py), issue the loads of the next step and the touches of the one after,
// barrier B, MFMAs.  After a segment's last step each wave shears its accumulators (d = x - j)
// block by block through a private 3-slot ring of 32 x 32 chunks -- no barrier -- and streams
// every completed chunk out: NDHW as 8 rows x 128 B per store instruction, NGHWD as 8 pixels x
// 128 B of d.
//
// Fused soft-argmin (FUSE).  While a chunk is in registers for its stores, each lane folds its
// 4 rows x 4 pixels into an online softmax (running max; sums of e and d*e per chunk in fp32
// relative to the chunk's first row, across chunks in fp64); the 8 lanes of a pixel column
// merge by cross-lane shuffles after the last chunk, so the segment's disparities leave the
// same pass -- with or without the volume.
#include "band_common.h"

#ifndef SMCV_STORE_THROTTLE
#define SMCV_STORE_THROTTLE 0
#endif

namespace smcv {
namespace h2band {

constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kKC = 16;             // channels per step (one 32x32x16 k-step)
constexpr int kRowB = 32;           // bytes per plane row: 16 x 16-bit
constexpr int kSlot = 32 * 32 * 4;  // one ring chunk: 32 x 32 fp32
constexpr int kRingW = 3 * kSlot;   // a wave's ring
enum { kNDHW = 0, kNGHWD = 1 };


template <typename T, int TMAX>
struct Geo {
  static constexpr int NP = sizeof(T) == 4 ? 2 : 1;  // operand planes
  static constexpr int DMAX = 32 * (TMAX - 1);
  static constexpr int RW = kXT + DMAX;   // right-window rows
  static constexpr int ROWS = RW + kXT;   // + left-tile rows
  static constexpr int PLANE = ROWS * kRowB;
  static constexpr int GROUPS = ROWS / 4; // 4-pixel groups per 8-channel chunk
  static constexpr int ITEMS = 2 * GROUPS;
  static constexpr int RING = NP * PLANE;              // the four wave rings
  static constexpr int MAXW = RING + kWaves * kRingW;  // max|L|, max|R| for segment parity 0/1
  static constexpr size_t SHM = (size_t)MAXW + 16;
  static_assert(ITEMS <= kThreads, "one staging item per lane");
  static_assert(GROUPS % 8 == 0, "8-lane write groups stay inside one chunk");
  static_assert(SHM * 2 <= 160 * 1024, "two workgroups per CU");
};






// Workgroups per CU: two (each wave owns 256 registers); the fused kernels too, since their
// soft-argmin runs on the accumulators themselves before the shear.
template <int FUSE>
constexpr int wg_per_cu() {
  return 2;
}

template <typename T, typename TO, int TMAX, bool MEAN, int LAYOUT, int FUSE>
__global__ __launch_bounds__(kThreads, wg_per_cu<FUSE>()) void band_h2(Args args) {
  using G = Geo<T, TMAX>;
  constexpr int DMAX = G::DMAX;
  constexpr int NP = G::NP;
  // Every instantiation (the fused ones too) runs two workgroups per CU with hand-counted asm
  // feature loads: vm_wait names how many younger vector-memory operations may stay in flight
  // after a segment -- 4 (T-1) volume stores (+1 disparity store for FUSE 1), one disparity
  // store for FUSE 2 -- and scripts/check_h2_asm.py verifies the count on the compiled asm.
  constexpr bool ASM = true;
  constexpr int PF = ASM ? kPF : 0;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const T* __restrict__ L = static_cast<const T*>(args.L);
  const T* __restrict__ R = static_cast<const T*>(args.R);
  TO* __restrict__ out = static_cast<TO*>(args.out);
  const int cpg = args.cpg, H = args.H, W = args.W, D = args.D;
  const Strides4 ls = args.ls, rs = args.rs;

  // the persistent schedule: XCD-grouped segment ranges, D passes consecutive (Sched)
  const Sched sched(args.nwork, args.npass);
  if (sched.none) return;  // the whole workgroup leaves together
  const int nitems = sched.nitems;
  auto witem = [&](int i) -> int { return sched.item(i); };
  const int nks = (cpg + kKC - 1) / kKC;
  const bool store_vol = FUSE != 2 && __builtin_amdgcn_readfirstlane(args.out != nullptr ? 1 : 0) != 0;
  // NGHWD quads are 16-B aligned only when D % 4 == 0
  const bool dq = LAYOUT == kNDHW || __builtin_amdgcn_readfirstlane(D & 3) == 0;

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
  const bool cfull = __builtin_amdgcn_readfirstlane(cpg % kKC) == 0;  // uniform: a scalar branch

  using QT = typename Quad<T>::type;
  struct Set {
    QT v[8];
    int nv;  // valid channels of v (0: pixels outside the image or an idle lane)
  };
  Set st;  // one set: the loads of step s+1 fly during step s's matrix work
  auto row_of = [&](const Work& k) {
    return isR ? R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h
               : L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;
  };
  auto load = [&](Set& st, const Work& k, int ks) {
    const int cl = ks * kKC + 8 * ch;  // channel within the group
    const int px = isR ? k.js + 4 * g : k.x0 + 4 * g - G::RW;
    const bool okp = active && px >= 0 && px < W;
    // W % 4 != 0 (fp32 only): the group holding a row's end reads the row's last 4 pixels
    // (W - 4 .. W - 1, in bounds) and put() moves its W % 4 valid pixels down; flagged in nv
    const bool strad = NP == 2 && okp && px + 4 > W;
    const T* p = row_of(k) + (okp ? (strad ? W - 4 : px) : 0) + ((int64_t)k.g * cpg + min(cl, cpg - 1)) * cs;
    if (SMCV_ABLATE & 2) p = L + 4 * (lane & 7);
    st.nv = (okp ? min(max(cpg - cl, 0), 8) : 0) | (strad ? 16 : 0);
    // channel tail: clamp to the group's last channel (one code path; put() zeroes the tail)
    const int lim = cfull ? 7 : min(max(cpg - 1 - cl, 0), 7);
    // the channel stride, opaque here: the 8 addresses are stepped, not 8 hoisted 64-bit offsets
    int64_t csl = cs;
    asm volatile("" : "+v"(csl));
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      gload<ASM>(st.v[kk], p);
      if (kk < lim) p += csl;
    }
  };
  // Touch every 128-B line a later step loads: lane (ch, g) loads one dword of channel
  // 8 ch + (g & 7) of its own pixel group -- the 8 groups of a line cover the line's 8
  // channels -- so that step's real loads find their lines in L2.  Lanes with nothing to touch
  // (and invalid steps) reload L[0]: every lane issues exactly kPF touches per step.
  unsigned pfd = 0;  // the touches' destination: never read, live until the final wait
  auto touch = [&](const Work& k, int ks, bool valid) {
    if constexpr (PF != 0) {
      const int cl = ks * kKC + 8 * ch + (g & 7);
      const int px = isR ? k.js + 4 * g : k.x0 + 4 * g - G::RW;
      const bool ok = valid && active && px >= 0 && px < W && cl < cpg;
      const T* p = ok ? row_of(k) + px + ((int64_t)k.g * cpg + cl) * cs : L;
      asm volatile("global_load_dword %0, %1, off" : "+v"(pfd) : "v"(p) : "memory");
    }
  };

  int kL = 0, kR = 0;  // per-segment scale exponents (workgroup-uniform; fp32 only)
  float mx = 0.f;      // this lane's max|x| over the current segment (fp32 only)
  // stage one step into the plane(s)
  auto put = [&](Set& st) {
    if (!active || (SMCV_ABLATE & 16)) return;
    if constexpr (NP == 2) {
      const float sc = __builtin_ldexpf(1.0f, isR ? kR : kL);  // 2^k (1.0 when unscaled)
      // max |x| and the split, straight from the loaded registers (no copies): v_max3 with |.|
      // modifiers, two values per instruction in two chains (fmaxf would canonicalise every
      // loaded value first), then four v_fma_mix per value pair
      auto stage = [&](const f32x4v (&v)[8]) {
        float m0 = mx, m1 = 0.f;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m0) : "v"(v[kk].x), "v"(v[kk].y));
          asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m1) : "v"(v[kk].z), "v"(v[kk].w));
        }
        mx = fmaxf(m0, m1);
        // swz(4g + p, ch) = swz(4g, ch) ^ 32 p (p only flips the row bits 5-6, which hold g & 3):
        // one opaque base per step, so the compiler keeps one register instead of four
        // loop-invariant offsets (which spilled, and every reload waited for vmcnt(0))
        unsigned o0 = (unsigned)swz(4 * g, ch);
        asm volatile("" : "+v"(o0));
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
      if (__builtin_expect(__any(st.nv != 8), 0)) {  // row edges / channel tail only
        f32x4v v[8];
        const int nv = st.nv & 15;
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) v[kk] = kk < nv ? st.v[kk] : f32x4v{0.f, 0.f, 0.f, 0.f};
        if (st.nv & 16) {  // loaded from W - 4: pixels W - r .. W - 1 move to lanes' slots 0 .. r-1
          const int r = W & 3;  // 1, 2 or 3 (uniform); element-wise selects
          const bool r1 = r == 1, r2 = r == 2;
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) {
            const f32x4v o = v[kk];
            f32x4v n;
            n.x = r1 ? o.w : (r2 ? o.z : o.y);
            n.y = r1 ? 0.f : (r2 ? o.w : o.z);
            n.z = (r1 || r2) ? 0.f : o.w;
            n.w = 0.f;
            v[kk] = n;
          }
        }
        stage(v);
      } else {
        stage(st.v);
      }
    } else {
      // 16-bit features as they are: 8 channels x 4 pixels -> 4 rows of 8 channels
      u32x2 qv[8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) qv[kk] = st.v[kk];
      if (__any(st.nv != 8)) {
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
          if (kk >= st.nv) qv[kk] = u32x2{0u, 0u};
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint4 w;
        unsigned* pw = reinterpret_cast<unsigned*>(&w);
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // channels 2j (low half), 2j+1 (high half) of pixel p
          const unsigned lo = p < 2 ? qv[2 * j].x : qv[2 * j].y;
          const unsigned hi = p < 2 ? qv[2 * j + 1].x : qv[2 * j + 1].y;
          pw[j] = __builtin_amdgcn_perm(hi, lo, (p & 1) ? 0x07060302u : 0x05040100u);
        }
        *reinterpret_cast<uint4*>(smem + swz(4 * g + p, ch)) = w;
      }
    }
  };

  // ------------------------------------------------------------------- MFMA role of a wave
  const int lr = lane & 31;
  const int hh = lane >> 5;
  const unsigned char* abase = smem + 32 * wave * kRowB + swz(lr, hh);  // + 1024 t
  const unsigned char* bbase = smem + (G::RW + 32 * wave) * kRowB + swz(lr, hh);
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
  auto band = [&](auto first) {
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
      if (!(SMCV_ABLATE & 1)) {
        f32x16 c;
        if constexpr (decltype(first)::value) {
          c = f32x16{};
        } else {
          c = acc[t];
        }
        if constexpr (NP == 2) {
          c = mma(am[t % NB], bh, c);
          c = mma(ah[t % NB], bm, c);
        }
        acc[t] = mma(ah[t % NB], bh, c);
      } else {  // diagnostic: operands consumed, accumulators opaque (the epilogue stays whole)
        asm volatile("" : "+v"(acc[t]) : "v"(ah[t % NB]), "v"(bh));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ------------------------------------------------------------------------------ epilogue
  // Lane (lr, hh) holds, in block t, element i at R row jj = c_i + 4 hh (c_i = (i & 3) +
  // 8 (i >> 2)) and L column lr: local disparity dl = 32 (a + 1) + u - c_i with a = T-2-t and
  // u = lr - 4 hh, i.e. chunk a+1 (row u - c_i) when u >= c_i, else chunk a (row 32 + u - c_i).
  // Block a completes chunk a of the wave (chunk -1 and chunk T-1 hold only rows no one reads).
  //   NDHW ring: [slot][32 d][32 x], chunk m in slot m % 3 (adjacent slots: one base + a
  //   compile-time offset; slot 2 -> 0 wraps with one select);
  //   NGHWD ring: [32 x][96 d, circular], chunk m at d-positions 32 (m % 3) .. +32.
  // Both write patterns are conflict-free (132 / 388 B lane strides in a 32-lane half), and so
  // are the 16-B readouts (scripts/check_h2_bounds.py).
  const unsigned ringw = lds_addr(smem + G::RING) + (unsigned)(wave * kRingW);
  const int u = lr - 4 * hh;
  const unsigned wbase = LAYOUT == kNDHW ? ringw + (unsigned)(4 * lr + 128 * u)
                                         : ringw + (unsigned)(384 * lr + 4 * u);
  const int rl = lane >> 3, cl = lane & 7;  // chunk readout: rows (NDHW) / pixels (NGHWD) 8qq + rl
  const size_t plane_stride = (size_t)H * W;
  const bool ntq = __builtin_amdgcn_readfirstlane(W & 3) == 0;  // see store_quad
  // lane parts of the chunk store addresses, in elements (32-bit: the host keeps 8 H W < 2^31);
  // the rest of each address is uniform (scalar registers)
  const int lane_st = LAYOUT == kNDHW ? rl * H * W + 4 * cl : rl * D + 4 * cl;
  const unsigned rdbase = LAYOUT == kNDHW ? ringw + (unsigned)(rl * 128 + 16 * cl)
                                          : ringw + (unsigned)(rl * 384 + 16 * cl);

  // Fused soft-argmin straight from the accumulators (fused_softargmin, band_common.h; shared
  // with band_h2db's FUSE 1).  No ring, no LDS: the volume-free kernel never shears.
  // (fp16 / bf16 features: exact products, no scale -- SCALE is false for them)
  // args.round (fp16 / bf16 features under autocast, the default): the fold sees each cell
  // rounded to the feature dtype, as the reference's volume holds it
  auto fuse_regs = [&](const Work& k, auto scale, auto xlt) {
    constexpr bool SC = decltype(scale)::value, XL = decltype(xlt)::value;
    if constexpr (std::is_same<T, float>::value) {
      fused_softargmin<TMAX, MEAN, SC, XL>(acc, args, k, kL, kR, wave, lr, hh);
    } else {
      if (args.round)
        fused_softargmin<TMAX, MEAN, SC, XL, true, T>(acc, args, k, kL, kR, wave, lr, hh);
      else
        fused_softargmin<TMAX, MEAN, SC, XL>(acc, args, k, kL, kR, wave, lr, hh);
    }
  };

  // SCALE: multiply back by 2^-(kL+kR); XLT: the segment has cells x < d (R pad rows), forced
  // to 0.  Compile-time, so the common case costs no VALU.
  auto epilogue_v = [&](const Work& k, bool fast, auto scale, auto xlt, auto ntc) {
    constexpr bool NTQ = decltype(ntc)::value;
    const int x0w = k.x0 + 32 * wave;  // this wave's first pixel
    const float mul = args.mul;
    const int kk = -(kL + kR);
    const int jlane = k.js + 32 * wave + 4 * hh;  // R row of element c_i of block 0, minus c_i
    if constexpr (FUSE != 0) {
      fuse_regs(k, scale, xlt);
      if (FUSE == 2 || !store_vol) return;  // the volume-free pass: no shear, no ring, no stores
    }
    // Block t writes its 16 cells into the ring (chunks a and a+1, a = T-2-t); chunk a is then
    // complete and is read back (4 x 16 B per lane) and stored.  Software-pipelined (PIPE): the
    // readout of chunk a is consumed only after block t-1's ring writes are issued, so its LDS
    // latency hides behind them instead of stalling the wave once per block (the 3-slot ring
    // keeps chunk a's slot apart from the chunks block t-1 writes, and a wave's LDS operations
    // execute in order anyway).
    constexpr bool PIPE = FUSE == 0;
    auto write_block = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int a = TMAX - 2 - t;
      // per block, opaque to the compiler: the per-element addresses and selects below are
      // recomputed in each block (two VALU each) instead of being hoisted out of the block loop
      // as 16+ loop-invariant registers (which spill at two workgroups per CU)
      unsigned wb = wbase;
      int uu = u, jl = jlane;
      asm volatile("" : "+v"(wb), "+v"(uu), "+v"(jl));
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ci = (i & 3) + 8 * (i >> 2);
        float val = acc[t][i];
        if (MEAN) val *= mul;
        if constexpr (decltype(scale)::value) val = __builtin_ldexpf(val, kk);
        if constexpr (decltype(xlt)::value) val = jl + 32 * t + ci >= 0 ? val : 0.f;
        unsigned addr;
        if constexpr (LAYOUT == kNDHW) {
          const int sA = (a + 3) % 3, sB = (a + 4) % 3;  // slots of chunks a, a+1
          if (sA != 2) {
            addr = wb + (unsigned)(sB * kSlot - ci * 128);
          } else {  // chunk a in slot 2, chunk a+1 in slot 0
            // the wrap amount is selected, kept opaque, and subtracted; the constant part folds
            // into the ds_write offset (left to itself the compiler hoists 32 constants, one pair
            // per element, into VGPRs for the whole kernel -- which then spilled)
            unsigned sel = uu >= ci ? 3u * kSlot : 0u;
            asm volatile("" : "+v"(sel));
            addr = (wb - sel) + (unsigned)(3 * kSlot - ci * 128);
          }
        } else {
          const int bp = 32 * ((a + 4) % 3);  // ring d-position of local disparity 32 (a+1)
          if (bp != 0) {
            addr = wb + (unsigned)(4 * (bp - ci));
          } else {  // u < c_i wraps to the top of the 96-entry circle (wrap kept opaque, as above)
            unsigned sel = uu >= ci ? 384u : 0u;
            asm volatile("" : "+v"(sel));
            addr = (wb - sel) + (unsigned)(4 * (96 - ci));
          }
        }
        if (!(SMCV_ABLATE & 32)) lds_store1(addr, val);
      }
      // the wave's own ring writes precede its reads (LDS executes a wave's operations in order)
      asm volatile("" ::: "memory");
    };
    auto read_chunk = [&](auto tc, f32x4v (&v)[4]) {
      constexpr int t = decltype(tc)::value;
      constexpr int a = TMAX - 2 - t;
      unsigned rb = rdbase;
      asm volatile("" : "+v"(rb));
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const unsigned ra = LAYOUT == kNDHW ? rb + (unsigned)((a % 3) * kSlot + 8 * qq * 128)
                                            : rb + (unsigned)(8 * qq * 384 + (a % 3) * 128);
        if constexpr ((SMCV_ABLATE & 32) != 0)
          v[qq] = f32x4v{acc[t][4 * qq], acc[t][4 * qq + 1], acc[t][4 * qq + 2], acc[t][4 * qq + 3]};
        else
          v[qq] = lds_load4(ra);
      }
    };
    auto store_chunk = [&](int a, const f32x4v (&v)[4]) {
      if (!store_vol) return;
      int ls_ = lane_st, rlo = rl, clo = cl;
      asm volatile("" : "+v"(ls_), "+v"(rlo), "+v"(clo));
      if constexpr (LAYOUT == kNDHW) {
        TO* ol = out + (((size_t)k.n * D + k.dp + 32 * a) * plane_stride +
                        (size_t)k.y * W + x0w) + ls_;
        // rows 8 apart: one uniform stride, the pointer stepped store by store (kept
        // opaque, so no 64-bit per-row offsets are hoisted into registers)
        const size_t st8 = (size_t)8 * plane_stride;
        if (fast) {  // every store valid: exactly 4 (T-1) per lane, counted by vm_wait
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            asm volatile("" : "+v"(ol));
            store_quad<NTQ>(ol, v[qq]);
            ol += st8;
          }
        } else {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            asm volatile("" : "+v"(ol));
            const int dl = 32 * a + 8 * qq + rlo;
            const int xq = x0w + 4 * clo;
            if (dl < k.Dp && xq < W && !(SMCV_ABLATE & 4)) {
              if (xq + 4 <= W) {
                store_quad<NTQ>(ol, v[qq]);
              } else {  // the row's last, partial quad (W % 4 != 0)
#pragma unroll
                for (int e = 0; e < 3; ++e)
                  if (xq + e < W) store_one<TO>(ol + e, v[qq][e]);
              }
            }
            ol += st8;
          }
        }
      } else {
        const size_t pix = (((size_t)k.n * args.G + k.g) * H + k.y) * (size_t)W + x0w;
        TO* ol = out + (pix * (size_t)D + k.dp + 32 * a) + ls_;
        asm volatile("" : "+v"(ol));
        if (fast) {
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) store_quad<true>(ol + (size_t)(8 * qq) * D, v[qq]);
        } else {
          const int d0 = 32 * a + 4 * clo;
#pragma unroll
          for (int qq = 0; qq < 4; ++qq) {
            if (x0w + 8 * qq + rlo >= W || (SMCV_ABLATE & 4)) continue;
            if (d0 + 4 <= k.Dp && dq) {
              store_quad<true>(ol + (size_t)(8 * qq) * D, v[qq]);
            } else {
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (d0 + e < k.Dp) store_one<TO>(ol + (size_t)(8 * qq) * D + e, v[qq][e]);
            }
          }
        }
      }
    };
    f32x4v vp[4];  // the readout of the previous block's chunk (PIPE)
    [&]<int... I_>(std::integer_sequence<int, I_...>) {
      (
          [&] {
            constexpr int t = TMAX - 1 - I_;
            constexpr int a = TMAX - 2 - t;
            write_block(std::integral_constant<int, t>{});
            if constexpr (PIPE) {
#if SMCV_STORE_THROTTLE
              // at most SMCV_STORE_THROTTLE of this wave's stores in flight (the feature loads,
              // older, complete first): experiment
              if constexpr (a >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(SMCV_STORE_THROTTLE) : "memory");
#endif
              if constexpr (a >= 1) store_chunk(a - 1, vp);
              if constexpr (a >= 0) read_chunk(std::integral_constant<int, t>{}, vp);
            } else if constexpr (a >= 0) {
              f32x4v v[4];
              read_chunk(std::integral_constant<int, t>{}, v);
              store_chunk(a, v);
            }
            // one block at a time (the live accumulators shrink block by block)
            __builtin_amdgcn_sched_barrier(0);
          }(),
          ...);
    }(std::make_integer_sequence<int, TMAX>{});
    if constexpr (PIPE && TMAX >= 2) store_chunk(TMAX - 2, vp);
  };

  auto epilogue_n = [&](const Work& k, bool fast, auto ntc) {
    using TT = std::true_type;
    using FF = std::false_type;
    const bool xl = __builtin_amdgcn_readfirstlane(k.js) < 0;
    if constexpr (NP == 2) {
      if (__builtin_amdgcn_readfirstlane(kL + kR) != 0) {
        if (xl)
          epilogue_v(k, fast, TT{}, TT{}, ntc);
        else
          epilogue_v(k, fast, TT{}, FF{}, ntc);
        return;
      }
    }
    if (xl)
      epilogue_v(k, fast, FF{}, TT{}, ntc);
    else
      epilogue_v(k, fast, FF{}, FF{}, ntc);
  };
  // non-temporal NDHW stores unless an fp32 row's 16-B pieces straddle lines (W % 4 != 0)
  auto epilogue = [&](const Work& k, bool fast) {
    if (LAYOUT != kNDHW || ntq)
      epilogue_n(k, fast, std::true_type{});
    else
      epilogue_n(k, fast, std::false_type{});
  };

  // exact fp32 path for a segment holding +-inf (or a scale fp32 cannot reach)
  auto slow_segment = [&](const Work& k) {
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
      for (int idx = tid; idx < k.Dp * kXT; idx += kThreads) {
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
    if constexpr (FUSE != 0) {
      for (int xx = tid; xx < kXT; xx += kThreads) {
        const int x = k.x0 + xx;
        if (x >= W) continue;
        float m = -INFINITY;
        double s = 0.0, t = 0.0;  // relative to m; t over the pass-local d
        bool nan = false;
        for (int d = 0; d < k.Dp; ++d) {
          const float v = cell(x, k.dp + d);
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
        const size_t px = ((size_t)k.n * H + k.y) * W + x;
        if (args.ws_m != nullptr) {
          // one of several D passes: the same partial state as fuse_regs (d global); a NaN cell or
          // a +inf maximum is carried as s = NaN, which fused_merge_kernel propagates; an all -inf
          // pass (s = 0, m = -inf) contributes nothing, and all -inf passes give 0 / 0 = NaN
          typedef __attribute__((address_space(1))) void gvoid;
          const size_t o = (size_t)k.pass * ((size_t)args.nhw) + px;
          const double sv = (nan || m == INFINITY) ? (double)NAN : s;
          *reinterpret_cast<__attribute__((address_space(1))) double*>((gvoid*)(args.ws_s + o)) = sv;
          *reinterpret_cast<__attribute__((address_space(1))) double*>((gvoid*)(args.ws_t + o)) =
              t + (double)k.dp * sv;
          store_one<float>(args.ws_m + o, m);
        } else {
          store_one<float>(args.disp + px,
                           (nan || m == INFINITY || m == -INFINITY) ? NAN : (float)(t / s));
        }
      }
    }
  };

  // ----------------------------------------------------------------------------- main loop
  // maxima words: [0] max|L| parity 0, [1] max|R| parity 0, [2], [3] parity 1
  const unsigned maxw = lds_addr(smem + G::MAXW);
  if (tid < 4) *lds_word(maxw + 4 * tid) = 0u;
  bool redone = false;  // the current segment is a recomputation
  bool pend = false;    // 4 (T-1) output stores were issued after the outstanding feature loads
  // One pipeline step: channel step ks of item it (work k); nx / ks1 name the next step, whose
  // loads this step issues (none after the last), pk / pks / pv the step after that, whose lines
  // it touches.  Returns true when the segment must be recomputed from its first step.
  auto body = [&](const Work& k, int it, int ks, const Work& nx, int ks1, bool more,
                  const Work& pk, int pks, bool pv) -> bool {
    if (ks == 0) mx = 0.f;
    __syncthreads();  // A: the previous step's fragment reads are done
    SM_STAMP(0);
    // after a segment: the volume kernel leaves 4 (T-1) chunk stores in flight, the volume-free
    // fused kernel its one disparity store per wave
    vm_wait<FUSE == 2 ? 1 : 4 * (TMAX - 1) + (FUSE == 1 ? 1 : 0), PF, ASM>(st.v, pfd,
                                                                     __builtin_amdgcn_readfirstlane((int)pend));
#ifdef SMCV_STAMPS
    if (ks == 0) SM_STAMP(5); else if (ks == 1) SM_STAMP(6); else SM_STAMP(7);
#endif
    pend = false;
    put(st);
    const unsigned par = (unsigned)(it & 1) * 8u;
    if constexpr (NP == 2) {
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
    }
    SM_STAMP(1);
    if (more) load(st, nx, ks1);
    touch(pk, pks, pv);  // unconditional: vm_wait counts exactly kPF touches after the loads
    SM_STAMP(2);
    __syncthreads();  // B: the planes of step s are complete
    SM_STAMP(0);
    // the matrix phase at raised wave priority: while one workgroup feeds its MFMAs, the
    // co-resident workgroup's staging / epilogue VALU yields issue slots to it (3-4 % faster on
    // cfg2, profiles/r02/band_experiments/prio_mfma_phase.log; raising it in or outside the
    // epilogue instead measured flat)
    __builtin_amdgcn_s_setprio(1);
    if (ks == 0)
      band(std::true_type{});
    else
      band(std::false_type{});
    __builtin_amdgcn_s_setprio(0);
    SM_STAMP(3);
    if (ks != nks - 1) return false;
    // ---- end of a segment: (fp32) range check, then the epilogue
    const bool fast =
        store_vol && dq && k.x0 + kXT <= W && k.Dp == DMAX && !(SMCV_ABLATE & 12);
    if constexpr (NP == 1) {
      if (!(SMCV_ABLATE & 8)) epilogue(k, fast);
      pend = FUSE == 2 ? k.x0 + 32 * wave + 32 <= W : fast;  // as below
      SM_STAMP(4);
      return false;
    } else {
      const float ml = __uint_as_float(*lds_word(maxw + par));
      const float mr = __uint_as_float(*lds_word(maxw + par + 4));
      const bool fin = ml <= 3.4e38f && mr <= 3.4e38f;  // no +-inf staged
      const int el = ml > 0.f ? exp_of(ml) : 0, er = mr > 0.f ? exp_of(mr) : 0;
      const bool okl = ml == 0.f || (el + kL <= 15 && el + kL >= -1);
      const bool okr = mr == 0.f || (er + kR <= 15 && er + kR >= -1);
      if (fin && okl && okr) {
        if (!(SMCV_ABLATE & 8)) epilogue(k, fast);
        // exactly 4 (T-1) stores per lane were issued after the loads; FUSE 2: one disparity
        // store per wave, certainly issued when all of the wave's pixels lie inside the row
        pend = FUSE == 2 ? k.x0 + 32 * wave + 32 <= W : fast;
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
    }
  };

  // the step m steps after (item i, step s): its work item and step; false past the last item
  auto ahead = [&](int i, int s, int m, Work& w, int& ws) -> bool {
    s += m;
    while (s >= nks) {
      s -= nks;
      ++i;
    }
    ws = s;
    if (i >= nitems) return false;
    w = decode(witem(i), args, DMAX);
    return true;
  };

  // items it = 0 .. nitems-1 (work index wbeg + gi + it gsz), channel steps ks = 0 .. nks-1;
  // every load() is followed by exactly kPF touches (of the step after the loaded one)
  Work cur = decode(witem(0), args, DMAX);
  {
    Work pk = cur;
    int pks = 0;
    const bool pv = ahead(0, 0, 1, pk, pks);
    load(st, cur, 0);
    touch(pk, pks, pv);
  }
  for (int it = 0, ks = 0; it < nitems;) {
    const bool last = ks == nks - 1;
    const bool more = !last || it + 1 < nitems;
    const Work nx = last && more ? decode(witem(it + 1), args, DMAX) : cur;
    Work pk = cur;
    int pks = 0;
    const bool pv = ahead(it, ks, 2, pk, pks);
    if (body(cur, it, ks, nx, last ? 0 : ks + 1, more, pk, pks, pv)) {  // recompute the segment
      vm_wait<0, 0, ASM>(st.v, pfd, 0);  // no load in flight when the registers are reloaded
      ks = 0;
      Work pk1 = cur;
      int pks1 = 0;
      const bool pv1 = ahead(it, 0, 1, pk1, pks1);
      load(st, cur, 0);
      touch(pk1, pks1, pv1);
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
  vm_wait<0, 0, ASM>(st.v, pfd, 0);  // nothing in flight when the registers die
  SM_STAMP_FLUSH
}

// Merge of the per-pass partial soft-argmin states (volume-free fused kernel, D > 192): the
// same shift-and-rescale as the lane-pair merge inside the band kernel, over the passes.
__global__ __launch_bounds__(256) void fused_merge_kernel(const double* __restrict__ S,
                                                          const double* __restrict__ T,
                                                          const float* __restrict__ Mv, int npass,
                                                          int64_t nhw, float* __restrict__ disp) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= nhw) return;
  constexpr float kL2E = 1.4426950408889634f;
  float M = -INFINITY;
  for (int p = 0; p < npass; ++p) M = fmaxf(M, Mv[p * nhw + i]);
  const float sh = fmaxf(M, -3.402823466e38f);
  double s = 0.0, t = 0.0;
  for (int p = 0; p < npass; ++p) {
    const double g = (double)__builtin_amdgcn_exp2f((Mv[p * nhw + i] - sh) * kL2E);
    s += S[p * nhw + i] * g;
    t += T[p * nhw + i] * g;
  }
  disp[i] = (float)(t / s);
}

template <typename T, typename TO, int TMAX, bool MEAN, int LAYOUT, int FUSE>
int launch(Args a, int64_t N, hipStream_t st) {
  using G = Geo<T, TMAX>;
  a.tiles = (int)ceil_div(a.W, kXT);
  const int64_t nwork = (int64_t)a.tiles * a.H * N * a.G * a.npass;
  if (nwork > INT32_MAX / 64) return fail(SM_EINVAL, "band kernel: too much work for one launch");
  a.nwork = (int)nwork;
  auto kern = band_h2<T, TO, TMAX, MEAN, LAYOUT, FUSE>;
  static std::atomic<unsigned long long> lds_done{0};  // per instantiation
  const int dev = stream_device(st);
  if (int rc = ensure_lds_limit(reinterpret_cast<const void*>(kern), (int)G::SHM, dev, lds_done))
    return rc;
  int64_t nwg = std::min<int64_t>(nwork, wg_per_cu<FUSE>() * (int64_t)device_cus(dev));
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(kThreads), G::SHM, st, a);
  return check_launch("band_h2");
}

// the smallest band geometry that holds one D pass of pw disparities
template <typename F>
int by_tmax(int64_t pw, F f) {
  if (pw <= 32) return f(std::integral_constant<int, 2>{});
  if (pw <= 64) return f(std::integral_constant<int, 3>{});
  if (pw <= 128) return f(std::integral_constant<int, 5>{});
  return f(std::integral_constant<int, 7>{});
}

}  // namespace h2band

int check_dot_args(const void* left, const void* right, const void* out, int dtype, int64_t N,
                   int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                   const int64_t* r_strides, Strides4* ls, Strides4* rs);

namespace h2band {
int band_h2db_run(const Args& a, int64_t N, bool mean, bool aligned4, hipStream_t st, bool* handled);
int band_sl_run(const Args& a, int64_t N, bool mean, bool aligned4, hipStream_t st, bool* handled,
                int fuse);
int band_rs_gw_run(const Args& a, int64_t N, int dtype, hipStream_t st, bool* handled);
#ifndef SMCV_RS_FUSE2
#define SMCV_RS_FUSE2 1  // the one-pass volume-free fused pass on band_rs (0: band_h2's FUSE 2;
                         // 2, diagnostic: also the D passes + merge)
#endif
int band_rs_run(const Args& a, int64_t N, bool mean, bool aligned4, hipStream_t st, bool* handled,
                int fuse);
int band_h2db_fused_run(const Args& a, int64_t N, bool mean, bool aligned4, hipStream_t st,
                        bool* handled);
}

namespace {
// Shared validation; *vec = the shape takes the band kernels (4-pixel groups: W % 4 == 0,
// 4-element aligned rows and feature pointers, a 16-B aligned output, channels > 0).
int h2_prepare(const void* left, const void* right, const void* out, int dtype, int64_t N,
               int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
               const int64_t* r_strides, h2band::Args* a, bool* vec, bool* al4 = nullptr) {
  Strides4 ls, rs;
  int rc = check_dot_args(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &ls, &rs);
  if (rc) return rc;
  const uintptr_t align = 4 * (uintptr_t)elem_size(dtype);
  const bool aligned4 = (W % 4 == 0) && ls.n % 4 == 0 && ls.c % 4 == 0 && ls.h % 4 == 0 &&
                       rs.n % 4 == 0 && rs.c % 4 == 0 && rs.h % 4 == 0 &&
                       ((reinterpret_cast<uintptr_t>(left) | reinterpret_cast<uintptr_t>(right)) % align == 0) &&
                       reinterpret_cast<uintptr_t>(out) % 16 == 0;
  if (al4) *al4 = aligned4;
  // fp32 rows of any width (and any element strides): the 16-B feature loads and volume stores
  // are then only dword-aligned, which gfx950 global memory accesses allow (unaligned mode);
  // the row-end group is handled in load() / put() and the row-end quad in the epilogue
  const bool any_w = dtype == SM_F32 && reinterpret_cast<uintptr_t>(out) % 4 == 0;
  *vec = (aligned4 || any_w) && W >= 4 && C > 0 && 8 * H * W < INT32_MAX &&
         8 * W * std::max<int64_t>(D, 1) < INT32_MAX;
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
  a->round = 0;
  a->ws_s = a->ws_t = nullptr;
  a->ws_m = nullptr;
  a->nhw = N * H * W;
  return SM_OK;
}
}  // namespace

// Inner product (mode 0, sum) / correlation (mode 1, mean) -> (N, D, H, W) in the input dtype.
// *handled = false when the shape needs the generic path.
int band_h2_entry(const void* left, const void* right, void* out, int dtype, int64_t N, int64_t C,
                  int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                  const int64_t* r_strides, int mode, void* stream, bool* handled, int variant) {
  using namespace h2band;
  *handled = false;
  Args a;
  bool vec = false, al4 = false;
  int rc = h2_prepare(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &a, &vec, &al4);
  if (rc) return rc;
  if (!vec) return SM_OK;
  *handled = true;
  if (N == 0 || H == 0 || D == 0) return SM_OK;
  const bool mean = mode == 1;
  a.mul = 1.0f / (float)C;
  hipStream_t st = as_stream(stream);
  // fp32 with aligned rows: variant 6 the sliding-window kernel (band_sl), variant 5 the
  // role-split kernel (band_rs; the shapes they do not take fall through to band_h2db), variant
  // 2 the double-buffered pipeline (band_h2db); other shapes (and variant 0) run band_h2
  if (variant != 0 && dtype == SM_F32) {
    bool done = false;
    if (variant == 6) {  // the sliding-window kernel; shapes it does not take: band_h2db
      rc = band_sl_run(a, N, mean, al4, st, &done, 0);
      if (done || rc != SM_OK) return rc;
    }
    if (variant == 5) {  // the role-split kernel; shapes it does not take: band_h2db
      rc = band_rs_run(a, N, mean, al4, st, &done, 0);
      if (done || rc != SM_OK) return rc;
    }
    rc = band_h2db_run(a, N, mean, al4, st, &done);
    if (done || rc != SM_OK) return rc;
  }
  SM_DISPATCH_DTYPE(dtype, T0, {
    using T = typename std::conditional<std::is_same<T0, bf16_t>::value, __bf16, T0>::type;
    return by_tmax(a.pw, [&](auto tm) {
      constexpr int TM = decltype(tm)::value;
      return mean ? launch<T, T, TM, true, h2band::kNDHW, false>(a, N, st)
                  : launch<T, T, TM, false, h2band::kNDHW, false>(a, N, st);
    });
  });
  return SM_OK;
}

// Groupwise (mean over C/G contiguous channels) -> (N, G, H, W, D) float32.
int band_h2_groupwise_entry(const void* left, const void* right, float* out, int dtype, int64_t N,
                            int64_t C, int64_t H, int64_t W, int64_t D, int64_t G,
                            const int64_t* l_strides, const int64_t* r_strides, void* stream,
                            bool* handled) {
  using namespace h2band;
  *handled = false;
  if (G <= 0 || C % G != 0) return fail(SM_EINVAL, "groupwise: C % G != 0");
  Args a;
  bool vec = false;
  int rc = h2_prepare(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &a, &vec);
  if (rc) return rc;
  if (!vec) return SM_OK;
  *handled = true;
  if (N == 0 || H == 0 || D == 0) return SM_OK;
  a.G = (int)G;
  a.cpg = (int)(C / G);
  a.mul = 1.0f / (float)a.cpg;
  hipStream_t st = as_stream(stream);
  {  // 16-bit features with 16-channel group steps: the role-split kernel
    bool done = false;
    rc = band_rs_gw_run(a, N, dtype, st, &done);
    if (done || rc != SM_OK) return rc;
  }
  SM_DISPATCH_DTYPE(dtype, T0, {
    using T = typename std::conditional<std::is_same<T0, bf16_t>::value, __bf16, T0>::type;
    return by_tmax(a.pw, [&](auto tm) {
      constexpr int TM = decltype(tm)::value;
      return launch<T, float, TM, true, h2band::kNGHWD, false>(a, N, st);
    });
  });
  return SM_OK;
}

// Inner product / correlation fused with soft-argmin: disparity (N, H, W) fp32, and the volume
// when out != nullptr.  fp32 features, one D pass (D <= 192); *handled = false otherwise.
int64_t band_h2_fused_workspace_bytes(int64_t N, int64_t H, int64_t W, int64_t D) {
  const int64_t npass = (std::max<int64_t>(D, 1) + 191) / 192;
  return npass > 1 ? npass * N * H * W * (8 + 8 + 4) : 0;
}

int band_h2_fused_entry(const void* left, const void* right, void* out, float* disp, int dtype,
                        int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                        const int64_t* l_strides, const int64_t* r_strides, int mode,
                        void* stream, bool* handled, void* workspace, int64_t ws_bytes) {
  using namespace h2band;
  *handled = false;
  if (disp == nullptr && N * H * W > 0) return fail(SM_EINVAL, "null disparity pointer");
  Args a;
  bool vec = false, al4 = false;
  // (the volume check of check_dot_args needs a pointer when only the disparity is wanted)
  int rc = h2_prepare(left, right, out ? out : disp, dtype, N, C, H, W, D, l_strides, r_strides,
                      &a, &vec, &al4);
  if (rc) return rc;
  if (N * H * W == 0) {
    *handled = true;
    return SM_OK;
  }
  vec = vec && reinterpret_cast<uintptr_t>(disp) % 16 == 0;
  // D > 192 (several passes): volume-free only, with a workspace for the partial states
  const bool multi = a.npass > 1 && out == nullptr && workspace != nullptr &&
                     ws_bytes >= band_h2_fused_workspace_bytes(N, H, W, D) &&
                     reinterpret_cast<uintptr_t>(workspace) % 8 == 0;
  // fp16 / bf16 features with fp32 disparities (SM_FUSED_DISP_F32: the reference's autocast
  // eval) take the band kernel's half instantiations; fp32 features the fp32 ones
  const bool f32disp = (mode & SM_FUSED_DISP_F32) != 0;
  // fp16 / bf16 features: the fold regresses the cells rounded to the feature dtype (the
  // reference's autocast result) unless SM_FUSED_EXACT_ACC asks for the fp32 accumulators
  a.round = dtype != SM_F32 && (mode & SM_FUSED_EXACT_ACC) == 0;
#ifndef SMCV_SL_FUSE
#define SMCV_SL_FUSE 1  // the fp32 fused passes on the sliding-window kernel where it takes them
#endif
  if (SMCV_SL_FUSE && vec && dtype == SM_F32 && D > 0) {
    // one D pass with or without the volume; two passes (C = 16) without it, the passes' states
    // merged in registers (no workspace)
    Args b = a;
    b.out = out;
    b.disp = disp;
    b.mul = 1.0f / (float)C;
    bool done = false;
    rc = band_sl_run(b, N, (mode & 1) != 0, al4, as_stream(stream), &done, out != nullptr ? 1 : 2);
    if (rc != SM_OK) return rc;
    if (done) {
      *handled = true;
      return SM_OK;
    }
  }
  if (!vec || (dtype != SM_F32 && !f32disp) || (a.npass != 1 && !multi) || D == 0) return SM_OK;
  if (multi) {
    const int64_t per = (int64_t)a.npass * a.nhw;
    a.ws_s = static_cast<double*>(workspace);
    a.ws_t = a.ws_s + per;
    a.ws_m = reinterpret_cast<float*>(a.ws_t + per);
  }
  *handled = true;
  a.out = out;
  a.disp = disp;
  a.mul = 1.0f / (float)C;
  const bool mean = (mode & 1) != 0;
  hipStream_t st = as_stream(stream);
  if (dtype != SM_F32) {  // exact products of the half features, one MFMA per block and step
    auto go_half = [&](auto tag) {
      using T = typename decltype(tag)::type;
      return by_tmax(a.pw, [&](auto tm) {
        constexpr int TM = decltype(tm)::value;
        if (out != nullptr)
          return mean ? launch<T, T, TM, true, h2band::kNDHW, 1>(a, N, st)
                      : launch<T, T, TM, false, h2band::kNDHW, 1>(a, N, st);
        const int rc2 = mean ? launch<T, T, TM, true, h2band::kNDHW, 2>(a, N, st)
                             : launch<T, T, TM, false, h2band::kNDHW, 2>(a, N, st);
        if (rc2 != SM_OK || a.ws_m == nullptr) return rc2;
        hipLaunchKernelGGL(fused_merge_kernel, dim3((unsigned)ceil_div(a.nhw, (int64_t)256)),
                           dim3(256), 0, st, a.ws_s, a.ws_t, a.ws_m, a.npass, a.nhw, disp);
        return check_launch("fused_merge_kernel");
      });
    };
    return dtype == SM_F16 ? go_half(std::type_identity<__half>{}) : go_half(std::type_identity<__bf16>{});
  }
#ifndef SMCV_NO_RS_FUSE  // (diagnostic builds: -DSMCV_NO_RS_FUSE keeps the band_h2db / band_h2 paths)
  // the role-split kernel for the shapes it takes, with the volume (FUSE 1: 1 % below
  // band_h2db's FUSE 1 on cfg2) and, for one D pass, without it (FUSE 2: 103.3 against band_h2's
  // 111.3-111.7 us per pair on 32-pair cfg2 launches, a tie at 8 pairs,
  // profiles/r04/band_experiments/fuse2_b32.jsonl; on cfg4's two passes it ran 4-7 % slower,
  // fuse_ab.jsonl, fuse2_cfg4_b32.jsonl: 381 against 364-366 us per pair at 32 pairs, so D > 192
  // stays on band_h2)
  if (out != nullptr || (SMCV_RS_FUSE2 && (a.npass == 1 || SMCV_RS_FUSE2 == 2))) {
    bool done = false;
    rc = band_rs_run(a, N, mean, al4, st, &done, out != nullptr ? 1 : 2);
    if (rc != SM_OK) return rc;
    if (done) {
      if (out != nullptr || a.ws_m == nullptr) return SM_OK;
      hipLaunchKernelGGL(fused_merge_kernel, dim3((unsigned)ceil_div(a.nhw, (int64_t)256)), dim3(256), 0,
                         st, a.ws_s, a.ws_t, a.ws_m, a.npass, a.nhw, disp);
      return check_launch("fused_merge_kernel");
    }
  }
#endif
#ifndef SMCV_NO_DB_FUSE  // (diagnostic builds: -DSMCV_NO_DB_FUSE keeps band_h2's FUSE 1 path)
  if (out != nullptr) {  // volume kept, aligned rows: the double-buffered kernel with the fold
    bool done = false;
    rc = band_h2db_fused_run(a, N, mean, al4, st, &done);
    if (done || rc != SM_OK) return rc;
  }
#endif
  return by_tmax(a.pw, [&](auto tm) {
    constexpr int TM = decltype(tm)::value;
    // FUSE 1: volume + disparities; FUSE 2: disparities only -- no shear, no ring, no volume
    // stores.  Both two workgroups per CU with hand-counted loads (see band_h2).
    if (out != nullptr)
      return mean ? launch<float, float, TM, true, h2band::kNDHW, 1>(a, N, st)
                  : launch<float, float, TM, false, h2band::kNDHW, 1>(a, N, st);
    const int rc = mean ? launch<float, float, TM, true, h2band::kNDHW, 2>(a, N, st)
                        : launch<float, float, TM, false, h2band::kNDHW, 2>(a, N, st);
    if (rc != SM_OK || a.ws_m == nullptr) return rc;
    hipLaunchKernelGGL(fused_merge_kernel, dim3((unsigned)ceil_div(a.nhw, (int64_t)256)), dim3(256), 0,
                       st, a.ws_s, a.ws_t, a.ws_m, a.npass, a.nhw, disp);
    return check_launch("fused_merge_kernel");
  });
}

}  // namespace smcv

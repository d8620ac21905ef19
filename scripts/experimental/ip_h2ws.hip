// Inner-product / correlation cost volume (N, D, H, W) from fp32 features with the volume stores
// decoupled from the compute ("h2ws"): band_h2db's step pipeline in 4 compute waves, plus 4 store
// waves that stream the previous segment's output while the compute waves run the next one.
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// band_h2 / band_h2db issue a segment's 96 KB of volume stores in a burst at its end, and the
// wave blocks on them while the memory drains; the compute and the stores then add up instead of
// overlapping (profiles/r03/band_experiments/: a memory pattern with separate reader and store
// waves moves a cfg2 pair 20 % faster than the kernel).  Here one 12-wave workgroup owns a CU,
// in three roles of 4 waves (one of each per SIMD):
//   * compute waves 0-3 run band_h2db's matrix phase (32x32x16 MFMA over double-buffered fp16
//     planes, one barrier per step); their epilogue only shears the accumulators into an LDS
//     FIFO holding the segment's whole output (4 waves x T-1 chunks of 32 d x 32 x fp32: 96 KB
//     for D = 192; no ring wrap, so an element's address is linear in its disparity);
//   * loader waves 4-7 stage the next step into the other plane buffer (wait for its feature
//     loads, track max|x|, split into the h and m planes) and issue the loads of the step after;
//   * store waves 8-11 drain the FIFO: during the next segment's steps, store wave s reads
//     compute wave s's chunks (4 x 16 B per lane) and writes them out (8 rows x 128 B per
//     instruction, non-temporal), a quota per step so that the segment is out before the next
//     epilogue.
// A wave only ever waits for its own kind of memory traffic: the compute waves have none, the
// loaders' vmcnt counts only loads (the compiler places those waits), the store waves' only
// stores.  Every wave runs the same loop skeleton (gfx950 has one workgroup barrier) and takes
// the same scale decisions from the LDS maxima, so the barrier counts always match.
#include "band_common.h"

// diagnostic builds only (scripts/build_ab_ws.sh): bit 0 no volume stores, bit 1 no feature
// loads after the first, bit 2 no MFMA phase, bit 3 no epilogue, bit 4 no staging (results
// are then wrong)
#ifndef SMCV_WS_ABL
#define SMCV_WS_ABL 0
#endif
// 1: a store wave drains a chunk as soon as its compute wave flags it complete (LDS counters, no
// barrier after the epilogue); 0: a barrier after the epilogue hands the whole FIFO over
#ifndef SMCV_WS_FLAGS
#define SMCV_WS_FLAGS 1
#endif

namespace smcv {
namespace h2band {

namespace ws {
constexpr int kCompute = 4;          // waves per role: compute 0-3, loader 4-7, store 8-11
constexpr int kThreads = 64 * 3 * kCompute;
constexpr int kCT = 64 * kCompute;    // threads per role
constexpr int kKC = 16;               // channels per step (one 32x32x16 k-step)
constexpr int kSlot = 32 * 32 * 4;    // one chunk: 32 d x 32 x fp32

template <int TMAX>
struct Geo {
  static constexpr int DMAX = 32 * (TMAX - 1);
  static constexpr int NC = TMAX - 1;      // chunks per wave and segment
  static constexpr int RW = kXT + DMAX;    // right-window rows
  static constexpr int ROWS = RW + kXT;    // + left-tile rows
  static constexpr int PLANE = ROWS * 32;  // one fp16 plane: rows of 16 channels
  static constexpr int BUF = 2 * PLANE;    // a plane buffer (h, m)
  static constexpr int GROUPS = ROWS / 4;
  static constexpr int ITEMS = 2 * GROUPS;
  static constexpr int FIFO = 2 * BUF;     // the segment's output: [wave 4][chunk NC][32][32]
  static constexpr int MAXW = FIFO + kCompute * NC * kSlot;  // 3 parity sets x (max|L|, max|R|)
  static constexpr int FLAGS = MAXW + 32;  // per compute wave: chunks completed so far
  static constexpr size_t SHM = (size_t)FLAGS + 16;
  static_assert(ITEMS <= kCT, "one staging item per loader lane");
  static_assert(GROUPS % 8 == 0, "8-lane write groups stay inside one chunk");
  static_assert(BUF % 1024 == 0, "plane buffers keep the swizzle's row bits");
  static_assert(SHM <= 160 * 1024, "one workgroup per CU");
};
}  // namespace ws

template <bool MEAN, int TMAX>
__global__ __launch_bounds__(ws::kThreads, 3) void band_h2ws(Args args) {
  using ws::kCompute;  // (block-scope declarations: they hide band_h2's namesakes in a one-file build)
  using ws::kCT;
  using ws::kKC;
  using ws::kSlot;
  using G = ws::Geo<TMAX>;
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
  const int nks = (cpg + kKC - 1) / kKC;

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const bool compute = wave < kCompute;                         // wave-uniform roles
  const bool loader = wave >= kCompute && wave < 2 * kCompute;
  const int sw = wave - 2 * kCompute;  // store wave: the compute wave whose chunks it drains

  // ---------------------------------------------------------------- staging role of a lane
  const int lid = tid - kCT;  // loader lane
  const bool active = loader && lid < G::ITEMS;
  const int ch = min(max(lid, 0) / G::GROUPS, 1);
  const int g = min(max(lid, 0) - ch * G::GROUPS, G::GROUPS - 1);
  const bool isR = 4 * g < G::RW;
  const int64_t cs = isR ? rs.c : ls.c;
  const bool cfull = __builtin_amdgcn_readfirstlane(cpg % kKC) == 0;

  struct Set {
    f32x4v v[8];
    int nv;
  };
  Set st;
  auto row_of = [&](const Work& k) {
    return isR ? R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h
               : L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;
  };
  auto load = [&](const Work& k, int ks) {
    const int cl = ks * kKC + 8 * ch;
    const int px = isR ? k.js + 4 * g : k.x0 + 4 * g - G::RW;
    const bool okp = active && px >= 0 && px < W;
    const float* p = row_of(k) + (okp ? px : 0) + (int64_t)min(cl, cpg - 1) * cs;
    st.nv = okp ? min(max(cpg - cl, 0), 8) : 0;
    const int lim = cfull ? 7 : min(max(cpg - 1 - cl, 0), 7);
    int64_t csl = cs;
    asm volatile("" : "+v"(csl));
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      gload<false>(st.v[kk], p);  // compiler-tracked: a loader wave has no stores to wait for
      if (kk < lim) p += csl;
    }
  };

  int kL = 0, kR = 0;  // per-segment scale exponents (workgroup-uniform)
  float mx = 0.f;      // this lane's max|x| over the segment being staged
  // Staging of one step into buffer `buf`, in pieces: piece 0 zeroes the invalid channels /
  // pixels and tracks max|x|; pieces 1-4 split pixel p = piece-1 into the h and m planes.
  auto put_piece = [&](int piece, unsigned buf) {
    if (!active) return;
    if (piece == 0) {
      if (__builtin_expect(__any(st.nv != 8), 0)) {
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
          if (kk >= st.nv) st.v[kk] = f32x4v{0.f, 0.f, 0.f, 0.f};
      }
      float m0 = mx, m1 = 0.f;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m0) : "v"(st.v[kk].x), "v"(st.v[kk].y));
        asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m1) : "v"(st.v[kk].z), "v"(st.v[kk].w));
      }
      mx = fmaxf(m0, m1);
      return;
    }
    const int p = piece - 1;
    const float sc = __builtin_ldexpf(1.0f, isR ? kR : kL);
    unsigned o0 = buf + (unsigned)swz(4 * g, ch);
    asm volatile("" : "+v"(o0));
    uint4 wh, wm;
    split_pair(st.v[0][p], st.v[1][p], sc, wh.x, wm.x);
    split_pair(st.v[2][p], st.v[3][p], sc, wh.y, wm.y);
    split_pair(st.v[4][p], st.v[5][p], sc, wh.z, wm.z);
    split_pair(st.v[6][p], st.v[7][p], sc, wh.w, wm.w);
    const unsigned off = o0 ^ (32u * p);
    *reinterpret_cast<uint4*>(smem + off) = wh;
    *reinterpret_cast<uint4*>(smem + G::PLANE + off) = wm;
  };
  // maxima words: set s (0..2) at MAXW + 8 s: max|L|, max|R|
  const unsigned maxw = lds_addr(smem + G::MAXW);
  auto publish_max = [&](int set) {  // after the staging of a segment's last step
    const float ml = wave_max(isR ? 0.f : mx), mr = wave_max(isR ? mx : 0.f);
    if (lane == 0) {
      __hip_atomic_fetch_max(lds_word(maxw + 8u * set), __float_as_uint(ml), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_fetch_max(lds_word(maxw + 8u * set + 4), __float_as_uint(mr), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  };

  // ------------------------------------------------------------------- MFMA role of a wave
  const int lr = lane & 31;
  const int hh = lane >> 5;
  f32x16 acc[TMAX];
  auto mma = [](f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  };
  // The matrix phase of one step on buffer `buf` (the fragments of block t + 1 are read while
  // block t multiplies)
  auto band = [&](unsigned buf) {
    const unsigned char* ab = smem + buf + 32 * wave * 32 + swz(lr, hh);
    const unsigned char* bb = smem + buf + (G::RW + 32 * wave) * 32 + swz(lr, hh);  // (wave < 4)
    const f16x8 bh = *reinterpret_cast<const f16x8*>(bb);
    const f16x8 bm = *reinterpret_cast<const f16x8*>(bb + G::PLANE);
    f16x8 ah = *reinterpret_cast<const f16x8*>(ab);
    f16x8 am = *reinterpret_cast<const f16x8*>(ab + G::PLANE);
#pragma unroll
    for (int t = 0; t < TMAX; ++t) {
      f16x8 nh = ah, nm = am;
      if (t + 1 < TMAX) {
        nh = *reinterpret_cast<const f16x8*>(ab + 1024 * (t + 1));
        nm = *reinterpret_cast<const f16x8*>(ab + G::PLANE + 1024 * (t + 1));
      }
      f32x16 c = acc[t];  // zero at a segment's first step (its consumer cleared it)
      c = mma(am, bh, c);
      c = mma(ah, bm, c);
      acc[t] = mma(ah, bh, c);
      ah = nh;
      am = nm;
    }
  };

  // ------------------------------------------------------------------------------ epilogue
  // Lane (lr, hh), element i of block t: R row c_i + 4 hh (c_i = (i & 3) + 8 (i >> 2)), pixel
  // x0w + lr, local disparity 32 (a + 1) + u - c_i with a = T-2-t, u = lr - 4 hh: in the FIFO
  // [chunk][32 d][32 x] of this wave, byte 4096 (a + 1) + 128 (u - c_i) + 4 lr.  Chunks -1 and
  // T-1 hold disparities outside 0 .. DMAX-1 (only the first and the last block have such cells):
  // not written.
  const int u = lr - 4 * hh;
  const int rl = lane >> 3, cl = lane & 7;
  const size_t plane_stride = (size_t)H * W;
  const int lane_st = rl * H * W + 4 * cl;
  const unsigned fifo = lds_addr(smem + G::FIFO);

  // Chunk hand-over (SMCV_WS_FLAGS): compute wave s counts the FIFO chunks it has completed
  // (over all fills) in LDS word FLAGS + 4 s; store wave s waits for a chunk's count before
  // reading it.  A wait only ever spans an interval without barriers in which the compute wave
  // completes that chunk (its epilogue, right after the segment-end barrier), and it is bounded
  // in any case: a wave never spins forever.
  const unsigned flagw = lds_addr(smem + G::FLAGS);
  auto flag_publish = [&](unsigned v) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the chunk's LDS writes are done
    if (lane == 0)
      *reinterpret_cast<volatile __attribute__((address_space(3))) unsigned*>(flagw + 4u * wave) = v;
  };
  auto flag_wait = [&](unsigned need) {
    const unsigned fa = flagw + 4u * (unsigned)sw;
    for (int spin = 0; spin < (1 << 16); ++spin) {
      unsigned v;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(fa) : "memory");
      if ((int)(__builtin_amdgcn_readfirstlane(v) - need) >= 0) break;
      __builtin_amdgcn_s_sleep(1);
    }
  };

  auto epilogue_v = [&](const Work& k, unsigned fbase, auto scale, auto xlt) {
    const float mul = args.mul;
    const int kk = -(kL + kR);
    const int jlane = k.js + 32 * wave + 4 * hh;
    // one register per lane: element (t, i) is at e0 + 4096 (a + 1) + 128 (27 - c_i), all
    // immediate offsets (u - 27 may be negative: the sum wraps back into the FIFO)
    unsigned e0 = fifo + (unsigned)(wave * G::NC * kSlot) + (unsigned)(128 * (u - 27) + 4 * lr);
    int uu = u, jl = jlane;
    asm volatile("" : "+v"(e0), "+v"(uu), "+v"(jl));
    [&]<int... I_>(std::integer_sequence<int, I_...>) {
      (
          [&] {
            constexpr int t = TMAX - 1 - I_;
            constexpr int a = TMAX - 2 - t;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int ci = (i & 3) + 8 * (i >> 2);
              float val = acc[t][i];
              if (MEAN) val *= mul;
              if constexpr (decltype(scale)::value) val = __builtin_ldexpf(val, kk);
              if constexpr (decltype(xlt)::value) val = jl + 32 * t + ci >= 0 ? val : 0.f;
              const unsigned addr = e0 + (unsigned)(4096 * (a + 1) + 128 * (27 - ci));
              if constexpr (a == -1) {
                if (uu >= ci) lds_store1(addr, val);
              } else if constexpr (a == TMAX - 2) {
                if (uu < ci) lds_store1(addr, val);
              } else {
                lds_store1(addr, val);
              }
            }
            acc[t] = f32x16{};  // ready for the next segment's first step
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (SMCV_WS_FLAGS && a >= 0) flag_publish(fbase + (unsigned)(a + 1));
          }(),
          ...);
    }(std::make_integer_sequence<int, TMAX>{});
  };
  auto epilogue = [&](const Work& k, unsigned fbase) {
    using TT = std::true_type;
    using FF = std::false_type;
    const bool xl = __builtin_amdgcn_readfirstlane(k.js) < 0;
    if (__builtin_amdgcn_readfirstlane(kL + kR) != 0) {
      if (xl)
        epilogue_v(k, fbase, TT{}, TT{});
      else
        epilogue_v(k, fbase, TT{}, FF{});
      return;
    }
    if (xl)
      epilogue_v(k, fbase, FF{}, TT{});
    else
      epilogue_v(k, fbase, FF{}, FF{});
  };

  // Store wave: chunks [c0, c1) of compute wave sw's FIFO for segment k (8 rows x 128 B per
  // store instruction, non-temporal: the volume is not re-read here)
  auto drain = [&](const Work& k, int c0, int c1, unsigned fbase) {
    const bool fast = k.x0 + kXT <= W && k.Dp == DMAX;
    const int x0w = k.x0 + 32 * sw;
    unsigned rb = fifo + (unsigned)(sw * G::NC * kSlot + rl * 128 + 16 * cl);
    asm volatile("" : "+v"(rb));
    int ls_ = lane_st;
    asm volatile("" : "+v"(ls_));
    float* ob = out + (((size_t)k.n * D + k.dp) * plane_stride + (size_t)k.y * W + x0w) + ls_;
    const size_t st8 = (size_t)8 * plane_stride;
    for (int a = c0; a < c1; ++a) {
      if constexpr (SMCV_WS_FLAGS) flag_wait(fbase + (unsigned)(a + 1));
      f32x4v v[4];
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) v[qq] = lds_load4(rb + (unsigned)(a * kSlot + 8 * qq * 128));
      float* ol = ob + (size_t)(32 * a) * plane_stride;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        asm volatile("" : "+v"(ol));
        if (fast || (32 * a + 8 * qq + rl < k.Dp && x0w + 4 * cl < W)) store_quad<true>(ol, v[qq]);
        ol += st8;
      }
    }
  };

  auto slow_segment = [&](const Work& k) {
    const float mul = MEAN ? args.mul : 1.0f;
    const float* lrow = L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;  // (compute waves)
    const float* rrow = R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h;
    for (int idx = tid; idx < k.Dp * kXT; idx += kCT) {  // compute waves only
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
  if (tid < 6) *lds_word(maxw + 4 * tid) = 0u;
  if (tid < kCompute) *lds_word(flagw + 4 * tid) = 0u;
  __syncthreads();  // cleared before any wave publishes
  // band_h2db's loop, one copy per role (ROLE 0 compute, 1 loader, 2 store): each copy carries
  // only its role's registers (the accumulators, the staged features, the drain pointers), and
  // all copies run the same barrier sequence, as their loop decisions come from the same
  // workgroup-uniform values.  An iteration multiplies step (it, ks) out of buffer bm when `mul`
  // (compute), stages step (sit, sks) into the other buffer and loads the step after it
  // (loader), and drains a quota of the previous segment's chunks (store).
  auto run = [&](auto role) {
    constexpr int ROLE = decltype(role)::value;
    SM_STAMP_DECL  // (diagnostic builds: phases 0 work, 1 load wait, 2 barrier, 3 segment end,
                   //  4 post-epilogue barrier, 5 loop head)
    bool redone = false;
    if constexpr (ROLE == 0) {
#pragma unroll
      for (int t = 0; t < TMAX; ++t) acc[t] = f32x16{};
    }
    int it = 0, ks = 0;        // the step multiplied this iteration (if mul)
    int sit = 0, sks = 0;      // the step staged this iteration
    int set = 0, sset = 0;     // maxima sets (item % 3) of it and sit
    bool mul = false;
    unsigned bm = (unsigned)G::BUF;  // buffer multiplied from; staging goes to the other one
    Work cur = decode(witem(0), args, DMAX);   // item it
    Work scur = cur;                           // item sit
    bool pending = false;  // a segment's output waits in the FIFO (store: item pit)
    int pit = 0;
    unsigned fills = 0, pfb = 0;  // FIFO fills so far; chunk-count base of the pending fill
    if constexpr (ROLE == 1) load(scur, 0);
    while (it < nitems) {
      const bool stage_ok = sit < nitems;
      const bool nk = sks + 1 < nks;
      const int lit = nk ? sit : sit + 1, lks = nk ? sks + 1 : 0;
      const bool load_ok = lit < nitems;
      const Work lw = nk ? scur : (load_ok ? decode(witem(lit), args, DMAX) : scur);
      const unsigned sb = bm ^ (unsigned)G::BUF;  // the other plane buffer
      SM_STAMP(5);
      if constexpr (ROLE == 0) {
        __builtin_amdgcn_s_setprio(1);
        if constexpr (!(SMCV_WS_ABL & 4)) band(bm);
        __builtin_amdgcn_s_setprio(0);
      } else if constexpr (ROLE == 1) {
#ifdef SMCV_STAMPS
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        SM_STAMP(1);
#endif
        if (sks == 0) mx = 0.f;
        if constexpr (!(SMCV_WS_ABL & 16)) {
#pragma unroll
          for (int piece = 0; piece < 5; ++piece) put_piece(piece, sb);
        }
        if (stage_ok && sks == nks - 1) publish_max(sset);
        if constexpr (!(SMCV_WS_ABL & 2)) {
          if (load_ok) load(lw, lks);
        }
      } else {
        if (!(SMCV_WS_ABL & 1) && mul && pending) {
          // the previous segment's chunks, spread over this segment's steps
          // flags: half the chunks while the compute waves run the epilogue and the first step,
          // the rest spread over the other steps; barrier hand-over: an even spread
          auto cend = [&](int s_) {
            if (s_ < 0) return 0;
            if constexpr (SMCV_WS_FLAGS) return G::NC / 2 + (G::NC - G::NC / 2) * s_ / max(nks - 1, 1);
            return (s_ + 1) * G::NC / nks;
          };
          const int c1 = ks == nks - 1 ? G::NC : cend(ks);
          drain(decode(witem(pit), args, DMAX), cend(ks - 1), c1, pfb);
          if (ks == nks - 1) pending = false;
        }
      }
      SM_STAMP(0);
      __syncthreads();  // fragment reads of bm done; staging complete; drain quota read out
      SM_STAMP(2);
      bool restart = false;
      if (!mul) {
        if constexpr (ROLE == 0) {
#pragma unroll
          for (int t = 0; t < TMAX; ++t) acc[t] = f32x16{};  // a (re)start: nothing multiplied
        }
      } else if (ks == nks - 1) {
        // ---- end of segment `it`: range check on its maxima (every wave), then the epilogue
        const unsigned mw = maxw + 8u * (unsigned)set;
        const float ml = __uint_as_float(*lds_word(mw));
        const float mr = __uint_as_float(*lds_word(mw + 4));
        const int set2 = set == 0 ? 2 : set - 1;  // (it + 2) % 3: cleared for segment it + 2
        if (tid < 2) *lds_word(maxw + 8u * (unsigned)set2 + 4 * tid) = 0u;
        const bool fin = ml <= 3.4e38f && mr <= 3.4e38f;
        const int el = ml > 0.f ? exp_of(ml) : 0, er = mr > 0.f ? exp_of(mr) : 0;
        const bool okl = ml == 0.f || (el + kL <= 15 && el + kL >= -1);
        const bool okr = mr == 0.f || (er + kR <= 15 && er + kR >= -1);
        if (fin && okl && okr) {
          // (the FIFO was drained during this segment's steps)
          if constexpr (ROLE == 0 && !(SMCV_WS_ABL & 8)) epilogue(cur, fills * (unsigned)G::NC);
          pending = true;
          pit = it;
          pfb = fills * (unsigned)G::NC;
          ++fills;
          redone = false;
        } else {
          const int nkl = ml > 0.f ? 13 - el : kL, nkr = mr > 0.f ? 13 - er : kR;
          if (!fin || redone || nkl < -100 || nkl > 100 || nkr < -100 || nkr > 100) {
            if constexpr (ROLE == 0) slow_segment(cur);  // the staged next step stays valid
            redone = false;
          } else {
            kL = nkl;  // recompute with the new scale: restart at this segment's first step
            kR = nkr;
            redone = true;
            restart = true;
          }
          if constexpr (ROLE == 0) {
#pragma unroll
            for (int t = 0; t < TMAX; ++t) acc[t] = f32x16{};
          }
        }
      }
      if (restart) {
        __syncthreads();  // every wave has read the maxima
        if (tid < 4) {    // this segment's set and the next one's (its staged step published)
          const int s4 = (tid >> 1) == 0 ? set : (set == 2 ? 0 : set + 1);
          *lds_word(maxw + 8u * (unsigned)s4 + 4 * (tid & 1)) = 0u;
        }
        __syncthreads();
        sit = it;
        sks = 0;
        sset = set;
        scur = cur;
        if constexpr (ROLE == 1) load(scur, 0);
        mul = false;
        continue;  // (it, ks) stays: its segment is multiplied again from step 0
      }
      SM_STAMP(3);
      if (!SMCV_WS_FLAGS && mul && ks == nks - 1) __syncthreads();  // the FIFO is complete
      SM_STAMP(4);
      // advance: the staged step is multiplied next, the step after it is staged
      cur = scur;
      mul = stage_ok;
      if (!stage_ok) break;
      bm = sb;
      it = sit;
      ks = sks;
      set = sset;
      if (nk) {
        ++sks;
      } else {
        ++sit;
        sks = 0;
        sset = sset == 2 ? 0 : sset + 1;
        scur = lw;
      }
    }
    if constexpr (ROLE == 2 && !(SMCV_WS_ABL & 1)) {
      if (pending) drain(decode(witem(pit), args, DMAX), 0, G::NC, pfb);  // the last segment
    }
    SM_STAMP_FLUSH
  };
  if (compute)
    run(std::integral_constant<int, 0>{});
  else if (loader)
    run(std::integral_constant<int, 1>{});
  else
    run(std::integral_constant<int, 2>{});
}

template <bool MEAN, int TMAX>
int launch_h2ws(Args a, int64_t N, hipStream_t st) {
  using G = ws::Geo<TMAX>;
  a.tiles = (int)ceil_div(a.W, kXT);
  const int64_t nwork = (int64_t)a.tiles * a.H * N * a.G * a.npass;
  if (nwork > INT32_MAX / 64) return fail(SM_EINVAL, "band kernel: too much work for one launch");
  a.nwork = (int)nwork;
  auto kern = band_h2ws<MEAN, TMAX>;
  static std::atomic<unsigned long long> lds_done{0};
  const int dev = stream_device(st);
  if (int rc = ensure_lds_limit(reinterpret_cast<const void*>(kern), (int)G::SHM, dev, lds_done))
    return rc;
  int64_t nwg = std::min<int64_t>(nwork, (int64_t)device_cus(dev));  // one workgroup per CU
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(ws::kThreads), G::SHM, st, a);
  return check_launch("band_h2ws");
}

// fp32 inner product / correlation volume on the store-decoupled band kernel; *handled = false
// when the shape is not one it takes (4-element aligned rows, one channel group).
int band_h2db_run(const Args& a, int64_t N, bool mean, bool aligned4, hipStream_t st, bool* handled);

int band_h2ws_run(const Args& a, int64_t N, bool mean, bool aligned4, hipStream_t st,
                  bool* handled) {
  *handled = false;
  if (!aligned4 || a.G != 1 || a.pw > 192) return SM_OK;
  *handled = true;
  auto go = [&](auto tm) {
    constexpr int TM = decltype(tm)::value;
    return mean ? launch_h2ws<true, TM>(a, N, st) : launch_h2ws<false, TM>(a, N, st);
  };
  // D <= 32: band_h2db (a 2-block band has little store burst to hide, and at T = 2 the register
  // allocator copies the staged features before their wait: check_h2_asm.py)
  if (a.pw <= 32) return band_h2db_run(a, N, mean, aligned4, st, handled);
  if (a.pw <= 64) return go(std::integral_constant<int, 3>{});
  if (a.pw <= 128) return go(std::integral_constant<int, 5>{});
  return go(std::integral_constant<int, 7>{});
}

}  // namespace h2band
}  // namespace smcv

// Inner-product / correlation cost volume (N, D, H, W) from fp32 features: band_h2 with
// double-buffered planes ("h2db"), so that the staging of step s+1 runs inside step s's matrix
// phase and a step needs one barrier instead of two.
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// Contraction, operands (per-segment power-of-two scale, round-to-nearest two-plane fp16 split,
// h*h' + h*m' + m*h' on v_mfma_f32_32x32x16_f16), tiling (4 waves x 32 pixels per 128-pixel
// segment, T = 1 + DMAX/32 blocks of 32 x 32 per wave), scale control and the exact fp32 path
// are band_h2's (ip_h2.hip).  What changes is the step pipeline:
//   * two plane buffers (32 KB each): while the waves multiply out of buffer b, they split the
//     next step's features (loaded into registers one step earlier) into buffer !b, piece by
//     piece between the band blocks' MFMAs, where the VALU and LDS issue slots are idle;
//   * one barrier per step: it orders this step's fragment reads of b before the next staging
//     into b, and the staging into !b before the next step's fragment reads;
//   * the shear ring of a segment's epilogue lives in the buffer the segment's last step was
//     multiplied from (free after the step's barrier): 2 slots x 4 KB per wave.  Two slots
//     suffice because a wave's LDS operations execute in order (block a+1's ring writes follow
//     chunk a's readout); chunk m is in slot m & 1, which makes the ring address of an element
//     the same for both of its chunks when a is even and one bit flip apart when a is odd.
//     One more barrier per segment keeps the next staging out of the ring until every wave's
//     readout is done: 5 barriers per 64-channel segment instead of 8;
//   * the segment maxima for the scale check are accumulated in three parity sets, because the
//     staging of a segment's last step now runs inside the previous step.
// A segment whose scale must change restarts the pipeline at its first step (the next
// segment's first step was already staged with the old scale).
#include "band_common.h"

namespace smcv {
namespace h2band {

namespace db {
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kKC = 16;             // channels per step (one 32x32x16 k-step)
constexpr int kSlot = 32 * 32 * 4;  // one ring chunk: 32 d x 32 x fp32
constexpr int kBuf = 32 * 1024;     // one plane buffer (h + m planes) or the 4 waves' rings

template <int TMAX>
struct Geo {
  static constexpr int DMAX = 32 * (TMAX - 1);
  static constexpr int RW = kXT + DMAX;    // right-window rows
  static constexpr int ROWS = RW + kXT;    // + left-tile rows
  static constexpr int PLANE = ROWS * 32;  // one fp16 plane: rows of 16 channels
  static constexpr int GROUPS = ROWS / 4;
  static constexpr int ITEMS = 2 * GROUPS;
  static constexpr int MAXW = 2 * kBuf;   // 3 parity sets x (max|L|, max|R|)
  static constexpr size_t SHM = (size_t)MAXW + 32;
  static_assert(2 * PLANE <= kBuf, "h and m planes fit one buffer");
  static_assert(kWaves * 2 * kSlot <= kBuf, "the 2-slot rings fit one buffer");
  static_assert(ITEMS <= kThreads, "one staging item per lane");
  static_assert(GROUPS % 8 == 0, "8-lane write groups stay inside one chunk");
  static_assert(SHM * 2 <= 160 * 1024, "two workgroups per CU");
};
}  // namespace db

// FUSE 1: the soft-argmin of the volume is folded from the accumulators before the shear
// (fused_softargmin, band_common.h) and stored beside it (f-1, volume kept, one D pass).
template <bool MEAN, int TMAX, int FUSE>
__global__ __launch_bounds__(db::kThreads, 2) void band_h2db(Args args) {
  using namespace db;
  using G = db::Geo<TMAX>;
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

  // ---------------------------------------------------------------- staging role of a lane
  const bool active = tid < G::ITEMS;
  const int ch = min(tid / G::GROUPS, 1);
  const int g = min(tid - ch * G::GROUPS, G::GROUPS - 1);
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
      gload<true>(st.v[kk], p);
      if (kk < lim) p += csl;
    }
  };
  auto vm_wait_st = [&](int after_stores) {  // the 8 feature loads (TMAX-1 chunk stores younger)
    asm volatile(
        "s_cmp_eq_u32 %8, 0\n\t"
        "s_cbranch_scc1 .Ldb_all%=\n\t"
        "s_waitcnt vmcnt(%9)\n\t"
        "s_branch .Ldb_done%=\n"
        ".Ldb_all%=:\n\t"
        "s_waitcnt vmcnt(0)\n"
        ".Ldb_done%=:"
        : "+v"(st.v[0]), "+v"(st.v[1]), "+v"(st.v[2]), "+v"(st.v[3]), "+v"(st.v[4]),
          "+v"(st.v[5]), "+v"(st.v[6]), "+v"(st.v[7])
        : "s"(after_stores), "n"(4 * (TMAX - 1))
        : "memory", "scc");
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
  // The matrix phase of one step on buffer `buf`, with the staging of the next step (into
  // `nbuf`) in pieces between the blocks: `stage_fn(piece)` is called after block piece+1.
  auto band = [&](unsigned buf, auto&& stage_fn) {
    const unsigned char* ab = smem + buf + 32 * wave * 32 + swz(lr, hh);
    const unsigned char* bb = smem + buf + (G::RW + 32 * wave) * 32 + swz(lr, hh);
    const f16x8 bh = *reinterpret_cast<const f16x8*>(bb);
    const f16x8 bm = *reinterpret_cast<const f16x8*>(bb + G::PLANE);
    f16x8 ah[2], am[2];
    auto rd = [&](int t) {
      ah[t & 1] = *reinterpret_cast<const f16x8*>(ab + 1024 * t);
      am[t & 1] = *reinterpret_cast<const f16x8*>(ab + G::PLANE + 1024 * t);
    };
    rd(0);
#pragma unroll
    for (int t = 0; t < TMAX; ++t) {
      if (t + 1 < TMAX) rd(t + 1);
      __builtin_amdgcn_sched_barrier(0);
      f32x16 c = acc[t];  // zero at a segment's first step (its consumer cleared it)
      c = mma(am[t & 1], bh, c);
      c = mma(ah[t & 1], bm, c);
      acc[t] = mma(ah[t & 1], bh, c);
      __builtin_amdgcn_sched_barrier(0);
      stage_fn(t);  // staging work behind this block's MFMAs
      __builtin_amdgcn_sched_barrier(0);
    }
    if constexpr (TMAX < 6) {
#pragma unroll
      for (int t = TMAX; t < 6; ++t) stage_fn(t);  // short bands: the remaining pieces
    }
  };

  // ------------------------------------------------------------------------------ epilogue
  // Lane (lr, hh), element i of block t: R row c_i + 4 hh (c_i = (i & 3) + 8 (i >> 2)), pixel
  // x0w + lr, local disparity 32 (a + 1) + u - c_i with a = T-2-t, u = lr - 4 hh.  Ring (in the
  // plane buffer just multiplied from) [slot][32 d][32 x], chunk m in slot m & 1.  With X =
  // 128 (u - c_i) + 4 lr: chunk a+1 row u - c_i (u >= c_i) and chunk a row 32 + u - c_i both sit
  // at 4096 + X when a is even; when a is odd they sit at X and 8192 + X, i.e. (4096 + X) ^ 4096.
  const int u = lr - 4 * hh;
  const int rl = lane >> 3, cl = lane & 7;
  const size_t plane_stride = (size_t)H * W;
  const int lane_st = rl * H * W + 4 * cl;

  auto epilogue_v = [&](const Work& k, bool fast, unsigned buf, auto scale, auto xlt) {
    // FUSE: the disparity store is issued after the next step's loads and before the chunk
    // stores, so vm_wait_st's count of younger stores stays a lower bound (the wait also covers it)
    if constexpr (FUSE == 1) {
      // the sum kernel folds with an explicit x 1.0 (exact): the register allocator then fits
      // the fold into 256 registers as it does for the mean (368 B of scratch otherwise)
      Args fa = args;
      float one = 1.0f;
      asm volatile("" : "+v"(one));
      if constexpr (!MEAN) fa.mul = one;
      fused_softargmin<TMAX, true, decltype(scale)::value, decltype(xlt)::value, false>(
          acc, fa, k, kL, kR, wave, lr, hh);
    }
    const int x0w = k.x0 + 32 * wave;
    const float mul = args.mul;
    const int kk = -(kL + kR);
    const int jlane = k.js + 32 * wave + 4 * hh;
    const unsigned ringw = lds_addr(smem + buf) + (unsigned)(wave * 2 * kSlot);
    float* ob = out + (((size_t)k.n * D + k.dp) * plane_stride + (size_t)k.y * W + x0w);
    const size_t st8 = (size_t)8 * plane_stride;
    auto write_block = [&](auto tc) {
      constexpr int t = decltype(tc)::value;
      constexpr int a = TMAX - 2 - t;
      int uu = u, jl = jlane;
      unsigned rw = ringw;
      asm volatile("" : "+v"(uu), "+v"(jl), "+v"(rw));
      const unsigned y0 = (unsigned)(4096 + 128 * uu + 4 * lr);  // 4096 + X + 128 c_i
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ci = (i & 3) + 8 * (i >> 2);
        float val = acc[t][i];
        if (MEAN) val *= mul;
        if constexpr (decltype(scale)::value) val = __builtin_ldexpf(val, kk);
        if constexpr (decltype(xlt)::value) val = jl + 32 * t + ci >= 0 ? val : 0.f;
        const unsigned yi = y0 - (unsigned)(128 * ci);
        const unsigned addr = rw + ((a & 1) ? (yi ^ 4096u) : yi);
        lds_store1(addr, val);
      }
      acc[t] = f32x16{};  // ready for the next segment's first step
      asm volatile("" ::: "memory");
    };
    auto read_chunk = [&](int a, f32x4v (&v)[4]) {
      unsigned rb = ringw + (unsigned)(rl * 128 + 16 * cl);
      asm volatile("" : "+v"(rb));
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) v[qq] = lds_load4(rb + (unsigned)((a & 1) * kSlot + 8 * qq * 128));
    };
    auto store_chunk = [&](int a, const f32x4v (&v)[4]) {
      int ls_ = lane_st;
      asm volatile("" : "+v"(ls_));
      float* ol = ob + (size_t)(32 * a) * plane_stride + ls_;
      if (fast) {  // every store valid: exactly 4 (T-1) per lane, counted by vm_wait_st
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          asm volatile("" : "+v"(ol));
          store_quad<true>(ol, v[qq]);
          ol += st8;
        }
      } else {
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          asm volatile("" : "+v"(ol));
          const int dl = 32 * a + 8 * qq + rl;
          if (dl < k.Dp && x0w + 4 * cl < W) store_quad<true>(ol, v[qq]);
          ol += st8;
        }
      }
    };
    // software-pipelined: chunk a's readout is consumed after block t-1's ring writes
    f32x4v vp[4];
    [&]<int... I_>(std::integer_sequence<int, I_...>) {
      (
          [&] {
            constexpr int t = TMAX - 1 - I_;
            constexpr int a = TMAX - 2 - t;
            write_block(std::integral_constant<int, t>{});
            if constexpr (a >= 1) store_chunk(a - 1, vp);
            if constexpr (a >= 0) read_chunk(a, vp);
            __builtin_amdgcn_sched_barrier(0);
          }(),
          ...);
    }(std::make_integer_sequence<int, TMAX>{});
    if constexpr (TMAX >= 2) store_chunk(TMAX - 2, vp);
  };
  auto epilogue = [&](const Work& k, bool fast, unsigned buf) {
    using TT = std::true_type;
    using FF = std::false_type;
    const bool xl = __builtin_amdgcn_readfirstlane(k.js) < 0;
    if (__builtin_amdgcn_readfirstlane(kL + kR) != 0) {
      if (xl)
        epilogue_v(k, fast, buf, TT{}, TT{});
      else
        epilogue_v(k, fast, buf, TT{}, FF{});
      return;
    }
    if (xl)
      epilogue_v(k, fast, buf, FF{}, TT{});
    else
      epilogue_v(k, fast, buf, FF{}, FF{});
  };

  auto slow_segment = [&](const Work& k) {
    const float mul = MEAN ? args.mul : 1.0f;
    const float* lrow = L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;
    const float* rrow = R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h;
    auto cell = [&](int x, int d) {
      float s = 0.f;
      if (x >= d) {
        for (int c = 0; c < cpg; ++c)
          s = __builtin_fmaf(ld1(lrow + (int64_t)c * ls.c + x), ld1(rrow + (int64_t)c * rs.c + x - d), s);
        s *= mul;
      }
      return s;
    };
    for (int idx = tid; idx < k.Dp * kXT; idx += kThreads) {
      const int dl = idx / kXT, x = k.x0 + idx % kXT, d = k.dp + dl;
      if (x >= W) continue;
      store_one<float>(out + (((size_t)k.n * D + d) * H + k.y) * W + x, cell(x, d));
    }
    if constexpr (FUSE == 1) {  // the pixel's soft-argmin from the same exact cells (one D pass)
      for (int xx = tid; xx < kXT; xx += kThreads) {
        const int x = k.x0 + xx;
        if (x >= W) continue;
        float m = -INFINITY;
        double s = 0.0, t = 0.0;  // relative to m
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
        store_one<float>(args.disp + ((size_t)k.n * H + k.y) * W + x,
                         (nan || m == INFINITY || m == -INFINITY) ? NAN : (float)(t / s));
      }
    }
  };

  // ----------------------------------------------------------------------------- main loop
  if (tid < 6) *lds_word(maxw + 4 * tid) = 0u;
  __syncthreads();  // cleared before any wave publishes
  // The loop runs one step per iteration: it multiplies step (it, ks) out of buffer bm (when
  // `mul`) and stages step (sit, sks) into buffer bm ^ kBuf between the blocks, issuing the loads
  // of the step after that.  The loads have one site before the loop, one in the loop and one
  // on the restart path, all merging at the loop head (scripts/check_h2_asm.py checks that no
  // loaded register is touched before its wait).  A pipeline (re)start is an iteration whose
  // multiply is discarded (`mul` false: its accumulators are cleared after the barrier).
  bool redone = false;
  bool pend = false;  // 4 (T-1) chunk stores were issued after the outstanding loads
#pragma unroll
  for (int t = 0; t < TMAX; ++t) acc[t] = f32x16{};
  int it = 0, ks = 0;        // the step multiplied this iteration (if mul)
  int sit = 0, sks = 0;      // the step staged this iteration
  int set = 0, sset = 0;     // maxima sets (item % 3) of it and sit
  bool mul = false;
  unsigned bm = kBuf;        // buffer multiplied from; staging goes to bm ^ kBuf
  Work cur = decode(witem(0), args, DMAX);   // item it
  Work scur = cur;                           // item sit
  load(scur, 0);
  while (it < nitems) {
    const bool stage_ok = sit < nitems;
    // the step after (sit, sks): its loads are issued behind this iteration's blocks
    const bool nk = sks + 1 < nks;
    const int lit = nk ? sit : sit + 1, lks = nk ? sks + 1 : 0;
    const bool load_ok = lit < nitems;
    const Work lw = nk ? scur : (load_ok ? decode(witem(lit), args, DMAX) : scur);
    const unsigned sb = bm ^ (unsigned)kBuf;
    auto stage_fn = [&](int piece) {
      if (piece == 0) {
        vm_wait_st(__builtin_amdgcn_readfirstlane((int)pend));
        pend = false;
        if (sks == 0) mx = 0.f;
      }
      if (piece < 5) put_piece(piece, sb);
      if (piece == 5) {
        if (stage_ok && sks == nks - 1) publish_max(sset);
        if (load_ok) load(lw, lks);
      }
    };
    __builtin_amdgcn_s_setprio(1);
    band(bm, stage_fn);
    __builtin_amdgcn_s_setprio(0);
    __syncthreads();  // fragment reads of bm done; staging of sb complete
    bool restart = false;
    if (!mul) {
#pragma unroll
      for (int t = 0; t < TMAX; ++t) acc[t] = f32x16{};  // a (re)start: nothing multiplied
    } else if (ks == nks - 1) {
      // ---- end of segment `it`: range check on its maxima, then the epilogue
      const unsigned mw = maxw + 8u * (unsigned)set;
      const float ml = __uint_as_float(*lds_word(mw));
      const float mr = __uint_as_float(*lds_word(mw + 4));
      const int set2 = set == 0 ? 2 : set - 1;  // (it + 2) % 3: cleared for segment it + 2
      if (tid < 2) *lds_word(maxw + 8u * (unsigned)set2 + 4 * tid) = 0u;
      const bool fin = ml <= 3.4e38f && mr <= 3.4e38f;
      const int el = ml > 0.f ? exp_of(ml) : 0, er = mr > 0.f ? exp_of(mr) : 0;
      const bool okl = ml == 0.f || (el + kL <= 15 && el + kL >= -1);
      const bool okr = mr == 0.f || (er + kR <= 15 && er + kR >= -1);
      const bool fast = cur.x0 + kXT <= W && cur.Dp == DMAX;
      if (fin && okl && okr) {
        epilogue(cur, fast, bm);
        pend = fast;
        redone = false;
      } else {
        const int nkl = ml > 0.f ? 13 - el : kL, nkr = mr > 0.f ? 13 - er : kR;
        if (!fin || redone || nkl < -100 || nkl > 100 || nkr < -100 || nkr > 100) {
          slow_segment(cur);  // scale unchanged: the staged next step stays valid
          redone = false;
        } else {
          kL = nkl;  // recompute with the new scale: restart at this segment's first step
          kR = nkr;
          redone = true;
          restart = true;
        }
#pragma unroll
        for (int t = 0; t < TMAX; ++t) acc[t] = f32x16{};
      }
    }
    if (restart) {
      vm_wait_st(0);
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
      load(scur, 0);
      mul = false;
      pend = false;
      continue;  // (it, ks) stays: its segment is multiplied again from step 0
    }
    if (mul && ks == nks - 1) __syncthreads();  // ring readouts done before bm is staged into
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
  vm_wait_st(0);  // nothing in flight when the registers die
}

template <bool MEAN, int TMAX, int FUSE>
int launch_h2db(Args a, int64_t N, hipStream_t st) {
  using G = db::Geo<TMAX>;
  a.tiles = (int)ceil_div(a.W, kXT);
  const int64_t nwork = (int64_t)a.tiles * a.H * N * a.G * a.npass;
  if (nwork > INT32_MAX / 64) return fail(SM_EINVAL, "band kernel: too much work for one launch");
  a.nwork = (int)nwork;
  auto kern = band_h2db<MEAN, TMAX, FUSE>;
  static std::atomic<unsigned long long> lds_done{0};
  const int dev = stream_device(st);
  if (int rc = ensure_lds_limit(reinterpret_cast<const void*>(kern), (int)G::SHM, dev, lds_done))
    return rc;
  int64_t nwg = std::min<int64_t>(nwork, 2 * (int64_t)device_cus(dev));
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(db::kThreads), G::SHM, st, a);
  return check_launch("band_h2db");
}

// fp32 inner product / correlation volume on the double-buffered band kernel; *handled = false
// when the shape is not one it takes (4-element aligned rows, one channel group).
int band_h2db_run(const Args& a, int64_t N, bool mean, bool aligned4, hipStream_t st,
                  bool* handled) {
  *handled = false;
  if (!aligned4 || a.G != 1 || a.pw > 192) return SM_OK;
  *handled = true;
  auto go = [&](auto tm) {
    constexpr int TM = decltype(tm)::value;
    return mean ? launch_h2db<true, TM, 0>(a, N, st) : launch_h2db<false, TM, 0>(a, N, st);
  };
  if (a.pw <= 32) return go(std::integral_constant<int, 2>{});
  if (a.pw <= 64) return go(std::integral_constant<int, 3>{});
  if (a.pw <= 128) return go(std::integral_constant<int, 5>{});
  return go(std::integral_constant<int, 7>{});
}

// The same kernel with the soft-argmin folded in (FUSE 1): volume and disparity (args.disp) in
// one pass; one D pass (D <= 192), fp32, aligned rows.
int band_h2db_fused_run(const Args& a, int64_t N, bool mean, bool aligned4, hipStream_t st,
                        bool* handled) {
  *handled = false;
  if (!aligned4 || a.G != 1 || a.pw > 192 || a.npass != 1 || a.out == nullptr ||
      a.disp == nullptr || a.ws_m != nullptr)
    return SM_OK;
  *handled = true;
  auto go = [&](auto tm) {
    constexpr int TM = decltype(tm)::value;
    return mean ? launch_h2db<true, TM, 1>(a, N, st) : launch_h2db<false, TM, 1>(a, N, st);
  };
  if (a.pw <= 32) return go(std::integral_constant<int, 2>{});
  if (a.pw <= 64) return go(std::integral_constant<int, 3>{});
  if (a.pw <= 128) return go(std::integral_constant<int, 5>{});
  return go(std::integral_constant<int, 7>{});
}

}  // namespace h2band
}  // namespace smcv

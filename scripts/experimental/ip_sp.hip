// Inner-product / correlation cost volume (N, D, H, W) from fp32 features: the software-
// pipelined band kernel ("sp"), one workgroup of four waves per CU, one wave per SIMD.
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// The contraction, the operands (per-segment power-of-two scale, round-to-nearest two-plane fp16
// split, h*h' + h*m' + m*h' on v_mfma_f32_32x32x16_f16), the tiling (4 waves x 32 pixels per
// 128-pixel segment, T = 1 + DMAX/32 blocks of 32 x 32 per wave) and the scale control are
// band_h2db's (ip_h2db.hip).  What changes is where the epilogue runs:
//   * band_h2db shears and stores a segment's volume at the segment's end, in a burst that stops
//     the wave's matrix work (and its co-resident workgroup's staging) for ~30 % of its time;
//   * here every wave keeps TWO accumulator sets in AGPRs (one wave per SIMD: 512 registers),
//     multiplies segment i into one while it shears and stores segment i-1 out of the other, one
//     "drain stage" per band block, spread over segment i's steps.  The MFMAs, the staging of the
//     next step, the shear and the volume stores all run in one instruction stream, and HBM sees
//     a steady store stream instead of bursts;
//   * the channel steps per segment (NKS) are a template parameter: every step of a segment is
//     its own straight-line code with its drain stages, staging pieces and loads fixed at
//     compile time, and nothing that holds the big register sets sits under a branch (the
//     register allocator then keeps both accumulator sets in place).  The feature loads and
//     the volume stores are ordinary compiler-visible memory operations, issued loads first:
//     the compiler's own vmcnt waits then leave a step's stores in flight while the next step
//     waits for its loads.  Work past the end is done on clamped, valid addresses and
//     discarded: the volume stores are raw-buffer stores whose masked lanes carry an
//     out-of-range offset, and a drain with nothing to drain gets a zero-size buffer;
//   * pad pixels (x < 0, x >= W) are loaded from the nearest valid pixel group of the row and
//     split with a zero scale, so the staging has no per-lane branches either; a non-finite
//     value there (or NaN in the segment's data, which the max|x| check does not see) can only
//     reach cells x < d, which the drain forces to 0 when the segment has any (js < 0), or
//     columns x >= W, which are not stored;
//   * the shear ring is per wave, 4 slots x 4 KB: chunk m (32 disparities x 32 pixels) lives in
//     slot (m + 1) & 3, so a block's two chunks are adjacent (ring address = lane base +
//     immediate) except for the block whose chunks wrap (slots 3 and 0), which masks its
//     addresses.
// One barrier per step: it orders this step's fragment reads of buffer b before the next
// staging into b, and the staging into !b before the next step's fragment reads.
#include "band_common.h"

#ifndef SMCV_SP_ABLATE
#define SMCV_SP_ABLATE 0  // diagnostics only (scripts/build_variants.py): 1 no drain stages, 2 no
#endif                    // staging, 4 feature loads from one line, 8 no MFMA, 16 no barrier,
                          // 32 no volume stores, 64 no ring writes / readouts (stores kept),
                          // 128 no feature loads
#ifndef SMCV_SP_SETS
#define SMCV_SP_SETS 4  // feature-load register sets (loads issued SETS - 1 steps ahead)
#endif

namespace smcv {
namespace h2band {

namespace sp {
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kKC = 16;             // channels per step (one 32x32x16 k-step)
constexpr int kSlot = 32 * 32 * 4;  // one ring chunk: 32 d x 32 x fp32
constexpr int kRingW = 4 * kSlot;   // one wave's ring
constexpr int kRings = kWaves * kRingW;

template <int TMAX>
struct Geo {
  static constexpr int DMAX = 32 * (TMAX - 1);
  static constexpr int RW = kXT + DMAX;    // right-window rows
  static constexpr int ROWS = RW + kXT;    // + left-tile rows
  static constexpr int PLANE = ROWS * 32;  // one fp16 plane: rows of 16 channels
  static constexpr int BUF = 2 * PLANE;    // h + m planes of one step
  static constexpr int GROUPS = ROWS / 4;
  static constexpr int ITEMS = 2 * GROUPS;
  static constexpr int PL0 = kRings;          // plane buffers after the rings (ring bases are
  static constexpr int MAXW = PL0 + 2 * BUF;  // multiples of kRingW)
  // 4 maxima sets x (max|L|, max|R|); then a dummy target (h and m) for the idle staging lanes
  static constexpr int DUMMY = MAXW + 64;
  static constexpr size_t SHM = (size_t)DUMMY + PLANE + 16;
  static_assert(ITEMS <= kThreads, "one staging item per lane");
  static_assert(GROUPS % 8 == 0, "8-lane write groups stay inside one chunk");
  static_assert(SHM <= 160 * 1024, "one workgroup per CU");
};

// Drain stage k (0 <= k < T) of a segment runs in step ks = floor(k NKS / T) of the next
// segment: step ks runs the stages [ceil(ks T / NKS), ceil((ks + 1) T / NKS)), spread over its
// block slots 2 .. T-1, i.e. after the step's feature loads (issued at slot 2, once the staging
// has consumed the previous ones), so that a step's loads never wait for its own stores.
constexpr int stage_lo(int ks, int T, int NKS) { return (ks * T + NKS - 1) / NKS; }
constexpr int stage_slot(int k, int T, int NKS) {
  const int ks = (k * NKS) / T, lo = stage_lo(ks, T, NKS), cnt = stage_lo(ks + 1, T, NKS) - lo;
  return 2 + ((k - lo) * (T - 2)) / cnt;
}
// Stage k >= 1 issues one chunk's 4 stores, all after the step's loads.
constexpr int stores_in_step(int ks, int T, int NKS) {
  int n = 0;
  for (int k = stage_lo(ks, T, NKS); k < stage_lo(ks + 1, T, NKS); ++k)
    if (k >= 1) n += 4;
  return n;
}
}  // namespace sp

template <bool MEAN, int TMAX, int NKS, int NSETS>
__global__ __launch_bounds__(sp::kThreads, 1) void band_sp(Args args) {
  using namespace sp;
  using G = sp::Geo<TMAX>;
  constexpr int T = TMAX;
  constexpr int DMAX = G::DMAX;
  static_assert(T >= 3, "the staging occupies block slots 0-2");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const float* __restrict__ L = static_cast<const float*>(args.L);
  const float* __restrict__ R = static_cast<const float*>(args.R);
  const int cpg = args.cpg, H = args.H, W = args.W, D = args.D;
  const Strides4 ls = args.ls, rs = args.rs;

  const Sched sched(args.nwork, args.npass);
  if (sched.none) return;  // the whole workgroup leaves together
  const int nitems = sched.nitems;
  // the work item of index i, clamped (work past the end is done on a valid item, discarded)
  auto witem = [&](int i) -> Work { return decode(sched.item(min(i, nitems - 1)), args, DMAX); };

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  const int lr = lane & 31;
  const int hh = lane >> 5;

  // ---------------------------------------------------------------- staging role of a lane
  const bool active = tid < G::ITEMS;
  const int ch = min(tid / G::GROUPS, 1);
  const int g = min(tid - ch * G::GROUPS, G::GROUPS - 1);
  const bool isR = 4 * g < G::RW;
  const int64_t cs = isR ? rs.c : ls.c;

  // NSETS feature-load register sets: the loads of step j land in set j % NSETS, issued
  // NSETS - 1 steps before the step that stages them
  f32x4v sv[NSETS][8];
  if constexpr (SMCV_SP_ABLATE & 128)
    for (int i = 0; i < NSETS; ++i)
      for (int kk = 0; kk < 8; ++kk) sv[i][kk] = f32x4v{1.f, -1.f, 0.5f, 2.f};
  bool okp[NSETS];  // the loaded pixel group is inside the row (else: split with a zero scale)
  auto load = [&](int set, const Work& k, int ks) __attribute__((always_inline)) {
    const int px = isR ? k.js + 4 * g : k.x0 + 4 * g - G::RW;
    okp[set] = active && px >= 0 && px < W;
    int pxc = min(max(px, 0), W - 4);  // pad groups: the nearest valid group
    if constexpr (SMCV_SP_ABLATE & 4) pxc = 0;
    const float* p = (isR ? R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h
                          : L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h) +
                     pxc + (SMCV_SP_ABLATE & 4 ? 0 : (int64_t)(ks * kKC + 8 * ch) * cs);
    int64_t csl = SMCV_SP_ABLATE & 4 ? 0 : cs;
    asm volatile("" : "+v"(csl));
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      if constexpr (SMCV_SP_ABLATE & 128)
        asm volatile("" : "+v"(sv[set][kk]));  // no load: the registers as they are
      else
        gload<false>(sv[set][kk], p);  // compiler-tracked: it places the vmcnt waits itself
      p += csl;
    }
  };
  int kL = 0, kR = 0;  // per-segment scale exponents of the staging side (workgroup-uniform)
  float mx = 0.f;      // this lane's max|x| over the segment being staged (valid groups only)
  float sc = 0.f;      // this lane's split scale: 2^k, or 0 for a pad group
  // Staging of one step into plane buffer `buf` (byte offset), in pieces: piece 0 tracks
  // max|x| and sets the scale; pieces 1-4 split pixel p = piece-1 into the h and m planes.
  auto put_piece = [&](int set, int piece, unsigned buf) __attribute__((always_inline)) {
    if constexpr (SMCV_SP_ABLATE & 2) return;
    f32x4v(&sv_)[8] = sv[set];
    if (piece == 0) {
      float m0 = 0.f, m1 = 0.f;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m0) : "v"(sv_[kk].x), "v"(sv_[kk].y));
        asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m1) : "v"(sv_[kk].z), "v"(sv_[kk].w));
      }
      mx = okp[set] ? fmaxf(mx, fmaxf(m0, m1)) : mx;
      sc = okp[set] ? __builtin_ldexpf(1.0f, isR ? kR : kL) : 0.f;
      return;
    }
    const int p = piece - 1;
    unsigned o0 = buf + (unsigned)swz(4 * g, ch);
    asm volatile("" : "+v"(o0));
    uint4 wh, wm;
    const float xs[8] = {sv_[0][p], sv_[1][p], sv_[2][p], sv_[3][p],
                         sv_[4][p], sv_[5][p], sv_[6][p], sv_[7][p]};
    split_quad(xs, sc, wh, wm);
    const unsigned off = active ? o0 ^ (32u * p) : (unsigned)G::DUMMY;  // (no branch)
    *reinterpret_cast<uint4*>(smem + off) = wh;
    *reinterpret_cast<uint4*>(smem + G::PLANE + off) = wm;
  };
  // maxima words: set s (0..3) at MAXW + 8 s: max|L|, max|R|
  const unsigned maxw = lds_addr(smem + G::MAXW);
  auto publish_max = [&](int set) __attribute__((always_inline)) {  // a segment fully staged
    const unsigned uml = __builtin_amdgcn_readfirstlane(__float_as_uint(wave_max(isR ? 0.f : mx)));
    const unsigned umr = __builtin_amdgcn_readfirstlane(__float_as_uint(wave_max(isR ? mx : 0.f)));
    if (lane == 0) {
      asm volatile("ds_max_u32 %0, %1\n\tds_max_u32 %0, %2 offset:4"
                   :
                   : "v"(maxw + 8u * (unsigned)set), "v"(uml), "v"(umr)
                   : "memory");
    }
  };

  // ------------------------------------------------------------------- MFMA role of a wave
  f32x16 acc0[T], acc1[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc0[t] = acc1[t] = f32x16{};
  auto mma = [](f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  };
  auto accp = [&]<int Q>() -> f32x16(&)[T] {
    if constexpr (Q == 0) return acc0; else return acc1;
  };

  // ------------------------------------------------------------- drain (shear + stores)
  // Lane (lr, hh), element i of block t: R row c_i + 4 hh (c_i = (i & 3) + 8 (i >> 2)), pixel
  // x0w + lr, local disparity 32 (a + 1) + u - c_i with a = T-2-t, u = lr - 4 hh.  Chunk m in
  // slot (m + 1) & 3 of the wave's ring ([slot][32 d][32 x] fp32): where the block's chunks a,
  // a+1 sit in adjacent slots the element's address is wbase + (slot(a) + 1) 4096 - 128 c_i -
  // 512 with wbase = ring + 512 + 128 u + 4 lr (>= ring: u >= -4), an immediate offset per
  // element; for a = 2 (slots 3, 0) it is ring + ((16384 + 128 (u - c_i) + 4 lr) & 16383).
  const int u = lr - 4 * hh;
  const unsigned ringw = lds_addr(smem) + (unsigned)(wave * kRingW);
  const int rl = lane >> 3, cl = lane & 7;
  const int64_t plane_stride = (int64_t)H * W;
  // the drained segment (workgroup-uniform); nothing to drain: a zero-size store buffer
  Work pw = witem(0);
  int p_kk = 0;
  bool p_special = false;  // scaled (kk != 0) or holding cells x < d (js < 0)
  int p_bytes = 0;        // 0x80000000 (valid) or 0 (every store dropped)
  bool p_full = false;    // the whole 128-pixel segment and all DMAX disparities are stored
  float* p_ob = static_cast<float*>(args.out);  // (n, dp, y, x0w) of the drained segment
  f32x4v vp[4];           // one chunk's readout, stored in the next stage

  // Ring writes as inline asm: an immediate offset per element (the compiler cannot prove the
  // opaque lane base non-negative, so it would not fold them), and the plain path stores the
  // accumulators straight from their AGPRs (no copy, no VALU).  LDS operations of a wave
  // execute in order, so the later (compiler-generated) readouts see them; extra LDS operations
  // only make the compiler's own lgkmcnt waits conservative.
  auto write_block = [&]<int Q, int t>() __attribute__((always_inline)) {
    if constexpr (SMCV_SP_ABLATE & 64) return;
    constexpr int a = T - 2 - t;
    constexpr bool wrap = ((a + 1) & 3) == 3;  // chunks a, a+1 in slots 3 and 0
    f32x16(&acc)[T] = accp.template operator()<Q>();
    // opaque here: the drained set is invariant over the steps of the next segment, and the
    // compiler would otherwise hoist its reads (and scaling) out of the step sequence
    asm volatile("" : "+a"(acc[t]));
    // lane bases, recomputed per block (opaque: not hoisted as invariants)
    int uu = u, ll = lr, jl = pw.js + 32 * wave + 4 * hh;
    asm volatile("" : "+v"(uu), "+v"(ll), "+v"(jl));
    const unsigned wb = ringw + (unsigned)(512 + 128 * uu + 4 * ll);
    const unsigned ww = (unsigned)(16384 + 128 * uu + 4 * ll);
    const bool special = p_special;
    if (special || MEAN) {  // values through VGPRs (scaled, forced to 0 at x < d, or the mean)
      asm volatile("" : "+a"(acc[t]));  // the copies to VGPRs stay inside this branch
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ci = (i & 3) + 8 * (i >> 2);
        float val = acc[t][i];
        if constexpr (MEAN) val *= args.mul;
        if (special) {
          val = __builtin_ldexpf(val, p_kk);
          val = jl + 32 * t + ci >= 0 ? val : 0.f;  // R pad rows: cells x < d
        }
        if constexpr (wrap) {
          const unsigned ad = ringw | ((ww - (unsigned)(128 * ci)) & 16383u);
          asm volatile("ds_write_b32 %0, %1" : : "v"(ad), "v"(val) : "memory");
        } else {
          asm volatile("ds_write_b32 %0, %1 offset:%2"
                       :
                       : "v"(wb), "v"(val), "n"((((a + 1) & 3) + 1) * 4096 - 128 * ci - 512)
                       : "memory");
        }
      }
    } else {  // straight from the AGPRs
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int ci = (i & 3) + 8 * (i >> 2);
        if constexpr (wrap) {
          const unsigned ad = ringw | ((ww - (unsigned)(128 * ci)) & 16383u);
          asm volatile("ds_write_b32 %0, %1" : : "v"(ad), "a"(acc[t][i]) : "memory");
        } else {
          asm volatile("ds_write_b32 %0, %1 offset:%2"
                       :
                       : "v"(wb), "a"(acc[t][i]), "n"((((a + 1) & 3) + 1) * 4096 - 128 * ci - 512)
                       : "memory");
        }
      }
    }
  };
  auto read_chunk = [&]<int a>() __attribute__((always_inline)) {
    if constexpr (SMCV_SP_ABLATE & 64) return;
    int rr = rl, cc = cl;
    asm volatile("" : "+v"(rr), "+v"(cc));
    const unsigned rb = ringw + (unsigned)(rr * 128 + 16 * cc);
#pragma unroll
    for (int qq = 0; qq < 4; ++qq)
      vp[qq] = lds_load4(rb + (unsigned)(((a + 1) & 3) * kSlot + qq * 1024));
  };
  auto store_chunk = [&]<int a>() __attribute__((always_inline)) {
    if constexpr (SMCV_SP_ABLATE & 32) return;
    float* cb = p_ob + (int64_t)(32 * a) * plane_stride;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(cb, (short)0, p_bytes, 0x00020000);
    int rr = rl, cc = cl;
    asm volatile("" : "+v"(rr), "+v"(cc));
    const unsigned q8 = (unsigned)(8 * plane_stride * 4);
    const unsigned lo = (unsigned)(rr * plane_stride * 4 + 16 * cc);
    if (p_full) {  // every cell of the segment is inside the volume
#pragma unroll
      for (int qq = 0; qq < 4; ++qq)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, vp[qq]), rsrc,
            lo + (unsigned)qq * q8, 0, SMCV_NT_STORE ? 2 : 0);
    } else {
      // masked lanes: the offset's top bit set (out of range; no select, which the compiler
      // would turn into branches around the stores)
      const unsigned xbad = (unsigned)(pw.x0 + 32 * wave + 4 * cc >= W) << 31;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const unsigned bad = xbad | ((unsigned)(32 * a + 8 * qq + rr >= pw.Dp) << 31);
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, vp[qq]), rsrc,
            (lo + (unsigned)qq * q8) | bad, 0, SMCV_NT_STORE ? 2 : 0);
      }
    }
  };
  // stage k: W(T-1) W(T-2) R(0) | S(k-1) W(T-2-k) R(k) | S(T-2)
  auto drain_stage = [&]<int Q, int k>() __attribute__((always_inline)) {
    if constexpr (SMCV_SP_ABLATE & 1) {
    } else if constexpr (k == 0) {
      write_block.template operator()<Q, T - 1>();
      write_block.template operator()<Q, T - 2>();
      read_chunk.template operator()<0>();
    } else if constexpr (k <= T - 2) {
      store_chunk.template operator()<k - 1>();
      write_block.template operator()<Q, T - 2 - k>();
      read_chunk.template operator()<k>();
    } else {
      store_chunk.template operator()<T - 2>();
    }
  };
  auto set_prev = [&](const Work& k, bool valid) __attribute__((always_inline)) {
    pw = k;
    p_kk = -(kL + kR);
    p_special = p_kk != 0 || k.js < 0;
    p_bytes = valid ? (int)0x80000000 : 0;
    p_full = k.Dp == DMAX && k.x0 + kXT <= W;
    p_ob = static_cast<float*>(args.out) +
           (((int64_t)k.n * D + k.dp) * plane_stride + (int64_t)k.y * W + k.x0 + 32 * wave);
  };

  auto barrier = []() __attribute__((always_inline)) {
    if constexpr (SMCV_SP_ABLATE & 16)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    else
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };

  // --------------------------------------------------------------------------- the steps
  // The loop body runs U segments (U even: both accumulator sets; U NKS a multiple of NSETS:
  // the load sets), so every step's accumulator set, load sets and drain stages are fixed at
  // compile time.  Step G (0 <= G < U NKS) of the body is step KS = G % NKS of the body's
  // segment G / NKS; wq[k] is the work item it + k (k < LA).
  constexpr int U = [] {
    int u = 2;
    while ((u * NKS) % NSETS != 0) u += 2;
    return u;
  }();
  constexpr int LA = 1 + (NKS - 1 + NSETS) / NKS;  // items a step's loads can reach
  int it = 0;            // the segment multiplied
  unsigned bm = G::PL0;  // plane buffer multiplied from (the other one is staged into)
  Work wq[LA];
#pragma unroll
  for (int k = 0; k < LA; ++k) wq[k] = witem(k);
  // Step G: multiply out of bm into acc<P>, issue the loads of step G + NSETS into the set that
  // step G's features were staged from (free since step G-1), stage step G + 1 from its set
  // into the other buffer, run the drain stages of the previous segment (acc<1-P>) that fall
  // into this step.
  auto step = [&]<int P, int GS>() __attribute__((always_inline)) {
    constexpr int KS = GS % NKS;
    f32x16(&acc)[T] = accp.template operator()<P>();
    constexpr int k0 = stage_lo(KS, T, NKS), k1 = stage_lo(KS + 1, T, NKS);
    // the staged step (it + sd, ss) and the loaded one (it + ld, lks)
    constexpr int sd = (KS + 1) / NKS, ss = (KS + 1) % NKS;
    constexpr int ld = (KS + NSETS) / NKS, lks = (KS + NSETS) % NKS;
    constexpr int sset = (GS + 1) % NSETS, lset = GS % NSETS;
    const unsigned sb = bm ^ (unsigned)(G::PL0 ^ (G::PL0 + G::BUF));
    auto slot = [&](auto tc) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value;
      if constexpr (t == 0) {
        load(lset, wq[ld], lks);
        if constexpr (ss == 0) mx = 0.f;  // the staged step opens its segment
        put_piece(sset, 0, sb);
        put_piece(sset, 1, sb);
      }
      if constexpr (t == 1) {
        put_piece(sset, 2, sb);
        put_piece(sset, 3, sb);
      }
      if constexpr (t == 2) {
        put_piece(sset, 4, sb);
        if constexpr (ss == NKS - 1) {  // the staged segment is complete: its maxima
          if (it + sd < nitems) publish_max((it + sd) & 3);
        }
      }
      [&]<int... K_>(std::integer_sequence<int, K_...>) __attribute__((always_inline)) {
        (
            [&]() __attribute__((always_inline)) {
              constexpr int k = k0 + K_;
              if constexpr (stage_slot(k, T, NKS) == t) drain_stage.template operator()<1 - P, k>();
            }(),
            ...);
      }(std::make_integer_sequence<int, k1 - k0>{});
    };
    const unsigned char* ab = smem + bm + 32 * wave * 32 + swz(lr, hh);
    const unsigned char* bb = smem + bm + (G::RW + 32 * wave) * 32 + swz(lr, hh);
    const f16x8 bh = *reinterpret_cast<const f16x8*>(bb);
    const f16x8 bmv = *reinterpret_cast<const f16x8*>(bb + G::PLANE);
    f16x8 ah[2], am[2];
    auto rd = [&](int t) __attribute__((always_inline)) {
      ah[t & 1] = *reinterpret_cast<const f16x8*>(ab + 1024 * t);
      am[t & 1] = *reinterpret_cast<const f16x8*>(ab + G::PLANE + 1024 * t);
    };
    rd(0);
    [&]<int... I_>(std::integer_sequence<int, I_...>) __attribute__((always_inline)) {
      (
          [&]() __attribute__((always_inline)) {
            constexpr int t = I_;
            if constexpr (t + 1 < T) rd(t + 1);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (SMCV_SP_ABLATE & 8) {
              asm volatile("" : : "v"(ah[t & 1]), "v"(am[t & 1]), "v"(bh), "v"(bmv));
            } else {
              f32x16 c;
              if constexpr (KS == 0)
                c = mma(am[t & 1], bh, f32x16{});
              else
                c = mma(am[t & 1], bh, acc[t]);
              c = mma(ah[t & 1], bmv, c);
              acc[t] = mma(ah[t & 1], bh, c);
            }
            __builtin_amdgcn_sched_barrier(0);
            slot(std::integral_constant<int, t>{});
            __builtin_amdgcn_sched_barrier(0);
          }(),
          ...);
    }(std::make_integer_sequence<int, T>{});
    barrier();
    bm = sb;
  };

  // exact fp32 FMA path for a segment holding a non-finite value or out of the scale range
  auto slow_segment = [&](const Work& k) __attribute__((always_inline)) {
    const float mul = MEAN ? args.mul : 1.0f;
    float* out = static_cast<float*>(args.out);
    const float* lrow = L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;
    const float* rrow = R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h;
    for (int idx = tid; idx < k.Dp * kXT; idx += kThreads) {
      const int dl = idx / kXT, x = k.x0 + idx % kXT, d = k.dp + dl;
      if (x >= W) continue;
      float s = 0.f;
      if (x >= d) {
        for (int c = 0; c < cpg; ++c)
          s = __builtin_fmaf(lrow[(int64_t)c * ls.c + x], rrow[(int64_t)c * rs.c + x - d], s);
        s *= mul;
      }
      store_one<float>(out + (((int64_t)k.n * D + d) * H + k.y) * W + x, s);
    }
  };

  // ----------------------------------------------------------------------------- main loop
  if (tid < 8) *lds_word(maxw + 4 * tid) = 0u;
  barrier();  // cleared before any wave publishes

  // (Re)start the pipeline at segment `it` (body step GS0 = its step 0): load and stage that
  // step into bm, publish its maxima when it is the segment's only step, issue the loads of
  // the NSETS - 1 steps after it.
  auto prologue = [&]<int GS0>() __attribute__((always_inline)) {
    load(GS0 % NSETS, wq[0], 0);
    mx = 0.f;
#pragma unroll
    for (int piece = 0; piece < 5; ++piece) put_piece(GS0 % NSETS, piece, bm);
    if constexpr (NKS == 1) publish_max(it & 3);
#pragma unroll
    for (int k = 1; k < NSETS; ++k) load((GS0 + k) % NSETS, wq[k / NKS], k % NKS);
    // nothing pending on this path at the loop join (see ip_rs.hip: the compiler's wait
    // placement would otherwise carry the restart's registers into every segment's first step)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    barrier();
  };
  prologue.template operator()<0>();
  set_prev(wq[0], false);
  bool redone = false;

  // Body segment SI: multiplied into acc<SI % 2> (the previous one drained out of the other
  // set meanwhile), then its range check; returns true when the workgroup's last segment is done.
  auto segment = [&]<int SI>() __attribute__((always_inline)) -> bool {
    constexpr int P = SI % 2;
    for (;;) {
      [&]<int... K_>(std::integer_sequence<int, K_...>) __attribute__((always_inline)) {
        (step.template operator()<P, SI * NKS + K_>(), ...);
      }(std::make_integer_sequence<int, NKS>{});
      // ---- end of segment `it`: the range check on its maxima
      const unsigned mw = maxw + 8u * (unsigned)(it & 3);
      const float ml = __uint_as_float(*lds_word(mw));
      const float mr = __uint_as_float(*lds_word(mw + 4));
      if (tid < 2) *lds_word(maxw + 8u * (unsigned)((it + 3) & 3) + 4 * tid) = 0u;
      const bool fin = ml <= 3.4e38f && mr <= 3.4e38f;
      const int el = ml > 0.f ? exp_of(ml) : 0, er = mr > 0.f ? exp_of(mr) : 0;
      const bool okl = ml == 0.f || (el + kL <= 15 && el + kL >= -1);
      const bool okr = mr == 0.f || (er + kR <= 15 && er + kR >= -1);
      if (fin && okl && okr) {
        set_prev(wq[0], true);  // drained by the next segment's steps (or after the loop)
        redone = false;
      } else {
        set_prev(wq[0], false);
        const int nkl = ml > 0.f ? 13 - el : kL, nkr = mr > 0.f ? 13 - er : kR;
        if (!fin || redone || nkl < -100 || nkl > 100 || nkr < -100 || nkr > 100) {
          slow_segment(wq[0]);  // scale unchanged: the staged next step stays valid
          redone = false;
        } else {
          // recompute with the new scale: restart at this segment's first step (the staged
          // step and the loads in flight used the old scale)
          kL = nkl;
          kR = nkr;
          redone = true;
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          barrier();  // every wave has read the maxima
          if (tid < 4) {  // this segment's set and the next one's (its staged step published)
            const int s4 = (tid >> 1) == 0 ? (it & 3) : ((it + 1) & 3);
            *lds_word(maxw + 8u * (unsigned)s4 + 4 * (tid & 1)) = 0u;
          }
          barrier();
          prologue.template operator()<SI * NKS>();
          continue;
        }
      }
      ++it;
#pragma unroll
      for (int k = 0; k + 1 < LA; ++k) wq[k] = wq[k + 1];
      wq[LA - 1] = witem(it + LA - 1);
      return it >= nitems;
    }
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
  // the last segment's drain (in acc<(it - 1) & 1>)
  auto all = [&]<int Q>() __attribute__((always_inline)) {
    [&]<int... K_>(std::integer_sequence<int, K_...>) __attribute__((always_inline)) {
      (drain_stage.template operator()<Q, K_>(), ...);
    }(std::make_integer_sequence<int, T>{});
  };
  if (it & 1)
    all.template operator()<0>();
  else
    all.template operator()<1>();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing in flight when the registers die
}

template <bool MEAN, int TMAX, int NKS, int NSETS>
int launch_sp(Args a, int64_t N, hipStream_t st) {
  using G = sp::Geo<TMAX>;
  a.tiles = (int)ceil_div(a.W, kXT);
  const int64_t nwork = (int64_t)a.tiles * a.H * N * a.G * a.npass;
  if (nwork > INT32_MAX / 64) return fail(SM_EINVAL, "band kernel: too much work for one launch");
  a.nwork = (int)nwork;
  auto kern = band_sp<MEAN, TMAX, NKS, NSETS>;
  static std::atomic<unsigned long long> lds_done{0};
  const int dev = stream_device(st);
  if (int rc = ensure_lds_limit(reinterpret_cast<const void*>(kern), (int)G::SHM, dev, lds_done))
    return rc;
  int64_t nwg = std::min<int64_t>(nwork, (int64_t)device_cus(dev));
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(sp::kThreads), G::SHM, st, a);
  return check_launch("band_sp");
}

// fp32 inner product / correlation volume on the software-pipelined band kernel; *handled =
// false when the shape is not one it takes: 4-element aligned rows of W >= 4, one channel group,
// C = 16 NKS channels with NKS in {1, 4} (other channel counts: band_h2db), a pass width of
// more than 64 disparities, and 32 disparity planes spanning < 2 GB (the store offsets).
int band_sp_run(const Args& a, int64_t N, bool mean, bool aligned4, hipStream_t st,
                bool* handled) {
  *handled = false;
  const int nks = a.cpg / 16;
  if (!aligned4 || a.G != 1 || a.W < 4 || a.cpg % 16 != 0 || (nks != 1 && nks != 4) ||
      a.pw <= 64 || a.pw > 192 || (int64_t)a.H * a.W * 4 * 32 >= ((int64_t)1 << 31))
    return SM_OK;
  *handled = true;
  auto go = [&](auto tm, auto nk) {
    constexpr int TM = decltype(tm)::value, NK = decltype(nk)::value;
    // T = 7 with one channel step: two load sets (four spill at 512 registers)
    constexpr int NS = (TM == 7 && NK == 1) ? 2 : SMCV_SP_SETS;
    return mean ? launch_sp<true, TM, NK, NS>(a, N, st) : launch_sp<false, TM, NK, NS>(a, N, st);
  };
  using I1 = std::integral_constant<int, 1>;
  using I4 = std::integral_constant<int, 4>;
  using T5 = std::integral_constant<int, 5>;
  using T7 = std::integral_constant<int, 7>;
  if (a.pw <= 128) return nks == 1 ? go(T5{}, I1{}) : go(T5{}, I4{});
  return nks == 1 ? go(T7{}, I1{}) : go(T7{}, I4{});
}

}  // namespace h2band
}  // namespace smcv

// Inner-product / correlation cost volume (N, D, H, W) from fp32 features: the role-split band
// kernel ("rs"), one workgroup of eight waves per CU, two per SIMD -- a compute wave and a
// memory wave.
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// The contraction, the operands (per-segment power-of-two scale, round-to-nearest two-plane fp16
// split, h*h' + h*m' + m*h' on v_mfma_f32_32x32x16_f16), the tiling (128-pixel segments, 32
// pixels and T = 1 + DMAX/32 blocks of 32 x 32 per compute wave) and the scale control are
// band_h2db's and band_sp's.  What changes is who does what:
//   * a wave counts its memory operations with ONE in-order counter (vmcnt): loads and stores
//     issued by the same wave retire in issue order, so a wave that both loads features and
//     stores the volume waits, at every staging, for volume stores it issued steps earlier.
//     band_sp (one wave per SIMD doing everything) measured 1170 us on cfg2; without its loads
//     910, without its stores 910, without both 782 (r04 ablations, profiles/r04/sp_ablations);
//   * here the two waves of a SIMD split the work by memory direction.  The compute wave (waves
//     0-3) holds the accumulators, reads the fragments, issues the MFMAs and writes finished
//     accumulators into its shear ring in LDS; it touches no global memory.  The memory wave
//     (waves 4-7) loads the features, splits them into the staged planes, reads the finished
//     ring out and stores the volume.  Its loads still queue behind its stores, but a late load
//     now delays only the staging, which has a whole step of slack, never the matrix pipe;
//   * per step: the memory waves issue the loads of the step NSETS ahead, stage the next step
//     into the idle plane buffer and drain their share of the previous segment's ring while
//     the compute waves multiply the current step; one barrier ends the step.  At a segment's
//     first step the compute waves first write the previous segment's accumulators into the
//     ring (one more barrier, after which the memory waves may read it);
//   * the ring holds one segment per compute wave, T-1 chunks of 32 disparities x 32 pixels
//     (chunk m at m x 4 KB), so each block's two chunks are adjacent (immediate offsets).  The
//     block straddling chunk -1 (t = T-1) and the one straddling chunk T-1 (t = 0) fold their
//     out-of-band half into chunk 0 / chunk T-2 at exactly the cells block T-2 / block 1 write
//     later (same lanes, same elements): written in the order T-1, 0, 1, ..., T-2, the ring
//     needs no dummy chunks;
//   * no inline asm names an accumulator register class, so the compiler keeps the accumulators
//     in ordinary VGPRs: both roles share one 256-register budget (2 waves per SIMD).
// Pad pixels, the restart on a scale change, the exact slow path for non-finite segments and
// the x < d forcing come from band_sp (round 4; scripts/experimental/ip_sp.hip).
#include "band_common.h"

#ifndef SMCV_RS_ABLATE
#define SMCV_RS_ABLATE 0  // diagnostics only (scripts/build_variants.py): 1 no ring writes,
#endif                    // 2 no readouts / stores, 4 no loads, 8 no MFMA, 16 no staging,
                          // 32 feature loads from a few L2-resident lines
#ifndef SMCV_RS_DRAIN_C
#define SMCV_RS_DRAIN_C 1  // 1: the compute wave reads its ring out and stores the volume (its
#endif                     // own LDS order suffices); 0: the memory wave does (extra barrier)
#ifndef SMCV_RS_SETS
#define SMCV_RS_SETS 4  // feature-load register sets (loads issued SETS - 1 steps ahead)
#endif

// Diagnostic per-phase cycle counts (scripts/rs_stamps.hip only; never in libstereocv.so):
// compute waves 0 barrier, 1 ring writes, 2 fragments + MFMA issue, 3 ring readout + store
// issue, 4 the rest; memory waves 5 barrier, 6 load issue, 7 staging (with its load waits),
// 8 publish + readout/stores, 9 the rest.
#ifdef SMCV_RS_STAMPS
namespace smcv {
extern __device__ unsigned long long g_rs_stamps[4096][10];
}
#define RS_STAMP(p)                                          \
  {                                                          \
    const unsigned long long n_ = __builtin_amdgcn_s_memtime(); \
    st_[p] += n_ - t_;                                       \
    t_ = n_;                                                 \
  }
#else
#define RS_STAMP(p)
#endif

namespace smcv {
namespace h2band {

namespace roles {
constexpr int kCW = 4;                 // compute waves (one per SIMD), as many memory waves
constexpr int kThreads = 2 * 64 * kCW;
constexpr int kKC = 16;                // channels per step (one 32x32x16 k-step)
constexpr int kSlot = 32 * 32 * 4;     // one ring chunk: 32 d x 32 x fp32

template <int TMAX, int FUSE = 0, int NPL = 2>
struct Geo {
  static constexpr int DMAX = 32 * (TMAX - 1);
  static constexpr int RW = kXT + DMAX;    // right-window rows
  static constexpr int ROWS = RW + kXT;    // + left-tile rows
  static constexpr int PLANE = ROWS * 32;  // one fp16 plane: rows of 16 channels
  static constexpr int BUF = NPL * PLANE;  // the planes of one step (fp32: h + m; 16-bit: one)
  static constexpr int GROUPS = ROWS / 4;
  static constexpr int ITEMS = 2 * GROUPS;
  // one compute wave's ring (the volume-free fused pass has none)
  static constexpr int RINGW = FUSE == 2 ? 0 : (TMAX - 1) * kSlot;
  static constexpr int PL0 = kCW * RINGW;           // plane buffers after the rings
  static constexpr int MAXW = PL0 + 2 * BUF;        // 4 maxima sets x (max|L|, max|R|)
  static constexpr size_t SHM = (size_t)MAXW + 64;
  static_assert(ITEMS <= 64 * kCW, "one staging item per memory-wave lane");
  static_assert(SHM <= 160 * 1024, "one workgroup per CU");
};

// the ring chunks a memory wave reads out and stores in step ks of the next segment
constexpr int chunk_lo(int ks, int T, int NKS) { return (ks * (T - 1) + NKS - 1) / NKS; }
}  // namespace roles

// One role's whole program.  Both roles run the same control flow (the same segments, range
// checks, restarts and barriers, all decided on workgroup-uniform data); what each does between
// the barriers is selected at compile time, so neither role's registers (the accumulators, the
// load sets) are live in the other's code.
template <bool CW, bool MEAN, int TMAX, int NKS, int NSETS, int FUSE, typename TI, bool GW>
__device__ __forceinline__ void rs_role(const Args& args, unsigned char* smem) {
  using namespace roles;
  constexpr bool F32 = std::is_same<TI, float>::value;  // else fp16 / bf16: exact products
  using G = roles::Geo<TMAX, FUSE, F32 ? 2 : 1>;
  static_assert(F32 || FUSE == 0, "the fused passes of 16-bit features run on band_h2");
  constexpr bool VOL = FUSE != 2;  // the volume is written (FUSE 0, 1)
  constexpr int T = TMAX;
  constexpr int DMAX = G::DMAX;
  static_assert(T >= 3, "blocks 0 and T-1 are distinct and fold into distinct chunks");
  constexpr bool isC = CW;
  const TI* __restrict__ L = static_cast<const TI*>(args.L);
  const TI* __restrict__ R = static_cast<const TI*>(args.R);
  const int cpg = args.cpg, H = args.H, W = args.W, D = args.D;
  const Strides4 ls = args.ls, rs = args.rs;

  const Sched sched(args.nwork, args.npass);
  if (sched.none) return;  // the whole workgroup leaves together
#ifdef SMCV_RS_PRIO  // diagnostics: 1 the compute waves, 2 the memory waves issue at priority 1
  if constexpr ((SMCV_RS_PRIO == 1) == isC) __builtin_amdgcn_s_setprio(1);
#endif
  const int nitems = sched.nitems;
  auto witem = [&](int i) -> Work {
    return decode_fd((unsigned)sched.item_fd(min(i, nitems - 1), args.fd_np), args, DMAX);
  };

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int rw = wave & (kCW - 1);  // the 32-pixel slice (and ring) of this wave pair
#ifdef SMCV_RS_STAMPS
  unsigned long long st_[10] = {}, t_ = __builtin_amdgcn_s_memtime();
#endif
  [[maybe_unused]] constexpr int SB = isC ? 0 : 5;  // this role's first stamp slot
  const int lane = tid & 63;
  const int lr = lane & 31;
  const int hh = lane >> 5;

  // ------------------------------------------------------- staging role of a memory-wave lane
  const int mt = max(tid - 64 * kCW, 0);
  const bool active = !isC && mt < G::ITEMS;
  const int ch = min(mt / G::GROUPS, 1);
  const int g = min(mt - ch * G::GROUPS, G::GROUPS - 1);
  const bool isR = 4 * g < G::RW;
  const int64_t cs = isR ? rs.c : ls.c;

  // NSETS feature-load register sets: the loads of step j land in set j % NSETS, issued
  // NSETS - 1 steps before the step that stages them
  using QT = typename Quad<TI>::type;  // 4 pixels of one channel row: 16 B fp32, 8 B 16-bit
  QT sv[NSETS][8];
  bool okp[NSETS];
  auto load = [&](int set, const Work& k, int ks) __attribute__((always_inline)) {
    const int px = isR ? k.js + 4 * g : k.x0 + 4 * g - G::RW;
    okp[set] = active && px >= 0 && px < W;
    if constexpr (SMCV_RS_ABLATE & 4) {
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        if constexpr (F32)
          sv[set][kk] = f32x4v{1.f, -1.f, 0.5f, 2.f};
        else
          sv[set][kk] = QT{0x3c003c00u, 0xbc00bc00u};
        asm volatile("" : "+v"(sv[set][kk]));
      }
      return;
    }
    int pxc = min(max(px, 0), W - 4);  // pad groups: the nearest valid group
    if constexpr (SMCV_RS_ABLATE & 32) pxc = 4 * (lane & 7);  // L2-resident lines only
    const TI* p = (isR ? R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h
                       : L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h) +
                  pxc + (SMCV_RS_ABLATE & 32 ? 0 : ((int64_t)k.g * cpg + ks * kKC + 8 * ch) * cs);
    int64_t csl = SMCV_RS_ABLATE & 32 ? 0 : cs;
    asm volatile("" : "+v"(csl));
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      gload<false>(sv[set][kk], p);  // compiler-tracked: it places the vmcnt waits itself
      p += csl;
    }
  };
  int kL = 0, kR = 0;  // per-segment scale exponents of the staging side (workgroup-uniform)
  float mx = 0.f;      // this lane's max|x| over the segment being staged (valid groups only)
  // Staging of one step into plane buffer `buf` (byte offset): max|x| of the step, then the
  // split of its four pixels into the h and m planes.
  auto stage = [&](int set, unsigned buf) __attribute__((always_inline)) {
    if constexpr (SMCV_RS_ABLATE & 16) return;
    if constexpr (!F32) {
      // 16-bit features as they are: pixel p's 8 channels -> 16 B of the one plane (pad groups
      // zeroed: they reach only cells x < d or columns x >= W)
      u32x2 qv[8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) qv[kk] = okp[set] ? sv[set][kk] : u32x2{0u, 0u};
      unsigned o0 = buf + (unsigned)swz(4 * g, ch);
      asm volatile("" : "+v"(o0));
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        uint4 w;
        unsigned* pw_ = reinterpret_cast<unsigned*>(&w);
#pragma unroll
        for (int j = 0; j < 4; ++j) {  // channels 2j (low half), 2j+1 (high half) of pixel p
          const unsigned lo = p < 2 ? qv[2 * j].x : qv[2 * j].y;
          const unsigned hi = p < 2 ? qv[2 * j + 1].x : qv[2 * j + 1].y;
          pw_[j] = __builtin_amdgcn_perm(hi, lo, (p & 1) ? 0x07060302u : 0x05040100u);
        }
        if (active) *reinterpret_cast<uint4*>(smem + (o0 ^ (32u * p))) = w;
      }
      return;
    } else {
    f32x4v(&sv_)[8] = sv[set];
    float m0 = 0.f, m1 = 0.f;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m0) : "v"(sv_[kk].x), "v"(sv_[kk].y));
      asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(m1) : "v"(sv_[kk].z), "v"(sv_[kk].w));
    }
    mx = okp[set] ? fmaxf(mx, fmaxf(m0, m1)) : mx;
    const float sc = okp[set] ? __builtin_ldexpf(1.0f, isR ? kR : kL) : 0.f;
    unsigned o0 = buf + (unsigned)swz(4 * g, ch);
    asm volatile("" : "+v"(o0));
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      uint4 wh, wm;
      const float xs[8] = {sv_[0][p], sv_[1][p], sv_[2][p], sv_[3][p],
                           sv_[4][p], sv_[5][p], sv_[6][p], sv_[7][p]};
      split_quad(xs, sc, wh, wm);
      if (active) {
        const unsigned off = o0 ^ (32u * p);
        *reinterpret_cast<uint4*>(smem + off) = wh;
        *reinterpret_cast<uint4*>(smem + G::PLANE + off) = wm;
      }
    }
    }
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

  // --------------------------------------------------------------- compute role of a wave
  f32x16 acc[T];
#pragma unroll
  for (int t = 0; t < T; ++t) acc[t] = f32x16{};
  auto mma = [](f16x8 a, f16x8 b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
  };

  // the segment whose accumulators go into the ring next (workgroup-uniform)
  Work pw = witem(0);
  int p_kk = 0;
  bool p_special = false;  // scaled (kk != 0) or holding cells x < d (js < 0)
  int p_bytes = 0;         // 0x80000000 (valid) or 0 (every store dropped)
  bool p_full = false;     // the whole 128-pixel segment and all DMAX disparities are stored
  float* p_ob = static_cast<float*>(args.out);  // (n, dp, y, x0 + 32 rw) of that segment
  const int64_t plane_stride = (int64_t)H * W;

  // ---------------------------------------------------------------------------- the ring
  // Lane (lr, hh), element i of block t: R row c_i + 4 hh (c_i = (i & 3) + 8 (i >> 2)), pixel
  // x0 + 32 rw + lr, local disparity 32 (a + 1) + u - c_i with a = T-2-t, u = lr - 4 hh, i.e.
  // chunk a + 1 row u - c_i (u >= c_i) or chunk a row 32 + u - c_i.  Chunk m at ring + m 4096
  // ([32 d][32 x] fp32): the element's address is wb + (a + 1) 4096 - 128 c_i - 512 with
  // wb = ring + 512 + 128 u + 4 lr (>= ring: u >= -4), an immediate offset per element.  Block
  // T-1 (a = -1) folds chunk -1 into chunk 0 and block 0 (a = T-2) chunk T-1 into chunk T-2:
  // ((128 (u - c_i) + 4 lr) mod 4096) within the chunk.
  //
  // GW (groupwise, (N, G, H, W, D) output): the ring is [32 px][DMAX d] fp32 per compute wave
  // (RS = 4 DMAX bytes per pixel), the layout of the output's pixel records, so a wave's 32
  // pixels read out as 1-KB contiguous pieces.  Element address ring + lr RS + 4 dl =
  // wbg + 128 (a + 1) - 4 c_i - 16 with wbg = ring + 16 + lr (RS + 4) - 16 hh; the straddling
  // blocks fold into chunk 0 / chunk T-2 with dl mod 32 (the same cells as in NDHW terms).
  // ds_write_b32: bank = (lr RS / 4 + dl) mod 32 = (const + lr) mod 32, conflict free.
  constexpr int RS = 4 * DMAX;
  const int u = lr - 4 * hh;
  const unsigned ring = lds_addr(smem) + (unsigned)(rw * G::RINGW);
  // lane constants of the ring writes: the plain base, and the 16 folded addresses of the two
  // straddling blocks (one per element row c_i; block 0 adds chunk T-2's offset)
  const unsigned wb = GW ? ring + (unsigned)(16 + lr * (RS + 4) - 16 * hh)
                         : ring + (unsigned)(512 + 128 * u + 4 * lr);
  unsigned fold[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const int ci = (i & 3) + 8 * (i >> 2);
    fold[i] = GW ? ring + (unsigned)(lr * RS) + 4u * ((unsigned)(u - ci) & 31u)
                 : ring + ((unsigned)(32768 + 128 * u + 4 * lr - 128 * ci) & 4095u);
  }
  // SPEC: the segment is scaled (kk != 0) or holds cells x < d (R pad rows, forced to 0); the
  // plain form is one ds_write_b32 per element with an immediate offset and no vector ALU work
  // (MEAN: one multiply)
  auto write_block = [&]<int t, bool SPEC>() __attribute__((always_inline)) {
    if constexpr (SMCV_RS_ABLATE & 1) return;
    constexpr int a = T - 2 - t;
    const int jl = pw.js + 32 * rw + 4 * hh;
    const unsigned wbl = wb;  // (locals: asm operands may not name the enclosing captures)
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int ci = (i & 3) + 8 * (i >> 2);
      const unsigned fl = fold[i];
      float val = acc[t][i];
      if constexpr (MEAN) val *= args.mul;
      if constexpr (SPEC) {
        if constexpr (F32) val = __builtin_ldexpf(val, p_kk);
        val = jl + 32 * t + ci >= 0 ? val : 0.f;  // R pad rows: cells x < d
      }
      constexpr int fold_off = a == -1 ? 0 : GW ? (T - 2) * 128 : (T - 2) * kSlot;
      const int imm = GW ? 128 * (a + 1) - 4 * ci - 16 : (a + 1) * kSlot - 128 * ci - 512;
      if constexpr (a == -1 || a == T - 2) {
        asm volatile("ds_write_b32 %0, %1 offset:%2" : : "v"(fl), "v"(val), "n"(fold_off) : "memory");
      } else {
        asm volatile("ds_write_b32 %0, %1 offset:%2" : : "v"(wbl), "v"(val), "n"(imm) : "memory");
      }
    }
  };
  // block T-1 first, then 0 .. T-2 (the folded halves are overwritten by later blocks)
  auto write_blocks = [&]<bool SPEC>() __attribute__((always_inline)) {
    write_block.template operator()<T - 1, SPEC>();
    [&]<int... K_>(std::integer_sequence<int, K_...>) __attribute__((always_inline)) {
      (write_block.template operator()<K_, SPEC>(), ...);
    }(std::make_integer_sequence<int, T - 1>{});
  };
  // two whole code paths on a workgroup-uniform flag (a per-element select would run the
  // special form's ldexp / compare / select on every segment)
  auto write_ring = [&]() __attribute__((always_inline)) {
    if constexpr (VOL) {
      if (__builtin_expect(p_special, 0))
        write_blocks.template operator()<true>();
      else
        write_blocks.template operator()<false>();
    }
  };
  // FUSE: the previous segment's soft-argmin straight from the accumulators (f-1, band_common.h)
  // before the next segment's first MFMAs overwrite them; nothing for an invalid segment
  auto fuse_regs = [&]() __attribute__((always_inline)) {
    if constexpr (FUSE != 0) {
      if (p_bytes == 0) return;
      auto go = [&](auto scale, auto xlt) __attribute__((always_inline)) {
        fused_softargmin<T, MEAN, decltype(scale)::value, decltype(xlt)::value>(
            acc, args, pw, -p_kk, 0, rw, lr, hh);
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
  const int rl = lane >> 3, cl = lane & 7;
  // chunk m of the ring: rows 8 qq + rl, pixels 4 cl .. 4 cl + 3 -> out[n, dp + 32 m + row, y,
  // x0 + 32 rw + 4 cl ..]
  // GW: unit m is the wave ring's bytes [4096 m, 4096 (m + 1)), four 1-KB pieces, lane l at
  // 16 l of a piece: byte o is pixel o / RS, disparity (o % RS) / 4 of the wave's 32 pixels
  auto drain_read = [&]<int m>(f32x4v(&vp)[4]) __attribute__((always_inline)) {
    if constexpr ((SMCV_RS_ABLATE & 2) || !VOL) return;
    if constexpr (GW) {
      unsigned rb = ring + 16u * (unsigned)lane;
      asm volatile("" : "+v"(rb));
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) vp[qq] = lds_load4(rb + (unsigned)(m * 4096 + qq * 1024));
      return;
    }
    int rr = rl, cc = cl;
    asm volatile("" : "+v"(rr), "+v"(cc));
    const unsigned rb = ring + (unsigned)(rr * 128 + 16 * cc);
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) vp[qq] = lds_load4(rb + (unsigned)(m * kSlot + qq * 1024));
  };
  auto drain_store = [&]<int m>(const f32x4v(&vp)[4]) __attribute__((always_inline)) {
    if constexpr ((SMCV_RS_ABLATE & 2) || !VOL) return;
    if constexpr (GW) {
      const __amdgpu_buffer_rsrc_t rsrc =
          __builtin_amdgcn_make_buffer_rsrc(p_ob, (short)0, p_bytes, 0x00020000);
      int ln = lane;
      asm volatile("" : "+v"(ln));
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const unsigned o = (unsigned)(m * 4096 + qq * 1024) + 16u * (unsigned)ln;
        unsigned off;
        if (p_full) {  // the wave's 32 pixel records are one contiguous range of the output
          off = o;
        } else {
          const unsigned px = o / (unsigned)RS, dd = (o % (unsigned)RS) / 4u;
          const unsigned bad = (unsigned)(pw.x0 + 32 * rw + (int)px >= W || (int)dd >= pw.Dp) << 31;
          off = (px * (unsigned)D + dd) * 4u | bad;
        }
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, vp[qq]), rsrc, off, 0,
            SMCV_NT_STORE ? 2 : 0);
      }
      return;
    }
    int rr = rl, cc = cl;
    asm volatile("" : "+v"(rr), "+v"(cc));
    float* cb = p_ob + (int64_t)(32 * m) * plane_stride;
    const __amdgpu_buffer_rsrc_t rsrc =
        __builtin_amdgcn_make_buffer_rsrc(cb, (short)0, p_bytes, 0x00020000);
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
      const unsigned xbad = (unsigned)(pw.x0 + 32 * rw + 4 * cc >= W) << 31;
#pragma unroll
      for (int qq = 0; qq < 4; ++qq) {
        const unsigned bad = xbad | ((unsigned)(32 * m + 8 * qq + rr >= pw.Dp) << 31);
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned, vp[qq]), rsrc,
            (lo + (unsigned)qq * q8) | bad, 0, SMCV_NT_STORE ? 2 : 0);
      }
    }
  };
  auto drain_range = [&]<int M0, int M1>() __attribute__((always_inline)) {
    [&]<int... K_>(std::integer_sequence<int, K_...>) __attribute__((always_inline)) {
      (
          [&]() __attribute__((always_inline)) {
            f32x4v vp[4];
            drain_read.template operator()<M0 + K_>(vp);
            drain_store.template operator()<M0 + K_>(vp);
          }(),
          ...);
    }(std::make_integer_sequence<int, M1 - M0>{});
  };
  auto set_prev = [&](const Work& k, bool valid) __attribute__((always_inline)) {
    pw = k;
    p_kk = -(kL + kR);
    p_special = p_kk != 0 || k.js < 0;
    p_bytes = valid ? (int)0x80000000 : 0;
    if constexpr (GW) {  // (N, G, H, W, D): the wave's first pixel record, from disparity dp
      p_full = k.Dp == DMAX && D == DMAX && k.x0 + kXT <= W;
      p_ob = static_cast<float*>(args.out) +
             ((((int64_t)k.n * args.G + k.g) * H + k.y) * W + k.x0 + 32 * rw) * D + k.dp;
    } else {
      p_full = k.Dp == DMAX && k.x0 + kXT <= W;
      p_ob = static_cast<float*>(args.out) +
             (((int64_t)k.n * D + k.dp) * plane_stride + (int64_t)k.y * W + k.x0 + 32 * rw);
    }
  };

  auto barrier = []() __attribute__((always_inline)) {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };

  // --------------------------------------------------------------------------- the steps
  // The loop body runs U segments (U NKS a multiple of NSETS: the load sets), so every step's
  // load set and drained chunks are fixed at compile time.  Step G (0 <= G < U NKS) of the body
  // is step KS = G % NKS of the body's segment G / NKS; wq[k] is the work item it + k (k < LA).
  constexpr int U = [] {
    int u = 1;
    while ((u * NKS) % NSETS != 0) ++u;
    return u;
  }();
  constexpr int LA = 1 + (NKS - 1 + NSETS) / NKS;  // items a step's loads can reach
  int it = 0;            // the segment multiplied
  unsigned bm = G::PL0;  // plane buffer multiplied from (the other one is staged into)
  Work wq[LA];
#pragma unroll
  for (int k = 0; k < LA; ++k) wq[k] = witem(k);

  auto step = [&]<int GS>() __attribute__((always_inline)) {
    constexpr int KS = GS % NKS;
    constexpr int sd = (KS + 1) / NKS, ss = (KS + 1) % NKS;           // the staged step
    constexpr int ld = (KS + NSETS) / NKS, lks = (KS + NSETS) % NKS;  // the loaded step
    constexpr int sset = (GS + 1) % NSETS, lset = GS % NSETS;
    const unsigned sb = bm ^ (unsigned)(G::PL0 ^ (G::PL0 + G::BUF));
    RS_STAMP(SB + 4);
    if constexpr (isC) {
      if constexpr (KS == 0) {  // the previous segment's accumulators
        write_ring();
        fuse_regs();
      }
      RS_STAMP(1);
    } else {
      load(lset, wq[ld], lks);
      RS_STAMP(6);
    }
    // the ring is complete (and its readers done before) -- when another wave reads it
    if constexpr (KS == 0 && !SMCV_RS_DRAIN_C) barrier();
    // the compute wave's ring chunks of this step: the first (up to) two read before the
    // matrix work, stored after it (the reads' latency hidden behind the MFMAs)
    constexpr int c0 = chunk_lo(KS, T, NKS), c1 = chunk_lo(KS + 1, T, NKS);
    constexpr int npre = SMCV_RS_DRAIN_C && VOL ? (c1 - c0 < 2 ? c1 - c0 : 2) : 0;
    [[maybe_unused]] f32x4v pv[2][4];
    if constexpr (isC && npre > 0) drain_read.template operator()<c0>(pv[0]);
    if constexpr (isC && npre > 1) drain_read.template operator()<c0 + 1>(pv[1]);
    if constexpr (isC && !F32) {  // 16-bit features: one exact product per block
      using FV = typename std::conditional<std::is_same<TI, __bf16>::value, bf16x8, f16x8>::type;
      const unsigned char* ab = smem + bm + 32 * rw * 32 + swz(lr, hh);
      const unsigned char* bb = smem + bm + (G::RW + 32 * rw) * 32 + swz(lr, hh);
      const FV bh = *reinterpret_cast<const FV*>(bb);
      FV ah[2];
      ah[0] = *reinterpret_cast<const FV*>(ab);
#pragma unroll
      for (int t = 0; t < T; ++t) {
        if (t + 1 < T) ah[(t + 1) & 1] = *reinterpret_cast<const FV*>(ab + 1024 * (t + 1));
        const f32x16 c0v = KS == 0 ? f32x16{} : acc[t];
        if constexpr (std::is_same<TI, __bf16>::value)
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah[t & 1], bh, c0v, 0, 0, 0);
        else
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[t & 1], bh, c0v, 0, 0, 0);
      }
      if constexpr (npre > 0) drain_store.template operator()<c0>(pv[0]);
      if constexpr (npre > 1) drain_store.template operator()<c0 + 1>(pv[1]);
      if constexpr (SMCV_RS_DRAIN_C) drain_range.template operator()<c0 + npre, c1>();
    } else if constexpr (isC) {
      const unsigned char* ab = smem + bm + 32 * rw * 32 + swz(lr, hh);
      const unsigned char* bb = smem + bm + (G::RW + 32 * rw) * 32 + swz(lr, hh);
      const f16x8 bh = *reinterpret_cast<const f16x8*>(bb);
      const f16x8 bmv = *reinterpret_cast<const f16x8*>(bb + G::PLANE);
      f16x8 ah[2], am[2];
      auto rd = [&](int t) __attribute__((always_inline)) {
        ah[t & 1] = *reinterpret_cast<const f16x8*>(ab + 1024 * t);
        am[t & 1] = *reinterpret_cast<const f16x8*>(ab + G::PLANE + 1024 * t);
      };
      rd(0);
#pragma unroll
      for (int t = 0; t < T; ++t) {
        if (t + 1 < T) rd(t + 1);
        if constexpr (SMCV_RS_ABLATE & 8) {
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
      }
      RS_STAMP(2);
      if constexpr (npre > 0) drain_store.template operator()<c0>(pv[0]);
      if constexpr (npre > 1) drain_store.template operator()<c0 + 1>(pv[1]);
      if constexpr (SMCV_RS_DRAIN_C) drain_range.template operator()<c0 + npre, c1>();
      RS_STAMP(3);
    } else {
      if constexpr (ss == 0) mx = 0.f;  // the staged step opens its segment
      stage(sset, sb);
      RS_STAMP(7);
      if constexpr (ss == NKS - 1 && F32) {  // the staged segment is complete: its maxima
        if (it + sd < nitems) publish_max((it + sd) & 3);
      }
      if constexpr (!SMCV_RS_DRAIN_C)
        drain_range.template operator()<chunk_lo(KS, T, NKS), chunk_lo(KS + 1, T, NKS)>();
      RS_STAMP(8);
    }
    barrier();
    RS_STAMP(SB);
    bm = sb;
  };

  // exact fp32 FMA path for a segment holding a non-finite value or out of the scale range
  // (16-bit features never take it: no scale, and their maxima stay 0)
  auto slow_segment = [&](const Work& k) __attribute__((always_inline)) {
    if constexpr (!F32 || GW) return;
    if constexpr (FUSE != 0) slow_softargmin_f32<MEAN>(args, k, tid, kThreads);
    if constexpr (!VOL) return;
    const float mul = MEAN ? args.mul : 1.0f;
    float* out = static_cast<float*>(args.out);
    const float* lrow = static_cast<const float*>(args.L) + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;
    const float* rrow = static_cast<const float*>(args.R) + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h;
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

  // (Re)start the pipeline at segment `it` (body step GS0 = its step 0): the memory waves load
  // and stage that step into bm, publish its maxima when it is the segment's only step, and
  // issue the loads of the NSETS - 1 steps after it.
  auto prologue = [&]<int GS0>() __attribute__((always_inline)) {
    if constexpr (!isC) {
      load(GS0 % NSETS, wq[0], 0);
      mx = 0.f;
      stage(GS0 % NSETS, bm);
      if constexpr (NKS == 1 && F32) publish_max(it & 3);
#pragma unroll
      for (int k = 1; k < NSETS; ++k) load((GS0 + k) % NSETS, wq[k / NKS], k % NKS);
      // A (re)start may land its loads in other registers than the steady-state loop, which
      // copies them over at the join; the compiler's wait placement merges both paths, and a
      // load pending in the restart's registers would become a wait at every segment's first
      // step (sets 1 and 2 forced complete: measured in the asm).  Waiting here (a compiler-
      // visible vmcnt(0); restarts are rare) leaves nothing pending on this path.
      __builtin_amdgcn_s_waitcnt(0x0F70);
    }
    barrier();
  };
  prologue.template operator()<0>();
  set_prev(wq[0], false);
  bool redone = false;

  // Body segment SI: its steps, then its range check; returns true when the workgroup's last
  // segment is done.
  auto segment = [&]<int SI>() __attribute__((always_inline)) -> bool {
    for (;;) {
      [&]<int... K_>(std::integer_sequence<int, K_...>) __attribute__((always_inline)) {
        (step.template operator()<SI * NKS + K_>(), ...);
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
        set_prev(wq[0], true);  // written to the ring at the next segment's first step
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
  // the last segment: into the ring, then out
  if constexpr (isC) {
    write_ring();
    fuse_regs();
  }
  if constexpr (!SMCV_RS_DRAIN_C) barrier();
  if constexpr (isC == (bool)SMCV_RS_DRAIN_C) drain_range.template operator()<0, T - 1>();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // nothing in flight when the registers die
#ifdef SMCV_RS_STAMPS
  RS_STAMP(SB + 4);
  if (lane == 0)
    for (int p = 0; p < 10; ++p) g_rs_stamps[(blockIdx.x * 8 + wave) & 4095][p] = st_[p];
#endif
}

// FUSE 0: the volume; 1: the volume and its soft-argmin; 2: the soft-argmin only (no ring, no
// volume stores)
// TI: the feature type (fp32: the split; fp16 / bf16: as they are); GW: the groupwise
// (N, G, H, W, D) fp32 output (else (N, D, H, W) in the feature type's fp32 form)
template <bool MEAN, int TMAX, int NKS, int NSETS, int FUSE, typename TI = float, bool GW = false>
__global__ __launch_bounds__(roles::kThreads, 1) void band_rs(Args args) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  if (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) < roles::kCW)
    rs_role<true, MEAN, TMAX, NKS, NSETS, FUSE, TI, GW>(args, smem);
  else
    rs_role<false, MEAN, TMAX, NKS, NSETS, FUSE, TI, GW>(args, smem);
}

template <bool MEAN, int TMAX, int NKS, int NSETS, int FUSE, typename TI = float, bool GW = false>
int launch_rs(Args a, int64_t N, hipStream_t st) {
  using G = roles::Geo<TMAX, FUSE, std::is_same<TI, float>::value ? 2 : 1>;
  a.tiles = (int)ceil_div(a.W, kXT);
  const int64_t nwork = (int64_t)a.tiles * a.H * N * a.G * a.npass;
  if (nwork > INT32_MAX / 64) return fail(SM_EINVAL, "band kernel: too much work for one launch");
  a.nwork = (int)nwork;
  a.fd_np = make_fastdiv((unsigned)a.npass);
  a.fd_tiles = make_fastdiv((unsigned)a.tiles);
  a.fd_g = make_fastdiv((unsigned)a.G);
  a.fd_h = make_fastdiv((unsigned)a.H);
  auto kern = band_rs<MEAN, TMAX, NKS, NSETS, FUSE, TI, GW>;
  static std::atomic<unsigned long long> lds_done{0};
  const int dev = stream_device(st);
  if (int rc = ensure_lds_limit(reinterpret_cast<const void*>(kern), (int)G::SHM, dev, lds_done))
    return rc;
  int64_t nwg = std::min<int64_t>(nwork, (int64_t)device_cus(dev));
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(roles::kThreads), G::SHM, st, a);
  return check_launch("band_rs");
}

// fp32 inner product / correlation volume on the role-split band kernel; *handled = false when
// the shape is not one it takes: 4-element aligned rows of W >= 4, one channel group, C = 16 NKS
// channels with NKS in {1, 4} (other channel counts: band_h2db), a pass width of more than 64
// disparities, and 32 disparity planes spanning < 2 GB (the store offsets).
int band_rs_run(const Args& a, int64_t N, bool mean, bool aligned4, hipStream_t st,
                bool* handled, int fuse) {
  *handled = false;
  const int nks = a.cpg / 16;
  if (!aligned4 || a.G != 1 || a.W < 4 || a.cpg % 16 != 0 || (nks != 1 && nks != 4) ||
      a.pw <= 64 || a.pw > 192 || (int64_t)a.H * a.W * 4 * 32 >= ((int64_t)1 << 31))
    return SM_OK;
  // the mean with the volume kept, one channel step, D > 128: its compute wave would spill
  if (fuse == 1 && mean && nks == 1 && a.pw > 128) return SM_OK;
  *handled = true;
  auto go = [&](auto tm, auto nk) {
    constexpr int TM = decltype(tm)::value, NK = decltype(nk)::value;
    // one channel step per segment: two load sets (four unroll the body over four segments,
    // whose work-item state spills)
    constexpr int NS = NK == 1 ? 2 : SMCV_RS_SETS;
    auto f = [&](auto fc) {
      constexpr int FU = decltype(fc)::value;
      if constexpr (FU == 1 && NK == 1 && TM == 7) {
        // (the mean is excluded above: its compute wave would spill; never a silent sum)
        if (mean) return fail(SM_EINVAL, "band_rs: unhandled fused mean shape");
        return launch_rs<false, TM, NK, NS, FU>(a, N, st);
      } else
        return mean ? launch_rs<true, TM, NK, NS, FU>(a, N, st)
                    : launch_rs<false, TM, NK, NS, FU>(a, N, st);
    };
    return fuse == 2   ? f(std::integral_constant<int, 2>{})
           : fuse == 1 ? f(std::integral_constant<int, 1>{})
                       : f(std::integral_constant<int, 0>{});
  };
  using I1 = std::integral_constant<int, 1>;
  using I4 = std::integral_constant<int, 4>;
  using T5 = std::integral_constant<int, 5>;
  using T7 = std::integral_constant<int, 7>;
  if (a.pw <= 128) return nks == 1 ? go(T5{}, I1{}) : go(T5{}, I4{});
  return nks == 1 ? go(T7{}, I1{}) : go(T7{}, I4{});
}

#ifndef SMCV_RS_GW
#define SMCV_RS_GW 1  // groupwise volumes of 16-bit features on band_rs (0: band_h2)
#endif
#ifndef SMCV_RS_GW_SETS
#define SMCV_RS_GW_SETS 4  // feature-load register sets of the groupwise instances (C/G >= 32)
#endif
// Groupwise volume (mean over C/G channels, (N, G, H, W, D) fp32) of fp16 / bf16 features on the
// role-split kernel; *handled = false when the shape is not one it takes: 4-element aligned
// rows, C/G a multiple of 16 (one or more 16-channel steps per group: 1, 2 or 4), one D pass of
// 65..192 disparities with D % 4 == 0 (whole 16-B quads of a pixel record).
int band_rs_gw_run(const Args& a, int64_t N, int dtype, hipStream_t st, bool* handled) {
  *handled = false;
  const int nks = a.cpg / 16;
  if (!SMCV_RS_GW || (dtype != SM_F16 && dtype != SM_BF16) || a.W < 4 || a.cpg % 16 != 0 ||
      (nks != 1 && nks != 2 && nks != 4) || a.npass != 1 || a.pw <= 64 || a.pw > 192 ||
      a.D % 4 != 0)
    return SM_OK;
  *handled = true;
  auto go = [&](auto tm, auto nk, auto ti) {
    constexpr int TM = decltype(tm)::value, NK = decltype(nk)::value;
    using TI = typename decltype(ti)::type;
    constexpr int NS = NK == 1 ? 2 : SMCV_RS_GW_SETS;
    return launch_rs<true, TM, NK, NS, 0, TI, true>(a, N, st);
  };
  auto by_t = [&](auto ti) {
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I4 = std::integral_constant<int, 4>;
    using T5 = std::integral_constant<int, 5>;
    using T7 = std::integral_constant<int, 7>;
    if (a.pw <= 128)
      return nks == 1 ? go(T5{}, I1{}, ti) : nks == 2 ? go(T5{}, I2{}, ti) : go(T5{}, I4{}, ti);
    return nks == 1 ? go(T7{}, I1{}, ti) : nks == 2 ? go(T7{}, I2{}, ti) : go(T7{}, I4{}, ti);
  };
  return dtype == SM_F16 ? by_t(std::type_identity<__half>{}) : by_t(std::type_identity<__bf16>{});
}

}  // namespace h2band
}  // namespace smcv

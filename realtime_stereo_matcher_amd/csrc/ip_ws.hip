// Inner-product / correlation cost volume, warp-specialised band kernel (gfx950 matrix cores).
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// Per image row the volume is a band of the contraction S[j][x] = sum_c R[c][j] L[c][x]
// (d = x - j).  A workgroup owns a 128-pixel row segment and runs two kinds of waves at once:
//
//   * 4 STAGE waves (one per SIMD) load the next 16-channel step of the right window
//     R[js .. js + 128 + DMAX) and the left tile into registers (16-B loads, one step ahead),
//     split every fp32 value exactly into three bf16 planes (x = h + m + l by truncation:
//     h = hi16(x), m = hi16(x - h), l = x - h - m, each exactly representable) and write the
//     planes to LDS under a row/chunk XOR swizzle that makes both their 16-B writes and the
//     MFMA fragment reads bank-conflict free (scripts/check_swizzle.py);
//   * 4 MATH waves (one per SIMD) each own a 32-pixel x-block and accumulate its
//     T = 1 + ceil((D-1)/32) 32x32 band blocks with v_mfma_f32_32x32x16_bf16: six products
//     per block (h*h, h*m, m*h, h*l, m*m, l*h; the dropped terms are O(2^-24) relative), so
//     the result is fp32-accurate and exact for small-integer features.
//
// The planes are double-buffered: during step s the math waves read buffer s&1 while the
// stage waves fill buffer (s+1)&1, and one workgroup barrier per step hands the buffers over.
// Stage waves never store and math waves never load from global memory, so neither role's
// vmcnt waits touch the other's traffic: the output stores stream out behind the MFMAs.
//
// Epilogue (math wave, after a segment's last step): the accumulators are sheared (d = x - j)
// block by block, in descending j, through a per-wave 64-row LDS ring; each block completes
// 32 output rows, which leave as full 128-B lines (8 rows per store instruction).  No
// workgroup-wide output tile, no barrier.
#include "common.h"

#include <type_traits>

// Diagnostic ablation bits, compile-time (scripts/ip_stamps.hip builds with -DSMCV_ABLATE=N;
// the library always has 0; outputs become garbage): 1 no MFMAs, 2 feature loads from one
// cached line, 4 no output stores, 8 no epilogue, 16 no plane staging.
#ifndef SMCV_ABLATE
#define SMCV_ABLATE 0
#endif

namespace smcv {
namespace wsband {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kMath = 4;                 // math waves (waves 0..3)
constexpr int kStage = 4;                // stage waves (waves 4..7)
constexpr int kThreads = 64 * (kMath + kStage);
constexpr int kXT = 32 * kMath;          // left pixels per row segment
constexpr int kKC = 16;                  // channels per step (one 32x32x16 k-step)
constexpr int kRowB = 32;                // bytes per plane row: 16 bf16
constexpr int kRingAll = 4 * 32 * 512;   // shared ring: 4 chunk slots x 32 rows x 512 B

// byte offset of (plane row r, 8-channel chunk h).  Reads: lane l -> row base + (l & 31),
// chunk l >> 5 (base a multiple of 32); writes: 8 consecutive lanes -> rows 4i + p of one
// 32-row block.  Both are conflict-free under the gfx950 ds_read_b128 / ds_write_b128 groups.
__device__ __forceinline__ int swz(int r, int h) {
  return ((r ^ ((r >> 2) & 3)) << 5) + ((h ^ ((r >> 4) & 1)) << 4);
}

template <int TMAX>
struct Geo {
  static constexpr int DMAX = 32 * (TMAX - 1);
  static constexpr int RW = kXT + DMAX;       // right-window rows
  static constexpr int ROWS = RW + kXT;       // + left-tile rows
  static constexpr int PLANE = ROWS * kRowB;
  static constexpr int BUF = 3 * PLANE;
  static constexpr int GROUPS = ROWS / 4;     // 4-pixel groups per chunk
  static constexpr int ITEMS = 2 * GROUPS;    // (group, 8-channel chunk) items per step
  static constexpr size_t SHM = 2 * (size_t)BUF + (size_t)kRingAll + 16;  // + counter
  static_assert(ITEMS <= 64 * kStage, "one staging item per stage lane");
  static_assert(GROUPS % 8 == 0, "8-lane write groups stay inside one chunk");
};

struct Work {
  int n, y, x0, dp, Dp, Tn, js;
};

__device__ __forceinline__ Work decode(int w, int tiles, int npass, int H, int D, int dmax) {
  Work k;
  const int pass = w % npass;
  const int rest = w / npass;
  const int tile = rest % tiles;
  const int row = rest / tiles;
  k.y = row % H;
  k.n = row / H;
  k.x0 = tile * kXT;
  k.dp = pass * dmax;
  k.Dp = min(dmax, D - k.dp);
  k.Tn = 1 + (k.Dp - 1 + 31) / 32;
  k.js = k.x0 - k.dp - 32 * (k.Tn - 1);
  return k;
}

typedef __attribute__((address_space(3))) unsigned char lds_u8;
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const lds_u8*)p;
}
// LDS accesses by byte address (the ring uses compile-time offsets on one base VGPR)
__device__ __forceinline__ void lds_store1(unsigned addr, float v) {
  *reinterpret_cast<__attribute__((address_space(3))) float*>(addr) = v;
}
typedef float f32x4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 lds_load4(unsigned addr) {
  const f32x4v v = *reinterpret_cast<__attribute__((address_space(3))) f32x4v*>(addr);
  return make_float4(v.x, v.y, v.z, v.w);
}

// output stores: streaming (nontemporal) by default -- the volume is written once and read by
// a later kernel, so it should not displace the feature rows the stage waves re-read from L2
#ifndef SMCV_NT
#define SMCV_NT 1
#endif
__device__ __forceinline__ void st_out(float* p, float4 v) {
  if (SMCV_NT) {
    f32x4v q = {v.x, v.y, v.z, v.w};
    __builtin_nontemporal_store(q, reinterpret_cast<f32x4v*>(p));
  } else {
    *reinterpret_cast<float4*>(p) = v;
  }
}

__device__ __forceinline__ unsigned hi_pack(float a, float b) {
  // bf16 truncations of a (low half) and b (high half)
  return __builtin_amdgcn_perm(__float_as_uint(b), __float_as_uint(a), 0x07060302u);
}
__device__ __forceinline__ float trunc16(float x) {
  return __uint_as_float(__float_as_uint(x) & 0xffff0000u);
}

// acc += A * B over the three-plane split, smallest products first
__device__ __forceinline__ void mma6(f32x16& acc, const bf16x8 (&a)[3], const bf16x8 (&b)[3]) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
}

template <int TMAX, bool MEAN>
__global__ __launch_bounds__(kThreads, 1) void ip_band_ws(
    const float* __restrict__ L, const float* __restrict__ R, float* __restrict__ out, int C,
    int H, int W, int D, Strides4 ls, Strides4 rs, int tiles, int npass, int pw, int nwork) {
  using G = Geo<TMAX>;
  constexpr int ablate = SMCV_ABLATE;
  constexpr int DMAX = G::DMAX;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  // work range of this workgroup's XCD group (blocks b and b+8 share an XCD)
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

  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lane = tid & 63;
  SM_STAMP_DECL

  if (wave >= kMath) {
    // =============================== stage waves ===============================
    const int sq = (wave - kMath) * 64 + lane;
    const bool active = sq < G::ITEMS;
    const int h = min(sq / G::GROUPS, 1);  // 8-channel chunk (idle lanes: clamped to 1, so
                                           // their loads stay inside the channel range)
    const int g = min(sq - h * G::GROUPS, G::GROUPS - 1);  // 4-pixel group: rows 4g .. 4g+3
    const bool isR = 4 * g < G::RW;
    const int64_t rsc = rs.c, lsc = ls.c;  // SGPR copies: a per-lane struct select is a VMEM load
    const int64_t cs = isR ? rsc : lsc;
    float4 va[8], vb[8];
    int oka = 0, okb = 0;  // valid channels (0..8) of va / vb; 0 also for out-of-image pixels
    const bool cfull = C % kKC == 0;  // uniform: no channel clamping anywhere
    // load() only issues the loads; the out-of-image / past-C zeroing is applied in put(),
    // so nothing consumes the data before the other register set's step has been written.
    auto load = [&](float4 (&v)[8], int& nv, int s) {
      s = min(s, S - 1);  // past the end: reload the last step (keeps the wait counts fixed)
      const int it = s / nks;
      const int c0 = (s - it * nks) * kKC + 8 * h;
      const Work k = decode(wbeg + gi + it * gsz, tiles, npass, H, D, pw);
      const int px = isR ? k.js + 4 * g : k.x0 + 4 * g - G::RW;
      const bool okp = active && px >= 0 && px < W;
      const float* row = isR ? R + (int64_t)k.n * rs.n + (int64_t)k.y * rs.h
                             : L + (int64_t)k.n * ls.n + (int64_t)k.y * ls.h;
      const float* p = row + (okp ? px : 0) + (int64_t)min(c0, C - 1) * cs;
      nv = okp ? min(max(C - c0, 0), 8) : 0;
      if (ablate & 2) p = L + 4 * (lane & 7);
      if (cfull) {
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) v[kk] = *reinterpret_cast<const float4*>(p + kk * cs);
      } else {
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
          v[kk] = *reinterpret_cast<const float4*>(p + min(kk, max(C - 1 - c0, 0)) * cs);
      }
    };
    auto put = [&](float4 (&v)[8], int nv, int b) {
      if (!active || (ablate & 16)) return;
      if (__any(nv != 8)) {  // row edges / channel tail only
#pragma unroll
        for (int kk = 0; kk < 8; ++kk)
          if (kk >= nv) v[kk] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      unsigned char* base = smem + b * G::BUF;
      float col[4][8];
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        col[0][kk] = v[kk].x;
        col[1][kk] = v[kk].y;
        col[2][kk] = v[kk].z;
        col[3][kk] = v[kk].w;
      }
      // h plane (truncation: the high halves) of the four pixels
      uint4 ph[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        ph[p].x = hi_pack(col[p][0], col[p][1]);
        ph[p].y = hi_pack(col[p][2], col[p][3]);
        ph[p].z = hi_pack(col[p][4], col[p][5]);
        ph[p].w = hi_pack(col[p][6], col[p][7]);
      }
      // residual planes: x = +-inf would leave a NaN residual, so waves holding an infinity
      // take a separate copy of the split that zeroes it (each branch writes its own planes:
      // no merged values, no copies on the common path)
      auto split_store = [&](auto guard) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          float r1[8], r2[8];
#pragma unroll
          for (int kk = 0; kk < 8; ++kk) {
            const float x = guard(col[p][kk]);
            r1[kk] = x - trunc16(x);
            r2[kk] = r1[kk] - trunc16(r1[kk]);
          }
          uint4 pm, pl;
          pm.x = hi_pack(r1[0], r1[1]);
          pm.y = hi_pack(r1[2], r1[3]);
          pm.z = hi_pack(r1[4], r1[5]);
          pm.w = hi_pack(r1[6], r1[7]);
          pl.x = hi_pack(r2[0], r2[1]);
          pl.y = hi_pack(r2[2], r2[3]);
          pl.z = hi_pack(r2[4], r2[5]);
          pl.w = hi_pack(r2[6], r2[7]);
          const int off = swz(4 * g + p, h);
          *reinterpret_cast<uint4*>(base + off) = ph[p];
          *reinterpret_cast<uint4*>(base + G::PLANE + off) = pm;
          *reinterpret_cast<uint4*>(base + 2 * G::PLANE + off) = pl;
        }
      };
      float mx = 0.f;
#pragma unroll
      for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) mx = fmaxf(mx, fabsf(col[p][kk]));
      if (__any(mx == __builtin_inff())) {
        asm volatile("" ::: "memory");
        split_store([](float x) { return __builtin_isinf(x) ? 0.f : x; });
      } else {
        split_store([](float x) { return x; });
      }
    };
    load(va, oka, 0);
    load(vb, okb, 1);
    put(va, oka, 0);
    load(va, oka, 2);
    __syncthreads();
    // step s: the math waves consume buffer s&1 while this wave fills (s+1)&1.  The body is
    // branch-free (steps past the end reload the last step into a buffer nobody reads), so
    // the compiler's vmcnt waits count exactly the other register set's 8 loads in flight.
    for (int s = 0; s < S; s += 2) {
      put(vb, okb, 1);
      SM_STAMP(4);
      load(vb, okb, s + 3);
      SM_STAMP(5);
      __syncthreads();
      SM_STAMP(6);
      put(va, oka, 0);
      SM_STAMP(4);
      load(va, oka, s + 4);
      SM_STAMP(5);
      __syncthreads();
      SM_STAMP(6);
    }
    SM_STAMP_FLUSH
    return;
  }

  // ================================ math waves =================================
  const int mw = wave;
  const int lr = lane & 31;
  const int hh = lane >> 5;
  // The math waves share a ring of 4 chunk slots, each 32 output rows x 128 pixels (512-B
  // rows); chunk m (local rows [32m, 32m+32)) lives in slot m & 3.  Element (t, i) of a lane --
  // local disparity dl = 32 (a+1) + u - c_i with a = Tn-2-t, u = lr - 4 hh,
  // c_i = (i & 3) + 8 (i >> 2) -- belongs to chunk a or a+1; for (a & 3) != 3 the two slots are
  // adjacent and the element's ring row is 32 (a&3) + 32 + u - c_i: one base VGPR per lane and
  // a compile-time offset per element.  When (a & 3) == 3 the pair wraps (slots 3, 0): one
  // select per element.  Rows of x < d (dl < 0, chunk -1) and dl >= Dp land in slots that hold
  // no live chunk.  A chunk is complete when all four waves have written both of its blocks:
  // an LDS counter (one increment per wave per block) orders the waves, and each wave then
  // stores a quarter of the chunk (8 rows) as 2 x 512-B rows per store instruction.
  const unsigned ring0 = lds_addr(smem + 2 * G::BUF);
  const unsigned ctr = ring0 + kRingAll;  // handshake counter (zeroed before the first barrier)
  const int u = lr - 4 * hh;
  const unsigned wbase = ring0 + (unsigned)(5 + u) * 512u + 4u * (32 * mw + lr);  // row 32+u-27
  const float rdiv = 1.0f / (float)C;  // MEAN (correlation): sum * (1/C)
  const int srow = 8 * mw + (lane >> 5);  // store lanes: this wave's rows 8mw + 2q + (lane >> 5)
  const int sc4 = 4 * lr;
  const unsigned rbase = ring0 + (unsigned)srow * 512u + 4u * sc4;
  const size_t dstride = (size_t)H * W;
  unsigned seq = 0;  // handshakes done by this wave
  // LDS executes one wave's DS instructions in order, so a wave's ring writes are performed
  // before its counter increment and a waiter's ring reads after its counter read: relaxed
  // (no-fence) atomics suffice, and no vmcnt wait ever holds the output stores.
  auto handshake = [&]() {
    ++seq;
    asm volatile("" ::: "memory");
    if (lane == 0)
      __hip_atomic_fetch_add(reinterpret_cast<__attribute__((address_space(3))) unsigned*>(ctr), 1u,
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    // bounded spin: a broken invariant yields wrong output, never a hung GPU
    for (int guard = 0; guard < (1 << 16); ++guard) {
      if (__hip_atomic_load(reinterpret_cast<__attribute__((address_space(3))) unsigned*>(ctr),
                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) >= (unsigned)kMath * seq)
        break;
    }
    asm volatile("" ::: "memory");
  };
  // Output schedule of a full band (Tn == TMAX, Dp == DMAX, whole 128-px segment):
  //   phase A: blocks a = -1 .. min(2, TMAX-2) are sheared (chunks 0..min(2,TMAX-2) complete),
  //            handshake, those chunks are stored;
  //   phase B: (TMAX >= 5) handshake -- every wave's reads of chunks 0..2 are done -- blocks
  //            a = 3 .. TMAX-2 are sheared into their slots, handshake; chunks 3 .. TMAX-2 are
  //            DEFERRED: they stay in the ring and leave during the next segment's MFMA steps
  //            (one read-ahead store per even band block), so the output stream overlaps the
  //            matrix work.  Deferred reads are scheduled in steps ks < nks-1, so the step
  //            barrier orders them before the next epilogue; leftovers (nks small) are flushed
  //            and fenced by a handshake.
  constexpr int kNA = TMAX - 1;                         // chunks of a full band
  constexpr int kLastA = kNA - 1 < 2 ? kNA - 1 : 2;     // last chunk of phase A
  constexpr int kDefer = 4 * (kNA - 1 - kLastA);        // deferred stores per segment
  constexpr int kChunk0 = kLastA + 1;                   // first deferred chunk
  constexpr int kSlotsPerStep = (TMAX + 1) / 2;         // even band blocks
  int pend_r = kDefer;                                  // next deferred read (kDefer: none)
  float* pend_o = out;                                  // lane pointer of the deferred segment
  float4 pv = make_float4(0.f, 0.f, 0.f, 0.f);
  float* pv_o = nullptr;                                // destination of pv (nullptr: none)
  auto pend_read = [&]() {
    const int m = kChunk0 + (pend_r >> 2);
    const int qq = pend_r & 3;
    pv = lds_load4(rbase + (unsigned)((m & 3) * 16384 + 1024 * qq));
    pv_o = pend_o + (size_t)(32 * m + 2 * qq) * dstride;
    ++pend_r;
  };
  auto pv_store = [&]() {
    if (pv_o != nullptr && !(ablate & 4)) st_out(pv_o, pv);
    pv_o = nullptr;
  };
  f32x16 acc[TMAX];
  if (mw == 0 && lane == 0)
    *reinterpret_cast<__attribute__((address_space(3))) unsigned*>(ctr) = 0u;
  __syncthreads();  // buffer 0 is staged (and the counter zeroed)
  SM_STAMP(0);
  for (int s = 0; s < S; ++s) {
    const int it = s / nks;
    const int ks = s - it * nks;
    const Work k = decode(wbeg + gi + it * gsz, tiles, npass, H, D, pw);
    const unsigned char* base = smem + (s & 1) * G::BUF;
    const int boff = (G::RW + 32 * mw) * kRowB + swz(lr, hh);
    const unsigned char* abase = base + 32 * mw * kRowB + swz(lr, hh);  // + 1024 t
    const bool pend_ok = ks < nks - 1;  // deferred reads allowed in this step
    // The full band always runs (a partial last D pass computes blocks it never stores: one
    // code path).  Fragments are read two blocks ahead of their MFMAs (sched_barrier keeps the
    // order), so each read's LDS latency hides behind twelve MFMAs; the first step of a segment
    // starts the accumulators from a zero C operand instead of zeroing 112 registers.
    auto band = [&](auto first) {
      bf16x8 bq[3], af[3][3];
      auto rd = [&](int t) {
#pragma unroll
        for (int p = 0; p < 3; ++p)
          af[t % 3][p] = *reinterpret_cast<const bf16x8*>(abase + p * G::PLANE + 1024 * t);
      };
#pragma unroll
      for (int p = 0; p < 3; ++p) bq[p] = *reinterpret_cast<const bf16x8*>(base + p * G::PLANE + boff);
      rd(0);
      if (TMAX > 1) rd(1);
#pragma unroll
      for (int t = 0; t < TMAX; ++t) {
        if (t + 2 < TMAX) rd(t + 2);
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (decltype(first)::value) {
          const f32x16 z = {};
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t % 3][2], bq[0], z, 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t % 3][1], bq[1], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t % 3][0], bq[2], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t % 3][1], bq[0], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t % 3][0], bq[1], acc[t], 0, 0, 0);
          acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[t % 3][0], bq[0], acc[t], 0, 0, 0);
        } else {
          mma6(acc[t], af[t % 3], bq);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (!(t & 1)) {
          pv_store();  // the value read one slot earlier: its LDS latency is long hidden
          if (pend_ok && pend_r < kDefer) pend_read();
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    };
    if (!(ablate & 1)) {
      if (ks == 0)
        band(std::true_type{});
      else
        band(std::false_type{});
    }
    pv_store();
    SM_STAMP(1);

    if (ks == nks - 1 && !(ablate & 8)) {
      // ---- epilogue: shear through the shared ring
      if (pend_r < kDefer) {  // leftovers of the previous segment (few channel steps)
        while (pend_r < kDefer) {
          pend_read();
          pv_store();
        }
        handshake();  // every wave's reads are done before any slot is rewritten
      }
      const bool fullx = k.x0 + kXT <= W;
      // this lane's output column group in row dl = 0; per chunk row offsets are uniform
      float* const olane = out + ((size_t)k.n * D + k.dp) * H * (size_t)W + (size_t)k.y * W +
                           k.x0 + sc4 + (size_t)srow * H * (size_t)W;
      auto store_chunk = [&](int m) {
        const unsigned rb = rbase + (unsigned)(m & 3) * 16384u;
        float* ol = olane;
        asm volatile("" : "+v"(ol));  // per chunk: not hoisted (and spilled) 64-bit addresses
        float4 v[4];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) v[qq] = lds_load4(rb + 1024u * qq);
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
          const int dl = 32 * m + 2 * qq + srow;
          if (dl < k.Dp) {
            float* o = ol + (size_t)(32 * m + 2 * qq) * dstride;
            if (ablate & 4) {
              if (v[qq].x == 12345.f) o[0] = v[qq].y;  // diagnostic: ring reads, no stream
            } else if (fullx) {
              st_out(o, v[qq]);
            } else {
              const float vv[4] = {v[qq].x, v[qq].y, v[qq].z, v[qq].w};
#pragma unroll
              for (int e = 0; e < 4; ++e)
                if (k.x0 + sc4 + e < W) o[e] = vv[e];
            }
          }
        }
      };
      auto elem = [&](int t, int i) {
        float val = acc[t][i];
        if (MEAN) val *= rdiv;
        return val;
      };
      // shear of block t into the ring (compile-time t, a = TMAX-2-t)
      auto shear_fast = [&](int t) {
        const int a = TMAX - 2 - t;
        const int sl = a & 3;
        if (sl != 3) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int ci = (i & 3) + 8 * (i >> 2);
            lds_store1(wbase + (unsigned)(sl * 16384 + (27 - ci) * 512), elem(t, i));
          }
        } else {
          // slots 3 and 0: rows u - c >= 0 wrap to slot 0 (64 KiB lower)
          unsigned wbt = wbase;
          int ut = u;
          asm volatile("" : "+v"(wbt), "+v"(ut));
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            const int ci = (i & 3) + 8 * (i >> 2);
            const unsigned wb = (ut >= ci) ? wbt - 65536u : wbt;
            lds_store1(wb + (unsigned)(3 * 16384 + (27 - ci) * 512), elem(t, i));
          }
        }
      };
      const bool fast = k.Tn == TMAX && k.js >= 0 && k.Dp == DMAX;
      const bool defer = fast && fullx;
      if (fast) {
        // phase A: blocks a = -1 .. kLastA
#pragma unroll
        for (int t = TMAX - 1; t >= TMAX - 2 - kLastA; --t) shear_fast(t);
        SM_STAMP(2);
        handshake();
#pragma unroll
        for (int m = 0; m <= kLastA; ++m) store_chunk(m);
        if (kDefer > 0) {
          handshake();  // chunks 0..kLastA have been read by every wave
#pragma unroll
          for (int t = TMAX - 3 - kLastA; t >= 0; --t) shear_fast(t);
          handshake();
          if (!defer) {
#pragma unroll
            for (int m = kChunk0; m < kNA; ++m) store_chunk(m);
          }
        }
        SM_STAMP(3);
      } else {
        // partial band, a row's first segment or a short pass: computed addresses, zeroes for
        // x < d, one handshake per block
#pragma unroll
        for (int t = TMAX - 1; t >= 0; --t) {
          if (t < k.Tn) {
            unsigned wbt = wbase;
            int ut = u;
            asm volatile("" : "+v"(wbt), "+v"(ut));  // per-block: not hoisted (and spilled)
            const int a = k.Tn - 2 - t;
            const int sl = a & 3;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
              const int ci = (i & 3) + 8 * (i >> 2);
              float val = elem(t, i);
              val = (k.js + 32 * (mw + t) + ci + 4 * hh >= 0) ? val : 0.f;  // x < d
              unsigned wb = wbt;
              if (sl == 3 && ut >= ci) wb -= 65536u;
              lds_store1(wb + (unsigned)(sl * 16384 + (27 - ci) * 512), val);
            }
            handshake();
            if (a >= 0) store_chunk(a);
          }
        }
        for (int m = max(k.Tn - 1, 0); 32 * m < k.Dp; ++m) store_chunk(m);
      }
      if (defer && kDefer > 0) {
        pend_r = 0;
        pend_o = olane;
      }
    }
    SM_STAMP(3);
    __syncthreads();  // hand buffer s&1 back to the stage waves
    SM_STAMP(0);
  }
  while (pend_r < kDefer) {
    pend_read();
    pv_store();
  }
  if (S & 1) __syncthreads();  // the stage waves run whole step pairs
  SM_STAMP_FLUSH
}

int device_cus() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cached[dev] == 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}

template <int TMAX>
int launch(const float* l, const float* r, float* o, int64_t N, int64_t C, int64_t H, int64_t W,
           int64_t D, int64_t npass, int64_t pw, Strides4 ls, Strides4 rs, bool mean, hipStream_t st) {
  using G = Geo<TMAX>;
  const int tiles = (int)ceil_div(W, kXT);
  const int64_t nwork = (int64_t)tiles * H * N * npass;
  if (nwork > INT32_MAX / 64) return fail(SM_EINVAL, "inner product: too much work for one launch");
  auto kern = mean ? ip_band_ws<TMAX, true> : ip_band_ws<TMAX, false>;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                                     hipFuncAttributeMaxDynamicSharedMemorySize, (int)G::SHM);
  if (e != hipSuccess)
    return fail(SM_ELAUNCH, std::string("hipFuncSetAttribute: ") + hipGetErrorString(e));
  int64_t nwg = std::min<int64_t>(nwork, (int64_t)device_cus());
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(kThreads), G::SHM, st, l, r, o, (int)C,
                     (int)H, (int)W, (int)D, ls, rs, tiles, (int)npass, (int)pw, (int)nwork);
  return check_launch("ip_band_ws");
}

}  // namespace wsband

int check_dot_args(const void* left, const void* right, const void* out, int dtype, int64_t N,
                   int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                   const int64_t* r_strides, Strides4* ls, Strides4* rs);

// fp32 warp-specialised band kernel; *handled = false when the shape needs the generic path
// (16-B pixel groups: W % 4 == 0, 4-float-aligned rows, C > 0).
int band_ws_entry(const void* left, const void* right, void* out, int dtype, int64_t N, int64_t C,
                  int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                  const int64_t* r_strides, int mode, void* stream, bool* handled) {
  *handled = false;
  if (dtype != SM_F32) return SM_OK;
  Strides4 ls, rs;
  int rc = check_dot_args(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &ls, &rs);
  if (rc) return rc;
  const bool vec = (W % 4 == 0) && W >= 4 && C > 0 && ls.n % 4 == 0 && ls.c % 4 == 0 &&
                   ls.h % 4 == 0 && rs.n % 4 == 0 && rs.c % 4 == 0 && rs.h % 4 == 0 &&
                   ((reinterpret_cast<uintptr_t>(left) | reinterpret_cast<uintptr_t>(right)) % 16 == 0);
  if (!vec) return SM_OK;
  *handled = true;
  if (N == 0 || H == 0 || D == 0) return SM_OK;
  const bool mean = mode == 1;
  hipStream_t st = as_stream(stream);
  const float* l = static_cast<const float*>(left);
  const float* r = static_cast<const float*>(right);
  float* o = static_cast<float*>(out);
  using namespace wsband;
  // D passes of at most 192 disparities, balanced (D = 256: two passes of 128), and the
  // smallest band geometry that holds one pass
  const int64_t npass = ceil_div(D, (int64_t)192);
  const int64_t pw = ceil_div(D, npass);
  if (pw <= 32) return launch<2>(l, r, o, N, C, H, W, D, npass, pw, ls, rs, mean, st);
  if (pw <= 64) return launch<3>(l, r, o, N, C, H, W, D, npass, pw, ls, rs, mean, st);
  if (pw <= 128) return launch<5>(l, r, o, N, C, H, W, D, npass, pw, ls, rs, mean, st);
  return launch<7>(l, r, o, N, C, H, W, D, npass, pw, ls, rs, mean, st);
}

}  // namespace smcv

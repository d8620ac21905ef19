// Inner-product / correlation cost volume on the gfx950 matrix cores.
//
// Reference: TorchInnerProductCost.forward  cost_volume/inner_product.py:11-42 (sum over C)
//            make_correlation_volume         model/mobile_disp_net_c.py:188-205 (mean over C)
//   out[n, d, y, x] = sum_c L[n,c,y,x] * R[n,c,y,x-d]   (x >= d),   0 (x < d)
//
// Per image row the volume is a BAND of the C-contraction S[j][x] = sum_c R[c][j] L[c][x]
// (d = x - j in [0, D)).  One workgroup (8 waves) owns a row segment of 128 left pixels; wave w
// owns the 16-pixel x-block w and accumulates the T = 1 + ceil((D-1)/16) 16x16 S-blocks of its
// band (8 % over-compute at D = 192) with v_mfma_f32_16x16x32_bf16, K = 32 channels per step.
//
// fp32 features are split EXACTLY into three bf16 planes (x = h + m + l, 8+8+8 significand
// bits); the six partial products h*h, h*m, m*h, h*l, m*m, l*h are accumulated in fp32 by the
// MFMA.  The three dropped terms are O(2^-24) relative, so the result is fp32-accurate
// (|err| ~ 1e-6 at C = 64, bar 1e-4) and EXACT for small-integer features (argmin bit-exact).
// fp16 features need two planes (11 bits) and 4 products (exact products); bf16 needs one.
// The matrix cores run at 16x the fp32 rate, so even 6 products leave the kernel HBM-bound.
//
// Staging per 32-channel step: the right WINDOW R[j0 .. j0+128+16(T-1)) and the left tile are
// loaded as (8 channels x 4 pixels) items -- eight 16-B loads per lane, coalesced along the
// row -- split, and written to LDS pixel-major ([pixel][32 ch], 64 B per row and plane) under an
// XOR chunk swizzle that makes every ds_read_b128 fragment read bank-conflict free (staging
// writes are at most 2-way).  The window is re-used by all T blocks of all eight waves, so the
// disparity sweep never re-reads HBM.  The workgroup is persistent: the loads of the next step
// (or the next row segment) are issued into registers before the current step's MFMAs and
// epilogue, hiding HBM latency.  Epilogue: the accumulators are sheared (d = x - j) into an LDS
// [D][128] fp32 tile and streamed out as 512-B row segments (out rows are x-contiguous).
// Workgroups b and b+8 share an XCD; each XCD group walks its own contiguous range of row
// segments, so concurrently running segments of one row share that XCD's L2.
#include "common.h"

#include <cstdlib>

namespace smcv {
namespace band {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));


typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kXT = 16 * kWaves;  // left pixels per row segment
constexpr int kKC = 32;           // channels per MFMA k-step
constexpr int kRowBytes = 64;     // one LDS pixel row of one plane: 32 bf16

// byte offset of (pixel row r, 16-B channel chunk ch) inside one plane.  With the chunk XOR
// f = {0,2,3,1}[(r>>2)&3] the 16x16x32 fragment read (lane l -> row l&15, chunk l>>4) is
// conflict-free under all four gfx950 ds_read_b128 lane groups, and the staging writes
// (8 contiguous lanes per LDS cycle) are at most 2-way (checked in scripts/check_swizzle.py).
__device__ __forceinline__ int swz(int r, int ch) {
  const int f = (0x78 >> (2 * ((r >> 2) & 3))) & 3;  // {0, 2, 3, 1}
  return r * kRowBytes + 16 * (ch ^ f);
}

// Exact split of 8 floats into P bf16 planes (x = h + m + l); non-finite values stay whole in h.
template <int P>
__device__ __forceinline__ void split8(const float (&v)[8], uint4 (&q)[P]) {
  union U {
    __bf16 b[8];
    uint4 u;
  };
  U h, m, l;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float x = v[i];
    const __bf16 bh = (__bf16)x;
    h.b[i] = bh;
    if (P > 1) {
      float r1 = x - (float)bh;
      r1 = __builtin_isfinite(x) ? r1 : 0.f;
      const __bf16 bm = (__bf16)r1;
      m.b[i] = bm;
      if (P > 2) l.b[i] = (__bf16)(r1 - (float)bm);
    }
  }
  q[0] = h.u;
  if (P > 1) q[1] = m.u;
  if (P > 2) q[2] = l.u;
}

template <typename T>
__device__ __forceinline__ void load4(const T* p, float (&o)[4]) {
  if constexpr (sizeof(T) == 4) {
    const float4 f = *reinterpret_cast<const float4*>(p);
    o[0] = f.x;
    o[1] = f.y;
    o[2] = f.z;
    o[3] = f.w;
  } else {
    union {
      uint2 u;
      T e[4];
    } q;
    q.u = *reinterpret_cast<const uint2*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = to_f(q.e[i]);
  }
}

// acc += A * B over the P-plane split: for P = 3 the six products l*h, m*m, h*l, m*h, h*m, h*h
// (smallest first); P = 2: m*m, m*h, h*m, h*h (exact for fp16 data); P = 1: h*h.
template <int P>
__device__ __forceinline__ void band_mma(f32x4& acc, const bf16x8 (&a)[P], const bf16x8 (&b)[P]) {
  if constexpr (P == 3) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[2], acc, 0, 0, 0);
  }
  if constexpr (P == 2) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[1], acc, 0, 0, 0);
  if constexpr (P >= 2) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[0], acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[1], acc, 0, 0, 0);
  }
  acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[0], acc, 0, 0, 0);
}

// ---- LDS-DMA staging (global_load_lds): the next step's raw feature data lands straight in
// an LDS region with no VGPR destination, issued by inline asm so hipcc does not drain it
// (or the epilogue's output stores, which vmcnt also counts) at every barrier.  The consumer
// retires it with a hand-counted s_waitcnt vmcnt(#stores issued after it).
typedef __attribute__((address_space(3))) unsigned char lds_u8;
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const lds_u8*)p;
}
// lanes land at lds_byte + 16 * lane (wave-uniform base in M0)
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_byte) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_byte)
      : "memory");
}
// lanes land at lds_byte + 4 * lane
__device__ __forceinline__ void glds4(const void* gsrc, unsigned lds_byte) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_byte)
      : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

// staging items (8 channels x 4 pixels) per wave for a TMAX-block band, and the raw LDS-DMA
// bytes one wave needs for them: 8 channel blocks of IPW lanes x 4 pixels
constexpr int band_ipw(int tmax) { return ((16 * 8 + 16 * (tmax - 1) + 16 * 8) / 8 + 3) / 4 * 4; }
template <typename T>
constexpr int raw_k_bytes(int tmax) { return band_ipw(tmax) * 4 * (int)sizeof(T); }
template <typename T>
constexpr int raw_wave_bytes(int tmax) { return 8 * raw_k_bytes<T>(tmax); }

// 4 consecutive outputs (16-B aligned for fp32, 8-B for 16-bit types) in one store.
template <typename T>
__device__ __forceinline__ void store4(T* o, float4 v) {
  if constexpr (sizeof(T) == 4) {
    *reinterpret_cast<float4*>(o) = v;
  } else {
    union {
      T e[4];
      uint2 u;
    } pk;
    pk.e[0] = from_f<T>(v.x);
    pk.e[1] = from_f<T>(v.y);
    pk.e[2] = from_f<T>(v.z);
    pk.e[3] = from_f<T>(v.w);
    *reinterpret_cast<uint2*>(o) = pk.u;
  }
}

// One unit of work: a 128-pixel segment of one image row and one pass of at most DMAX
// disparities.  Consecutive work ids are the segments of one row (they share right columns).
struct BandWork {
  int n, y, x0, dp, Dp, Tn, rwin, js;
};

__device__ __forceinline__ BandWork band_decode(int w, int tiles, int npass, int H, int D,
                                                int dmax) {
  BandWork k;
  const int pass = w % npass;
  const int rest = w / npass;
  const int tile = rest % tiles;
  const int row = rest / tiles;
  k.y = row % H;
  k.n = row / H;
  k.x0 = tile * kXT;
  k.dp = pass * dmax;
  k.Dp = min(dmax, D - k.dp);
  k.Tn = 1 + (k.Dp - 1 + 15) / 16;       // 16x16 band blocks per x-block
  k.rwin = kXT + 16 * (k.Tn - 1);        // right-window rows
  k.js = k.x0 - k.dp - 16 * (k.Tn - 1);  // right column held in window row 0
  return k;
}

template <typename T>
struct StageItem {
  const T* row;  // feature row (n, c = 0, y) of L or R
  int64_t cstride;
  int j0;     // first pixel of the 4-pixel group
  int chunk;  // 8-channel chunk inside the 32-channel step
  int lrow;   // first LDS pixel row
  bool isR, active;
};

template <typename T, int P, int TMAX, bool VEC, bool MEAN>
__global__ __launch_bounds__(kThreads, 1) void ip_band_mfma(
    const T* __restrict__ L, const T* __restrict__ R, T* __restrict__ out, int C, int H, int W,
    int D, Strides4 ls, Strides4 rs, int tiles, int npass, int nwork, int ablate) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int DMAX = 16 * (TMAX - 1);
  constexpr int RWMAX = kXT + DMAX;           // window rows at Tn = TMAX
  constexpr int PLANE_R = RWMAX * kRowBytes;  // compile-time plane strides
  constexpr int PLANE_L = kXT * kRowBytes;
  constexpr int IPW = band_ipw(TMAX);  // staging items per wave
  constexpr int RAWK = raw_k_bytes<T>(TMAX);
  static_assert(IPW == ((RWMAX + kXT) / kWaves + 3) / 4 * 4, "band_ipw mismatch");
  static_assert(IPW <= 64 && IPW * kWaves >= RWMAX + kXT, "one staging item per lane");
  // planes (aliased by the epilogue's [DMAX + 1][128] fp32 tile) | per-wave raw DMA slots
  constexpr int IN_BYTES = P * (RWMAX + kXT) * kRowBytes;
  constexpr int OUT_BYTES = (DMAX + 1) * kXT * 4;
  constexpr int RAW_OFF = IN_BYTES > OUT_BYTES ? IN_BYTES : OUT_BYTES;  // + 8 raw slots
  unsigned char* const Rt = smem;
  unsigned char* const Lt = smem + P * PLANE_R;

  // work range of this workgroup's XCD group (blocks b and b+8 share an XCD)
  const int grp = blockIdx.x & 7;
  const int gi = blockIdx.x >> 3;
  const int gsz = gridDim.x >> 3;
  const int q = nwork >> 3, rr = nwork & 7;
  const int wbeg = grp < rr ? grp * (q + 1) : rr * (q + 1) + (grp - rr) * q;
  const int wend = wbeg + q + (grp < rr ? 1 : 0);
  int w = wbeg + gi;
  if (w >= wend) return;  // the whole workgroup leaves together

  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int fr = lane & 15;  // fragment row / column
  const int fk = lane >> 4;  // fragment k-chunk (8 channels)
  const float fdiv = (float)C;  // MEAN: torch divides the channel sum by C
  SM_STAMP_DECL

  // ---- this thread's staging item: (8-channel chunk, 4-pixel group) of the window or tile.
  // VEC path: the item's 8 channel rows x 4 pixels arrive by LDS-DMA into this wave's raw slot
  // (lane-linear), issued one step ahead; non-VEC path: plain register loads by the compiler.
  float v[8][4];
  bool okj = true, cfull = true;
  int cbi = 0;
  unsigned char* const raw_slot = smem + RAW_OFF + wave * raw_wave_bytes<T>(TMAX);
  const unsigned raw_lds = __builtin_amdgcn_readfirstlane(lds_addr(smem + RAW_OFF)) +
                           (unsigned)__builtin_amdgcn_readfirstlane(wave) * raw_wave_bytes<T>(TMAX);
  // items are dealt in contiguous blocks of IPW per wave so every wave stages the same amount
  // (lanes >= IPW idle); within a wave, consecutive lanes walk pixel groups of one row
  const int item_id = wave * IPW + lane;
  auto make_item = [&](const BandWork& k) {
    StageItem<T> it;
    const bool isR = item_id < k.rwin;
    const int i = isR ? item_id : item_id - k.rwin;
    it.isR = isR;
    it.active = lane < IPW && item_id < k.rwin + kXT;
    it.chunk = i & 3;
    it.lrow = 4 * (i >> 2);
    it.j0 = (isR ? k.js : k.x0) + it.lrow;
    it.row = isR ? R + k.n * rs.n + (int64_t)k.y * rs.h : L + k.n * ls.n + (int64_t)k.y * ls.h;
    it.cstride = isR ? rs.c : ls.c;
    return it;
  };
  // VEC: issue_prep() latches the item's DMA source; issue_piece(k) sends channel k of the
  // item (one LDS-DMA wave instruction).  The eight pieces are spread over the MFMA stream.
  const T* dma_src = L;
  int64_t dma_cs = 0;
  bool dma_on = false;
  auto issue_piece = [&](int k) {
    if (VEC && dma_on) {
      const int c = cfull ? cbi + k : min(cbi + k, C - 1);
      const T* src = dma_src + (int64_t)c * dma_cs;
      if constexpr (sizeof(T) == 4) {
        glds16(src, raw_lds + k * RAWK);
      } else {
        glds4(src, raw_lds + k * RAWK);
        glds4(src + 2, raw_lds + k * RAWK + RAWK / 2);
      }
    }
  };
  auto issue_prep = [&](const StageItem<T>& it, int c0, bool on) {
    const int cb = c0 + 8 * it.chunk;
    cbi = cb;
    if (VEC) {
      // W % 4 == 0 and j0 % 4 == 0: the 4-pixel group is entirely inside or outside the row
      okj = it.j0 >= 0 && it.j0 < W;
      cfull = cb + 8 <= C;
      dma_on = on && it.active;
      dma_src = it.row + (okj ? it.j0 : 0);
      dma_cs = it.cstride;
    } else {
      if (!on || !it.active) return;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int c = min(cb + k, C - 1);
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int j = it.j0 + p;
          const int jc = min(max(j, 0), W - 1);
          const float x = to_f(it.row[(int64_t)c * it.cstride + jc]);
          v[k][p] = (j >= 0 && j < W && cb + k < C) ? x : 0.f;
        }
      }
    }
  };
  auto issue = [&](const StageItem<T>& it, int c0) {
    issue_prep(it, c0, true);
#pragma unroll
    for (int k = 0; k < 8; ++k) issue_piece(k);
  };
  auto stage = [&](const StageItem<T>& it, bool after_epilogue) {
    if (VEC) {
      // retire this wave's LDS-DMA; only the epilogue's DMAX/16 row stores may stay in flight
      if (after_epilogue)
        vm_wait<DMAX / 16>();
      else
        vm_wait<0>();
    }
    SM_STAMP_IN(8);
    if (!it.active) return;
    if (VEC && C > 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        if constexpr (sizeof(T) == 4) {
          const float4 f = *reinterpret_cast<const float4*>(raw_slot + k * RAWK + 16 * lane);
          v[k][0] = f.x;
          v[k][1] = f.y;
          v[k][2] = f.z;
          v[k][3] = f.w;
        } else {
          union {
            unsigned u[2];
            T e[4];
          } q;
          q.u[0] = *reinterpret_cast<const unsigned*>(raw_slot + k * RAWK + 4 * lane);
          q.u[1] = *reinterpret_cast<const unsigned*>(raw_slot + k * RAWK + RAWK / 2 + 4 * lane);
#pragma unroll
          for (int p = 0; p < 4; ++p) v[k][p] = to_f(q.e[p]);
        }
      }
      if (!cfull || !__all(okj)) {  // row edges / channel tail only
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const bool ok = okj && (cbi + k < C);
#pragma unroll
          for (int p = 0; p < 4; ++p) v[k][p] = ok ? v[k][p] : 0.f;
        }
      }
    }
    unsigned char* base = it.isR ? Rt : Lt;
    const int pstride = it.isR ? PLANE_R : PLANE_L;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float col[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) col[k] = v[k][p];
      uint4 pk[P];
      split8<P>(col, pk);
      const int off = swz(it.lrow + p, it.chunk);
#pragma unroll
      for (int pl = 0; pl < P; ++pl) *reinterpret_cast<uint4*>(base + pl * pstride + off) = pk[pl];
    }
  };

  f32x4 acc[TMAX];
  BandWork cur = band_decode(w, tiles, npass, H, D, DMAX);
  StageItem<T> item = make_item(cur);
  int c0 = 0;
  bool counted_epi = false;  // the previous step ended with exactly DMAX/16 full-row stores
  const bool no_hbm = (ablate & 2) != 0;
#pragma unroll
  for (int k = 0; k < 8; ++k)
#pragma unroll
    for (int p = 0; p < 4; ++p) v[k][p] = 0.f;  // C == 0: zero sum (mean: 0/0 = NaN, as torch)
  if (C > 0) issue(item, 0);

  while (true) {
    __syncthreads();  // previous fragment reads / out-tile reads are done
    SM_STAMP(0);
    stage(item, counted_epi);
    SM_STAMP(1);
    __syncthreads();
    SM_STAMP(2);

    // prefetch the next (segment, channel step) before this step's MFMAs and epilogue
    const bool last_step = c0 + kKC >= C;
    const int nw = last_step ? w + gsz : w;
    const int nc0 = last_step ? 0 : c0 + kKC;
    const bool has_next = nw < wend;
    const BandWork nxt = last_step ? band_decode(has_next ? nw : w, tiles, npass, H, D, DMAX) : cur;
    const StageItem<T> nitem = last_step ? make_item(nxt) : item;
    // the next step's DMA: latched here, its 8 pieces interleaved with the band blocks below
    const bool dma_next = C > 0 && has_next && !no_hbm;
    issue_prep(nitem, nc0, dma_next);
    const bool interleave = VEC && cur.Tn == TMAX && !(ablate & 1);
    if (!interleave) {
#pragma unroll
      for (int k = 0; k < 8; ++k) issue_piece(k);
    }
    SM_STAMP(9);

    if (c0 == 0) {
#pragma unroll
      for (int t = 0; t < TMAX; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    // ---- band MMA: B = left x-block (cols x), A = right j-block (rows j).  The full band
    // (Tn == TMAX, every work item but the last pass of a D > DMAX split) runs a compile-time
    // loop that reads block t+1's fragments while block t's six MFMAs issue.
    if (!(ablate & 1)) {
      bf16x8 bq[P];
      const int boff = swz(16 * wave + fr, fk);
#pragma unroll
      for (int p = 0; p < P; ++p) bq[p] = *reinterpret_cast<const bf16x8*>(Lt + p * PLANE_L + boff);
      const unsigned char* abase = Rt + swz(16 * wave + fr, fk);  // + 1024 t: 16-row periodic
      if (cur.Tn == TMAX) {
        bf16x8 a0[P], a1[P];
#pragma unroll
        for (int p = 0; p < P; ++p) a0[p] = *reinterpret_cast<const bf16x8*>(abase + p * PLANE_R);
#pragma unroll
        for (int t = 0; t < TMAX; t += 2) {
          if (t + 1 < TMAX) {
#pragma unroll
            for (int p = 0; p < P; ++p)
              a1[p] = *reinterpret_cast<const bf16x8*>(abase + p * PLANE_R + 1024 * (t + 1));
          }
          band_mma<P>(acc[t], a0, bq);
#pragma unroll
          for (int k = (8 * t + TMAX - 1) / TMAX; k < (8 * (t + 1) + TMAX - 1) / TMAX; ++k)
            issue_piece(k);  // DMA pieces spread evenly over the band blocks
          if (t + 1 < TMAX) {
            if (t + 2 < TMAX) {
#pragma unroll
              for (int p = 0; p < P; ++p)
                a0[p] = *reinterpret_cast<const bf16x8*>(abase + p * PLANE_R + 1024 * (t + 2));
            }
            band_mma<P>(acc[t + 1], a1, bq);
#pragma unroll
            for (int k = (8 * (t + 1) + TMAX - 1) / TMAX; k < (8 * (t + 2) + TMAX - 1) / TMAX; ++k)
              issue_piece(k);
          }
        }
      } else {
#pragma unroll
        for (int t = 0; t < TMAX; ++t) {
          if (t < cur.Tn) {
            bf16x8 aq[P];
#pragma unroll
            for (int p = 0; p < P; ++p)
              aq[p] = *reinterpret_cast<const bf16x8*>(abase + p * PLANE_R + 1024 * t);
            band_mma<P>(acc[t], aq, bq);
          }
        }
      }
    }

    SM_STAMP(3);
    if (last_step) {
      // ---- epilogue: shear S[j][x] -> out[d = x - j][x] through an LDS [Dp][128] fp32 tile
      __syncthreads();
      SM_STAMP(4);
      float* ot = reinterpret_cast<float*>(smem);
      const int xl = 16 * wave + fr;
      // local disparity of accumulator (t, r): dl = b0 - 16 t - r.  Elements outside
      // [0, Dp) go to a trash row (row DMAX) instead of a divergent branch.
      const int b0 = fr - 4 * fk + 16 * (cur.Tn - 1);
      const int j_b = cur.js + 16 * wave + 4 * fk;  // right column of (t = 0, r = 0)
      float* const olane = ot + b0 * kXT + xl;      // element (t, r) at olane - (16t + r) * kXT
      if (cur.Tn == TMAX && cur.Dp == DMAX && cur.js >= 0) {
        // interior segment: only the first and last band blocks straddle [0, DMAX)
#pragma unroll
        for (int t = 0; t < TMAX; ++t) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float val = acc[t][r];
            if (MEAN) val = val / fdiv;
            if (t == 0 || t == TMAX - 1) {
              const int dl = b0 - 16 * t - r;
              const bool keep = (unsigned)dl < (unsigned)DMAX;
              ot[(keep ? dl : DMAX) * kXT + xl] = val;
            } else {
              olane[-(16 * t + r) * kXT] = val;
            }
          }
        }
      } else {
#pragma unroll
        for (int t = 0; t < TMAX; ++t) {
          if (t < cur.Tn) {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const int dl = b0 - 16 * t - r;
              const bool keep = (unsigned)dl < (unsigned)cur.Dp;
              const bool inside = j_b + 16 * t + r >= 0;  // j < 0 <=> x < d: exact zero
              float val = acc[t][r];
              if (MEAN) val = val / fdiv;
              ot[(keep ? dl : DMAX) * kXT + xl] = inside ? val : 0.f;
            }
          }
        }
      }
      SM_STAMP(5);
      __syncthreads();
      SM_STAMP(6);
      const int c4 = tid & 31;
      const int x = cur.x0 + 4 * c4;
      const bool fullrow = (cur.x0 + kXT <= W) && ((W & 3) == 0);
      if (ablate & 4) {
        // diagnostic path: no output stream
      } else if (fullrow && cur.Dp == DMAX) {  // the counted case: DMAX/16 stores per lane
#pragma unroll
        for (int it16 = 0; it16 < DMAX / 16; ++it16) {
          const int dl = (tid >> 5) + 16 * it16;
          const float4 val = *reinterpret_cast<const float4*>(ot + dl * kXT + 4 * c4);
          store4(out + (((size_t)cur.n * D + cur.dp + dl) * H + cur.y) * (size_t)W + x, val);
        }
      } else if (fullrow) {  // 16-B aligned row segments: one wide store per lane per row
        for (int dl = tid >> 5; dl < cur.Dp; dl += kThreads / 32) {
          const float4 val = *reinterpret_cast<const float4*>(ot + dl * kXT + 4 * c4);
          store4(out + (((size_t)cur.n * D + cur.dp + dl) * H + cur.y) * (size_t)W + x, val);
        }
      } else {
        for (int dl = tid >> 5; dl < cur.Dp; dl += kThreads / 32) {
          const float4 val = *reinterpret_cast<const float4*>(ot + dl * kXT + 4 * c4);
          T* o = out + (((size_t)cur.n * D + cur.dp + dl) * H + cur.y) * (size_t)W + x;
          const float vv[4] = {val.x, val.y, val.z, val.w};
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (x + k < W) o[k] = from_f<T>(vv[k]);
        }
      }
    }
    counted_epi = last_step && !(ablate & 4) && cur.Dp == DMAX && (cur.x0 + kXT <= W) &&
                  ((W & 3) == 0);
    if (last_step) SM_STAMP(7);
    if (!has_next) break;
    w = nw;
    c0 = nc0;
    cur = nxt;
    item = nitem;
  }
  SM_STAMP_FLUSH
}

// Diagnostic ablation bits (STEREOCV_ABLATE, timing studies only; outputs become garbage):
// 1 = skip MFMAs, 2 = skip the global loads of the pipelined steps, 4 = skip output stores.
int ablate_bits() {
  const char* e = getenv("STEREOCV_ABLATE");
  return e ? atoi(e) : 0;
}

template <typename T, int P, int TMAX>
int launch_band(const void* l, const void* r, void* o, int64_t N, int64_t C, int64_t H, int64_t W,
                int64_t D, Strides4 ls, Strides4 rs, int divisor, hipStream_t st) {
  constexpr int DMAX = 16 * (TMAX - 1);
  constexpr int RWMAX = kXT + DMAX;
  const int tiles = (int)ceil_div(W, kXT);
  const int npass = (int)ceil_div(D, DMAX);
  const int64_t nwork = (int64_t)tiles * H * N * npass;
  if (nwork > INT32_MAX) return fail(SM_EINVAL, "inner product: too much work for one launch");
  const int Dp = (int)std::min<int64_t>(D, DMAX);
  const size_t in_bytes = (size_t)P * (RWMAX + kXT) * kRowBytes;
  const size_t out_bytes = (size_t)(DMAX + 1) * kXT * 4;  // + trash row
  const size_t shm = std::max(in_bytes, out_bytes) + (size_t)kWaves * raw_wave_bytes<T>(TMAX);
  (void)Dp;
  // 4-pixel vector loads need W % 4 == 0 and 4-element-aligned rows on both sides
  const bool vec = (W % 4 == 0) && ls.n % 4 == 0 && ls.c % 4 == 0 && ls.h % 4 == 0 &&
                   rs.n % 4 == 0 && rs.c % 4 == 0 && rs.h % 4 == 0 &&
                   ((reinterpret_cast<uintptr_t>(l) | reinterpret_cast<uintptr_t>(r)) %
                        (4 * sizeof(T)) == 0);
  const bool mean = divisor >= 0;
  auto kern = vec ? (mean ? ip_band_mfma<T, P, TMAX, true, true> : ip_band_mfma<T, P, TMAX, true, false>)
                  : (mean ? ip_band_mfma<T, P, TMAX, false, true> : ip_band_mfma<T, P, TMAX, false, false>);
  static std::atomic<unsigned long long> lds_done[4];
  const int dev = stream_device(st);
  if (int rc = ensure_lds_limit(reinterpret_cast<const void*>(kern), (int)shm, dev,
                                lds_done[2 * vec + mean]))
    return rc;
  // persistent grid: one 8-wave workgroup per CU (LDS-limited), a multiple of 8
  int64_t nwg = std::min<int64_t>(nwork, (int64_t)device_cus(dev));
  nwg = std::max<int64_t>(8, (nwg + 7) / 8 * 8);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(kThreads), shm, st, static_cast<const T*>(l),
                     static_cast<const T*>(r), static_cast<T*>(o), (int)C, (int)H, (int)W, (int)D,
                     ls, rs, tiles, npass, (int)nwork, ablate_bits());
  return check_launch("ip_band_mfma");
}

template <typename T, int P>
int launch_band_d(const void* l, const void* r, void* o, int64_t N, int64_t C, int64_t H, int64_t W,
                  int64_t D, Strides4 ls, Strides4 rs, int divisor, hipStream_t st) {
  if (D <= 64) return launch_band<T, P, 5>(l, r, o, N, C, H, W, D, ls, rs, divisor, st);
  if (D <= 128) return launch_band<T, P, 9>(l, r, o, N, C, H, W, D, ls, rs, divisor, st);
  if (D <= 192) return launch_band<T, P, 13>(l, r, o, N, C, H, W, D, ls, rs, divisor, st);
  // D > 192: passes of 128 disparities (the 192-wide tile plus DMA slots would exceed LDS)
  return launch_band<T, P, 9>(l, r, o, N, C, H, W, D, ls, rs, divisor, st);
}

}  // namespace band

using namespace band;

int check_dot_args(const void* left, const void* right, const void* out, int dtype, int64_t N,
                   int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                   const int64_t* r_strides, Strides4* ls, Strides4* rs);

// mode 0: inner product (sum); mode 1: correlation (mean over C).
int band_mfma_entry(const void* left, const void* right, void* out, int dtype, int64_t N, int64_t C,
                    int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                    const int64_t* r_strides, int mode, void* stream) {
  Strides4 ls, rs;
  int rc = check_dot_args(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, &ls, &rs);
  if (rc) return rc;
  if (N == 0 || H == 0 || W == 0 || D == 0) return SM_OK;
  const int divisor = mode == 0 ? -1 : (int)C;
  hipStream_t st = as_stream(stream);
  switch (dtype) {
    case SM_F32: return launch_band_d<float, 3>(left, right, out, N, C, H, W, D, ls, rs, divisor, st);
    case SM_F16: return launch_band_d<__half, 2>(left, right, out, N, C, H, W, D, ls, rs, divisor, st);
    case SM_BF16: return launch_band_d<bf16_t, 1>(left, right, out, N, C, H, W, D, ls, rs, divisor, st);
    default: return fail(SM_EDTYPE, "unsupported dtype code");
  }
}

}  // namespace smcv

// Round 6: how the HBM takes the cfg2 volume's write stream and the features' read stream, by the
// width of the x-range a workgroup owns (the piece of each plane row it touches per unit).
// One 512-thread workgroup per CU (256), band_rs's XCD-contiguous unit schedule: unit =
// (pair, row y, x-range of PX pixels); XCD group b & 7 owns a contiguous range of units, its 32
// workgroups take units gi, gi + 32, ...
//   writes: a unit writes its PX pixels of all 192 volume planes (1 KiB per store instruction:
//           PX = 128: 8 rows x 128 B per wave (band_rs's shape); PX >= 256: one row, 1 KiB per
//           instruction), non-temporal unless PLAIN;
//   reads:  a unit reads its PX pixels (+ the 192-column right window when WIN) of 64 L and 64 R
//           planes, 16 channels per step, 1 KiB per load instruction, 3 steps in flight.
// Also a transposed write order (TR): unit = (pair, y, block of 24 planes), the whole 3,840-B row
// of each plane (what a workgroup owning every pixel of a row for a few disparities would write).
//   hipcc -O3 --offload-arch=gfx950 -shared -fPIC scripts/micro/mem_shapes.hip -o scripts/micro/libmem_shapes.so
#include <hip/hip_runtime.h>

namespace {
constexpr int C = 64, D = 192, H = 540, W = 960;
typedef float f4 __attribute__((ext_vector_type(4)));

// ORDER 0: units as band_rs (XCD-contiguous unit ranges, 32 workgroups on consecutive units);
// 1: row walk, XCD-contiguous row ranges (workgroup gi walks rows gi, gi + 32, ... of its XCD's
// range, each row's tiles left to right: band_sl with map 2); 2: row walk, rows b, b + 256, ...
template <int ORDER, int TPR>
__device__ __forceinline__ void unit_rc(int ub, int us, int k, int& row, int& tile) {
  if constexpr (ORDER == 0) {
    const int u = ub + k * us;
    row = u / TPR;
    tile = u % TPR;
  } else {
    row = ub + (k / TPR) * us;
    tile = k % TPR;
  }
}
template <int ORDER, int TPR>
__device__ __forceinline__ void sched_o(int np, int& ub, int& us, int& uc) {
  const int b = blockIdx.x, nwg = gridDim.x;
  if constexpr (ORDER == 2) {
    const int rows = np * H;
    ub = b;
    us = nwg;
    uc = max(0, (rows - b + nwg - 1) / nwg) * TPR;
    return;
  }
  const int units = ORDER == 0 ? np * H * TPR : np * H;
  const int grp = b & 7, gi = b >> 3, gsz = nwg >> 3;
  const int q = units / 8, r = units % 8;
  const int gb = grp * q + min(grp, r), gc = q + (grp < r ? 1 : 0);
  ub = gb + gi;
  us = gsz;
  uc = max(0, (gc - gi + gsz - 1) / gsz) * (ORDER == 0 ? 1 : TPR);
}

__device__ __forceinline__ void sched(int units, int& ubeg, int& ustep, int& ucnt) {
  const int b = blockIdx.x, nwg = gridDim.x;
  const int grp = b & 7, gi = b >> 3, gsz = nwg >> 3;
  const int q = units / 8, r = units % 8;
  const int gb = grp * q + min(grp, r), gc = q + (grp < r ? 1 : 0);
  ubeg = gb + gi;
  ustep = gsz;
  ucnt = max(0, (gc - gi + gsz - 1) / gsz);
}

// STAGGER (PX = 128): 1 each workgroup starts its unit's d-order at a different 8-row block
// (instruction i -> (i + b) % 12), so the chip's concurrent stores spread over all 192 planes;
// 2 the same, rotated per unit (k) as well
template <int PX, bool PLAIN, int ORDER = 0, int STAGGER = 0>
__global__ __launch_bounds__(512) void wr(float* __restrict__ out, int np) {
  constexpr int TPR = (W + PX - 1) / PX;  // units per row
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int ub, us, uc;
  sched_o<ORDER, TPR>(np, ub, us, uc);
  const size_t plane = (size_t)H * W;
  const f4 v = {1.f, 2.f, 3.f, (float)lane};
  for (int k = 0; k < uc; ++k) {
    int row, tile;
    unit_rc<ORDER, TPR>(ub, us, k, row, tile);
    const int n = row / H, y = row % H, x0 = tile * PX;
    float* ob = out + (size_t)n * D * plane + (size_t)y * W + x0;
    if constexpr (PX == 128) {  // 8 waves x 24 instructions; 8 rows x 128 B each
      const int w4 = wave & 3, dh = wave >> 2;
      for (int i0 = 0; i0 < 12; ++i0) {
        const int i = STAGGER == 0 ? i0 : STAGGER == 1 ? (i0 + (int)blockIdx.x) % 12 : (i0 + (int)blockIdx.x + 5 * k) % 12;
        const int d = 96 * dh + 8 * i + (lane >> 3), x = 32 * w4 + 4 * (lane & 7);
        if (x0 + x < W) {
          f4* p = reinterpret_cast<f4*>(ob + (size_t)d * plane + x);
          if (PLAIN) *p = v; else __builtin_nontemporal_store(v, p);
        }
      }
    } else {  // one plane row piece per instruction group: PX / 256 instructions of 1 KiB
      for (int d = wave; d < D; d += 8) {
#pragma unroll
        for (int c = 0; c < PX / 256; ++c) {
          const int x = 256 * c + 4 * lane;
          if (x0 + x < W) {
            f4* p = reinterpret_cast<f4*>(ob + (size_t)d * plane + x);
            if (PLAIN) *p = v; else __builtin_nontemporal_store(v, p);
          }
        }
      }
    }
  }
}

// transposed: unit = (n, y, 24-plane block): whole rows
template <bool PLAIN>
__global__ __launch_bounds__(512) void wr_tr(float* __restrict__ out, int np) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int ub, us, uc;
  sched(np * H * 8, ub, us, uc);
  const size_t plane = (size_t)H * W;
  const f4 v = {1.f, 2.f, 3.f, (float)lane};
  for (int k = 0; k < uc; ++k) {
    const int u = ub + k * us, row = u / 8, n = row / H, y = row % H, db = (u % 8) * 24;
    float* ob = out + ((size_t)n * D + db) * plane + (size_t)y * W;
    for (int d = wave; d < 24; d += 8)
      for (int x = 4 * lane; x < W; x += 256) {
        f4* p = reinterpret_cast<f4*>(ob + (size_t)d * plane + x);
        if (PLAIN) *p = v; else __builtin_nontemporal_store(v, p);
      }
  }
}

// reads: 8 waves; per step (16 channels) each lane loads 16 B from each of the unit's L and R
// plane rows it covers; 3 steps in flight (compiler-tracked), consumed into a register sum
template <int PX, bool WIN, int ORDER = 0, bool HOTWIN = false>
__global__ __launch_bounds__(512) void rd(const float* __restrict__ L, const float* __restrict__ R,
                                          float* __restrict__ sink, int np) {
  constexpr int TPR = (W + PX - 1) / PX;
  constexpr int RC = PX + (WIN ? 192 : 0);  // right-window columns
  constexpr int GL = PX / 4, GR = RC / 4, G = GL + GR;  // 16-B groups per channel row
  constexpr int ITEMS = 16 * G;                         // (channel, group) per step
  constexpr int PER = (ITEMS + 511) / 512;              // loads per lane and step
  int ub, us, uc;
  sched_o<ORDER, TPR>(np, ub, us, uc);
  const size_t plane = (size_t)H * W;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < uc; ++k) {
    int row, tile;
    unit_rc<ORDER, TPR>(ub, us, k, row, tile);
    const int n = row / H, y = row % H, x0 = tile * PX;
    // 4 steps x PER loads per lane, issued in batches of 8 (64 KiB in flight per workgroup)
    for (int b0 = 0; b0 < 4 * PER; b0 += 8) {
      f4 t[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int jj = b0 + j, ks = jj / PER, it = threadIdx.x + 512 * (jj % PER);
        const int cidx = it / G, g = it % G;
        const bool isR = g < GR;
        // HOTWIN: the window's loads re-read the unit's own R columns (same instruction count,
        // no lines of the neighbouring units)
        int px = isR ? (HOTWIN ? x0 + 4 * (g % (PX / 4)) : x0 - (WIN ? 192 : 0) + 4 * g) : x0 + 4 * (g - GR);
        px = min(max(px, 0), W - 4);
        const float* p = (isR ? R : L) + ((size_t)n * C + 16 * min(ks, 3) + min(cidx, 15)) * plane + (size_t)y * W + px;
        t[j] = *reinterpret_cast<const f4*>(p);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += t[j];
    }
  }
  if (acc.x == 12345.f) sink[threadIdx.x] = acc.y;
}

// reads and writes at once, band_rs's role split without its barriers: waves 0-3 write each
// unit's 192 x 128 px (8 rows x 128 B per instruction), waves 4-7 read it (PX = 128)
template <int ORDER, bool WIN>
__global__ __launch_bounds__(512) void rw(const float* __restrict__ L, const float* __restrict__ R,
                                          float* __restrict__ out, int np) {
  constexpr int PX = 128, TPR = 8;
  constexpr int RC = PX + (WIN ? 192 : 0);
  constexpr int GL = PX / 4, GR = RC / 4, G = GL + GR;
  constexpr int ITEMS = 16 * G, PER = (ITEMS + 255) / 256;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int ub, us, uc;
  sched_o<ORDER, TPR>(np, ub, us, uc);
  const size_t plane = (size_t)H * W;
  if (wave < 4) {
    const f4 v = {1.f, 2.f, 3.f, (float)lane};
    for (int k = 0; k < uc; ++k) {
      int row, tile;
      unit_rc<ORDER, TPR>(ub, us, k, row, tile);
      const int n = row / H, y = row % H, x0 = tile * PX;
      float* ob = out + (size_t)n * D * plane + (size_t)y * W + x0;
      for (int i = 0; i < 24; ++i) {
        const int d = 8 * i + (lane >> 3), x = 32 * wave + 4 * (lane & 7);
        if (x0 + x < W) __builtin_nontemporal_store(v, reinterpret_cast<f4*>(ob + (size_t)d * plane + x));
      }
    }
    return;
  }
  const int t = threadIdx.x - 256;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < uc; ++k) {
    int row, tile;
    unit_rc<ORDER, TPR>(ub, us, k, row, tile);
    const int n = row / H, y = row % H, x0 = tile * PX;
    for (int b0 = 0; b0 < 4 * PER; b0 += 8) {
      f4 tv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int jj = b0 + j, ks = jj / PER, it = t + 256 * (jj % PER);
        const int cidx = it / G, g = it % G;
        const bool isR = g < GR;
        int px = isR ? x0 - (WIN ? 192 : 0) + 4 * g : x0 + 4 * (g - GR);
        px = min(max(px, 0), W - 4);
        const float* p = (isR ? R : L) + ((size_t)n * C + 16 * min(ks, 3) + min(cidx, 15)) * plane + (size_t)y * W + px;
        tv[j] = *reinterpret_cast<const f4*>(p);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += tv[j];
    }
  }
  if (acc.x == 12345.f) out[threadIdx.x] = acc.y;
}

// cfg3's groupwise output (N, G, H, W, D) fp32, G = 8, D = 192: a unit (n, g, y, 128-px tile)
// is 128 pixel records of 768 B, 96 KB contiguous; NW waves of the workgroup write it, 1 KiB per
// store instruction (band_rs GW: 4 compute waves, 24 pieces each).  ORDER 0: units in band_rs's
// XCD-contiguous order; 1: the units of one (n, g, y) row walked by one workgroup (row walk)
template <int NW, bool PLAIN, int ORDER>
__global__ __launch_bounds__(512) void wr_gw(float* __restrict__ out, int np) {
  constexpr int G = 8, TPR = 8;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  if (wave >= NW) return;
  int ub, us, uc;
  // rows here are (n, g, y): np G H of them
  sched_o<ORDER, TPR>(np * G, ub, us, uc);
  const f4 v = {1.f, 2.f, 3.f, (float)lane};
  for (int k = 0; k < uc; ++k) {
    int row, tile;
    unit_rc<ORDER, TPR>(ub, us, k, row, tile);
    const int x0 = tile * 128;
    const int npx = min(128, W - x0);
    float* ob = out + ((size_t)row * W + x0) * D;  // row = (n G + g) H + y
    const int nb = npx * D * 4 / 1024;               // 1-KiB pieces of the unit
    for (int i = wave; i < nb; i += NW) {
      f4* p = reinterpret_cast<f4*>(ob + (size_t)i * 256 + 4 * lane);
      if (PLAIN) *p = v; else __builtin_nontemporal_store(v, p);
    }
  }
}

template <typename K, typename... A>
int launch(K k, hipStream_t st, A... a) {
  hipLaunchKernelGGL(k, dim3(256), dim3(512), 0, st, a...);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}
}  // namespace

extern "C" int mem_run(int variant, const float* L, const float* R, float* out, int np, hipStream_t st) {
  switch (variant) {
    case 0: return launch(wr<128, false>, st, out, np);
    case 1: return launch(wr<256, false>, st, out, np);
    case 2: return launch(wr<512, false>, st, out, np);
    case 3: return launch(wr<1024, false>, st, out, np);
    case 4: return launch(wr_tr<false>, st, out, np);
    case 5: return launch(wr<128, true>, st, out, np);
    case 6: return launch(wr<1024, true>, st, out, np);
    case 7: return launch(wr_tr<true>, st, out, np);
    case 10: return launch(rd<128, true>, st, L, R, out, np);
    case 11: return launch(rd<128, false>, st, L, R, out, np);
    case 12: return launch(rd<256, false>, st, L, R, out, np);
    case 13: return launch(rd<512, false>, st, L, R, out, np);
    case 14: return launch(rd<1024, false>, st, L, R, out, np);
    case 15: return launch(rd<256, true>, st, L, R, out, np);
    case 16: return launch(rd<128, true, 0, true>, st, L, R, out, np);
    case 20: return launch(wr<128, false, 1>, st, out, np);
    case 21: return launch(wr<128, false, 2>, st, out, np);
    case 22: return launch(rd<128, false, 1>, st, L, R, out, np);
    case 23: return launch(rd<128, false, 2>, st, L, R, out, np);
    case 24: return launch(rd<128, true, 1>, st, L, R, out, np);
    case 25: return launch(wr<128, false, 1, 1>, st, out, np);
    case 26: return launch(wr<128, false, 1, 2>, st, out, np);
    case 27: return launch(wr<128, false, 0, 1>, st, out, np);
    case 40: return launch(wr_gw<4, false, 0>, st, out, np);
    case 41: return launch(wr_gw<4, true, 0>, st, out, np);
    case 42: return launch(wr_gw<8, false, 0>, st, out, np);
    case 43: return launch(wr_gw<8, true, 0>, st, out, np);
    case 44: return launch(wr_gw<4, false, 1>, st, out, np);
    case 45: return launch(wr_gw<4, true, 1>, st, out, np);
    case 30: return launch(rw<0, true>, st, L, R, out, np);
    case 31: return launch(rw<0, false>, st, L, R, out, np);
    case 32: return launch(rw<1, true>, st, L, R, out, np);
    case 33: return launch(rw<1, false>, st, L, R, out, np);
    default: return -1;
  }
}

// The sliding-window band kernel's memory pattern (csrc/ip_sl.hip) without its arithmetic, to
// find what the kernel's structure costs against a free-running read + write stream.
// One 512-thread workgroup per CU walks whole rows (rows b, b + 256, ...) of NP cfg2 pairs
// (64 x 540 x 960 fp32, D = 192), 8 segments of 128 pixels per row, 4 steps of 16 channels per
// segment.  Waves 4-7 (readers) load per step 16 channels x 128 columns of L and of R (4 x 16-B
// loads per lane, register sets SETS deep) and write them to LDS; waves 0-3 (writers) store the
// segment's 192 x 128-pixel output rows as 8 rows x 128 B per instruction.
//   MODE bits: 1 readers, 2 writers, 4 a barrier per step (else free-running), 8 the writers'
//   stores bunched as the kernel's (16 in step 0, 4 in steps 1 and 2; else 6 per step),
//   16 non-temporal stores (else plain), 32 readers use LDS-DMA (no registers)
//   hipcc -O3 --offload-arch=gfx950 scripts/micro/sl_pattern.hip -o /tmp/slp && /tmp/slp [NP]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int C = 64, D = 192, H = 540, W = 960, TILES = 8;
typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_byte) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_byte)
      : "memory");
}

// the kernel's barrier: LDS only, memory operations stay in flight
__device__ __forceinline__ void bar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// MAP: which rows a workgroup walks -- 0 rows b, b + nwg, ... (all workgroups on adjacent rows
// at once); 1 a contiguous block of rows per workgroup (256 regions spread over the batch);
// 2 XCD groups (b & 7) on 8 contiguous ranges, their 32 workgroups interleaved within each
template <int MODE, int SETS, int MAP = 0>
__global__ __launch_bounds__(512) void slp(const float* __restrict__ L, const float* __restrict__ R,
                                           float* __restrict__ out, int rows) {
  extern __shared__ unsigned char smem[];
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x, nwg = gridDim.x;
  int rbeg, rstep, rcnt;
  if (MAP == 0) {
    rbeg = b; rstep = nwg; rcnt = (rows - b + nwg - 1) / nwg;
  } else if (MAP == 1) {
    const int q = rows / nwg, r = rows % nwg;
    rbeg = b * q + min(b, r); rstep = 1; rcnt = q + (b < r ? 1 : 0);
  } else if (MAP == 2) {
    const int grp = b & 7, gi = b >> 3, gsz = nwg >> 3;
    const int q = rows / 8, r = rows % 8;
    const int gb = grp * q + min(grp, r), gc = q + (grp < r ? 1 : 0);
    rbeg = gb + gi; rstep = gsz; rcnt = (gc - gi + gsz - 1) / gsz;
  } else if (MAP == 6) {
    // MAP 6: units in one chip-wide sweep: unit u on workgroup u % 256 at time u / 256, so the
    // chip works on 32 consecutive whole rows at a time (the most linear write order)
    rbeg = b; rstep = nwg; rcnt = (rows * TILES - b + nwg - 1) / nwg;
  } else if (MAP >= 4) {
    // MAP 4 / 5: runs of TG = 2 / 4 tiles: unit = (row, run); XCD group b & 7 owns a contiguous
    // range of units, its 32 workgroups take units gi, gi + 32, ...: 8 / TG workgroups of one
    // XCD on the runs of a row at once, each walking its run's tiles in order (a sliding window)
    constexpr int TG = MAP == 4 ? 2 : 4;
    const int grp = b & 7, gi = b >> 3, gsz = nwg >> 3;
    const int units = rows * (TILES / TG), q = units / 8, r = units % 8;
    const int gb = grp * q + min(grp, r), gc = q + (grp < r ? 1 : 0);
    rbeg = gb + gi; rstep = gsz; rcnt = ((gc - gi + gsz - 1) / gsz) * TG;
  } else {
    // MAP 3 (units, not rows: the band_rs / r03-micro schedule): unit = (row, tile); XCD group
    // b & 7 owns a contiguous range of units, its 32 workgroups take units gi, gi + 32, ... of it,
    // so the 8 tiles of a row run on 8 workgroups of one XCD at the same time
    const int grp = b & 7, gi = b >> 3, gsz = nwg >> 3;
    const int units = rows * TILES, q = units / 8, r = units % 8;
    const int gb = grp * q + min(grp, r), gc = q + (grp < r ? 1 : 0);
    rbeg = gb + gi; rstep = gsz; rcnt = (gc - gi + gsz - 1) / gsz;
  }
  const int nseg = MAP >= 3 ? rcnt : rcnt * TILES;  // (MAP 6 as MAP 3: one tile per unit)
  const size_t plane = (size_t)H * W;
  auto seg_row = [&](int s, int& n, int& y, int& x0) {
    if (MAP == 6) {
      const int u = rbeg + s * rstep, row = u / TILES;
      n = row / H;
      y = row % H;
      x0 = (u % TILES) * 128;
      return;
    }
    if (MAP >= 4) {
      constexpr int TG = MAP == 4 ? 2 : 4;
      const int u = rbeg + (s / TG) * rstep, row = u / (TILES / TG);
      n = row / H;
      y = row % H;
      x0 = ((u % (TILES / TG)) * TG + s % TG) * 128;
      return;
    }
    if (MAP == 3) {
      const int u = rbeg + s * rstep, row = u / TILES;
      n = row / H;
      y = row % H;
      x0 = (u % TILES) * 128;
      return;
    }
    const int row = rbeg + (s / TILES) * rstep;
    n = row / H;
    y = row % H;
    x0 = (s % TILES) * 128;
  };
  if (wave >= 4) {  // readers
    const int mw = wave - 4;
    const bool isR = mw >= 2;
    const int wp = mw & 1;
    const int g = (lane & 7) | (((lane >> 4) & 3) << 3);
    const int c4 = (lane >> 3) & 1;
    const float* base = isR ? R : L;
    f4 sv[SETS][4];
    auto load = [&](int set, int j) {  // the loads of global step j
      const int s = min(j >> 2, nseg - 1), k = j & 3;
      int n, y, x0;
      seg_row(s, n, y, x0);
      const int px = min(x0 + 4 * g, W - 4);
      const float* p = base + ((size_t)n * C + 16 * k + 8 * wp + 4 * c4) * plane + (size_t)y * W + px;
      if constexpr (MODE & 64) {  // band_rs's right window: 320 columns from x0 - 192 (3 rounds)
        if (isR) {
#pragma unroll
          for (int rr = 0; rr < 3; ++rr) {
            const int gg = g + 32 * rr;
            const int pxr = min(max(x0 - 192 + 4 * min(gg, 79), 0), W - 4);
            const float* pr = base + ((size_t)n * C + 16 * k + 8 * wp + 4 * c4) * plane + (size_t)y * W + pxr;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const f4 t = *reinterpret_cast<const f4*>(pr + q * plane);
              sv[set][q] = rr == 0 ? t : sv[set][q] + t;
            }
          }
          return;
        }
      }
      if constexpr (MODE & 32) {
        const unsigned lb = 4096u * (unsigned)(j % SETS) + 1024u * (unsigned)mw;
#pragma unroll
        for (int q = 0; q < 4; ++q) glds16(p + q * plane, lb + 16384u * (unsigned)q);
      } else {
#pragma unroll
        for (int q = 0; q < 4; ++q)
          sv[set][q] = *reinterpret_cast<const f4*>(p + q * plane);
      }
    };
    const int nsteps = nseg * 4;
    if (!(MODE & 1)) {
      if (MODE & 4)
        for (int j = 0; j < nsteps; ++j) bar();
      return;
    }
#pragma unroll
    for (int q = 0; q < SETS - 1; ++q) load(q, q);
    for (int j0 = 0; j0 < nsteps; j0 += SETS) {
#pragma unroll
      for (int q = 0; q < SETS; ++q) {
        const int j = j0 + q;
        if (j < nsteps) {
          load((q + SETS - 1) % SETS, j + SETS - 1);
          if constexpr (MODE & 32) {
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (SETS - 1)) : "memory");
          } else {
            // consume set q: write 4 x 8 B to LDS (as the staging does)
            unsigned* d = reinterpret_cast<unsigned*>(smem + 2048 * mw + 8 * lane);
#pragma unroll
            for (int p = 0; p < 4; ++p)
              *reinterpret_cast<u2*>(d + 512 * p) =
                  u2{__float_as_uint(sv[q][p].x + sv[q][p].y), __float_as_uint(sv[q][p].z + sv[q][p].w)};
          }
          if (MODE & 4) bar();
        }
      }
    }
    return;
  }
  // writers: wave w owns pixels 32 w .. 32 w + 31 of each segment
  const int rl = lane >> 3, cl = lane & 7;
  f4 v = {1.f, 2.f, 3.f, (float)lane};
  const int nsteps = nseg * 4;
  int pend = 0;  // stores of the previous segment not yet issued
  for (int j = 0; j < nsteps; ++j) {
    if (MODE & 2) {
      const int k = j & 3;
      const int s = (j >> 2) - 1;  // stores of the previous segment
      if (s >= 0) {
        int n, y, x0;
        seg_row(s, n, y, x0);
        int j0, j1;
        if (MODE & 8) {  // as the kernel: 16 stores in step 0, 4 in steps 1 and 2
          j0 = k == 0 ? 0 : k == 1 ? 16 : k == 2 ? 20 : 24;
          j1 = k == 0 ? 16 : k == 1 ? 20 : 24;
        } else {
          j0 = 6 * k;
          j1 = 6 * k + 6;
        }
        const int x = x0 + 32 * wave + 4 * cl;
        for (int jj = j0; jj < j1; ++jj) {
          const int d = 8 * jj + rl;
          f4* o = reinterpret_cast<f4*>(out + ((size_t)n * D + d) * plane + (size_t)y * W + x);
          if (x < W) {
            if (MODE & 16) __builtin_nontemporal_store(v, o); else *o = v;
          }
        }
      }
    }
    (void)pend;
    if (MODE & 4) bar();
  }
}

template <typename F>
float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  float ts[7];
  for (int i = 0; i < 7; ++i) {
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    hipEventElapsedTime(&ts[i], a, b);
  }
  for (int i = 0; i < 7; ++i)
    for (int j = i + 1; j < 7; ++j)
      if (ts[j] < ts[i]) { float t = ts[i]; ts[i] = ts[j]; ts[j] = t; }
  return ts[3] * 1e3f;  // median
}

int main(int argc, char** argv) {
  const int NP = argc > 1 ? atoi(argv[1]) : 32;
  float *L, *R, *out;
  const size_t fb = (size_t)NP * C * H * W * 4, ob = (size_t)NP * D * H * W * 4;
  if (hipMalloc(&L, fb) || hipMalloc(&R, fb) || hipMalloc(&out, ob)) { printf("alloc failed\n"); return 1; }
  hipMemset(L, 0, fb);
  hipMemset(R, 0, fb);
  const int rows = NP * H;
  auto rep = [&](const char* name, float us, size_t bytes) {
    printf("{\"np\": %d, \"case\": \"%s\", \"us\": %.1f, \"us_per_pair\": %.2f, \"TBps\": %.3f, \"frac\": %.4f}\n",
           NP, name, us, us / NP, bytes / us / 1e6, bytes / us / 1e6 / 8.0);
    fflush(stdout);
  };
#define RUN(MODE, SETS, MAP, BYTES)                                                                 \
  {                                                                                                 \
    auto k = slp<MODE, SETS, MAP>;                                                                  \
    hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);         \
    rep("mode=" #MODE " sets=" #SETS " map=" #MAP, timeit([&] { k<<<256, 512, 65536>>>(L, R, out, rows); }), BYTES); \
  }
  const size_t rd = 2 * fb, wr = ob;
  for (int rep2 = 0; rep2 < 2; ++rep2) {
    RUN(1 + 2 + 4 + 8 + 16, 4, 0, rd + wr) RUN(2 + 16, 4, 0, wr)        // rows (sliding)
    RUN(1 + 2 + 4 + 8 + 16, 4, 3, rd + wr) RUN(2 + 16, 4, 3, wr)        // XCD units
    RUN(1 + 2 + 4 + 8 + 16 + 64, 4, 3, rd + wr) RUN(1 + 4 + 16 + 64, 4, 3, rd)  // XCD units, rs reads
    RUN(1 + 2 + 4 + 8 + 16, 4, 6, rd + wr) RUN(2 + 16, 4, 6, wr) RUN(2, 4, 6, wr)  // chip-wide units
  }
  return 0;
}

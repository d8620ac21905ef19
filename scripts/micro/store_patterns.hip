// Store-bandwidth microbenchmark for the cost-volume output pattern (D, H, W) fp32 = 192 x 540
// x 960: which store shapes reach the HBM write roofline on MI355X.
//   hipcc -O3 --offload-arch=gfx950 scripts/micro/store_patterns.hip -o /tmp/store_patterns
// Every kernel writes the whole volume once from registers (no loads, no LDS).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int D = 192, H = 540, W = 960;
typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__device__ __forceinline__ void st(float* p, f4 v) {
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<f4*>(p));
  else *reinterpret_cast<f4*>(p) = v;
}

// A: persistent WGs of NW waves; unit = (y, 128-px segment); each store instruction covers
//    ROWS rows x (1024/ROWS) bytes; the NW waves split the 192 rows of the unit.
template <int NW, int ROWS, bool NT>
__global__ __launch_bounds__(64 * NW) void seg_store(float* out, int nunits) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lpr = 64 / ROWS;                 // lanes per row
  const int rr = lane / lpr, cc = lane % lpr;  // row within instruction, 16-B column
  const int seg_px = 128;
  f4 v = {1.f, 2.f, 3.f, (float)lane};
  for (int u = blockIdx.x; u < nunits; u += gridDim.x) {
    const int y = u / 8, tile = u % 8;
    const int x0 = tile * seg_px;
    if (x0 >= W) continue;
    // this wave's share: rows [wave*192/NW, (wave+1)*192/NW), instruction covers ROWS rows
    // and (lpr*16) bytes of each; a row of 512 B needs 512/(lpr*16) column passes
    const int cols = 512 / (lpr * 16);
    for (int d = wave * (D / NW); d < (wave + 1) * (D / NW); d += ROWS)
      for (int c = 0; c < cols; ++c) {
        const int x = x0 + 4 * (c * lpr + cc);
        if (x < W) st<NT>(out + ((size_t)(d + rr) * H + y) * W + x, v);
      }
  }
}

// C: full rows: one WG (4 waves) per (d-group of 16 rows, y); each instruction 1 KB contiguous
template <bool NT>
__global__ __launch_bounds__(256) void row_store(float* out) {
  const int y = blockIdx.x, dg = blockIdx.y;
  f4 v = {1.f, 2.f, 3.f, 4.f};
  for (int d = dg * 16; d < dg * 16 + 16; ++d)
    for (int x = 4 * threadIdx.x; x < W; x += 4 * 256) st<NT>(out + ((size_t)d * H + y) * W + x, v);
}

template <typename F>
float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  float best = 1e9;
  for (int i = 0; i < 5; ++i) {
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best * 1e3f;
}

int main() {
  float* out;
  const size_t bytes = (size_t)D * H * W * 4;
  hipMalloc(&out, bytes);
  const int nunits = H * 8;
  auto rep = [&](const char* name, float us) {
    printf("%-44s %8.1f us  %6.2f TB/s\n", name, us, bytes / us / 1e6);
  };
#define SEG(NW, ROWS, NT, G)                                                                  \
  rep("seg NW=" #NW " rows/instr=" #ROWS " nt=" #NT " grid=" #G,                              \
      timeit([&] { seg_store<NW, ROWS, NT><<<G, 64 * NW>>>(out, nunits); }));
  SEG(4, 2, true, 256) SEG(4, 2, false, 256) SEG(4, 8, true, 256) SEG(8, 2, true, 256)
  SEG(8, 2, false, 256) SEG(16, 2, true, 256) SEG(4, 2, true, 512) SEG(4, 2, true, 1024)
  SEG(8, 2, true, 512) SEG(4, 4, true, 256) SEG(8, 8, true, 512)
  SEG(4, 2, true, 4320) SEG(8, 2, true, 4320)
  // the band kernel's chunk stores: 8 rows x 128 B (32-pixel waves) vs 16 rows x 64 B (16-pixel)
  SEG(4, 8, true, 512) SEG(4, 8, false, 512) SEG(4, 16, true, 512) SEG(4, 16, false, 512)
  SEG(8, 8, true, 512)  // (ROWS must divide D / NW = 24 rows per wave: no 16-row variant at NW=8)
  rep("rows nt", timeit([&] { row_store<true><<<dim3(H, D / 16), 256>>>(out); }));
  rep("rows", timeit([&] { row_store<false><<<dim3(H, D / 16), 256>>>(out); }));
  hipFree(out);
  return 0;
}

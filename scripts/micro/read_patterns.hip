// Read-bandwidth microbenchmark for the regression access pattern: a (D, H*W) fp32 volume,
// D = 192, H*W = 540*960, read once (no math beyond a running sum that is stored per lane).
//   hipcc -O3 --offload-arch=gfx950 scripts/micro/read_patterns.hip -o /tmp/read_patterns
// Compares a plain grid-stride stream with the plane-chunk walk of softargmin_f32x4_kernel.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <string>

constexpr int D = 192, P = 540 * 960;

// plain stream: every lane reads float4s, grid-stride over the whole buffer
__global__ __launch_bounds__(256) void stream_read(const float4* __restrict__ v, size_t n4,
                                                   float* __restrict__ sink) {
  float acc = 0.f;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const float4 a = v[i];
    acc += a.x + a.y + a.z + a.w;
  }
  sink[(size_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

// the soft-argmin walk: block = 4 waves over 256*PXV*... pixels; wave w owns the D quarter;
// KC planes in flight per wave; each lane reads V float4s per plane (V*64*16 B per wave row)
template <int KC, int V>
__global__ __launch_bounds__(256) void plane_walk(const float* __restrict__ vol,
                                                  float* __restrict__ sink) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int px0 = blockIdx.x * (64 * 4 * V);
  const int Dq = D / 4, d0 = wave * Dq;
  float acc = 0.f;
  for (int d = d0; d < d0 + Dq; d += KC) {
    float4 a[KC][V];
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int u = 0; u < V; ++u)
        a[k][u] = *reinterpret_cast<const float4*>(vol + (size_t)(d + k) * P + px0 + (u * 64 + lane) * 4);
#pragma unroll
    for (int k = 0; k < KC; ++k)
#pragma unroll
      for (int u = 0; u < V; ++u) acc += a[k][u].x + a[k][u].y + a[k][u].z + a[k][u].w;
  }
  sink[(size_t)blockIdx.x * 256 + threadIdx.x] = acc;
}

template <typename F>
float timeit(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  f();
  hipDeviceSynchronize();
  float best = 1e9;
  for (int i = 0; i < 10; ++i) {
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
  float *vol, *sink;
  const size_t bytes = (size_t)D * P * 4;
  hipMalloc(&vol, bytes);
  hipMalloc(&sink, (size_t)64 << 20);
  hipMemset(vol, 0, bytes);
  auto rep = [&](const char* name, float us) {
    printf("%-40s %8.1f us  %6.2f TB/s  frac %.3f\n", name, us, bytes / us / 1e6, bytes / us / 8e6);
  };
  const size_t n4 = bytes / 16;
  for (int g : {1024, 2048, 4096, 8192, 16384})
    rep((std::string("stream grid=") + std::to_string(g)).c_str(),
        timeit([&] { stream_read<<<g, 256>>>(reinterpret_cast<const float4*>(vol), n4, sink); }));
#define WALK(KC, V)                                                                        \
  rep("walk KC=" #KC " V=" #V, timeit([&] {                                                \
        plane_walk<KC, V><<<P / (256 * V), 256>>>(vol, sink);                              \
      }));
  WALK(8, 1) WALK(4, 1) WALK(16, 1) WALK(4, 2) WALK(8, 2) WALK(2, 4) WALK(4, 4)
  hipFree(vol);
  hipFree(sink);
  return 0;
}

// Diagnostic A/B driver for the fp32 soft-argmin kernels on the cfg2 volume (1x192x540x960):
// the library kernel (softargmin_wave_kernel<8,1>) against software-pipelined variants that keep
// the next chunk's plane loads in flight while the current chunk is folded.
//   hipcc -O3 -std=c++20 --offload-arch=gfx950 -Iinclude scripts/regress_ab.hip -o bin/regress_ab
//   bin/regress_ab            (GPU box)
#include "../realtime_stereo_matcher_amd/csrc/common.hip"
#include "../realtime_stereo_matcher_amd/csrc/regress.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>

namespace smcv {
namespace {

// ping-pong over two KC-plane register sets: loads of chunk c+1 fly while chunk c is folded
template <int KC, bool PRESOFT>
__global__ __launch_bounds__(64) void sa_pipe(const float* __restrict__ vol, float* __restrict__ out,
                                              int D, int W, int64_t vsn, int64_t vsd, int nunits) {
  const int P = (W + 255) >> 8;
  const int unit = blockIdx.x;
  if (unit >= nunits) return;
  const int n = unit / P;
  const int lane = threadIdx.x & 63;
  const int x0 = ((unit - n * P) * 64 + lane) * 4;
  if (x0 >= W) return;
  const float* base = vol + n * vsn + x0;
  float m[4];
  double S[4], T[4];
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    m[p] = -INFINITY;
    S[p] = 0.0;
    T[p] = 0.0;
  }
  auto load = [&](float4 (&v4)[KC], int d0) {
#pragma unroll
    for (int k = 0; k < KC; ++k)
      v4[k] = *reinterpret_cast<const float4*>(base + (int64_t)min(d0 + k, D - 1) * vsd);
  };
  auto fold = [&](const float4 (&v4)[KC], int d0) {
    const int nd = min(KC, D - d0);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      float v[KC];
#pragma unroll
      for (int k = 0; k < KC; ++k) v[k] = p == 0 ? v4[k].x : p == 1 ? v4[k].y : p == 2 ? v4[k].z : v4[k].w;
      if (PRESOFT) {
#pragma unroll
        for (int k = 0; k < KC; ++k)
          if (k < nd) T[p] += (double)(d0 + k) * (double)v[k];
      } else if (nd == KC) {
        fold_chunk<KC, true>(v, nd, d0, m[p], S[p], T[p]);
      } else {
        fold_chunk<KC, false>(v, nd, d0, m[p], S[p], T[p]);
      }
    }
  };
  float4 a[KC], b[KC];
  load(a, 0);
  for (int d0 = 0; d0 < D; d0 += 2 * KC) {
    if (d0 + KC < D) load(b, d0 + KC);
    fold(a, d0);
    if (d0 + KC >= D) break;
    if (d0 + 2 * KC < D) load(a, d0 + 2 * KC);
    fold(b, d0 + KC);
  }
  float res[4];
#pragma unroll
  for (int p = 0; p < 4; ++p)
    res[p] = PRESOFT ? (float)T[p]
             : (D == 0) ? 0.f : (m[p] == INFINITY || m[p] == -INFINITY) ? NAN : (float)(T[p] / S[p]);
  *reinterpret_cast<float4*>(out + (int64_t)n * W + x0) = make_float4(res[0], res[1], res[2], res[3]);
}

}  // namespace
}  // namespace smcv

int main() {
  const int64_t N = 1, D = 192, H = 540, W = 960, HW = H * W;
  float *vol, *o1, *o2;
  hipMalloc(&vol, N * D * HW * 4);
  hipMalloc(&o1, N * HW * 4);
  hipMalloc(&o2, N * HW * 4);
  std::vector<float> h(N * D * HW);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 4001) / 500.f - 4.f;
  hipMemcpy(vol, h.data(), h.size() * 4, hipMemcpyHostToDevice);
  const int nunits = (int)((HW + 255) / 256 * N);
  auto lib = [&]() {
    hipLaunchKernelGGL((smcv::softargmin_wave_kernel<8, 1>), dim3(nunits), dim3(64), 0, nullptr, vol, o1,
                       (int)D, (int)HW, D * HW, HW, nunits);
  };
  auto p8 = [&]() {
    hipLaunchKernelGGL((smcv::sa_pipe<8, false>), dim3(nunits), dim3(64), 0, nullptr, vol, o2, (int)D, (int)HW,
                       D * HW, HW, nunits);
  };
  auto p4 = [&]() {
    hipLaunchKernelGGL((smcv::sa_pipe<4, false>), dim3(nunits), dim3(64), 0, nullptr, vol, o2, (int)D, (int)HW,
                       D * HW, HW, nunits);
  };
  auto p6 = [&]() {
    hipLaunchKernelGGL((smcv::sa_pipe<6, false>), dim3(nunits), dim3(64), 0, nullptr, vol, o2, (int)D, (int)HW,
                       D * HW, HW, nunits);
  };
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto time = [&](auto f) {
    for (int i = 0; i < 3; ++i) f();
    hipDeviceSynchronize();
    std::vector<float> ts;
    for (int i = 0; i < 30; ++i) {
      hipEventRecord(a);
      f();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms;
      hipEventElapsedTime(&ms, a, b);
      ts.push_back(ms * 1e3f);
    }
    std::sort(ts.begin(), ts.end());
    return std::make_pair(ts[ts.size() / 2], ts[0]);
  };
  auto check = [&]() {
    std::vector<float> r1(N * HW), r2(N * HW);
    hipMemcpy(r1.data(), o1, r1.size() * 4, hipMemcpyDeviceToHost);
    hipMemcpy(r2.data(), o2, r2.size() * 4, hipMemcpyDeviceToHost);
    double e = 0;
    for (size_t i = 0; i < r1.size(); ++i) e = std::max(e, (double)std::fabs(r1[i] - r2[i]));
    return e;
  };
  const double bytes = (double)N * D * HW * 4 + N * HW * 4;
  for (int rep = 0; rep < 2; ++rep) {
    auto t = time(lib);
    printf("lib wave<8>   median %.1f us min %.1f us  frac %.3f\n", t.first, t.second, bytes / t.first / 8e6);
    t = time(p8);
    lib();
    printf("pipe<8>       median %.1f us min %.1f us  frac %.3f  max|diff| %.3g\n", t.first, t.second,
           bytes / t.first / 8e6, check());
    t = time(p4);
    printf("pipe<4>       median %.1f us min %.1f us  frac %.3f  max|diff| %.3g\n", t.first, t.second,
           bytes / t.first / 8e6, check());
    t = time(p6);
    printf("pipe<6>       median %.1f us min %.1f us  frac %.3f  max|diff| %.3g\n", t.first, t.second,
           bytes / t.first / 8e6, check());
  }
  printf("err=%s\n", hipGetErrorString(hipGetLastError()));
  return 0;
}

// Diagnostic A/B driver for the concatenate volume (cfg5: 1x128x540x960 fp16, D=64, out
// (N, 2C, H, W, D) fp16 = 17.25 GB): the library kernel against
//   zeros     the same grid and store loop writing zeros (the pattern's write ceiling),
//   pow2      the library kernel with x = v >> log2(D/8) instead of a runtime division,
//   pixel     one lane per (x, 8-disparity vector) with the R values read as one 16-B LDS load
//             of a reversed row copy.
//   hipcc -O3 -std=c++20 --offload-arch=gfx950 -Iinclude -c scripts/concat_ab.hip -o /tmp/cab.o && hipcc --offload-arch=gfx950 /tmp/cab.o build/stereocv/cv_dot.o -o bin/concat_ab
#include "../realtime_stereo_matcher_amd/csrc/common.hip"
#include "../realtime_stereo_matcher_amd/csrc/cv_copy.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

namespace smcv {
namespace {

__global__ __launch_bounds__(kThreads) void cc_zeros(uint16_t* __restrict__ out, int C, int H, int W, int D) {
  const int row = blockIdx.x;
  const int y = row % H;
  const int nc = row / H;
  const int c = nc % C;
  const int n = nc / C;
  const size_t span = (size_t)W * D;
  uint16_t* outL = out + (((size_t)n * 2 * C + c) * H + y) * span;
  uint16_t* outR = out + (((size_t)n * 2 * C + C + c) * H + y) * span;
  const unsigned nvec = (unsigned)(span / 8);
  for (unsigned v = threadIdx.x; v < nvec; v += kThreads) {
    *reinterpret_cast<uint4*>(outL + v * 8) = make_uint4(0, 0, 0, 0);
    *reinterpret_cast<uint4*>(outR + v * 8) = make_uint4(0, 0, 0, 0);
  }
}

// D / 8 = 1 << LG vectors per pixel; the R row is staged reversed (Rr[j] = R[W-1-j]) so the 8
// values R[x-d0-7 .. x-d0] of a vector are 8 consecutive halves Rr[W-1-x+d0 .. +7] in LDS
template <int LG>
__global__ __launch_bounds__(kThreads) void cc_pow2(const uint16_t* __restrict__ L, const uint16_t* __restrict__ R,
                                                    uint16_t* __restrict__ out, int C, int H, int W, int D,
                                                    Strides4 ls, Strides4 rs) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_c[];
  uint16_t* Ls = reinterpret_cast<uint16_t*>(smem_c);
  uint16_t* Rr = Ls + W + 8;  // reversed R, 8 zero halves after it
  const int row = blockIdx.x;
  const int y = row % H;
  const int nc = row / H;
  const int c = nc % C;
  const int n = nc / C;
  const uint16_t* Lrow = L + n * ls.n + (int64_t)c * ls.c + (int64_t)y * ls.h;
  const uint16_t* Rrow = R + n * rs.n + (int64_t)c * rs.c + (int64_t)y * rs.h;
  for (int x = threadIdx.x; x < W; x += kThreads) {
    Ls[x] = Lrow[x];
    Rr[W - 1 - x] = Rrow[x];
  }
  if (threadIdx.x < 8) Rr[W + threadIdx.x] = 0;
  __syncthreads();
  const size_t span = (size_t)W * D;
  uint16_t* outL = out + (((size_t)n * 2 * C + c) * H + y) * span;
  uint16_t* outR = out + (((size_t)n * 2 * C + C + c) * H + y) * span;
  const unsigned nvec = (unsigned)(span / 8);
  for (unsigned v = threadIdx.x; v < nvec; v += kThreads) {
    const unsigned x = v >> LG;
    const unsigned d0 = (v & ((1u << LG) - 1)) * 8;
    const uint16_t lx = Ls[x];
    vec16<uint16_t> a, b;
    // R values: Rr[W-1-x+d0+k] = R[x-d0-k] for k = 0..7 (zero past the row end: x-d0-k < 0)
    const int j0 = W - 1 - (int)x + (int)d0;
    uint16_t rv[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) rv[k] = Rr[min(j0 + k, W + 7)];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const bool ok = d0 + k <= x;
      a.v[k] = ok ? lx : (uint16_t)0;
      b.v[k] = ok ? rv[k] : (uint16_t)0;
    }
    store16(outL + (size_t)v * 8, a);
    store16(outR + (size_t)v * 8, b);
  }
}

}  // namespace
}  // namespace smcv

int main() {
  const int64_t N = 1, C = 128, H = 540, W = 960, D = 64;
  const size_t nin = N * C * H * W, nout = N * 2 * C * H * W * D;
  uint16_t *L, *R, *O1, *O2;
  hipMalloc(&L, nin * 2);
  hipMalloc(&R, nin * 2);
  hipMalloc(&O1, nout * 2);
  hipMalloc(&O2, nout * 2);
  std::vector<uint16_t> h(nin);
  for (size_t i = 0; i < nin; ++i) h[i] = (uint16_t)(i * 2654435761u >> 7);
  hipMemcpy(L, h.data(), nin * 2, hipMemcpyHostToDevice);
  for (size_t i = 0; i < nin; ++i) h[i] = (uint16_t)(i * 40503u + 7);
  hipMemcpy(R, h.data(), nin * 2, hipMemcpyHostToDevice);
  smcv::Strides4 ls{C * H * W, H * W, W}, rs = ls;
  auto lib = [&]() { return smcv::concat_entry(L, R, O1, SM_F16, N, C, H, W, D, nullptr, nullptr, nullptr); };
  dim3 grid((unsigned)(N * C * H));
  auto zeros = [&]() {
    hipLaunchKernelGGL(smcv::cc_zeros, grid, dim3(smcv::kThreads), 0, nullptr, O2, (int)C, (int)H, (int)W, (int)D);
    return 0;
  };
  auto pow2 = [&]() {
    hipLaunchKernelGGL((smcv::cc_pow2<3>), grid, dim3(smcv::kThreads), (size_t)(2 * W + 16) * 2, nullptr, L, R, O2,
                       (int)C, (int)H, (int)W, (int)D, ls, rs);
    return 0;
  };
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  auto time = [&](auto f) {
    for (int i = 0; i < 2; ++i) f();
    hipDeviceSynchronize();
    std::vector<float> ts;
    for (int i = 0; i < 10; ++i) {
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
  const double bytes = (double)nout * 2 + 2.0 * nin * 2;
  for (int rep = 0; rep < 2; ++rep) {
    auto t = time(lib);
    printf("lib concat  median %.1f us min %.1f us  frac %.3f\n", t.first, t.second, bytes / t.first / 8e6);
    t = time(zeros);
    printf("zeros       median %.1f us min %.1f us  frac %.3f\n", t.first, t.second, bytes / t.first / 8e6);
    t = time(pow2);
    printf("pow2        median %.1f us min %.1f us  frac %.3f\n", t.first, t.second, bytes / t.first / 8e6);
  }
  lib();
  pow2();
  hipDeviceSynchronize();
  // compare a sample of the two outputs (every 4099th element)
  std::vector<uint16_t> s1(nout / 4099 + 1), s2(nout / 4099 + 1);
  size_t bad = 0;
  std::vector<uint16_t> c1(1 << 20), c2(1 << 20);
  for (size_t off = 0; off < nout; off += (size_t)97 << 20) {
    const size_t cnt = std::min<size_t>(1 << 20, nout - off);
    hipMemcpy(c1.data(), O1 + off, cnt * 2, hipMemcpyDeviceToHost);
    hipMemcpy(c2.data(), O2 + off, cnt * 2, hipMemcpyDeviceToHost);
    for (size_t i = 0; i < cnt; ++i) bad += c1[i] != c2[i];
  }
  printf("pow2 vs lib: %zu mismatches in sampled blocks; err=%s\n", bad, hipGetErrorString(hipGetLastError()));
  return 0;
}

// Diagnostic driver: per-role, per-phase s_memtime breakdown of the role-split band kernel
// (csrc/ip_rs.hip) on the cfg2 launch (8 pairs of 64 x 540 x 960 fp32, D = 192; arguments
// N C D H W MEAN WARM for other shapes), and the spread of the waves' finishing times per XCD.
//   hipcc -O3 -std=c++20 --offload-arch=gfx950 -DSMCV_RS_STAMPS -Iinclude scripts/rs_stamps.hip -o rs_stamps
// Stamps execute only in this build (never in libstereocv.so).
#include "../realtime_stereo_matcher_amd/csrc/common.hip"
#include "../realtime_stereo_matcher_amd/csrc/ip_rs.hip"

namespace smcv {
__device__ unsigned long long g_rs_stamps[4096][10];
}

#include <cstdio>
#include <cstring>
#include <vector>
#include <algorithm>

int main(int argc, char** argv) {
  const int64_t N = argc > 1 ? atoi(argv[1]) : 8, C = argc > 2 ? atoi(argv[2]) : 64,
                D = argc > 3 ? atoi(argv[3]) : 192, H = argc > 4 ? atoi(argv[4]) : 540,
                W = argc > 5 ? atoi(argv[5]) : 960;
  const bool mean = argc > 6 && atoi(argv[6]) != 0;
  const int warm = argc > 7 ? atoi(argv[7]) : 3;  // launches before the stamped one
  const size_t nin = N * C * H * W, nout = N * D * H * W;
  float *L, *R, *O;
  hipMalloc(&L, nin * 4);
  hipMalloc(&R, nin * 4);
  hipMalloc(&O, nout * 4);
  std::vector<float> h(nin);
  for (size_t i = 0; i < nin; ++i) h[i] = (float)((i * 2654435761u) % 2001) / 1000.f - 1.f;
  hipMemcpy(L, h.data(), nin * 4, hipMemcpyHostToDevice);
  hipMemcpy(R, h.data(), nin * 4, hipMemcpyHostToDevice);
  smcv::h2band::Args a{};
  a.L = L;
  a.R = R;
  a.out = O;
  a.C = a.cpg = (int)C;
  a.G = 1;
  a.H = (int)H;
  a.W = (int)W;
  a.D = (int)D;
  a.ls = {C * H * W, H * W, W};
  a.rs = a.ls;
  a.npass = (int)((D + 191) / 192);
  a.pw = (int)(((D + a.npass - 1) / a.npass + 3) / 4 * 4);
  a.mul = mean ? 1.0f / (float)C : 1.0f;
  bool handled = false;
  auto run = [&]() { return smcv::h2band::band_rs_run(a, N, mean, true, nullptr, &handled, 0); };
  for (int it = 0; it < warm; ++it) run();
  hipDeviceSynchronize();
  static unsigned long long st[4096][10];
  memset(st, 0, sizeof(st));
  hipMemcpyToSymbol(HIP_SYMBOL(smcv::g_rs_stamps), st, sizeof(st));
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  int rc = run();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  hipMemcpyFromSymbol(st, HIP_SYMBOL(smcv::g_rs_stamps), sizeof(st));
  const char* names[10] = {"C barrier", "C ring writes", "C frags+mfma", "C readout+stores", "C other",
                           "M barrier", "M load issue", "M staging (+load waits)", "M publish/drain",
                           "M other"};
  double sum[10] = {0};
  int nw[2] = {0, 0};
  for (int w = 0; w < 4096; ++w) {
    const int role = (w & 7) < 4 ? 0 : 1;
    unsigned long long t = 0;
    for (int p = 0; p < 10; ++p) t += st[w][p];
    if (!t) continue;
    ++nw[role];
    for (int p = 0; p < 10; ++p) sum[p] += st[w][p];
  }
  printf("band_rs rc=%d handled=%d: %.1f us after %d launches, waves C %d M %d\n", rc, (int)handled, ms * 1e3,
         warm, nw[0], nw[1]);
  for (int r = 0; r < 2; ++r) {
    double tt = 0;
    for (int p = 5 * r; p < 5 * r + 5; ++p) tt += sum[p];
    printf(" %s: %.0f cycles/wave\n", r ? "memory waves" : "compute waves", tt / (nw[r] ? nw[r] : 1));
    for (int p = 5 * r; p < 5 * r + 5; ++p)
      printf("  %-28s %10.0f cycles/wave %5.1f %%\n", names[p], sum[p] / (nw[r] ? nw[r] : 1), 100.0 * sum[p] / tt);
  }
  // finishing-time spread: a wave's stamps sum to its lifetime (the grid is resident at once)
  for (int r = 0; r < 2; ++r) {
    std::vector<double> all;
    double xmax[8] = {0}, xsum[8] = {0};
    int xn[8] = {0};
    for (int w = 0; w < 4096; ++w) {
      if (((w & 7) < 4 ? 0 : 1) != r) continue;
      unsigned long long t = 0;
      for (int p = 0; p < 10; ++p) t += st[w][p];
      if (!t) continue;
      all.push_back((double)t);
      const int x = (w >> 3) & 7;
      xmax[x] = std::max(xmax[x], (double)t);
      xsum[x] += (double)t;
      ++xn[x];
    }
    std::sort(all.begin(), all.end());
    if (all.empty()) continue;
    const size_t n = all.size();
    printf(" %s lifetime cycles: min %.0f p10 %.0f median %.0f p90 %.0f max %.0f (clock %.2f GHz: max / event time)\n",
           r ? "memory" : "compute", all[0], all[n / 10], all[n / 2], all[9 * n / 10], all[n - 1],
           all[n - 1] / (ms * 1e6));
    printf("  per XCD mean/max:");
    for (int x = 0; x < 8; ++x) printf(" %.0f/%.0f", xsum[x] / (xn[x] ? xn[x] : 1), xmax[x]);
    printf("\n");
  }
  return 0;
}

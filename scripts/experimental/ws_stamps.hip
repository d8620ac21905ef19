// Diagnostic driver: per-role phase stamps (s_memtime) of band_h2ws on the cfg2 shape (8 pairs,
// 1x64x540x960 fp32, D=192).  Build here, run on the GPU box:
//   hipcc -O3 -std=c++20 --offload-arch=gfx950 -DSMCV_STAMPS [-DSMCV_WS_ABL=N] -Iinclude \
//         scripts/ws_stamps.hip -o bin/stamps/ws_stamps && bin/stamps/ws_stamps
// Stamps execute only in this build (never in libstereocv.so).
#include "../realtime_stereo_matcher_amd/csrc/common.hip"
#include "../realtime_stereo_matcher_amd/csrc/cv_dot.hip"
#include "../realtime_stereo_matcher_amd/csrc/ip_h2.hip"
#include "../realtime_stereo_matcher_amd/csrc/ip_h2ws.hip"

namespace smcv {
namespace h2band {  // the other fp32 variants are not in this one-file build
int band_b16_run(const Args&, int64_t, bool, bool, hipStream_t, bool* handled) {
  *handled = false;
  return SM_OK;
}
int band_h2db_run(const Args&, int64_t, bool, bool, hipStream_t, bool* handled) {
  *handled = false;
  return SM_OK;
}
}  // namespace h2band
}  // namespace smcv

#ifdef SMCV_STAMPS
namespace smcv {
__device__ unsigned long long g_stamps[4096][kStampPhases];
}
#endif

#include <cstdio>
#include <cstring>
#include <vector>

int main() {
  const int64_t N = 8, C = 64, H = 540, W = 960, D = 192;
  const size_t nin = N * C * H * W, nout = N * D * H * W;
  void *L, *R, *O;
  hipMalloc(&L, nin * 4);
  hipMalloc(&R, nin * 4);
  hipMalloc(&O, nout * 4);
  std::vector<float> h(nin);
  for (size_t i = 0; i < nin; ++i) h[i] = (float)((i * 2654435761u) % 2001) / 1000.f - 1.f;
  hipMemcpy(L, h.data(), nin * 4, hipMemcpyHostToDevice);
  hipMemcpy(R, h.data(), nin * 4, hipMemcpyHostToDevice);
  bool handled = false;
  auto run = [&](int variant) {
    return smcv::band_h2_entry(L, R, O, SM_F32, N, C, H, W, D, nullptr, nullptr, 0, nullptr,
                               &handled, variant);
  };
  for (int it = 0; it < 3; ++it) run(3);
  hipDeviceSynchronize();
  static unsigned long long st[4096][smcv::kStampPhases];
  memset(st, 0, sizeof(st));
  hipMemcpyToSymbol(HIP_SYMBOL(smcv::g_stamps), st, sizeof(st));
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  const int rc = run(3);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  hipMemcpyFromSymbol(st, HIP_SYMBOL(smcv::g_stamps), sizeof(st));
  const char* ph[6] = {"work", "load wait", "step barrier", "segment end", "post-epilogue barrier",
                       "loop head"};
  const char* roles[3] = {"compute", "loader", "store"};
  printf("band_h2ws cfg2: %.1f us rc=%d handled=%d\n", ms * 1e3, rc, (int)handled);
  for (int r = 0; r < 3; ++r) {
    double sum[6] = {0}, tot = 0;
    int n = 0;
    for (int w = 0; w < 4096; ++w) {
      if ((w % 12) / 4 != r) continue;
      unsigned long long t = 0;
      for (int p = 0; p < 6; ++p) t += st[w][p];
      if (!t) continue;
      ++n;
      for (int p = 0; p < 6; ++p) sum[p] += st[w][p];
    }
    for (int p = 0; p < 6; ++p) tot += sum[p];
    printf("%s waves: %d, %.0f ticks/wave\n", roles[r], n, tot / (n ? n : 1));
    for (int p = 0; p < 6; ++p)
      printf("  %-24s %10.0f ticks/wave  %5.1f %%\n", ph[p], sum[p] / (n ? n : 1), tot ? 100.0 * sum[p] / tot : 0.0);
  }
  return 0;
}

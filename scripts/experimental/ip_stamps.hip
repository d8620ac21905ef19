// Diagnostic driver: per-phase s_memtime breakdown of the inner-product band kernel
// (cfg2 shape).  Build + run on the GPU box:
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DSMCV_STAMPS -Iinclude scripts/ip_stamps.hip -o /tmp/ip_stamps && /tmp/ip_stamps
// Stamps execute only in this build (never in libstereocv.so).
#include "../realtime_stereo_matcher_amd/csrc/common.hip"
#include "../realtime_stereo_matcher_amd/csrc/cv_dot.hip"
#include "../realtime_stereo_matcher_amd/csrc/ip_mfma.hip"
#include "../realtime_stereo_matcher_amd/csrc/ip_f32.hip"
#include "../realtime_stereo_matcher_amd/csrc/ip_h2.hip"
#include "../realtime_stereo_matcher_amd/csrc/ip_b16.hip"
#include "../realtime_stereo_matcher_amd/csrc/ip_h2db.hip"

#ifdef SMCV_STAMPS
namespace smcv {
__device__ unsigned long long g_stamps[4096][kStampPhases];
}
#endif

#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>

int main(int argc, char** argv) {
  // modes: bf16x3 (default), f32, h2 (inner product), fused (+ soft-argmin, volume kept),
  // fusednv (soft-argmin only), gw (groupwise bf16 cfg3: C=256, G=8, fp32 (N,G,H,W,D) out)
  const char* mode = argc > 2 ? argv[2] : "bf16x3";
  const bool gw = !strcmp(mode, "gw");
  const int64_t N = argc > 3 ? atoi(argv[3]) : 1, C = gw ? 256 : 64, H = 540, W = 960,
                D = argc > 1 ? atoi(argv[1]) : 192;
  const int64_t G = 8;
  const size_t nin = N * C * H * W, nout = gw ? N * G * H * W * D : N * D * H * W;
  const size_t esz = gw ? 2 : 4;
  void *L, *R;
  float *O, *disp;
  hipMalloc(&L, nin * esz);
  hipMalloc(&R, nin * esz);
  hipMalloc(&O, nout * 4);
  hipMalloc(&disp, N * H * W * 4);
  const bool f32 = !strcmp(mode, "f32");
  const bool b16 = !strcmp(mode, "b16"), db = !strcmp(mode, "h2db");
  const bool h2 = !strcmp(mode, "h2") || b16 || db;
  const bool fused = !strcmp(mode, "fused"), fusednv = !strcmp(mode, "fusednv");
  const bool band = h2 || fused || fusednv || gw;
  bool handled = false;
  auto run = [&]() {
    if (h2) return smcv::band_h2_entry(L, R, O, SM_F32, N, C, H, W, D, nullptr, nullptr, 0, nullptr, &handled, b16 ? 1 : db ? 2 : 0);
    if (fused || fusednv)
      return smcv::band_h2_fused_entry(L, R, fused ? O : nullptr, disp, SM_F32, N, C, H, W, D, nullptr,
                                       nullptr, 0, nullptr, &handled, nullptr, 0);
    if (gw)
      return smcv::band_h2_groupwise_entry(L, R, O, SM_BF16, N, C, H, W, D, G, nullptr, nullptr, nullptr,
                                           &handled);
    if (f32) return smcv::band_f32_entry(L, R, O, SM_F32, N, C, H, W, D, nullptr, nullptr, 0, nullptr, &handled);
    return smcv::band_mfma_entry(L, R, O, SM_F32, N, C, H, W, D, nullptr, nullptr, 0, nullptr);
  };
  std::vector<float> h(nin);
  for (size_t i = 0; i < nin; ++i) h[i] = (float)((i * 2654435761u) % 2001) / 1000.f - 1.f;
  if (gw) {
    std::vector<uint16_t> hb(nin);
    for (size_t i = 0; i < nin; ++i) {
      uint32_t u;
      memcpy(&u, &h[i], 4);
      hb[i] = (uint16_t)(u >> 16);
    }
    hipMemcpy(L, hb.data(), nin * 2, hipMemcpyHostToDevice);
    hipMemcpy(R, hb.data(), nin * 2, hipMemcpyHostToDevice);
  } else {
    hipMemcpy(L, h.data(), nin * 4, hipMemcpyHostToDevice);
    hipMemcpy(R, h.data(), nin * 4, hipMemcpyHostToDevice);
  }
  for (int it = 0; it < 3; ++it)
    run();
  hipDeviceSynchronize();
  static unsigned long long zero[4096][12];
  memset(zero, 0, sizeof(zero));
#ifdef SMCV_STAMPS
  hipMemcpyToSymbol(HIP_SYMBOL(smcv::g_stamps), zero, sizeof(zero));
#endif
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  int rc = run();
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  static unsigned long long st[4096][12];
#ifdef SMCV_STAMPS
  hipMemcpyFromSymbol(st, HIP_SYMBOL(smcv::g_stamps), sizeof(st));
#else
  memset(st, 0, sizeof(st));
#endif
  const char* names[12] = {"top barrier", "stage (split+lds)", "stage barrier", "mfma",
                           "epi barrier 1", "shear writes", "epi barrier 2", "store loop",
                           "stage: dma wait", "dma issue", "-", "-"};
  if (band) {
    const char* hn[12] = {"barrier waits", "wait+stage (split, lds write)", "load+touch issue",
                          "frags+mfma", "epilogue (shear, ring, stores)", "vm_wait step 0",
                          "vm_wait step 1", "vm_wait steps 2+", "-", "-", "-", "-"};
    double sm[12] = {0};
    int n = 0;
    for (int w = 0; w < 4096; ++w) {
      unsigned long long t = 0;
      for (int p = 0; p < 12; ++p) t += st[w][p];
      if (!t) continue;
      ++n;
      for (int p = 0; p < 12; ++p) sm[p] += st[w][p];
    }
    double tt = 0;
    for (int p = 0; p < 12; ++p) tt += sm[p];
    printf("kernel %s %.1f us rc=%d, waves: %d, %.0f cycles/wave\n", mode, ms * 1e3, rc, n, tt / (n ? n : 1));
    for (int p = 0; p < 12; ++p)
      if (sm[p] > 0) printf("  %-30s %10.0f cycles/wave  %5.1f %%\n", hn[p], sm[p] / n, 100.0 * sm[p] / tt);
    return 0;
  }
  printf("kernel: %s\n", f32 ? "f32 band" : "bf16x3 band");
  double sum[12] = {0};
  int nw = 0;
  for (int w = 0; w < 4096; ++w) {
    unsigned long long t = 0;
    for (int p = 0; p < 12; ++p) t += st[w][p];
    if (!t) continue;
    ++nw;
    for (int p = 0; p < 12; ++p) sum[p] += st[w][p];
  }
  double tot = 0;
  for (int p = 0; p < 12; ++p) tot += sum[p];
  printf("rc=%d kernel %.1f us, %d waves with stamps\n", rc, ms * 1e3, nw);
  for (int p = 0; p < 10; ++p)
    printf("  %-26s %10.0f cycles/wave  %5.1f %%\n", names[p], sum[p] / nw, 100.0 * sum[p] / tot);
  printf("  total %.0f cycles/wave\n", tot / nw);
  return 0;
}

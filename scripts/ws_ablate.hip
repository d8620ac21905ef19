// Diagnostic driver: median kernel time (HIP events) of one band-kernel launch on the cfg2 shape
// (1x64x540x960 fp32, D=192) for ablation builds of csrc/ip_ws.hip.  Build + run on the GPU box:
//   hipcc -O3 -std=c++20 --offload-arch=gfx950 -DSMCV_ABLATE=N -Iinclude scripts/ws_ablate.hip -o /tmp/wsa && /tmp/wsa [mode]
// modes: ws (default), wsfused, wsfusednv, wsgw (cfg3 bf16 groupwise), h2, h2fused, h2fusednv, h2gw (cfg3), h2corr4 (cfg4 one pair)
#include "../realtime_stereo_matcher_amd/csrc/common.hip"
#include "../realtime_stereo_matcher_amd/csrc/cv_dot.hip"
#include "../realtime_stereo_matcher_amd/csrc/ip_h2.hip"
#include "../realtime_stereo_matcher_amd/csrc/ip_ws.hip"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "ws";
  const bool gw = !strcmp(mode, "wsgw") || !strcmp(mode, "h2gw");
  const bool c4 = !strcmp(mode, "h2corr4");  // cfg4: 1x16x1080x1920 fp32, correlation D=256
  const bool x8 = !strcmp(mode, "h2x8");  // cfg2, 8 pairs per launch (the bench's chunk)
  const int64_t N = x8 ? 8 : 1, C = gw ? 256 : c4 ? 16 : 64, H = c4 ? 1080 : 540, W = c4 ? 1920 : 960,
                D = c4 ? 256 : 192, G = 8;
  const size_t nin = N * C * H * W, nout = gw ? N * G * H * W * D : N * D * H * W;
  const size_t esz = gw ? 2 : 4;
  void *L, *R;
  float *O, *disp;
  hipMalloc(&L, nin * esz);
  hipMalloc(&R, nin * esz);
  hipMalloc(&O, nout * 4);
  hipMalloc(&disp, N * H * W * 4);
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
  bool handled = false;
  auto run = [&]() {
    if (!strcmp(mode, "h2gw"))
      return smcv::band_h2_groupwise_entry(L, R, O, SM_BF16, N, C, H, W, D, G, nullptr, nullptr, nullptr, &handled);
    if (c4) return smcv::band_h2_entry(L, R, O, SM_F32, N, C, H, W, D, nullptr, nullptr, 1, nullptr, &handled);
    if (!strcmp(mode, "h2") || x8) return smcv::band_h2_entry(L, R, O, SM_F32, N, C, H, W, D, nullptr, nullptr, 0, nullptr, &handled);
    if (!strcmp(mode, "h2fused") || !strcmp(mode, "h2fusednv"))
      return smcv::band_h2_fused_entry(L, R, !strcmp(mode, "h2fused") ? O : nullptr, disp, SM_F32, N, C, H, W, D,
                                       nullptr, nullptr, 0, nullptr, &handled, nullptr, 0);
    if (!strcmp(mode, "wsfused") || !strcmp(mode, "wsfusednv"))
      return smcv::band_ws_fused_entry(L, R, !strcmp(mode, "wsfused") ? O : nullptr, disp, SM_F32, N, C, H, W, D,
                                       nullptr, nullptr, 0, nullptr, &handled);
    if (gw)
      return smcv::band_ws_groupwise_entry(L, R, O, SM_BF16, N, C, H, W, D, G, nullptr, nullptr, nullptr, &handled);
    return smcv::band_ws_entry(L, R, O, SM_F32, N, C, H, W, D, nullptr, nullptr, 0, nullptr, &handled);
  };
  for (int it = 0; it < 3; ++it) run();
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  std::vector<float> ts;
  int rc = 0;
  for (int it = 0; it < 25; ++it) {
    hipEventRecord(a);
    rc |= run();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    ts.push_back(ms * 1e3f);
  }
  std::sort(ts.begin(), ts.end());
  printf("%-10s ablate=%-3d median %.1f us  min %.1f us  rc=%d err=%s\n", mode, SMCV_ABLATE, ts[ts.size() / 2], ts[0], rc,
         hipGetErrorString(hipGetLastError()));
  return 0;
}

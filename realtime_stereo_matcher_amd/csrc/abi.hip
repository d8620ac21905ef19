// extern "C" entry points of libstereocv.so (declared in include/stereocv.h).
#include "common.h"

namespace smcv {
int dot_volume_valu_entry(const void* left, const void* right, void* out, int dtype, int64_t N,
                          int64_t C, int64_t H, int64_t W, int64_t D, int64_t G,
                          const int64_t* l_strides, const int64_t* r_strides, int mode,
                          void* stream);
int band_f32_entry(const void* left, const void* right, void* out, int dtype, int64_t N,
                   int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                   const int64_t* r_strides, int mode, void* stream, bool* handled);
int band_h2_entry(const void* left, const void* right, void* out, int dtype, int64_t N, int64_t C,
                  int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                  const int64_t* r_strides, int mode, void* stream, bool* handled,
                  int variant);
int band_h2_groupwise_entry(const void* left, const void* right, float* out, int dtype, int64_t N,
                            int64_t C, int64_t H, int64_t W, int64_t D, int64_t G,
                            const int64_t* l_strides, const int64_t* r_strides, void* stream,
                            bool* handled);
int band_h2_fused_entry(const void* left, const void* right, void* out, float* disp, int dtype,
                        int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                        const int64_t* l_strides, const int64_t* r_strides, int mode,
                        void* stream, bool* handled, void* workspace, int64_t ws_bytes);
int64_t band_h2_fused_workspace_bytes(int64_t N, int64_t H, int64_t W, int64_t D);
size_t v4_workspace_bytes(int64_t N, int64_t H, int64_t W);
int v4_volume_entry(const float* L, const float* R, float* out, int64_t N, int64_t C, int64_t H,
                    int64_t W, int64_t D, const int64_t* l_strides, const int64_t* r_strides,
                    const float* w1, const float* b1, const float* w2, const float* b2,
                    const float* w3, const float* b3, const float* w4, const float* b4,
                    void* workspace, size_t workspace_bytes, hipStream_t st);
int concat_entry(const void* left, const void* right, void* out, int dtype, int64_t N,
                 int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                 const int64_t* r_strides, void* stream);
int interweave_entry(const void* left, const void* right, void* out, int dtype, int64_t N,
                     int64_t C, int64_t H, int64_t W, const int64_t* l_strides,
                     const int64_t* r_strides, void* stream);
int shifted_entry(const void* left, const void* right, void* out, int dtype, int64_t N,
                  int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                  const int64_t* r_strides, int mode, void* stream);
int softargmin_entry(const void* volume, void* out, int dtype, int64_t N, int64_t D, int64_t H,
                     int64_t W, int flags, const int64_t* vol_strides, void* stream);
int argext_entry(const void* volume, int64_t* out, int dtype, int64_t N, int64_t D, int64_t H,
                 int64_t W, int mode, const int64_t* vol_strides, void* stream);
int warp_entry(const void* image, const void* flow, void* out, int dtype, int64_t N, int64_t C,
               int64_t Hi, int64_t Wi, int64_t H, int64_t W, int64_t flow_channels,
               const int64_t* image_strides, const int64_t* flow_strides, void* stream,
               void* workspace, int64_t workspace_bytes);
int64_t warp_workspace_bytes(int64_t N, int64_t C, int64_t Hi, int64_t Wi, int64_t flow_channels);
}  // namespace smcv

using namespace smcv;

#ifndef SMCV_AUTO_SL
// AUTO's volume kernel for the shapes both take: the role-split band (0) or the sliding-window
// band (1).  The volume is bound by how HBM takes its mixed read + write stream.  band_rs reads
// each segment's 192-column right window again (from L2: the counted traffic stays 1.0x), and
// those re-reads of lines a neighbouring workgroup is fetching cost 540 us of a 32-pair cfg2
// launch's read stream (scripts/micro/mem_shapes.hip: 1,964 vs 1,422 us); band_sl reads every
// feature column once.  Round 5's band_sl walked rows strided over the whole grid and lost on the
// write stream; with each XCD on a contiguous eighth of the rows (SMCV_SL_MAP 1) it is the faster
// kernel: cfg2 32 pairs 3,642-3,672 vs 3,847-3,870 us, cfg4 11,988-12,045 vs 12,375-12,448 us,
// same process and buffers (profiles/r06/ab/), and equal on a slowly mapped volume buffer
#define SMCV_AUTO_SL 1
#endif
namespace {
// band_h2_entry's kernel choice for an algo: 6 band_sl, 5 band_rs, 2 band_h2db, 0 band_h2
int algo_variant(int algo) {
  switch (algo) {
    case SM_IP_AUTO: return SMCV_AUTO_SL ? 6 : 5;
    case SM_IP_MFMA_SL: return 6;
    case SM_IP_MFMA_RS: return 5;
    case SM_IP_MFMA_H2DB: return 2;
    default: return 0;
  }
}
}  // namespace

#define SM_ENTRY_BEGIN last_error().clear();

extern "C" int sm_cv_inner_product_ex(const void* left, const void* right, void* out, int dtype,
                                      int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                                      const int64_t* l_strides, const int64_t* r_strides,
                                      int algo, void* stream) {
  SM_ENTRY_BEGIN
  if (dtype == SM_F64) {  // fp64 features: fp64 products and sums whatever the algo (f64.hip)
    if (algo != SM_IP_AUTO && algo != SM_IP_VALU && algo != SM_IP_MFMA_F32 && algo != SM_IP_MFMA_H2 &&
        algo != SM_IP_MFMA_H2DB && algo != SM_IP_MFMA_RS && algo != SM_IP_MFMA_SL)
      return fail(SM_EINVAL, "unknown inner-product algo");
    return dot_volume_valu_entry(left, right, out, dtype, N, C, H, W, D, 1, l_strides, r_strides,
                                 0, stream);
  }
  switch (algo) {
    case SM_IP_MFMA_F32: {
      // exact fp32 MFMA band kernel; shapes the DMA path cannot take go to the VALU kernel
      bool handled = false;
      int rc = band_f32_entry(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, 0,
                              stream, &handled);
      if (handled || rc != SM_OK) return rc;
      return dot_volume_valu_entry(left, right, out, dtype, N, C, H, W, D, 1, l_strides,
                                   r_strides, 0, stream);
    }
    case SM_IP_AUTO:  // the two-plane fp16 band kernel; odd shapes: the exact VALU kernel
    case SM_IP_MFMA_H2:
    case SM_IP_MFMA_H2DB:
    case SM_IP_MFMA_RS:
    case SM_IP_MFMA_SL: {
      bool handled = false;
      // AUTO / SL: fp32 aligned rows with C = 16 or 64 and 65..192 disparities per pass (and
      // C = 16 with two passes of <= 128) take the sliding-window band (band_sl); RS: the
      // role-split band (band_rs); shapes they do not take: the double-buffered band (band_h2db)
      // for fp32 aligned rows, band_h2 for the rest
      const int variant = algo_variant(algo);
      int rc = band_h2_entry(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, 0,
                             stream, &handled, variant);
      if (handled || rc != SM_OK) return rc;
      return dot_volume_valu_entry(left, right, out, dtype, N, C, H, W, D, 1, l_strides,
                                   r_strides, 0, stream);
    }
    case SM_IP_VALU:
      return dot_volume_valu_entry(left, right, out, dtype, N, C, H, W, D, 1, l_strides,
                                   r_strides, 0, stream);
    default:
      return fail(SM_EINVAL, "unknown inner-product algo");
  }
}

extern "C" int sm_cv_inner_product(const void* left, const void* right, void* out, int dtype,
                                   int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                                   const int64_t* l_strides, const int64_t* r_strides,
                                   void* stream) {
  return sm_cv_inner_product_ex(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides,
                                SM_IP_AUTO, stream);
}

extern "C" int sm_cv_correlation_mean_ex(const void* left, const void* right, void* out,
                                         int dtype, int64_t N, int64_t C, int64_t H, int64_t W,
                                         int64_t D, const int64_t* l_strides,
                                         const int64_t* r_strides, int algo, void* stream) {
  SM_ENTRY_BEGIN
  bool handled = false;
  int rc = SM_OK;
  if (dtype == SM_F64) algo = SM_IP_VALU;  // fp64: the fp64 kernel below (f64.hip)
  switch (algo) {
    case SM_IP_MFMA_F32:
      rc = band_f32_entry(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, 1,
                          stream, &handled);
      break;
    case SM_IP_AUTO:
    case SM_IP_MFMA_H2:
    case SM_IP_MFMA_H2DB:
    case SM_IP_MFMA_RS:
    case SM_IP_MFMA_SL: {
      const int variant = algo_variant(algo);
      rc = band_h2_entry(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, 1, stream,
                         &handled, variant);
      break;
    }
    case SM_IP_VALU:
      break;
    default:
      return fail(SM_EINVAL, "unknown inner-product algo");
  }
  if (handled || rc != SM_OK) return rc;
  return dot_volume_valu_entry(left, right, out, dtype, N, C, H, W, D, 1, l_strides, r_strides,
                               1, stream);
}

extern "C" int sm_cv_correlation_mean(const void* left, const void* right, void* out, int dtype,
                                      int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                                      const int64_t* l_strides, const int64_t* r_strides,
                                      void* stream) {
  return sm_cv_correlation_mean_ex(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides,
                                   SM_IP_AUTO, stream);
}

extern "C" int sm_cv_groupwise(const void* left, const void* right, float* out, int dtype,
                               int64_t N, int64_t C, int64_t H, int64_t W, int64_t D, int64_t G,
                               const int64_t* l_strides, const int64_t* r_strides,
                               void* stream) {
  SM_ENTRY_BEGIN
  if (dtype == SM_F64)  // fp64 means rounded once into the float32 volume (f64.hip)
    return dot_volume_valu_entry(left, right, out, dtype, N, C, H, W, D, G, l_strides, r_strides,
                                 2, stream);
  // the MFMA band kernel (D-innermost epilogue); shapes it does not take: the VALU kernel
  bool handled = false;
  int rc = band_h2_groupwise_entry(left, right, out, dtype, N, C, H, W, D, G, l_strides,
                                   r_strides, stream, &handled);
  if (handled || rc != SM_OK) return rc;
  return dot_volume_valu_entry(left, right, out, dtype, N, C, H, W, D, G, l_strides, r_strides,
                               2, stream);
}

namespace {
int fused_softargmin(const void* left, const void* right, void* out_volume, void* disparity,
                     int dtype, int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                     const int64_t* l_strides, const int64_t* r_strides, int mode,
                     void* workspace, int64_t ws_bytes, void* stream) {
  if ((mode & ~(1 | SM_FUSED_DISP_F32 | SM_FUSED_EXACT_ACC)) != 0)
    return fail(SM_EINVAL,
                "mode must be 0 (sum) or 1 (mean), optionally | SM_FUSED_DISP_F32 | SM_FUSED_EXACT_ACC");
  const bool f32disp = (mode & SM_FUSED_DISP_F32) != 0;
  if (!valid_dtype(dtype) && dtype != SM_F64) return fail(SM_EDTYPE, "unsupported dtype code");
  if (ws_bytes < 0) return fail(SM_EINVAL, "negative workspace size");
  if (D == 0 && N * H * W > 0) {  // softmax over an empty axis: the weighted sum is 0
    if (disparity == nullptr) return fail(SM_EINVAL, "null disparity pointer");
    const hipError_t e = hipMemsetAsync(disparity, 0,
                                        (size_t)(N * H * W) * (f32disp ? 4 : elem_size(dtype)),
                                        as_stream(stream));
    return e == hipSuccess ? SM_OK : fail(SM_ELAUNCH, hipGetErrorString(e));
  }
  bool handled = false;
  int rc = SM_OK;
  if (dtype != SM_F64) {  // fp64: the volume and the fp64 regression below
    rc = band_h2_fused_entry(left, right, out_volume, static_cast<float*>(disparity), dtype, N, C,
                             H, W, D, l_strides, r_strides, mode, stream, &handled, workspace,
                             ws_bytes);
    if (handled || rc != SM_OK) return rc;
  }
  if (out_volume == nullptr)
    return fail(SM_EUNSUPPORTED,
                "fused cost volume + soft-argmin needs fp32 features (W >= 4) and D <= 192, or a "
                "workspace of sm_cv_inner_product_softargmin_workspace_bytes() for D > 192; pass "
                "a volume buffer for the two-kernel path");
  rc = (mode & 1) ? sm_cv_correlation_mean(left, right, out_volume, dtype, N, C, H, W, D,
                                            l_strides, r_strides, stream)
                   : sm_cv_inner_product(left, right, out_volume, dtype, N, C, H, W, D, l_strides,
                                         r_strides, stream);
  if (rc != SM_OK) return rc;
  return softargmin_entry(out_volume, disparity, dtype, N, D, H, W,
                          SM_REGRESS_SOFTMAX | (f32disp ? SM_REGRESS_OUT_F32 : 0), nullptr, stream);
}
}  // namespace

extern "C" int sm_cv_inner_product_softargmin(const void* left, const void* right,
                                              void* out_volume, void* disparity, int dtype,
                                              int64_t N, int64_t C, int64_t H, int64_t W,
                                              int64_t D, const int64_t* l_strides,
                                              const int64_t* r_strides, int mode, void* stream) {
  SM_ENTRY_BEGIN
  return fused_softargmin(left, right, out_volume, disparity, dtype, N, C, H, W, D, l_strides,
                          r_strides, mode, nullptr, 0, stream);
}

extern "C" int64_t sm_cv_inner_product_softargmin_workspace_bytes(int64_t N, int64_t H, int64_t W,
                                                                  int64_t D) {
  if (N < 0 || H < 0 || W < 0 || D < 0) return 0;
  return band_h2_fused_workspace_bytes(N, H, W, D);
}

extern "C" int sm_cv_inner_product_softargmin_ws(const void* left, const void* right,
                                                 void* out_volume, void* disparity, int dtype,
                                                 int64_t N, int64_t C, int64_t H, int64_t W,
                                                 int64_t D, const int64_t* l_strides,
                                                 const int64_t* r_strides, int mode,
                                                 void* workspace, int64_t workspace_bytes,
                                                 void* stream) {
  SM_ENTRY_BEGIN
  return fused_softargmin(left, right, out_volume, disparity, dtype, N, C, H, W, D, l_strides,
                          r_strides, mode, workspace, workspace_bytes, stream);
}

extern "C" int sm_cv_concat(const void* left, const void* right, void* out, int dtype, int64_t N,
                            int64_t C, int64_t H, int64_t W, int64_t D,
                            const int64_t* l_strides, const int64_t* r_strides, void* stream) {
  SM_ENTRY_BEGIN
  return concat_entry(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, stream);
}

extern "C" int sm_cv_interweave(const void* left, const void* right, void* out, int dtype,
                                int64_t N, int64_t C, int64_t H, int64_t W,
                                const int64_t* l_strides, const int64_t* r_strides,
                                void* stream) {
  SM_ENTRY_BEGIN
  return interweave_entry(left, right, out, dtype, N, C, H, W, l_strides, r_strides, stream);
}

extern "C" int sm_cv_interweave_shifted(const void* left, const void* right, void* out,
                                        int dtype, int64_t N, int64_t C, int64_t H, int64_t W,
                                        int64_t D, const int64_t* l_strides,
                                        const int64_t* r_strides, void* stream) {
  SM_ENTRY_BEGIN
  return shifted_entry(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, 0, stream);
}

extern "C" int sm_cv_diff(const void* left, const void* right, void* out, int dtype, int64_t N,
                          int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                          const int64_t* r_strides, void* stream) {
  SM_ENTRY_BEGIN
  return shifted_entry(left, right, out, dtype, N, C, H, W, D, l_strides, r_strides, 1, stream);
}

extern "C" int sm_regress_softargmin(const void* volume, void* out, int dtype, int64_t N,
                                     int64_t D, int64_t H, int64_t W, int flags,
                                     const int64_t* vol_strides, void* stream) {
  SM_ENTRY_BEGIN
  return softargmin_entry(volume, out, dtype, N, D, H, W, flags, vol_strides, stream);
}

extern "C" int sm_regress_argext(const void* volume, int64_t* out, int dtype, int64_t N,
                                 int64_t D, int64_t H, int64_t W, int mode,
                                 const int64_t* vol_strides, void* stream) {
  SM_ENTRY_BEGIN
  return argext_entry(volume, out, dtype, N, D, H, W, mode, vol_strides, stream);
}

extern "C" int sm_warp_by_flow(const void* image, const void* flow, void* out, int dtype,
                               int64_t N, int64_t C, int64_t Hi, int64_t Wi, int64_t H, int64_t W,
                               int64_t flow_channels, const int64_t* image_strides,
                               const int64_t* flow_strides, void* stream) {
  SM_ENTRY_BEGIN
  return warp_entry(image, flow, out, dtype, N, C, Hi, Wi, H, W, flow_channels, image_strides,
                    flow_strides, stream, nullptr, 0);
}

extern "C" int64_t sm_warp_by_flow_workspace_bytes(int64_t N, int64_t C, int64_t Hi, int64_t Wi,
                                                   int64_t flow_channels) {
  return warp_workspace_bytes(N, C, Hi, Wi, flow_channels);
}

extern "C" int sm_warp_by_flow_ws(const void* image, const void* flow, void* out, int dtype,
                                  int64_t N, int64_t C, int64_t Hi, int64_t Wi, int64_t H, int64_t W,
                                  int64_t flow_channels, const int64_t* image_strides,
                                  const int64_t* flow_strides, void* workspace,
                                  int64_t workspace_bytes, void* stream) {
  SM_ENTRY_BEGIN
  if (workspace_bytes < 0) return fail(SM_EINVAL, "warp_by_flow_map: negative workspace size");
  return warp_entry(image, flow, out, dtype, N, C, Hi, Wi, H, W, flow_channels, image_strides,
                    flow_strides, stream, workspace, workspace_bytes);
}

extern "C" int64_t sm_v4_volume_workspace_bytes(int64_t N, int64_t H, int64_t W) {
  if (N < 0 || H < 0 || W < 0) return -1;
  return (int64_t)v4_workspace_bytes(N, H, W);
}

extern "C" int sm_v4_volume(const void* featL, const void* featR, void* out, int dtype, int64_t N,
                            int64_t C, int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                            const int64_t* r_strides, const float* w1, const float* b1,
                            const float* w2, const float* b2, const float* w3, const float* b3,
                            const float* w4, const float* b4, void* workspace,
                            int64_t workspace_bytes, void* stream) {
  SM_ENTRY_BEGIN
  if (dtype != SM_F32) return fail(SM_EDTYPE, "v4_volume: float32 features only");
  if (workspace_bytes < 0) return fail(SM_EINVAL, "v4_volume: negative workspace size");
  return v4_volume_entry(static_cast<const float*>(featL), static_cast<const float*>(featR),
                         static_cast<float*>(out), N, C, H, W, D, l_strides, r_strides, w1, b1, w2,
                         b2, w3, b3, w4, b4, workspace, (size_t)workspace_bytes, as_stream(stream));
}

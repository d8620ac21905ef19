/*
 * stereocv.h -- C ABI of libstereocv.so, the MI355X (gfx950) stereo cost-volume and
 * disparity-regression engine.
 *
 * Every entry point replaces one operator of babiking/realtime_stereo_matcher's hot
 * path (file:line cited per function).  Conventions shared by all entry points:
 *
 *   - Pointers are DEVICE pointers (HIP).  The library never allocates, frees or
 *     synchronises caller memory; all work is enqueued on `stream` (a hipStream_t
 *     passed as void*, NULL = the null stream) and is stream-ordered.  No host sync;
 *     the only state besides the thread-local error string is a per-device cache
 *     (atomics) of the CU count and of the kernels whose LDS limit was raised.
 *   - Feature maps are 4-D (N, C, H, W).  `l_strides` / `r_strides` give the element
 *     strides of (N, C, H, W); the W stride must be 1 (the caller makes rows
 *     contiguous).  NULL strides mean contiguous.
 *   - Outputs are dense, contiguous, in the layout stated per function.
 *   - dtype codes: SM_F32, SM_F16, SM_BF16 (the output dtype equals the input dtype
 *     unless the function says otherwise).  Accumulation is always fp32 or wider.
 *     SM_F64 (round 6): the cost volumes (a-1 .. a-6, computed in fp64; groupwise into its
 *     float32 volume), the regressions (a-7, a-8, fp64 arithmetic) and the fused call's
 *     two-kernel path, as torch computes an fp64 input; the warp and the V4 volume are float32
 *     only (SM_EDTYPE).
 *   - Return 0 on success, a negative SM_E* code on failure; sm_last_error() then
 *     returns a thread-local, human-readable message.
 */
#ifndef STEREOCV_H_
#define STEREOCV_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum sm_dtype { SM_F32 = 0, SM_F16 = 1, SM_BF16 = 2, SM_F64 = 3 };
enum sm_status {
  SM_OK = 0,
  SM_EINVAL = -1,
  SM_EDTYPE = -2,
  SM_ELAUNCH = -3,
  SM_EUNSUPPORTED = -4 /* sm_cv_inner_product_softargmin without a volume: shape not fused */
};
enum sm_argext_mode { SM_ARGMIN = 0, SM_ARGMAX = 1 };
/* sm_cv_inner_product_softargmin*: mode = 0 (sum) or 1 (mean), optionally OR'd with */
enum sm_fused_flags {
  SM_FUSED_DISP_F32 = 2, /* the disparity is float32 whatever the feature dtype: the reference's
                            autocast eval, where the volume keeps the fp16 / bf16 feature dtype and
                            F.softmax + torch.sum run in fp32 (evaluate_stereo.py:48,
                            mobile_disp_net_c.py:208-220); fp16 / bf16 features then take the
                            fused band kernel too, which regresses each cell rounded to the
                            feature dtype -- the volume the reference's two calls regress */
  SM_FUSED_EXACT_ACC = 4 /* with SM_FUSED_DISP_F32 and fp16 / bf16 features: regress the fp32
                            accumulators of the exact products instead (no rounding to the
                            feature dtype; shapes the fused kernel does not take still regress
                            the rounded volume) */
};
enum sm_regress_flags {         /* bit flags */
  SM_REGRESS_SOFTMAX = 0,      /* softmax over D inside (mobile_disp_net_c.py:208-220) */
  SM_REGRESS_PRESOFTMAXED = 1, /* input already softmaxed (mobile_stereo_net_v4.py:10-14) */
  SM_REGRESS_OUT_F32 = 2       /* fp32 output from an fp16 / bf16 volume: the reference's autocast
                                  eval, where F.softmax and torch.sum run in fp32
                                  (mobile_stereo_net.py:144-147 under evaluate_stereo.py:48) */
};
/* Inner-product kernel selection (sm_cv_inner_product_ex). */
enum sm_ip_algo {
  SM_IP_AUTO = 0,        /* library default for the shape/dtype */
  SM_IP_VALU = 1,        /* fp32 VALU, LDS-staged right window reused across the D sweep */
  SM_IP_MFMA_F32 = 2,    /* banded C-contraction on v_mfma_f32_16x16x4_f32 (exact fp32 fma) */
  /* 3: reserved (the bf16 3-way split kernel, retired in round 4: slower than MFMA_H2) */
  /* 4: reserved (a retired warp-specialised variant of the bf16 split) */
  SM_IP_MFMA_H2 = 5,     /* banded contraction on 32x32x16 MFMA, two workgroups per CU, every wave
                            loads, stages, multiplies and stores (the default for fp16 / bf16
                            features and for fp32 rows that are not 4-element aligned) */
  /* 6: reserved (a retired warp-specialised variant, removed in round 3) */
  /* 7: reserved (16-pixel waves on 16x16x32 MFMA, retired in round 4: slower than MFMA_H2DB) */
  SM_IP_MFMA_H2DB = 8,   /* MFMA_H2 with double-buffered planes: the next step is staged inside
                            the current step's MFMA phase (fp32, aligned rows; else MFMA_H2; the
                            fallback of MFMA_SP, MFMA_RS and AUTO) */
  /* 9: reserved (store waves fed through an LDS queue, retired in round 4: slower) */
  /* 10: reserved (one-wave-per-SIMD software-pipelined band, retired in round 5: slower than
         MFMA_RS; source under scripts/experimental/) */
  SM_IP_MFMA_RS = 11,    /* role-split band kernel: per SIMD a compute wave (MFMAs, shear ring,
                            volume stores) and a memory wave (feature loads and staging); fp32,
                            aligned rows, C = 16 or 64, D in 65..192 per pass; other shapes:
                            MFMA_H2DB.  AUTO's volume kernel in rounds 4-5; since round 6 AUTO
                            takes MFMA_SL, and MFMA_RS keeps the groupwise 16-bit volumes */
  SM_IP_MFMA_SL = 12     /* sliding-window role-split band kernel: a workgroup walks whole rows
                            and keeps the right window of all channels in LDS, so a 128-pixel
                            segment stages only its own 128 left and 128 new right columns;
                            shapes of MFMA_RS plus (C = 16) two passes of <= 128 disparities
                            (D = 256); others: MFMA_H2DB.  Each XCD walks a contiguous eighth of
                            the rows.  AUTO's volume kernel for fp32 features since round 6, and
                            the fused volume + soft-argmin calls (sm_cv_inner_product_softargmin*)
                            take it for fp32 features */
};

/* Library version (major*10000 + minor*100 + patch). */
int sm_version(void);
/* Thread-local message for the last failing call on this thread ("" if none). */
const char* sm_last_error(void);

/* a-1: TorchInnerProductCost(max_disparity)(left, right)
 *      -- cost_volume/inner_product.py:11-42
 * out[n,d,y,x] = sum_c L[n,c,y,x] * R[n,c,y,x-d] (x >= d), 0 (x < d).
 * out: (N, D, H, W), dtype = dtype. */
int sm_cv_inner_product(const void* left, const void* right, void* out, int dtype,
                        int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                        const int64_t* l_strides, const int64_t* r_strides, void* stream);
/* Same with an explicit kernel choice (enum sm_ip_algo). */
int sm_cv_inner_product_ex(const void* left, const void* right, void* out, int dtype,
                           int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                           const int64_t* l_strides, const int64_t* r_strides, int algo,
                           void* stream);

/* a-6: make_correlation_volume(l_fmap, r_fmap, max_disp)
 *      -- model/mobile_disp_net_c.py:188-205
 * out[n,d,y,x] = mean_c L*R(x-d) (x >= d), 0 (x < d).  out: (N, D, H, W). */
int sm_cv_correlation_mean(const void* left, const void* right, void* out, int dtype,
                           int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                           const int64_t* l_strides, const int64_t* r_strides, void* stream);
/* sm_cv_correlation_mean with an explicit kernel (enum sm_ip_algo; AUTO is the plain call). */
int sm_cv_correlation_mean_ex(const void* left, const void* right, void* out, int dtype,
                              int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                              const int64_t* l_strides, const int64_t* r_strides, int algo,
                              void* stream);

/* f-1: cost volume + soft-argmin regression in one pass.
 *   mode 0: TorchInnerProductCost -- cost_volume/inner_product.py:11-42; mode 1:
 *   make_correlation_volume -- model/mobile_disp_net_c.py:188-205; each followed by
 *   disparity_regression -- model/mobile_disp_net_c.py:208-220 (= the inline soft-argmin of
 *   model/mobile_stereo_net.py:144-147).
 * disparity[n,y,x] = sum_d d * softmax_d(vol[n,:,y,x]): (N, H, W) in `dtype` (float32 with
 * mode | SM_FUSED_DISP_F32); the (N, D, H, W) volume (in `dtype`) is written too when
 * out_volume != NULL.  fp32 features (W >= 4) with D <= 192 take the fused band kernel, and so
 * do fp16 / bf16 features (4-element aligned rows) with SM_FUSED_DISP_F32 (the volume is never
 * read back; with out_volume == NULL it is never written).  Other shapes run the volume and the regression as
 * two kernels, which needs out_volume: with out_volume == NULL they return SM_EUNSUPPORTED.
 * D == 0: the disparity is 0 (an empty softmax axis). */
int sm_cv_inner_product_softargmin(const void* left, const void* right, void* out_volume,
                                   void* disparity, int dtype, int64_t N, int64_t C, int64_t H,
                                   int64_t W, int64_t D, const int64_t* l_strides,
                                   const int64_t* r_strides, int mode, void* stream);

/* f-1 for D > 192 without the volume (e.g. make_correlation_volume followed by
 * disparity_regression at D = 256, model/mobile_disp_net_c.py:188-220): the band kernel runs D in
 * passes of <= 192 disparities, each pass writes its partial softmax state per pixel into a
 * caller-provided device workspace (8-byte aligned, at least
 * sm_cv_inner_product_softargmin_workspace_bytes(N, H, W, D) bytes; 0 for D <= 192) and a
 * second kernel merges them.  Otherwise as sm_cv_inner_product_softargmin. */
int64_t sm_cv_inner_product_softargmin_workspace_bytes(int64_t N, int64_t H, int64_t W, int64_t D);
int sm_cv_inner_product_softargmin_ws(const void* left, const void* right, void* out_volume,
                                      void* disparity, int dtype, int64_t N, int64_t C,
                                      int64_t H, int64_t W, int64_t D, const int64_t* l_strides,
                                      const int64_t* r_strides, int mode, void* workspace,
                                      int64_t workspace_bytes, void* stream);

/* a-2: TorchGroupwiseCost(n_groups, max_disparity)(left, right)
 *      -- cost_volume/groupwise.py:24-56
 * out[n,g,y,x,d] = mean_{c in group g} L*R(x-d) (x >= d), 0 (x < d);
 * groups are contiguous channel blocks of C/G.  out: (N, G, H, W, D) float32 always
 * (groupwise.py:39).  C % G != 0 -> SM_EINVAL. */
int sm_cv_groupwise(const void* left, const void* right, float* out, int dtype,
                    int64_t N, int64_t C, int64_t H, int64_t W, int64_t D, int64_t G,
                    const int64_t* l_strides, const int64_t* r_strides, void* stream);

/* a-3: TorchConcatenateCost(max_disparity)(left, right)
 *      -- cost_volume/concatenate.py:11-41
 * out[n,c,y,x,d] = L (x >= d) ; out[n,C+c,y,x,d] = R(x-d) (x >= d) ; 0 (x < d).
 * out: (N, 2C, H, W, D), bit-exact copy. */
int sm_cv_concat(const void* left, const void* right, void* out, int dtype,
                 int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                 const int64_t* l_strides, const int64_t* r_strides, void* stream);

/* a-4: TorchInterweaveCost()(left, right) -- cost_volume/interweave.py:10-22,
 *      = interweave_tensors -- model/mobile_stereo_net_v4.py:17-23
 * out[n,2c] = L[n,c], out[n,2c+1] = R[n,c].  out: (N, 2C, H, W), bit-exact. */
int sm_cv_interweave(const void* left, const void* right, void* out, int dtype,
                     int64_t N, int64_t C, int64_t H, int64_t W,
                     const int64_t* l_strides, const int64_t* r_strides, void* stream);

/* a-4': the v4 per-disparity shifted interweave materialised as one volume
 *      -- model/mobile_stereo_net_v4.py:443-461 (input of the Conv3d stack)
 * out[n,2c,d,y,x] = L[n,c,y,x], out[n,2c+1,d,y,x] = R[n,c,y,x-d] (x >= d), 0 (x < d).
 * out: (N, 2C, D, H, W), bit-exact. */
int sm_cv_interweave_shifted(const void* left, const void* right, void* out, int dtype,
                             int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                             const int64_t* l_strides, const int64_t* r_strides, void* stream);

/* a-5: make_cost_volume(left, right, max_disp) -- model/mobile_stereo_net.py:8-27
 * out[n,c,d,y,x] = L[n,c,y,x] - R[n,c,y,x-d] (x >= d), 1.0 (x < d).
 * out: (N, C, D, H, W), bit-exact (one subtraction in the input dtype). */
int sm_cv_diff(const void* left, const void* right, void* out, int dtype,
               int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
               const int64_t* l_strides, const int64_t* r_strides, void* stream);

/* a-7: soft-argmin regression over D of a (N, D, H, W) volume
 *   flags = SM_REGRESS_SOFTMAX:      sum_d d * softmax_d(v)   (mobile_disp_net_c.py:208-220,
 *                                    inline mobile_stereo_net.py:144-147)
 *   flags = SM_REGRESS_PRESOFTMAXED: sum_d d * v              (mobile_stereo_net_v4.py:10-14)
 * out: (N, H, W) in `dtype` (keepdim is a caller-side view), or float32 with
 * SM_REGRESS_OUT_F32 (flags may OR it with either mode).  fp64 accumulation.
 * vol_strides: element strides of (N, D, H, W), W stride must be 1 (NULL = contiguous).
 * Any 4-byte aligned out works; fp32 planes with a 16-B aligned volume AND out take the
 * vectorised one-wave kernel, other alignments the generic kernel (same results). */
int sm_regress_softargmin(const void* volume, void* out, int dtype,
                          int64_t N, int64_t D, int64_t H, int64_t W, int flags,
                          const int64_t* vol_strides, void* stream);

/* a-8: hard argmin / argmax over D (build-defined): first index on ties,
 * NaN counts as the extreme (torch.argmin/argmax semantics).  out: (N, H, W) int64. */
int sm_regress_argext(const void* volume, int64_t* out, int dtype,
                      int64_t N, int64_t D, int64_t H, int64_t W, int mode,
                      const int64_t* vol_strides, void* stream);

/* §8f-4: warp an image / feature map by a disparity (1-channel) or flow (2-channel) map,
 * replacing warp_by_flow_map (tools/warp.py:5-42; model/mobile_stereo_net_v2.py:59-96 and
 * _v3.py:60-97, called by RefineNet _v3.py:136 / _v2.py:127): the reference's grid
 * (x - fx, y - fy) normalised by (w - 1, h - 1), sampled by grid_sample bilinear, zero padding,
 * align_corners=False.  image: (N, C, Hi, Wi); flow: (N, flow_channels, H, W) with
 * flow_channels 1 or 2; out: (N, C, H, W) contiguous.  float32 only (SM_EDTYPE otherwise).
 * Strides: element strides of (N, C, H, W) for image and flow (W stride 1; NULL = contiguous). */
int sm_warp_by_flow(const void* image, const void* flow, void* out, int dtype,
                    int64_t N, int64_t C, int64_t Hi, int64_t Wi, int64_t H, int64_t W,
                    int64_t flow_channels, const int64_t* image_strides,
                    const int64_t* flow_strides, void* stream);
/* The same warp with a caller-provided device workspace (16-B aligned): two-channel flows over
 * at most 64 channels then sample a channel-last copy of the image (one 128-B line per corner
 * and pixel at C = 32 instead of one per corner, pixel and channel).  Same results.
 * sm_warp_by_flow_workspace_bytes gives the size (0: the shape does not use one; any workspace,
 * or none, is then accepted and ignored). */
int64_t sm_warp_by_flow_workspace_bytes(int64_t N, int64_t C, int64_t Hi, int64_t Wi,
                                        int64_t flow_channels);
int sm_warp_by_flow_ws(const void* image, const void* flow, void* out, int dtype,
                       int64_t N, int64_t C, int64_t Hi, int64_t Wi, int64_t H, int64_t W,
                       int64_t flow_channels, const int64_t* image_strides,
                       const int64_t* flow_strides, void* workspace, int64_t workspace_bytes,
                       void* stream);

/* §8f-2: MobileStereoNetV4's cost volume -- model/mobile_stereo_net_v4.py:443-461 with the
 * stacks :317-335 (replaces the 48-iteration interweave -> conv3d -> volume11 loop).
 * For every disparity i < D: interweave(L[..., i:], R[..., :-i]) as a depth-64 volume ->
 * Conv3d(1->16, (8,3,3), stride (8,1,1)) -> Conv3d(16->32, (4,3,3), /4) -> Conv3d(32->16,
 * (2,3,3), /2), each with its eval-mode BatchNorm folded in and ReLU, zero padding 1 at the
 * crop's borders -> 1x1 conv 16->1 (+BN folded) + ReLU, at x >= i of out (N, D, H, W)
 * (0 at x < i).  featL/featR: (N, 32, H, W) float32 (strides as above); out contiguous float32.
 * Folded weights, float32 device pointers in PyTorch layouts: w1 (16,8,3,3) b1 (16),
 * w2 (32,16,4,3,3) b2 (32), w3 (16,32,2,3,3) b3 (16), w4 (16) b4 (1).
 * workspace: device scratch of at least sm_v4_volume_workspace_bytes(N, H, W) bytes (per-pixel
 * layer-1 tables + packed MFMA weights); the library allocates nothing.
 * Arithmetic: layer 1 fp32; layers 2-3 fp16 MFMA over per-layer power-of-two scaled, hi/lo-split
 * fp32 operands (3 products, fp32 accumulation). */
int64_t sm_v4_volume_workspace_bytes(int64_t N, int64_t H, int64_t W);
int sm_v4_volume(const void* featL, const void* featR, void* out, int dtype,
                 int64_t N, int64_t C, int64_t H, int64_t W, int64_t D,
                 const int64_t* l_strides, const int64_t* r_strides,
                 const float* w1, const float* b1, const float* w2, const float* b2,
                 const float* w3, const float* b3, const float* w4, const float* b4,
                 void* workspace, int64_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* STEREOCV_H_ */

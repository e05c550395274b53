/*
 * pose6d — C ABI of the MI355X (gfx950) hot path of SFR-Vision/6d-pose-estimation.
 *
 * The reference exposes this path as Python classes (models/pose_net_*.py,
 * models/pose_loss.py, models/add_loss.py); this library is what those classes'
 * forward()/backward() call in the build.  Each entry point names the reference
 * code it replaces (path:line in the reference tree).
 *
 * Conventions (all entry points):
 *  - plain device pointers + sizes; no torch types; no allocation inside: the
 *    caller passes every output and workspace buffer (sizes documented or
 *    queried with the *_workspace() functions);
 *  - `stream` is a hipStream_t (torch's current stream); every call is
 *    stream-ordered and graph-capturable (no sync, no malloc);
 *  - return 0 on success or a POSE6D_E* code; pose6d_last_error() then holds a
 *    message (thread-local);
 *  - activations are NHWC, dtype given by a POSE6D_DT_* code; parameters and
 *    statistics are fp32; conv weights for the kernels are packed OHWI
 *    (K-contiguous per output channel), see pose6d_pack_conv_weight().
 */
#ifndef POSE6D_H
#define POSE6D_H
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define POSE6D_OK 0
#define POSE6D_EINVAL 1
#define POSE6D_ELAUNCH 2
#define POSE6D_EUNSUPPORTED 3

#define POSE6D_DT_F32 0
#define POSE6D_DT_BF16 1

int pose6d_version(void);
const char *pose6d_last_error(void);

/* ------------------------------------------------------------------------
 * ADD / ADD-S evaluation — replaces ADDLoss.eval_metrics (add_loss.py:156-201)
 * and ADDLoss.forward (add_loss.py:101-150).
 *
 * Meshes are packed: points[3*(off[o] + k) + {0,1,2}] for object slot o,
 * npts[o] == 0 marks an absent object (the reference skips such samples,
 * add_loss.py:171-172); obj_ids outside [0, n_slots) are absent too.
 * sym[o] != 0 for SYMMETRIC_OBJECT_IDS (add_loss.py:10); diam[o] in metres.
 * Per sample b the kernels write
 *   add[b]   = mean_k ||Q_k - G_k||                         (add_loss.py:182)
 *   adds[b]  = mean_k min_j ||Q_k - G_j||                    (add_loss.py:186-189)
 *   valid[b] = 1 if the object is known, else 0
 *   correct[b] = (sym ? adds : add) < 0.1 * diam             (add_loss.py:193-195)
 * with Q = P R_pred^T + t_pred, G = P R_gt^T + t_gt computed with torch-CPU's
 * rounding (fma order, unfused _quat_to_mat) so that the per-point minimum
 * distance and its FIRST-index argmin are bit-exact.  min_dist/argmin are
 * [B][max_npts] (argmin may be NULL); pt_add is a [B][max_npts] workspace.
 * ---------------------------------------------------------------------- */
int pose6d_add_eval(const float *pred_rot, const float *pred_trans, const float *gt_rot,
                    const float *gt_trans, const int64_t *obj_ids, int64_t B,
                    const float *points, const int32_t *off, const int32_t *npts,
                    const uint8_t *sym, const double *diam, int32_t n_slots, int32_t max_npts,
                    float *min_dist, int32_t *argmin, float *pt_add,
                    double *add, double *adds, int32_t *valid, int32_t *correct, void *stream);

/* pose6d_add_eval with a neighbour table (round 6): nbr [total points][K] uint16
 * (K = 8, 16 or 32; 16-byte aligned; <= 65536 points per mesh) lists, for every mesh
 * point, other points of the same mesh near it in model space (pose6d_add_neighbors).
 * The ADD-S search first visits each point's own ground-truth point and those
 * neighbours, so the full sweep seldom finds a better candidate; its first-index tie
 * rule does not depend on the visiting order, so the results are identical (bit for
 * bit) to pose6d_add_eval whatever the table holds.  nbr == NULL: pose6d_add_eval. */
int pose6d_add_eval_nbr(const float *pred_rot, const float *pred_trans, const float *gt_rot,
                        const float *gt_trans, const int64_t *obj_ids, int64_t B,
                        const float *points, const int32_t *off, const int32_t *npts,
                        const uint8_t *sym, const double *diam, int32_t n_slots, int32_t max_npts,
                        const uint16_t *nbr, int32_t K, float *min_dist, int32_t *argmin, float *pt_add,
                        double *add, double *adds, int32_t *valid, int32_t *correct, void *stream);

/* The neighbour table of a packed mesh table (points / off / npts as pose6d_add_eval):
 * nbr[off[o] + k][0..K) = the K nearest other points of mesh o to its point k (local
 * indices; fp32 model-space distances; a mesh of fewer than K + 1 points repeats k).
 * One launch, a setup step per table (not per evaluation). */
int pose6d_add_neighbors(const float *points, const int32_t *off, const int32_t *npts, int32_t n_slots,
                         int32_t max_npts, int32_t K, uint16_t *nbr, void *stream);

/* Backward of ADDLoss.forward (add_loss.py:101-150) w.r.t. the predicted pose:
 * loss = mean over known samples of mean_k ||Q_k - G*_k|| (G* = G_k, or the
 * nearest ground-truth point for SYMMETRIC_OBJECT_IDS, taken from the `argmin`
 * [B][max_npts] a pose6d_add_eval call on the same inputs produced); dloss is a
 * device scalar.  grad_rot [B][4] (through _quat_to_mat, add_loss.py:203-215),
 * grad_trans [B][3]; unknown objects get zero gradient. */
int pose6d_add_loss_bwd(const float *pred_rot, const float *pred_trans, const float *gt_rot,
                        const float *gt_trans, const int64_t *obj_ids, int64_t B, const float *points,
                        const int32_t *off, const int32_t *npts, const uint8_t *sym, int32_t n_slots,
                        int32_t max_npts, const int32_t *argmin, const float *dloss, float *grad_rot,
                        float *grad_trans, void *stream);

/* ------------------------------------------------------------------------
 * Pose heads and loss
 * ---------------------------------------------------------------------- */
/* F.normalize(x, p=2, dim=1) (mode 0: x / max(||x||, 1e-12), pose_net_rgb.py:61,
 * pose_net_rgbd.py:138, pose_net_rgbd_geometric.py:45) or the RGB-Geometric form
 * x / (||x|| + 1e-8) (mode 1, pose_net_rgb_geometric.py:75).  x, y: [B][D]. */
int pose6d_rownorm_fwd(const float *x, float *y, int64_t B, int32_t D, int32_t mode, void *stream);
int pose6d_rownorm_bwd(const float *x, const float *dy, float *dx, int64_t B, int32_t D, int32_t mode,
                       void *stream);

/* PoseNetRGBDGeometric._compute_pinhole_translation (pose_net_rgbd_geometric.py:56-85):
 * depth_raw [B][H][W] fp32 (sampled at the clamped int pixel, 223 hard-coded as in
 * the reference), bbox_center [B][2], K [B][3][3] (K_batched=1) or [3][3] (0) -> t [B][3]. */
int pose6d_pinhole_depth(const float *depth_raw, int32_t H, int32_t W, const float *bbox_center,
                         const float *K, int32_t K_batched, int64_t B, float *t, void *stream);

/* PoseNetRGBGeometric._compute_pinhole_translation (pose_net_rgb_geometric.py:93-109):
 * z [B] -> t [B][3]; backward gives dz from dt. */
int pose6d_pinhole_z_fwd(const float *z, const float *bbox_center, const float *K, int32_t K_batched,
                         int64_t B, float *t, void *stream);
int pose6d_pinhole_z_bwd(const float *dt, const float *bbox_center, const float *K, int32_t K_batched,
                         int64_t B, float *dz, void *stream);

/* PoseLoss.forward (pose_loss.py:19-28): rot_mode 0 = geodesic (:30-50),
 * 1 = quaternion L1 (:52-61); trans = l1_loss mean.  loss: one float.
 * Backward: dloss (device scalar) -> grad_rot [B][4], grad_trans [B][3]. */
int pose6d_pose_loss_fwd(const float *pred_rot, const float *pred_trans, const float *gt_rot,
                         const float *gt_trans, int64_t B, float rot_weight, float trans_weight,
                         int32_t rot_mode, float *loss, void *stream);
int pose6d_pose_loss_bwd(const float *pred_rot, const float *pred_trans, const float *gt_rot,
                         const float *gt_trans, int64_t B, float rot_weight, float trans_weight,
                         int32_t rot_mode, const float *dloss, float *grad_rot, float *grad_trans,
                         void *stream);

/* The RGBD-Geometric training step's head + loss in one launch: rot =
 * F.normalize(raw) (pose_net_rgbd_geometric.py:45), trans = pinhole(depth_raw)
 * (:56-85), loss = PoseLoss(rot, trans) (pose_loss.py:19-28) and its gradient for
 * dloss = 1: grad_raw (through the normalize) and grad_trans.  Same formulas as the
 * separate pose6d_rownorm_* / pinhole_depth / pose_loss_* calls. */
int pose6d_geo_head_loss(const float *raw, const float *depth_raw, int32_t H, int32_t W, const float *bbox_center,
                         const float *K, int32_t K_batched, const float *gt_rot, const float *gt_trans, int64_t B,
                         float rot_weight, float trans_weight, int32_t rot_mode, float *rot, float *trans,
                         float *loss, float *grad_raw, float *grad_trans, void *stream);

/* ------------------------------------------------------------------------
 * Input crops -- replaces the per-sample body of LineMODDatasetRGBD.__getitem__
 * after the file reads (data/dataset_rgbd.py:104-206; dataset_rgb.py:95-145 for
 * the RGB models): square crop x1.2 around the (jittered) bbox with zero padding,
 * cv2.resize(..., (S, S)) INTER_LINEAR, ToTensor + Normalize, depth / 1000 and
 * the (d - 0.1) / 1.5 normalisation, crop-adjusted centre and intrinsics.
 * rgb [B][H][W][3] uint8 (RGB; bgr != 0: cv2.imread's BGR order, the
 * cvtColor of dataset_rgbd.py:90 folded in); depth [B][H][W] uint16 mm or NULL
 * (= zeros, :94-95); bbox_orig / bbox_aug [B][4] int32 (x, y, w, h) before /
 * after the jitter of :110-118 (drawn on the host, np.random order); K [B][3][3].
 * mean_std: 6 device floats (mean[3], std[3]) or NULL (ToTensor only).
 * Outputs (each may be NULL): rgb_out [B][3][S][S], depth_out [B][1][S][S],
 * depth_raw_out [B][S][S], center_out [B][2], K_out [B][3][3], all fp32.
 * ---------------------------------------------------------------------- */
int pose6d_crop_rgbd(const uint8_t *rgb, int32_t bgr, const uint16_t *depth, int32_t B, int32_t H, int32_t W,
                     const int32_t *bbox_orig, const int32_t *bbox_aug, const float *K, int32_t S,
                     const float *mean_std, float *rgb_out, float *depth_out, float *depth_raw_out,
                     float *center_out, float *K_out, void *stream);

/* ----------------------------------------------------------------------
 * Train transform of the same crops (train_rgbd_geometric.py:41-47, applied by
 * dataset_rgbd.py:196-197): pose6d_crop_rgbd's crop + resize, then on the uint8
 * crop ColorJitter(brightness, contrast, saturation, hue) with torchvision's op
 * order / factor draws and Pillow's arithmetic, ToTensor + Normalize, then
 * RandomErasing(erase_p, (erase_scale_lo, _hi), (erase_ratio_lo, _hi), value 0).
 * A jitter value of 0 switches that op off (torchvision's None).  Random draws:
 * counter-based (seed, crop, draw) -- the same seed gives the same crops; each crop's
 * drawn parameters go to params_out [B][16] (may be NULL): perm[4], brightness,
 * contrast, saturation, hue factor (NaN = off), erase i, j, h, w (-1 = none), 0 x 4.
 * workspace: pose6d_crop_train_workspace(B, S) bytes (the uint8 crops).  S <= 232.
 * rgb_out is required; the depth / centre / K outputs as pose6d_crop_rgbd.
 * ---------------------------------------------------------------------- */
int64_t pose6d_crop_train_workspace(int32_t B, int32_t S);
int pose6d_crop_rgbd_train(const uint8_t *rgb, int32_t bgr, const uint16_t *depth, int32_t B, int32_t H, int32_t W,
                           const int32_t *bbox_orig, const int32_t *bbox_aug, const float *K, int32_t S,
                           const float *mean_std, float brightness, float contrast, float saturation, float hue,
                           float erase_p, float erase_scale_lo, float erase_scale_hi, float erase_ratio_lo,
                           float erase_ratio_hi, uint64_t seed, uint8_t *workspace, float *rgb_out, float *depth_out,
                           float *depth_raw_out, float *center_out, float *K_out, float *params_out, void *stream);

/* ------------------------------------------------------------------------
 * ResNet50 trunk — replaces torchvision.models.resnet50 children[:-1] as
 * wrapped by every model (pose_net_rgb.py:18-20, pose_net_rgb_geometric.py:18-20,
 * pose_net_rgbd.py:48-61, pose_net_rgbd_geometric.py:23-25) and the z-CNN of
 * pose_net_rgb_geometric.py:36-55.  NHWC activations of `dtype`.
 * ---------------------------------------------------------------------- */
/* model input (B, C, H, W) fp32 -> NHWC with channels zero-padded to Cpad */
int pose6d_nchw_to_nhwc(int32_t dtype, const float *x, void *y, int32_t N, int32_t C, int32_t H, int32_t W,
                        int32_t Cpad, void *stream);

/* One launch packs every conv's OIHW fp32 master weight into the kernel layouts:
 * wp [O][Kpad] (K = (kh, kw', ci): ci padded to Ip, KWp packed taps kw' per kernel
 * row with filter tap kw at kw' = kw + KWp - KW, zeros elsewhere and beyond K) and,
 * when non-null, wt [I][KH][KW][O] for the data gradient.  `descs` is a device array of
 * n_desc records of pose6d_pack_desc_size() bytes:
 *   { const float *w; void *wp; void *wt; int32 O, I, Ip, KH, KW, Kpad, KWp, reserved; int64 start; }
 * (start: the caller's bookkeeping, unused; total: sum of O*Kpad, unused).  KWp and
 * Kpad of a forward conv come from pose6d_conv_pack_geom. */
int pose6d_pack_desc_size(void);
int pose6d_pack_conv_weights(int32_t dtype, const void *descs, int32_t n_desc, int64_t total, void *stream);
/* Packed layout of a conv's forward filter (wp): taps per kernel row (*kw_packed: KW,
 * or 8 for the row-tap stems -- Cin 4, stride 2, a kernel row of <= 8 taps: 7x7 / pad 3,
 * read by the LDS-DMA kernel as 64-byte input rows) and the padded K (*Kpad). */
int pose6d_conv_pack_geom(int32_t dtype, int32_t Cin, int32_t KH, int32_t KW, int32_t stride, int32_t pad,
                          int32_t *kw_packed, int32_t *Kpad);

/* nn.Conv2d forward (implicit GEMM on MFMA).  x [N][H][W][Cin] (Cin = 4 for the
 * padded stem, else a power of two), wp packed [Cout][Kpad], y [N][Ho][Wo][Cout].
 * bias may be NULL.  stats (NULL = none) receives BatchNorm partials over blocks of
 * 32 output pixels, rows = pose6d_conv_stats_rows(...), stored channel-major
 * [2][Cout][rows] fp32: stats[c][r] = sum, stats[Cout + c][r] = M2 about the block
 * mean. */
int pose6d_conv_stats_rows(int32_t N, int32_t Ho, int32_t Wo, int32_t Cout);
int pose6d_conv2d_fwd(int32_t dtype, const void *x, const void *wp, const float *bias, void *y, float *stats,
                      int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH, int32_t KW,
                      int32_t stride, int32_t pad, int32_t Ho, int32_t Wo, void *splitk_ws, int64_t splitk_ws_bytes,
                      void *stream);
/* Split-K workspace (caller-provided; the library keeps no device state of its own).
 * A forward plan on a small grid with a long K loop (pose6d_conv_variant >> 16 > 1)
 * divides each output tile's K-steps over several workgroups of one launch; their
 * fp32 partial tiles and the tiles' arrival counters live in splitk_ws:
 *   bytes = pose6d_conv_splitk_workspace(dtype, pass 0 = forward / 1 = data gradient, geometry...)
 * (0 = the plan does not split: splitk_ws may be NULL).  Layout: 32 KiB of arrival
 * counters, then the partial tiles.  The counter block must be ZERO before the first
 * use of a workspace (e.g. allocate it zeroed); every launch leaves it zero, so one
 * workspace serves any sequence of stream-ordered convs.  Launches that may run
 * concurrently (other streams, other threads) need workspaces of their own.  256-byte
 * aligned.  A plan that splits and gets no (or too small a) workspace fails with
 * POSE6D_ERR_ARG; data gradients split only under an explicit pose6d_tuning_t. */
int64_t pose6d_conv_splitk_workspace(int32_t dtype, int32_t pass, int32_t N, int32_t H, int32_t W, int32_t Cin,
                                     int32_t Cout, int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho,
                                     int32_t Wo);
/* kernel variant a conv launch selects (profiling joins): fwd/dgrad (pass 0/1):
 * (splits << 16) | (stages << 12) | (fast << 8) | (mode << 4) | tile (tile 0..3 = 128x128, 128x64,
 * 64x128, 64x64; mode 0 gemm, 1 im2col, 2 narrow stem, 3 dgrad, 4 stride-2 dgrad
 * split into output parity classes; fast = LDS-DMA bf16 kernel with an LDS ring
 * of `stages` K-steps, 0 on the register-staged kernel; splits = workgroups per output
 * tile of the in-launch split-K, 1 = none);
 * wgrad (pose6d_wgrad_variant, Cin = the padded channel count): (stages << 12) |
 * (fast << 8) | (BM == 128) << 1 | (BN == 128); fast = the LDS-DMA weight-gradient
 * kernel (bf16: 64x64 tiles; fp32: 64x64 or 128x128 tiles, bits 1 and 0), 0 = the
 * register-staged kernel. */
int pose6d_conv_variant(int32_t dtype, int32_t pass, int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout,
                        int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo);
int pose6d_wgrad_variant(int32_t dtype, int32_t M, int32_t Cout, int32_t K, int32_t Cin);
/* 3x3 / stride 1 / pad 1 bf16 forwards WITHOUT BatchNorm statistics (eval: pose6d_conv2d_fwd
 * with stats == NULL, pose6d_conv2d_fwd_act) on >= 64-channel slices run the patch kernel
 * (conv3x3_patch_kernel: each workgroup stages its input patch once per 64-channel slice
 * instead of once per filter tap): its workgroup count, or 0 when the geometry takes the
 * implicit-GEMM plans pose6d_conv_variant describes. */
int pose6d_conv_patch_plan(int32_t dtype, int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH,
                           int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo);
/* eval-mode forward with the BatchNorm folded into the store: out = act(T(conv(x) [+ bias]) * scale + shift
 * [+ res | + res * res_scale + res_shift]), act = ReLU if relu -- pose6d_conv2d_fwd followed by
 * pose6d_bn_act_fwd bit for bit, one launch, no raw-output round trip.  res: NHWC like out (or NULL). */
int pose6d_conv2d_fwd_act(int32_t dtype, const void *x, const void *w, const float *bias, void *out, int32_t N,
                          int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
                          int32_t pad, int32_t Ho, int32_t Wo, const float *scale, const float *shift, const void *res,
                          const float *res_scale, const float *res_shift, int32_t relu, void *splitk_ws,
                          int64_t splitk_ws_bytes, void *stream);
/* eval-mode output of a torchvision Bottleneck with a downsample branch, ONE launch
 * (replaces, at pose_net_*.py's `self.backbone(x)`, the block's conv3 + bn3 and the
 * downsample conv + bn + add + ReLU):
 *   out = act(T(x . w) * scale + shift + T(xd_s . wd) * scale_d + shift_d),
 * x [N][Ho][Wo][Cin] (conv3 input), w [Cout][Cin]; xd [N][Hd][Wd][Cind] (block input),
 * wd [Cout][Cind], xd_s = xd sampled every stride_d pixels; both 1x1, no bias.  Bit for
 * bit pose6d_conv2d_fwd of the downsample then pose6d_conv2d_fwd_act with
 * res_scale/res_shift, without the downsample output's HBM round trip.  Rejected
 * (POSE6D_ERR_ARG) when either separate launch's plan splits K (pose6d_conv_variant). */
int pose6d_conv2d_fwd_act_dual(int32_t dtype, const void *x, const void *w, const void *xd, const void *wd, void *out,
                               int32_t N, int32_t Ho, int32_t Wo, int32_t Cin, int32_t Cout, int32_t Hd, int32_t Wd,
                               int32_t Cind, int32_t stride_d, const float *scale, const float *shift,
                               const float *scale_d, const float *shift_d, int32_t relu, void *stream);
/* data gradient: dx [N][H][W][Cin] = conv_transpose(dy [N][Ho][Wo][Cout], wt) (+ dres if non-NULL).
 * dres may be dx itself (accumulate in place); a stride-2 1x1 conv then writes only the
 * pixels its taps reach (the other three parity classes are left as they are). */
int pose6d_conv2d_dgrad(int32_t dtype, const void *dy, const void *wt, const void *dres, void *dx, int32_t N,
                        int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
                        int32_t pad, int32_t Ho, int32_t Wo, void *stream);
/* weight gradient into OIHW fp32 dw (Cin_real channels of the Cin-padded input);
 * workspace: pose6d_conv2d_wgrad_workspace(...) bytes of fp32 split slabs, its
 * size passed as ws_bytes (a plan needing more fails with POSE6D_EINVAL). */
int64_t pose6d_conv2d_wgrad_workspace(int32_t dtype, int32_t N, int32_t Ho, int32_t Wo, int32_t Cin, int32_t Cout,
                                      int32_t KH, int32_t KW);
int pose6d_conv2d_wgrad(int32_t dtype, const void *x, const void *dy, float *dw, int32_t accumulate,
                        float *workspace, int64_t ws_bytes, int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cin_real,
                        int32_t Cout, int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo,
                        void *stream);

/* Data + weight gradient of one conv in one call (pose6d_conv2d_dgrad followed by
 * pose6d_conv2d_wgrad, same arguments and workspace): on the bf16 LDS-DMA paths
 * both run as ONE launch whose workgroups split between the two passes, then
 * the slab reduce.  dx == NULL skips the data gradient. */
int pose6d_conv2d_backward(int32_t dtype, const void *x, const void *dy, const void *wt, const void *dres,
                           void *dx, float *dw, int32_t accumulate, float *workspace, int64_t ws_bytes, int32_t N,
                           int32_t H, int32_t W, int32_t Cin, int32_t Cin_real, int32_t Cout, int32_t KH,
                           int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo, void *stream);
/* Explicit plan overrides for the conv entry points' *_tuned forms -- used by the
 * tests (every tile / ring depth / kernel of a shape must agree) and the tuning tools,
 * never by the product path: without one, each conv geometry has exactly one plan,
 * so one summation order.  Every field -1 = the default plan.
 *   conv_tile     fast path 0 = 128x128, 1 = 128x64, 3 = 64x64 (4 waves), 4 = 128x128, 5 = 128x64 (8 waves);
 *                 register-staged path 0..3 = 128x128, 128x64, 64x128, 64x64
 *   conv_stages   LDS ring slots of the fast path (2, 3, 4, 6)
 *   conv_s2       0: the stride-2 data gradient as one masked gather instead of 4 parity classes
 *   conv_base     1: the register-staged conv kernels instead of the LDS-DMA path
 *   wgrad_stages  LDS ring slots of the bf16 weight-gradient kernel (2..4)
 *   wgrad_base    1: the register-staged weight-gradient kernel (other split plan)
 *   bwd_separate  1: data and weight gradient as separate launches (not the fused kernel)
 *   conv_splitk   fast path (1x1 / KxK forward, stride-1 data gradient): K-steps of each output tile
 *                 split over this many workgroups of one launch (1 = none)
 *   wgrad_splits  weight gradient: pixel splits (slabs) of the plan (>= 1; tools only)
 *   bwd_order     fused backward: 1 = weight-gradient workgroups dispatched first, 0 = data gradient first
 *   conv_patch    3x3 stride-1 bf16 forwards without BatchNorm statistics: 0 = the implicit-GEMM plan,
 *                 1 or -1 = the patch plan (-1 only while no conv_tile / conv_stages / conv_base /
 *                 conv_splitk is forced)
 * A tuned plan that splits K needs pose6d_conv_splitk_workspace_tuned(...) bytes of
 * split-K workspace (see pose6d_conv_splitk_workspace). */
typedef struct {
  int32_t conv_tile, conv_stages, conv_s2, conv_base, wgrad_stages, wgrad_base, bwd_separate, conv_splitk;
  int32_t wgrad_splits, bwd_order, conv_patch;
} pose6d_tuning_t;
int64_t pose6d_conv_splitk_workspace_tuned(int32_t dtype, int32_t pass, int32_t N, int32_t H, int32_t W,
                                           int32_t Cin, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
                                           int32_t pad, int32_t Ho, int32_t Wo, const pose6d_tuning_t *tuning);
int pose6d_conv2d_fwd_tuned(int32_t dtype, const void *x, const void *w, const float *bias, void *y, float *stats,
                            int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH, int32_t KW,
                            int32_t stride, int32_t pad, int32_t Ho, int32_t Wo, const pose6d_tuning_t *tuning,
                            void *splitk_ws, int64_t splitk_ws_bytes, void *stream);
int pose6d_conv2d_dgrad_tuned(int32_t dtype, const void *dy, const void *wt, const void *dres, void *dx, int32_t N,
                              int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
                              int32_t pad, int32_t Ho, int32_t Wo, const pose6d_tuning_t *tuning, void *splitk_ws,
                              int64_t splitk_ws_bytes, void *stream);
int64_t pose6d_conv2d_wgrad_workspace_tuned(int32_t dtype, int32_t N, int32_t Ho, int32_t Wo, int32_t Cin,
                                            int32_t Cout, int32_t KH, int32_t KW, const pose6d_tuning_t *tuning);
int pose6d_conv2d_wgrad_tuned(int32_t dtype, const void *x, const void *dy, float *dw, int32_t accumulate,
                              float *workspace, int64_t ws_bytes, int32_t N, int32_t H, int32_t W, int32_t Cin,
                              int32_t Cin_real, int32_t Cout, int32_t KH, int32_t KW, int32_t stride, int32_t pad,
                              int32_t Ho, int32_t Wo, const pose6d_tuning_t *tuning, void *stream);
int pose6d_conv2d_backward_tuned(int32_t dtype, const void *x, const void *dy, const void *wt, const void *dres,
                                 void *dx, float *dw, int32_t accumulate, float *workspace, int64_t ws_bytes,
                                 int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cin_real, int32_t Cout,
                                 int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo,
                                 const pose6d_tuning_t *tuning, void *stream);
/* pose6d_conv2d_backward in phases (profiling): bit 0 = the gradient launch(es) that
 * fill the fp32 slabs (and dx), bit 1 = the slab reduce into dw; 3 = the whole call.
 * On the unfused path bit 0 runs the complete dgrad + wgrad and bit 1 nothing.  A
 * fused 1x1 conv whose weight gradient has ONE split and K = Cin = Cin_real, not
 * accumulating (layer4's 1x1 convs), writes dw directly during bit 0 (its single slab
 * is the OIHW gradient): bit 1 then does nothing. */
int pose6d_conv2d_backward_ex(int32_t dtype, const void *x, const void *dy, const void *wt, const void *dres,
                              void *dx, float *dw, int32_t accumulate, float *workspace, int64_t ws_bytes, int32_t N,
                              int32_t H, int32_t W, int32_t Cin, int32_t Cin_real, int32_t Cout, int32_t KH,
                              int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo, int32_t phases,
                              void *stream);
/* Backward chaining across convs: a weight-gradient slab reduce described by
 * pose6d_wgrad_reduce_t (the conv's geometry as passed to pose6d_conv2d_backward,
 * its workspace of slabs and its dW) can ride on the NEXT conv's fused launch as
 * extra workgroups instead of a launch of its own.
 * pose6d_conv2d_backward_chain = pose6d_conv2d_backward that (a) also reduces
 * `prev` (NULL = none; its slabs must be in a different workspace) and (b) when
 * this conv runs the fused kernel, leaves its OWN reduce pending: *deferred = 1,
 * and the caller passes it as `prev` to the next call or flushes it with
 * pose6d_wgrad_reduce.  *deferred = 0: this conv's dW is complete (also the case of
 * the direct-dW plans described at pose6d_conv2d_backward_ex). */
typedef struct {
  const float *ws;
  float *dw;
  int32_t dtype, N, H, W, Cin, Cin_real, Cout, KH, KW, stride, pad, Ho, Wo, accumulate;
} pose6d_wgrad_reduce_t;
int pose6d_wgrad_reduce(const pose6d_wgrad_reduce_t *job, void *stream);
int pose6d_conv2d_backward_chain(int32_t dtype, const void *x, const void *dy, const void *wt, const void *dres,
                                 void *dx, float *dw, int32_t accumulate, float *workspace, int64_t ws_bytes,
                                 int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cin_real, int32_t Cout,
                                 int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo,
                                 const pose6d_wgrad_reduce_t *prev, int32_t *deferred, void *stream);
/* pose6d_conv2d_backward_chain whose residual contribution is dres * mask instead of
 * dres: dres_mask = pose6d_bn_act_fwd_mask's ReLU bits for dres (bit e of byte i masks
 * element i * E + e, E = 8 bf16 / 4 fp32), i.e. dres = the block output's gradient and
 * the product = the dz a residual BN backward would otherwise write out; dres != dx. */
int pose6d_conv2d_backward_chain_masked(int32_t dtype, const void *x, const void *dy, const void *wt,
                                        const void *dres, const uint8_t *dres_mask, void *dx, float *dw,
                                        int32_t accumulate, float *workspace, int64_t ws_bytes, int32_t N, int32_t H,
                                        int32_t W, int32_t Cin, int32_t Cin_real, int32_t Cout, int32_t KH,
                                        int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo,
                                        const pose6d_wgrad_reduce_t *prev, int32_t *deferred, void *stream);

/* A BatchNorm backward's reduce pass folded into the data gradient that completes
 * its output gradient (the BN + ReLU producing this conv's input): while storing dX
 * (+ dres * mask), the epilogue also sums, per channel over each output tile,
 * dz = dX * relu and dz * (y - mean) * invstd into partial[2][C][rows] -- what
 * pose6d_bn_bwd's first launch computes from dX re-read.  relu = the stored bits
 * (relu_mask, pose6d_bn_act_fwd_mask) or T(y * relu_scale + relu_shift) > 0;
 * y2 / mean2 / invstd2 / partial2: a second BN fed the same dz (a downsampling
 * block's branch BN; needs relu_mask).  rows = pose6d_conv2d_backward_bn_rows.
 * pose6d_bn_bwd_partials then finishes the backward (finalize + apply). */
typedef struct {
  const void *y;
  const float *mean, *invstd;
  const float *relu_scale, *relu_shift;
  const uint8_t *relu_mask;
  float *partial;
  const void *y2;
  const float *mean2, *invstd2;
  float *partial2;
  int32_t rows;
} pose6d_bn_reduce_t;

int pose6d_conv2d_backward_bn_rows(int32_t dtype, int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout,
                                   int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo);

/* pose6d_conv2d_backward_chain (dres_mask as in _masked, or NULL) whose data gradient
 * also produces the BatchNorm-reduce partials `bn` describes (NULL = none); dX must be
 * written whole (dres != dx). */
int pose6d_conv2d_backward_chain_bn(int32_t dtype, const void *x, const void *dy, const void *wt, const void *dres,
                                    const uint8_t *dres_mask, void *dx, float *dw, int32_t accumulate,
                                    float *workspace, int64_t ws_bytes, int32_t N, int32_t H, int32_t W, int32_t Cin,
                                    int32_t Cin_real, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
                                    int32_t pad, int32_t Ho, int32_t Wo, const pose6d_wgrad_reduce_t *prev,
                                    int32_t *deferred, const pose6d_bn_reduce_t *bn, void *stream);
/* (1 << 16) | (data-gradient mode << 4) | ring stages when pose6d_conv2d_backward
 * runs ONE fused conv_bwd_kernel<mode, stages, 3> launch (+ the reduce), else 0 */
int pose6d_bwd_variant(int32_t dtype, int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH,
                       int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo);

/* nn.BatchNorm2d: finalize the conv-epilogue statistics (training) or use the
 * running statistics (eval) -> scale/shift (+ saved mean / invstd); running
 * stats, num_batches_tracked updated in training (torch semantics).
 * partial: [2][C][rows] (rows = ceil(count / 32); sum, M2 about the block's mean)
 * over 32-pixel blocks, as pose6d_conv2d_fwd writes them, folded in fp64 as shifted sums about the first row's
 * mean in ONE launch; workspace: unused (kept in the ABI, may be NULL). */
int pose6d_bn_finalize(const float *partial, int32_t rows, int32_t C, int64_t count, const float *gamma,
                       const float *beta, float *running_mean, float *running_var, int64_t *num_batches,
                       float momentum, float eps, int32_t training, float *scale, float *shift, float *save_mean,
                       float *save_invstd, double *workspace, void *stream);
/* pose6d_bn_finalize (training) of two BatchNorms over the same output grid -- a
 * downsampling Bottleneck's bn3 and its downsample BN (same rows, count) -- in ONE
 * launch; each BN's results bit for bit those of its own pose6d_bn_finalize call. */
typedef struct {
  const float *partial;   /* [2][C][rows] conv-epilogue statistics */
  const float *gamma, *beta;
  float *running_mean, *running_var;
  int64_t *num_batches;   /* may be NULL */
  float *scale, *shift, *save_mean, *save_invstd;
  float momentum, eps;
  int32_t C;
} pose6d_bn_stats_t;
int pose6d_bn_finalize_dual(const pose6d_bn_stats_t *a, const pose6d_bn_stats_t *b, int32_t rows, int64_t count,
                            void *stream);
/* Eval-mode fold of a table of BatchNorms in one launch: per entry and channel c,
 * scale = gamma / sqrt(running_var + eps), shift = beta - running_mean * scale,
 * save_mean = running_mean, save_invstd = 1 / sqrt(running_var + eps) -- pose6d_bn_finalize
 * with training = 0, for all entries.  descs: device array of n pose6d_bn_fold_t
 * (pose6d_bn_fold_desc_size() bytes each), max_c >= every entry's C. */
typedef struct {
  const float *gamma, *beta, *running_mean, *running_var;
  float *scale, *shift, *save_mean, *save_invstd;
  float eps;
  int32_t C;
} pose6d_bn_fold_t;
int pose6d_bn_fold_desc_size(void);
int pose6d_bn_eval_fold(const void *descs, int32_t n, int32_t max_c, void *stream);
/* out = act(y * scale + shift [+ res | + res * res_scale + res_shift]); act = ReLU if relu */
int pose6d_bn_act_fwd(int32_t dtype, const void *y, const float *scale, const float *shift, const void *res,
                      const float *res_scale, const float *res_shift, int32_t relu, void *out, int64_t M, int32_t C,
                      void *stream);
/* bn_act_fwd that also writes relu_mask[M * C / E] (E = 8 bf16 / 4 fp32 elements per
 * byte, bit e of byte i = out[i * E + e] > 0) for pose6d_bn_bwd_mask. */
int pose6d_bn_act_fwd_mask(int32_t dtype, const void *y, const float *scale, const float *shift, const void *res,
                           const float *res_scale, const float *res_shift, int32_t relu, void *out, uint8_t *relu_mask,
                           int64_t M, int32_t C, void *stream);
/* Training BatchNorm finalize + apply in ONE launch: pose6d_bn_finalize(bn, training = 1)
 * followed by pose6d_bn_act_fwd_mask(y, bn->scale, bn->shift, res, NULL, NULL, relu, out,
 * relu_mask), bit for bit (the identity-residual / no-residual forms; C a multiple of 64,
 * rows = ceil(count / 32) as the conv epilogue wrote them).  The apply workgroups wait for
 * the finalize workgroups of their channels through `flags` (pose6d_bn_finalize_act_flags
 * int32, zeroed ONCE by the caller, then left to the launches) and `epoch`, a device
 * int64 the caller advances (+1) between two launches on the same flags and never
 * changes while one runs; an apply workgroup that does not see its flags in time
 * computes its channels itself (same arithmetic), so nothing depends on dispatch order
 * (a NEGATIVE epoch sends every apply workgroup that way at once: tests).
 * Replaces pose6d_bn_finalize + pose6d_bn_act_fwd_mask of the trunk's training forward
 * (bn_stats_finalize / bn_act, BatchNorm2d + ReLU [+ residual] of every Bottleneck). */
int32_t pose6d_bn_finalize_act_flags(int32_t rows, int32_t C);
int pose6d_bn_finalize_act(int32_t dtype, const pose6d_bn_stats_t *bn, int32_t rows, int64_t count, const void *y,
                           const void *res, int32_t relu, void *out, uint8_t *relu_mask, int32_t *flags,
                           const int64_t *epoch, void *stream);
/* backward of bn_act_fwd for one BN: dz = dout * mask, mask = out > 0 when `out` is
 * given, else (relu_scale/relu_shift given: a ReLU BN without residual) the sign
 * bn_act_fwd stored, recomputed from y as round(y * relu_scale + relu_shift) > 0
 * (no read of the forward output), else 1; dgamma/dbeta (accumulate or
 * overwrite); dy; dz_out (if non-NULL) = dz.
 * workspace: (pose6d_bn_bwd_workspace_rows(M) * 2 + 3) * C floats. */
int pose6d_bn_bwd_workspace_rows(int64_t M);
/* pose6d_bn_bwd with the ReLU mask taken from pose6d_bn_act_fwd_mask's bits instead of
 * re-reading the forward output (the residual BNs: 1/16 of the bytes). */
int pose6d_bn_bwd_mask(int32_t dtype, const void *dout, const uint8_t *relu_mask, const void *y, const float *mean,
                       const float *invstd, const float *gamma, float *dgamma, float *dbeta, int32_t accumulate,
                       void *dy, void *dz_out, float *workspace, int64_t M, int32_t C, void *stream);
/* The rest of a BatchNorm backward whose reduce pass ran in the data gradient that
 * produced dout (pose6d_conv2d_backward_chain_bn's `partial`, [2][C][rows]): the
 * finalize (dgamma, dbeta written or accumulated) and the apply (dy), two launches.
 * relu = relu_mask bits or T(y * relu_scale + relu_shift) > 0.  partial2 / y2 / mean2 /
 * invstd2 / gamma2 / dgamma2 / dbeta2 / dy2 (or NULL partial2): a second BN fed the
 * same dout * mask (needs relu_mask).  coef: 3 * C floats (6 * C with the second BN). */
int pose6d_bn_bwd_partials(int32_t dtype, const float *partial, int32_t rows, const void *dout,
                           const uint8_t *relu_mask, const float *relu_scale, const float *relu_shift, const void *y,
                           const float *mean, const float *invstd, const float *gamma, float *dgamma, float *dbeta,
                           void *dy, const float *partial2, const void *y2, const float *mean2, const float *invstd2,
                           const float *gamma2, float *dgamma2, float *dbeta2, void *dy2, int32_t accumulate,
                           float *coef, int64_t M, int32_t C, void *stream);

/* The backward of a downsampling block's two BatchNorms (the block's last BN and its
 * downsample branch's BN, both fed dout * relu_mask): pose6d_bn_bwd_mask for (y, mean,
 * invstd, gamma -> dgamma, dbeta, dy) and for (y2, ... -> dy2), bit for bit, in three
 * launches (one reduce, one finalize, one apply: dout and the mask read once per pass).
 * workspace: 2 * (pose6d_bn_bwd_workspace_rows(M) * 2 + 3) * C floats. */
int pose6d_bn_bwd_mask_dual(int32_t dtype, const void *dout, const uint8_t *relu_mask, const void *y,
                            const float *mean, const float *invstd, const float *gamma, float *dgamma, float *dbeta,
                            void *dy, const void *y2, const float *mean2, const float *invstd2, const float *gamma2,
                            float *dgamma2, float *dbeta2, void *dy2, int32_t accumulate, float *workspace, int64_t M,
                            int32_t C, void *stream);
int pose6d_bn_bwd(int32_t dtype, const void *dout, const void *out, const float *relu_scale,
                  const float *relu_shift, const void *y, const float *mean, const float *invstd, const float *gamma,
                  float *dgamma, float *dbeta, int32_t accumulate, void *dy, void *dz_out, float *workspace,
                  int64_t M, int32_t C, void *stream);

/* conv bias gradient: out[c] (+)= sum_m x[m][c] over an NHWC tensor of M pixels */
int pose6d_channel_sum(int32_t dtype, const void *x, int64_t M, int32_t C, float *out, int32_t accumulate,
                       void *stream);

/* nn.MaxPool2d(k, s, p) on NHWC; argmax = window index (uint8) of the first max */
int pose6d_maxpool_fwd(int32_t dtype, const void *x, void *y, uint8_t *argmax, int32_t N, int32_t H, int32_t W,
                       int32_t C, int32_t k, int32_t s, int32_t p, int32_t Ho, int32_t Wo, void *stream);
/* pose6d_bn_act_fwd (ReLU, no residual) followed by pose6d_maxpool_fwd in one pass: y, argmax
 * as that pair would produce them (bit for bit), without the full-resolution activation. */
int pose6d_bn_relu_maxpool_fwd(int32_t dtype, const void *x, const float *scale, const float *shift, void *y,
                               uint8_t *argmax, int32_t N, int32_t H, int32_t W, int32_t C, int32_t k, int32_t s,
                               int32_t p, int32_t Ho, int32_t Wo, void *stream);
int pose6d_maxpool_bwd(int32_t dtype, const void *dy, const uint8_t *argmax, void *dx, int32_t N, int32_t H,
                       int32_t W, int32_t C, int32_t k, int32_t s, int32_t p, int32_t Ho, int32_t Wo, void *stream);
/* nn.AdaptiveAvgPool2d(1) + view(B, -1): x [N][HW][C] -> y [N][C] fp32 */
int pose6d_avgpool_fwd(int32_t dtype, const void *x, float *y, int32_t N, int32_t HW, int32_t C, void *stream);
int pose6d_avgpool_bwd(int32_t dtype, const float *dy, void *dx, int32_t N, int32_t HW, int32_t C, void *stream);

/* ------------------------------------------------------------------------
 * Fully-connected heads (fp32) — nn.Linear / BatchNorm1d / ReLU / GELU / Dropout
 * of the rot/trans/z heads (pose_net_rgb.py:23-50, pose_net_rgbd_geometric.py:28-38,
 * pose_net_rgb_geometric.py:23-33,58-65, pose_net_rgbd.py:73-103).
 * ---------------------------------------------------------------------- */
/* C[m][n] = alpha * sum_k A[m*sam + k*sak] * B[k*sbk + n*sbn] (+ bias[n]) + beta * C[m][n]
 * workspace (may be NULL): ws_floats fp32 for split-K partials of skinny GEMMs
 * (reduced in fixed order; >= 16 * M * N floats enables the full split). */
int pose6d_gemm_f32(const float *A, int64_t sam, int64_t sak, const float *B, int64_t sbk, int64_t sbn, float *C,
                    int64_t ldc, const float *bias, int32_t M, int32_t N, int32_t K, float alpha, float beta,
                    float *workspace, int64_t ws_floats, void *stream);
/* eval-mode nn.Linear followed by nn.BatchNorm1d (running statistics) [+ ReLU], one
 * launch path (replaces the rot/trans heads' Linear -> BatchNorm1d -> ReLU of
 * pose_net_rgb.py:27-35 / pose_net_rgbd_geometric.py:28-38 at eval):
 *   C[m][n] = act((A W^T + bias)[m][n] - rmean[n]) * (1 / sqrt(rvar[n] + eps)) * gamma[n] + beta[n])
 * with pose6d_gemm_f32 + pose6d_bn1d_fwd(training = 0)'s arithmetic bit for bit.  A [M][sam]
 * (K used), W [N][K] (nn.Linear weight), batch M <= 32. */
int pose6d_gemm_f32_bn_eval(const float *A, int64_t sam, const float *W, float *C, int64_t ldc, const float *bias,
                            int32_t M, int32_t N, int32_t K, const float *gamma, const float *beta,
                            const float *running_mean, const float *running_var, float eps, int32_t relu,
                            float *workspace, int64_t ws_floats, void *stream);
/* nn.Linear parameter gradients in one launch: dW[n][k] (+)= sum_b dy[b*ldy + n] x[b*ldx + k],
 * db[n] (+)= sum_b dy[b*ldy + n] (db may be NULL); dW [N][K] contiguous. */
int pose6d_linear_wgrad(const float *dy, int64_t ldy, const float *x, int64_t ldx, float *dw, float *db, int32_t N,
                        int32_t K, int32_t B, int32_t accumulate, void *stream);
/* db[n] (+)= sum_m dy[m * ldy + n]  (Linear bias gradient; ldy >= N) */
int pose6d_colsum_f32(const float *dy, int64_t ldy, float *db, int32_t M, int32_t N, int32_t accumulate,
                      void *stream);
/* BatchNorm1d (+ReLU) (+Dropout p_drop with a counter-based RNG keyed by the
 * device word *seed xor salt -- a device word so graph replays draw new masks) */
int pose6d_bn1d_fwd(const float *x, float *y, int32_t M, int32_t C, const float *gamma, const float *beta,
                    float *running_mean, float *running_var, int64_t *num_batches, float momentum, float eps,
                    int32_t training, int32_t relu, float p_drop, const uint64_t *seed, uint64_t salt, uint8_t *mask,
                    float *save_mean, float *save_invstd, void *stream);
int pose6d_bn1d_bwd(const float *dy, const float *x, const float *y, int32_t M, int32_t C, const float *gamma,
                    const float *save_mean, const float *save_invstd, int32_t training, int32_t relu, float p_drop,
                    const uint8_t *mask, float *dx, float *dgamma, float *dbeta, int32_t accumulate, void *stream);
/* act: 0 identity, 1 ReLU, 2 GELU (erf); optional dropout */
int pose6d_act_fwd(const float *x, float *y, int64_t n, int32_t act, float p_drop, const uint64_t *seed,
                   uint64_t salt, uint8_t *mask, void *stream);
int pose6d_act_bwd(const float *dy, const float *x, float *dx, int64_t n, int32_t act, float p_drop,
                   const uint8_t *mask, void *stream);

/* ------------------------------------------------------------------------
 * RGB-D fusion (PoseNetRGBD, pose_net_rgbd.py:66-103,118-142), fp32.
 * LayerNorm over rows of D (nn.LayerNorm(D): biased variance, eps), fused with
 * act (0 none, 1 ReLU, 2 exact GELU) and Dropout(p) — the nn.Sequential runs
 * LayerNorm -> GELU -> Dropout of `fusion` / `rot_head` / `trans_head`
 * (pose_net_rgbd.py:72-103) and rgb_norm / depth_norm (:68-69, :127-128, act 0).
 * Row strides (ld*) let the two normalised features land side by side in the
 * (B, 2D) concatenation (:134) without a copy; y2 (optional, contiguous)
 * receives a second copy.  mean / rstd (B each) are saved for the backward.
 * Backward: dy (+ dy2 when non-null: a second gradient flowing into the same
 * output, e.g. the residual and the concatenation branch) -> dx (+= when
 * accumulate_dx), dgamma / dbeta (+= when accumulate).
 * ---------------------------------------------------------------------- */
int pose6d_layernorm_fwd(const float *x, int64_t ldx, float *y, int64_t ldy, float *y2, int32_t B, int32_t D,
                         const float *gamma, const float *beta, float eps, int32_t act, float p_drop,
                         const uint64_t *seed, uint64_t salt, uint8_t *mask, float *mean, float *rstd,
                         void *stream);
int pose6d_layernorm_bwd(const float *dy, int64_t lddy, const float *dy2, int64_t lddy2, const float *x,
                         int64_t ldx, int32_t B, int32_t D, const float *gamma, const float *beta,
                         const float *mean, const float *rstd, int32_t act, float p_drop, const uint8_t *mask,
                         float *dx, int64_t lddx, int32_t accumulate_dx, float *dgamma, float *dbeta,
                         int32_t accumulate, void *stream);

/* CrossModalAttention core (pose_net_rgbd.py:23-35): per sample b,
 *   attn = softmax((q_b k_b^T) * scale), q_b, k_b, v_b = (H, hd) views of rows
 *   of the projections; out_b = dropout(attn) v_b, flattened back to H*hd.
 * probs (B*H*H) keeps the pre-dropout softmax for the backward; mask (B*H*H)
 * the dropout draw.  H <= 16. */
int pose6d_xattn_fwd(const float *q, const float *k, const float *v, float *out, int32_t B, int32_t H, int32_t hd,
                     float scale, float p_drop, const uint64_t *seed, uint64_t salt, float *probs, uint8_t *mask,
                     void *stream);
int pose6d_xattn_bwd(const float *dout, const float *q, const float *k, const float *v, const float *probs,
                     const uint8_t *mask, int32_t B, int32_t H, int32_t hd, float scale, float p_drop, float *dq,
                     float *dk, float *dv, void *stream);

/* ------------------------------------------------------------------------
 * Optimiser — clip_grad_norm_(params, max_norm) + AdamW.step() of the callers
 * (train_rgbd_geometric.py:65,111-112) over one flat fp32 buffer.
 * hp (device) = {lr, beta1, beta2, eps, weight_decay, step t (>= 1; bias
 *                corrections 1 - beta^t computed in-kernel), grad scale (applied to
 *                grad before the norm; 0 reads as 1 — the DDP trainer's 1/world),
 *                max_norm (<= 0: no clipping)}
 * ---------------------------------------------------------------------- */
int pose6d_sumsq_partial(const float *g, int64_t n, float *partials, int32_t nparts, void *stream);
/* the same, and (each optional) step[0] += 1 (the hp[5] counter pose6d_adamw_step reads next) and
 * seed[0] += 1 (the trainer's dropout seed word): the per-step counters without launches of their own */
int pose6d_sumsq_partial_step(const float *g, int64_t n, float *partials, int32_t nparts, float *step,
                              int64_t *seed, void *stream);
int pose6d_adamw_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n,
                      const float *partials, int32_t nparts, const float *hp, float *norm_out, void *stream);
/* The same update (bit-identical), that also writes every conv's packed compute-dtype
 * copies (wp / wt of pose6d_pack_conv_weights) from the updated values: the next
 * forward reads them without a packing launch.  Each conv's OIHW master must be a
 * 16-B aligned slice of param; wp's padding entries are never written (pack once,
 * with pose6d_pack_conv_weights, before the first step and after any write to the
 * masters from outside this call).  descs: device copy of the pack table (n_desc
 * records, see pose6d_pack_conv_weights).  jobs: device copy of the int32 [n_jobs][4]
 * work table pose6d_adamw_packed_jobs builds on the host from a HOST copy of the same
 * table (device addresses compared as integers) -- it returns the job count (cap /
 * jobs may be 0 / NULL to size the table), or a negative error code. */
int pose6d_adamw_packed_jobs(const void *descs, int32_t n_desc, const float *param, int64_t n, int32_t *jobs,
                             int32_t cap);
int pose6d_adamw_step_packed(float *param, const float *grad, float *exp_avg, float *exp_avg_sq,
                             const float *partials, int32_t nparts, const float *hp, float *norm_out, int32_t dtype,
                             const void *descs, const int32_t *jobs, int32_t n_jobs, void *stream);

#ifdef __cplusplus
}
#endif
#endif

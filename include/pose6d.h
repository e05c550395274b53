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

#ifdef __cplusplus
}
#endif
#endif

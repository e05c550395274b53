// Quaternion-normalise heads, pinhole translation heads and PoseLoss fwd/bwd.
// Reference: models/pose_net_*.py (normalise / pinhole), models/pose_loss.py.
// Batch sizes here are tiny (B = 32 per GPU): one launch per op, one lane per row,
// block-level fixed-order reductions for the means (deterministic).
#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr float kNormEps = 1e-12f;   // F.normalize default eps
constexpr float kGeoEps = 1e-8f;     // pose_net_rgb_geometric.py:75

__device__ __forceinline__ float l2(const float* x, int D) {
  float s = 0.f;
  for (int i = 0; i < D; ++i) s = fmaf(x[i], x[i], s);
  return sqrtf(s);
}

__global__ void rownorm_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t B, int D, int mode) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* xr = x + b * D;
  const float n = l2(xr, D);
  const float d = mode == 0 ? fmaxf(n, kNormEps) : n + kGeoEps;
  for (int i = 0; i < D; ++i) y[b * D + i] = xr[i] / d;
}

// mode 0: y = x / max(n, eps);   mode 1: y = x / (n + eps)
__global__ void rownorm_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ dx,
                                   int64_t B, int D, int mode) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float* xr = x + b * D;
  const float* g = dy + b * D;
  const float n = l2(xr, D);
  float xg = 0.f;
  for (int i = 0; i < D; ++i) xg = fmaf(xr[i], g[i], xg);
  if (mode == 0) {
    if (n > kNormEps) {
      // dx = dy / n - x (x.dy) / n^3
      const float inv = 1.0f / n;
      const float c = xg * inv * inv * inv;
      for (int i = 0; i < D; ++i) dx[b * D + i] = g[i] * inv - xr[i] * c;
    } else {
      for (int i = 0; i < D; ++i) dx[b * D + i] = g[i] / kNormEps;   // clamp_min: no grad to n
    }
  } else {
    const float d = n + kGeoEps;
    const float c = n > 0.f ? xg / (d * d * n) : 0.f;                 // norm grad is 0 at 0
    for (int i = 0; i < D; ++i) dx[b * D + i] = g[i] / d - xr[i] * c;
  }
}

__device__ __forceinline__ void load_K(const float* K, int batched, int64_t b, float& fx, float& fy, float& cx,
                                       float& cy) {
  const float* k = batched ? K + 9 * b : K;
  fx = k[0]; cx = k[2]; fy = k[4]; cy = k[5];
}

// pose_net_rgbd_geometric.py:56-85
__global__ void pinhole_depth_kernel(const float* __restrict__ depth, int H, int W, const float* __restrict__ bbox,
                                     const float* __restrict__ K, int Kb, int64_t B, float* __restrict__ t) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= B) return;
  float fx, fy, cx, cy;
  load_K(K, Kb, b, fx, fy, cx, cy);
  const float u = fminf(fmaxf(bbox[2 * b], 0.f), 223.f);
  const float v = fminf(fmaxf(bbox[2 * b + 1], 0.f), 223.f);
  const int ui = min(max((int)u, 0), 223);          // .long() truncation, then clamp
  const int vi = min(max((int)v, 0), 223);
  float z = depth[(int64_t)b * H * W + (int64_t)vi * W + ui];
  z = z > 0.01f ? z : 0.5f;
  z = fminf(fmaxf(z, 0.1f), 2.0f);
  t[3 * b + 0] = (u - cx) * z / fx;
  t[3 * b + 1] = (v - cy) * z / fy;
  t[3 * b + 2] = z;
}

// pose_net_rgb_geometric.py:93-109: x = ((u - cx) * z) / fx
__global__ void pinhole_z_fwd_kernel(const float* __restrict__ z, const float* __restrict__ bbox,
                                     const float* __restrict__ K, int Kb, int64_t B, float* __restrict__ t) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= B) return;
  float fx, fy, cx, cy;
  load_K(K, Kb, b, fx, fy, cx, cy);
  const float zz = z[b];
  t[3 * b + 0] = (bbox[2 * b] - cx) * zz / fx;
  t[3 * b + 1] = (bbox[2 * b + 1] - cy) * zz / fy;
  t[3 * b + 2] = zz;
}

__global__ void pinhole_z_bwd_kernel(const float* __restrict__ dt, const float* __restrict__ bbox,
                                     const float* __restrict__ K, int Kb, int64_t B, float* __restrict__ dz) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= B) return;
  float fx, fy, cx, cy;
  load_K(K, Kb, b, fx, fy, cx, cy);
  dz[b] = dt[3 * b + 0] * (bbox[2 * b] - cx) / fx + dt[3 * b + 1] * (bbox[2 * b + 1] - cy) / fy + dt[3 * b + 2];
}

__device__ __forceinline__ void normalize4(const float* x, float* y, float& n) {
  n = l2(x, 4);
  const float d = fmaxf(n, kNormEps);
  for (int i = 0; i < 4; ++i) y[i] = x[i] / d;
}

// per-row rotation term and its gradient w.r.t. the (unnormalised) prediction
__device__ float rot_term(const float* pr, const float* gr, int mode, float* dpr /*nullable*/, float g) {
  float q1[4], q2[4], n1, n2;
  normalize4(pr, q1, n1);
  normalize4(gr, q2, n2);
  float dq1[4] = {0.f, 0.f, 0.f, 0.f};
  float val;
  if (mode == 0) {
    // pose_loss.py:30-50
    float dot = 0.f;
    for (int i = 0; i < 4; ++i) dot = fmaf(q1[i], q2[i], dot);
    if (dot < 0.f)
      for (int i = 0; i < 4; ++i) q2[i] = -q2[i];
    float u[4], v[4];
    for (int i = 0; i < 4; ++i) { u[i] = q1[i] - q2[i]; v[i] = q1[i] + q2[i]; }
    const float dn = l2(u, 4), sn = l2(v, 4);
    val = 2.0f * atan2f(dn, sn);
    if (dpr) {
      const float den = dn * dn + sn * sn;
      const float gdn = 2.0f * g * sn / den, gsn = -2.0f * g * dn / den;
      for (int i = 0; i < 4; ++i) {
        if (dn > 0.f) dq1[i] += gdn * u[i] / dn;
        if (sn > 0.f) dq1[i] += gsn * v[i] / sn;
      }
    }
  } else {
    // pose_loss.py:52-61
    float dp = 0.f, dm = 0.f;
    for (int i = 0; i < 4; ++i) { dp += fabsf(q1[i] - q2[i]); dm += fabsf(q1[i] + q2[i]); }
    val = fminf(dp, dm);
    if (dpr) {
      const float wp = dp < dm ? g : (dp == dm ? 0.5f * g : 0.f);   // torch.minimum splits ties
      const float wm = dm < dp ? g : (dp == dm ? 0.5f * g : 0.f);
      for (int i = 0; i < 4; ++i) {
        const float a = q1[i] - q2[i], c = q1[i] + q2[i];
        dq1[i] += wp * (a > 0.f ? 1.f : (a < 0.f ? -1.f : 0.f)) + wm * (c > 0.f ? 1.f : (c < 0.f ? -1.f : 0.f));
      }
    }
  }
  if (dpr) {
    // back through F.normalize of the prediction
    if (n1 > kNormEps) {
      float xg = 0.f;
      for (int i = 0; i < 4; ++i) xg = fmaf(pr[i], dq1[i], xg);
      const float inv = 1.0f / n1, c = xg * inv * inv * inv;
      for (int i = 0; i < 4; ++i) dpr[i] = dq1[i] * inv - pr[i] * c;
    } else {
      for (int i = 0; i < 4; ++i) dpr[i] = dq1[i] / kNormEps;
    }
  }
  return val;
}

__global__ __launch_bounds__(kThreads) void pose_loss_fwd_kernel(const float* __restrict__ pr, const float* __restrict__ pt,
                                                                 const float* __restrict__ gr, const float* __restrict__ gt,
                                                                 int64_t B, float wr, float wt, int mode,
                                                                 float* __restrict__ loss) {
  __shared__ float red[2][kThreads / 64];
  float sr = 0.f, st = 0.f;
  for (int64_t b = threadIdx.x; b < B; b += kThreads) {
    sr += rot_term(pr + 4 * b, gr + 4 * b, mode, nullptr, 0.f);
    for (int i = 0; i < 3; ++i) st += fabsf(pt[3 * b + i] - gt[3 * b + i]);
  }
  sr = p6::wave_sum(sr);
  st = p6::wave_sum(st);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = sr; red[1][threadIdx.x >> 6] = st; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, c = 0.f;
    for (int i = 0; i < kThreads / 64; ++i) { a += red[0][i]; c += red[1][i]; }
    loss[0] = wr * (a / (float)B) + wt * (c / (float)(3 * B));
  }
}

__global__ void pose_loss_bwd_kernel(const float* __restrict__ pr, const float* __restrict__ pt,
                                     const float* __restrict__ gr, const float* __restrict__ gt, int64_t B, float wr,
                                     float wt, int mode, const float* __restrict__ dloss, float* __restrict__ grot,
                                     float* __restrict__ gtr) {
  const int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (b >= B) return;
  const float dl = dloss ? dloss[0] : 1.0f;
  rot_term(pr + 4 * b, gr + 4 * b, mode, grot + 4 * b, wr * dl / (float)B);
  const float c = wt * dl / (float)(3 * B);
  for (int i = 0; i < 3; ++i) {
    const float d = pt[3 * b + i] - gt[3 * b + i];
    gtr[3 * b + i] = d > 0.f ? c : (d < 0.f ? -c : 0.f);
  }
}

// The whole quaternion / translation head + PoseLoss forward and backward of the
// RGBD-Geometric training step in ONE single-block launch (it was five launches of
// a few threads each): per sample, exactly the arithmetic of rownorm_fwd,
// pinhole_depth, pose_loss_fwd / _bwd (dloss = 1) and rownorm_bwd above, and the
// loss reduced in pose_loss_fwd's order (rot / trans / loss bit-identical; the
// normalize backward may differ by fp contraction).
__global__ __launch_bounds__(kThreads) void geo_head_loss_kernel(
    const float* __restrict__ raw, const float* __restrict__ depth, int H, int W, const float* __restrict__ bbox,
    const float* __restrict__ K, int Kb, const float* __restrict__ gr, const float* __restrict__ gt, int64_t B,
    float wr, float wt, int mode, float* __restrict__ rot, float* __restrict__ trans, float* __restrict__ loss,
    float* __restrict__ draw, float* __restrict__ dtrans) {
  __shared__ float red[2][kThreads / 64];
  float sr = 0.f, st = 0.f;
  const float grot_scale = wr / (float)B, c = wt / (float)(3 * B);
  for (int64_t b = threadIdx.x; b < B; b += kThreads) {
    // F.normalize(raw) -> rot (pose_net_rgbd_geometric.py:45)
    const float* xr = raw + 4 * b;
    const float n = l2(xr, 4);
    const float d = fmaxf(n, kNormEps);
    float q[4];
    for (int i = 0; i < 4; ++i) { q[i] = xr[i] / d; rot[4 * b + i] = q[i]; }
    // pinhole translation (pose_net_rgbd_geometric.py:56-85)
    float fx, fy, cx, cy;
    load_K(K, Kb, b, fx, fy, cx, cy);
    const float u = fminf(fmaxf(bbox[2 * b], 0.f), 223.f);
    const float v = fminf(fmaxf(bbox[2 * b + 1], 0.f), 223.f);
    const int ui = min(max((int)u, 0), 223);
    const int vi = min(max((int)v, 0), 223);
    float z = depth[(int64_t)b * H * W + (int64_t)vi * W + ui];
    z = z > 0.01f ? z : 0.5f;
    z = fminf(fmaxf(z, 0.1f), 2.0f);
    const float t[3] = {(u - cx) * z / fx, (v - cy) * z / fy, z};
    // PoseLoss forward + backward w.r.t. rot / trans
    float drot[4];
    sr += rot_term(q, gr + 4 * b, mode, drot, grot_scale);
    for (int i = 0; i < 3; ++i) {
      trans[3 * b + i] = t[i];
      st += fabsf(t[i] - gt[3 * b + i]);
      const float e = t[i] - gt[3 * b + i];
      dtrans[3 * b + i] = e > 0.f ? c : (e < 0.f ? -c : 0.f);
    }
    // back through F.normalize (rownorm_bwd mode 0)
    if (n > kNormEps) {
      float xg = 0.f;
      for (int i = 0; i < 4; ++i) xg = fmaf(xr[i], drot[i], xg);
      const float inv = 1.0f / n, cc = xg * inv * inv * inv;
      for (int i = 0; i < 4; ++i) draw[4 * b + i] = drot[i] * inv - xr[i] * cc;
    } else {
      for (int i = 0; i < 4; ++i) draw[4 * b + i] = drot[i] / kNormEps;
    }
  }
  sr = p6::wave_sum(sr);
  st = p6::wave_sum(st);
  if ((threadIdx.x & 63) == 0) { red[0][threadIdx.x >> 6] = sr; red[1][threadIdx.x >> 6] = st; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float a = 0.f, cc = 0.f;
    for (int i = 0; i < kThreads / 64; ++i) { a += red[0][i]; cc += red[1][i]; }
    loss[0] = wr * (a / (float)B) + wt * (cc / (float)(3 * B));
  }
}

inline unsigned nblk(int64_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

}  // namespace

extern "C" int pose6d_rownorm_fwd(const float* x, float* y, int64_t B, int32_t D, int32_t mode, void* stream) {
  P6_CHECK_ARG(D > 0 && (mode == 0 || mode == 1), "pose6d_rownorm_fwd: bad D/mode");
  if (B == 0) return POSE6D_OK;
  rownorm_fwd_kernel<<<nblk(B), kThreads, 0, p6::stream_of(stream)>>>(x, y, B, D, mode);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_rownorm_bwd(const float* x, const float* dy, float* dx, int64_t B, int32_t D, int32_t mode,
                                  void* stream) {
  P6_CHECK_ARG(D > 0 && (mode == 0 || mode == 1), "pose6d_rownorm_bwd: bad D/mode");
  if (B == 0) return POSE6D_OK;
  rownorm_bwd_kernel<<<nblk(B), kThreads, 0, p6::stream_of(stream)>>>(x, dy, dx, B, D, mode);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_pinhole_depth(const float* depth_raw, int32_t H, int32_t W, const float* bbox_center,
                                    const float* K, int32_t K_batched, int64_t B, float* t, void* stream) {
  P6_CHECK_ARG(H >= 224 && W >= 224, "pose6d_pinhole_depth: the reference clamps to 223, needs H,W >= 224 (got %d x %d)",
               H, W);
  if (B == 0) return POSE6D_OK;
  pinhole_depth_kernel<<<nblk(B), kThreads, 0, p6::stream_of(stream)>>>(depth_raw, H, W, bbox_center, K, K_batched, B, t);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_pinhole_z_fwd(const float* z, const float* bbox_center, const float* K, int32_t K_batched,
                                    int64_t B, float* t, void* stream) {
  if (B == 0) return POSE6D_OK;
  pinhole_z_fwd_kernel<<<nblk(B), kThreads, 0, p6::stream_of(stream)>>>(z, bbox_center, K, K_batched, B, t);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_pinhole_z_bwd(const float* dt, const float* bbox_center, const float* K, int32_t K_batched,
                                    int64_t B, float* dz, void* stream) {
  if (B == 0) return POSE6D_OK;
  pinhole_z_bwd_kernel<<<nblk(B), kThreads, 0, p6::stream_of(stream)>>>(dt, bbox_center, K, K_batched, B, dz);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_pose_loss_fwd(const float* pred_rot, const float* pred_trans, const float* gt_rot,
                                    const float* gt_trans, int64_t B, float rot_weight, float trans_weight,
                                    int32_t rot_mode, float* loss, void* stream) {
  P6_CHECK_ARG(rot_mode == 0 || rot_mode == 1, "pose6d_pose_loss_fwd: bad rot_mode %d", rot_mode);
  P6_CHECK_ARG(B > 0, "pose6d_pose_loss_fwd: empty batch (the reference's mean would be NaN)");
  pose_loss_fwd_kernel<<<1, kThreads, 0, p6::stream_of(stream)>>>(pred_rot, pred_trans, gt_rot, gt_trans, B, rot_weight,
                                                                   trans_weight, rot_mode, loss);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_pose_loss_bwd(const float* pred_rot, const float* pred_trans, const float* gt_rot,
                                    const float* gt_trans, int64_t B, float rot_weight, float trans_weight,
                                    int32_t rot_mode, const float* dloss, float* grad_rot, float* grad_trans,
                                    void* stream) {
  P6_CHECK_ARG(rot_mode == 0 || rot_mode == 1, "pose6d_pose_loss_bwd: bad rot_mode %d", rot_mode);
  if (B == 0) return POSE6D_OK;
  pose_loss_bwd_kernel<<<nblk(B), kThreads, 0, p6::stream_of(stream)>>>(pred_rot, pred_trans, gt_rot, gt_trans, B,
                                                                        rot_weight, trans_weight, rot_mode, dloss,
                                                                        grad_rot, grad_trans);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_geo_head_loss(const float* raw, const float* depth_raw, int32_t H, int32_t W,
                                    const float* bbox_center, const float* K, int32_t K_batched, const float* gt_rot,
                                    const float* gt_trans, int64_t B, float rot_weight, float trans_weight,
                                    int32_t rot_mode, float* rot, float* trans, float* loss, float* grad_raw,
                                    float* grad_trans, void* stream) {
  P6_CHECK_ARG(H >= 224 && W >= 224, "pose6d_geo_head_loss: the reference clamps to 223, needs H,W >= 224");
  P6_CHECK_ARG(B > 0 && (rot_mode == 0 || rot_mode == 1), "pose6d_geo_head_loss: bad B / rot_mode");
  geo_head_loss_kernel<<<1, kThreads, 0, p6::stream_of(stream)>>>(raw, depth_raw, H, W, bbox_center, K, K_batched,
                                                                  gt_rot, gt_trans, B, rot_weight, trans_weight,
                                                                  rot_mode, rot, trans, loss, grad_raw, grad_trans);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

// RGB-D fusion kernels of PoseNetRGBD (pose_net_rgbd.py): LayerNorm (+ exact GELU
// / ReLU + Dropout) forward/backward, and the per-sample cross-modal attention
// core of CrossModalAttention (pose_net_rgbd.py:8-35):
//   q, k, v : (B, H, hd) rows of the q/k/v projections (H = 8, hd = 256)
//   attn    = softmax((q k^T) * scale) over the depth heads      (B, H, H)
//   out     = dropout(attn) v                                     (B, H * hd)
// Batch 32 x 2048-wide rows: everything here is a few hundred KB, so these are
// latency kernels (one workgroup per sample row), not bandwidth kernels; the
// projections themselves run on pose6d_gemm_f32.
#include "common.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float act_apply(float z, int act) {
  if (act == 1) return fmaxf(z, 0.f);
  if (act == 2) return 0.5f * z * (1.0f + erff(z * 0.70710678118654752f));
  return z;
}

__device__ __forceinline__ float act_grad(float z, int act) {
  if (act == 1) return z > 0.f ? 1.f : 0.f;
  if (act == 2) {
    const float cdf = 0.5f * (1.0f + erff(z * 0.70710678118654752f));
    const float pdf = 0.39894228040143268f * expf(-0.5f * z * z);
    return cdf + z * pdf;
  }
  return 1.f;
}

// one workgroup per row: mean, biased variance (two passes over the row), then
// y = drop(act(gamma * (x - mean) * rstd + beta)); y2 (contiguous) gets a copy
__global__ __launch_bounds__(kThreads) void ln_fwd_kernel(const float* __restrict__ x, int64_t ldx,
                                                          float* __restrict__ y, int64_t ldy, float* __restrict__ y2,
                                                          int D, const float* __restrict__ gamma,
                                                          const float* __restrict__ beta, float eps, int act,
                                                          float p_drop, const uint64_t* __restrict__ seedp,
                                                          uint64_t salt, uint8_t* __restrict__ mask,
                                                          float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  __shared__ float red[kThreads / 64];
  const int b = blockIdx.x;
  const float* xr = x + b * ldx;
  float s = 0.f;
  for (int d = threadIdx.x; d < D; d += kThreads) s += xr[d];
  const float mean = p6::block_sum<kThreads>(s, red) / (float)D;
  float q = 0.f;
  for (int d = threadIdx.x; d < D; d += kThreads) {
    const float t = xr[d] - mean;
    q = fmaf(t, t, q);
  }
  const float var = p6::block_sum<kThreads>(q, red) / (float)D;
  const float rstd = 1.0f / sqrtf(var + eps);
  if (threadIdx.x == 0) {
    mean_out[b] = mean;
    rstd_out[b] = rstd;
  }
  const float keep_scale = p_drop > 0.f ? 1.0f / (1.0f - p_drop) : 1.0f;
  for (int d = threadIdx.x; d < D; d += kThreads) {
    float v = act_apply((xr[d] - mean) * rstd * gamma[d] + beta[d], act);
    if (p_drop > 0.f) {
      const int64_t o = (int64_t)b * D + d;
      const bool keep = p6::uniform01(seedp[0] ^ salt, (uint64_t)o) >= p_drop;
      mask[o] = keep;
      v = keep ? v * keep_scale : 0.f;
    }
    y[b * ldy + d] = v;
    if (y2) y2[(int64_t)b * D + d] = v;
  }
}

// gradient reaching the LayerNorm output z (before act / dropout): (dy + dy2) -> dz
__device__ __forceinline__ float ln_dz(const float* __restrict__ dy, int64_t lddy, const float* __restrict__ dy2,
                                       int64_t lddy2, int b, int d, int D, float z, int act, float p_drop,
                                       const uint8_t* __restrict__ mask) {
  float g = dy[b * lddy + d];
  if (dy2) g += dy2[b * lddy2 + d];
  if (p_drop > 0.f) g = mask[(int64_t)b * D + d] ? g / (1.0f - p_drop) : 0.f;
  return act ? g * act_grad(z, act) : g;
}

// dx = rstd * (dxh - mean(dxh) - xh * mean(dxh * xh)),  dxh = dz * gamma
__global__ __launch_bounds__(kThreads) void ln_bwd_dx_kernel(
    const float* __restrict__ dy, int64_t lddy, const float* __restrict__ dy2, int64_t lddy2,
    const float* __restrict__ x, int64_t ldx, int D, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ mean_in, const float* __restrict__ rstd_in, int act, float p_drop,
    const uint8_t* __restrict__ mask, float* __restrict__ dx, int64_t lddx, int accumulate_dx) {
  __shared__ float red[kThreads / 64];
  const int b = blockIdx.x;
  const float mean = mean_in[b], rstd = rstd_in[b];
  const float* xr = x + b * ldx;
  float s1 = 0.f, s2 = 0.f;
  for (int d = threadIdx.x; d < D; d += kThreads) {
    const float xh = (xr[d] - mean) * rstd;
    const float dxh = ln_dz(dy, lddy, dy2, lddy2, b, d, D, xh * gamma[d] + beta[d], act, p_drop, mask) * gamma[d];
    s1 += dxh;
    s2 = fmaf(dxh, xh, s2);
  }
  const float m1 = p6::block_sum<kThreads>(s1, red) / (float)D;
  const float m2 = p6::block_sum<kThreads>(s2, red) / (float)D;
  for (int d = threadIdx.x; d < D; d += kThreads) {
    const float xh = (xr[d] - mean) * rstd;
    const float dxh = ln_dz(dy, lddy, dy2, lddy2, b, d, D, xh * gamma[d] + beta[d], act, p_drop, mask) * gamma[d];
    const float v = rstd * (dxh - m1 - xh * m2);
    float* o = dx + b * lddx + d;
    *o = accumulate_dx ? *o + v : v;
  }
}

// dgamma[d] = sum_b dz * xh, dbeta[d] = sum_b dz (one thread per column, fixed order)
__global__ __launch_bounds__(kThreads) void ln_bwd_param_kernel(
    const float* __restrict__ dy, int64_t lddy, const float* __restrict__ dy2, int64_t lddy2,
    const float* __restrict__ x, int64_t ldx, int B, int D, const float* __restrict__ gamma,
    const float* __restrict__ beta, const float* __restrict__ mean_in, const float* __restrict__ rstd_in, int act,
    float p_drop, const uint8_t* __restrict__ mask, float* __restrict__ dgamma, float* __restrict__ dbeta,
    int accumulate) {
  const int d = blockIdx.x * kThreads + threadIdx.x;
  if (d >= D) return;
  const float g = gamma[d], bt = beta[d];
  float sg = 0.f, sb = 0.f;
  for (int b = 0; b < B; ++b) {
    const float xh = (x[b * ldx + d] - mean_in[b]) * rstd_in[b];
    const float dz = ln_dz(dy, lddy, dy2, lddy2, b, d, D, xh * g + bt, act, p_drop, mask);
    sg = fmaf(dz, xh, sg);
    sb += dz;
  }
  dgamma[d] = accumulate ? dgamma[d] + sg : sg;
  dbeta[d] = accumulate ? dbeta[d] + sb : sb;
}

// ---- cross-modal attention core ------------------------------------------
constexpr int kMaxHeads = 16;

// one workgroup per sample: S = q k^T * scale (H x H dot products of length hd,
// one wave per product), row softmax, dropout, out = P v
__global__ __launch_bounds__(kThreads) void xattn_fwd_kernel(const float* __restrict__ q,
                                                             const float* __restrict__ k,
                                                             const float* __restrict__ v, float* __restrict__ out,
                                                             int H, int hd, float scale, float p_drop,
                                                             const uint64_t* __restrict__ seedp, uint64_t salt,
                                                             float* __restrict__ probs, uint8_t* __restrict__ mask) {
  __shared__ float S[kMaxHeads * kMaxHeads];
  __shared__ float P[kMaxHeads * kMaxHeads];
  const int b = blockIdx.x, D = H * hd;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* qb = q + (int64_t)b * D;
  const float* kb = k + (int64_t)b * D;
  const float* vb = v + (int64_t)b * D;
  for (int p = wave; p < H * H; p += kThreads / 64) {
    const int i = p / H, j = p - i * H;
    float s = 0.f;
    for (int d = lane; d < hd; d += 64) s = fmaf(qb[i * hd + d], kb[j * hd + d], s);
    s = p6::wave_sum(s);
    if (lane == 0) S[p] = s * scale;
  }
  __syncthreads();
  if (threadIdx.x < H) {
    const int i = threadIdx.x;
    float mx = -INFINITY;
    for (int j = 0; j < H; ++j) mx = fmaxf(mx, S[i * H + j]);
    float den = 0.f;
    for (int j = 0; j < H; ++j) den += expf(S[i * H + j] - mx);
    const float keep_scale = p_drop > 0.f ? 1.0f / (1.0f - p_drop) : 1.0f;
    for (int j = 0; j < H; ++j) {
      const int64_t o = (int64_t)b * H * H + i * H + j;
      const float a = expf(S[i * H + j] - mx) / den;
      probs[o] = a;
      float pv = a;
      if (p_drop > 0.f) {
        const bool keep = p6::uniform01(seedp[0] ^ salt, (uint64_t)o) >= p_drop;
        mask[o] = keep;
        pv = keep ? a * keep_scale : 0.f;
      }
      P[i * H + j] = pv;
    }
  }
  __syncthreads();
  for (int e = threadIdx.x; e < D; e += kThreads) {
    const int i = e / hd, d = e - i * hd;
    float acc = 0.f;
    for (int j = 0; j < H; ++j) acc = fmaf(P[i * H + j], vb[j * hd + d], acc);
    out[(int64_t)b * D + e] = acc;
  }
}

// backward: dP = dO v^T, dV = P^T dO, dA = dropout-bwd(dP), dS = A * (dA - rowsum(A dA)),
// dq = scale * dS k, dk = scale * dS^T q
__global__ __launch_bounds__(kThreads) void xattn_bwd_kernel(
    const float* __restrict__ dout, const float* __restrict__ q, const float* __restrict__ k,
    const float* __restrict__ v, const float* __restrict__ probs, const uint8_t* __restrict__ mask, int H, int hd,
    float scale, float p_drop, float* __restrict__ dq, float* __restrict__ dk, float* __restrict__ dv) {
  __shared__ float P[kMaxHeads * kMaxHeads];
  __shared__ float dS[kMaxHeads * kMaxHeads];
  const int b = blockIdx.x, D = H * hd;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const float* ob = dout + (int64_t)b * D;
  const float* vb = v + (int64_t)b * D;
  const float keep_scale = p_drop > 0.f ? 1.0f / (1.0f - p_drop) : 1.0f;
  for (int p = wave; p < H * H; p += kThreads / 64) {
    const int i = p / H, j = p - i * H;
    float s = 0.f;
    for (int d = lane; d < hd; d += 64) s = fmaf(ob[i * hd + d], vb[j * hd + d], s);
    s = p6::wave_sum(s);
    if (lane == 0) {
      const int64_t o = (int64_t)b * H * H + p;
      const bool keep = p_drop > 0.f ? mask[o] != 0 : true;
      dS[p] = keep ? s * keep_scale : 0.f;                 // dA
      P[p] = keep ? probs[o] * keep_scale : 0.f;           // dropped probabilities (forward's P)
    }
  }
  __syncthreads();
  if (threadIdx.x < H) {
    const int i = threadIdx.x;
    const float* A = probs + (int64_t)b * H * H + i * H;
    float r = 0.f;
    for (int j = 0; j < H; ++j) r = fmaf(A[j], dS[i * H + j], r);
    for (int j = 0; j < H; ++j) dS[i * H + j] = A[j] * (dS[i * H + j] - r) * scale;
  }
  __syncthreads();
  const float* qb = q + (int64_t)b * D;
  const float* kb = k + (int64_t)b * D;
  for (int e = threadIdx.x; e < D; e += kThreads) {
    const int i = e / hd, d = e - i * hd;   // head row i of q / k / v
    float gq = 0.f, gk = 0.f, gv = 0.f;
    for (int j = 0; j < H; ++j) {
      gq = fmaf(dS[i * H + j], kb[j * hd + d], gq);
      gk = fmaf(dS[j * H + i], qb[j * hd + d], gk);
      gv = fmaf(P[j * H + i], ob[j * hd + d], gv);
    }
    dq[(int64_t)b * D + e] = gq;
    dk[(int64_t)b * D + e] = gk;
    dv[(int64_t)b * D + e] = gv;
  }
}

}  // namespace

extern "C" int pose6d_layernorm_fwd(const float* x, int64_t ldx, float* y, int64_t ldy, float* y2, int32_t B,
                                    int32_t D, const float* gamma, const float* beta, float eps, int32_t act,
                                    float p_drop, const uint64_t* seed, uint64_t salt, uint8_t* mask, float* mean,
                                    float* rstd, void* stream) {
  P6_CHECK_ARG(B >= 0 && D > 0 && ldx >= D && ldy >= D, "pose6d_layernorm_fwd: bad shape");
  P6_CHECK_ARG(act >= 0 && act <= 2, "pose6d_layernorm_fwd: act must be 0 (none), 1 (ReLU) or 2 (GELU)");
  P6_CHECK_ARG(p_drop >= 0.f && p_drop < 1.f, "pose6d_layernorm_fwd: p_drop out of [0, 1)");
  P6_CHECK_ARG(p_drop == 0.f || (seed && mask), "pose6d_layernorm_fwd: dropout needs seed and mask");
  if (B == 0) return POSE6D_OK;
  ln_fwd_kernel<<<B, kThreads, 0, p6::stream_of(stream)>>>(x, ldx, y, ldy, y2, D, gamma, beta, eps, act, p_drop,
                                                           seed, salt, mask, mean, rstd);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_layernorm_bwd(const float* dy, int64_t lddy, const float* dy2, int64_t lddy2, const float* x,
                                    int64_t ldx, int32_t B, int32_t D, const float* gamma, const float* beta,
                                    const float* mean, const float* rstd, int32_t act, float p_drop,
                                    const uint8_t* mask, float* dx, int64_t lddx, int32_t accumulate_dx,
                                    float* dgamma, float* dbeta, int32_t accumulate, void* stream) {
  P6_CHECK_ARG(B >= 0 && D > 0 && ldx >= D && lddy >= D, "pose6d_layernorm_bwd: bad shape");
  P6_CHECK_ARG(act >= 0 && act <= 2, "pose6d_layernorm_bwd: bad act");
  P6_CHECK_ARG(p_drop == 0.f || mask, "pose6d_layernorm_bwd: dropout needs the forward mask");
  if (B == 0) return POSE6D_OK;
  hipStream_t s = p6::stream_of(stream);
  if (dgamma && dbeta) {
    ln_bwd_param_kernel<<<p6::ceil_div(D, kThreads), kThreads, 0, s>>>(dy, lddy, dy2, lddy2, x, ldx, B, D, gamma,
                                                                       beta, mean, rstd, act, p_drop, mask, dgamma,
                                                                       dbeta, accumulate);
    P6_LAUNCH_CHECK();
  }
  if (dx) {
    P6_CHECK_ARG(lddx >= D, "pose6d_layernorm_bwd: bad lddx");
    ln_bwd_dx_kernel<<<B, kThreads, 0, s>>>(dy, lddy, dy2, lddy2, x, ldx, D, gamma, beta, mean, rstd, act, p_drop,
                                            mask, dx, lddx, accumulate_dx);
    P6_LAUNCH_CHECK();
  }
  return POSE6D_OK;
}

extern "C" int pose6d_xattn_fwd(const float* q, const float* k, const float* v, float* out, int32_t B, int32_t H,
                                int32_t hd, float scale, float p_drop, const uint64_t* seed, uint64_t salt,
                                float* probs, uint8_t* mask, void* stream) {
  P6_CHECK_ARG(B >= 0 && H > 0 && H <= kMaxHeads && hd > 0, "pose6d_xattn_fwd: need 0 < H <= %d", kMaxHeads);
  P6_CHECK_ARG(p_drop >= 0.f && p_drop < 1.f, "pose6d_xattn_fwd: p_drop out of [0, 1)");
  P6_CHECK_ARG(p_drop == 0.f || (seed && mask), "pose6d_xattn_fwd: dropout needs seed and mask");
  P6_CHECK_ARG(probs != nullptr, "pose6d_xattn_fwd: probs buffer required");
  if (B == 0) return POSE6D_OK;
  xattn_fwd_kernel<<<B, kThreads, 0, p6::stream_of(stream)>>>(q, k, v, out, H, hd, scale, p_drop, seed, salt, probs,
                                                              mask);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_xattn_bwd(const float* dout, const float* q, const float* k, const float* v,
                                const float* probs, const uint8_t* mask, int32_t B, int32_t H, int32_t hd,
                                float scale, float p_drop, float* dq, float* dk, float* dv, void* stream) {
  P6_CHECK_ARG(B >= 0 && H > 0 && H <= kMaxHeads && hd > 0, "pose6d_xattn_bwd: need 0 < H <= %d", kMaxHeads);
  P6_CHECK_ARG(p_drop == 0.f || mask, "pose6d_xattn_bwd: dropout needs the forward mask");
  if (B == 0) return POSE6D_OK;
  xattn_bwd_kernel<<<B, kThreads, 0, p6::stream_of(stream)>>>(dout, q, k, v, probs, mask, H, hd, scale, p_drop, dq,
                                                              dk, dv);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

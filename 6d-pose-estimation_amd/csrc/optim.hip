// Gradient clipping + AdamW over one flat fp32 parameter buffer.
// Replaces the callers' torch.nn.utils.clip_grad_norm_(params, 1.0) and
// optim.AdamW(lr=1e-4, weight_decay=1e-4).step() (train_rgbd_geometric.py:65,111-112)
// with two launches for all 26 M parameters:
//   pose6d_sumsq_partial : fixed grid of NPART blocks, per-block sum of g^2 (fp32)
//   pose6d_adamw_step    : every block re-reduces the NPART partials (4 KB, L2-hot)
//                          in fixed order -> same norm everywhere, deterministic;
//                          clip coefficient min(1, max_norm/(norm+1e-6)); AdamW
//                          update in torch's operation order.
// Hyper-parameters come from a device array (graph replays pick up lr changes):
//   hp = {lr, beta1, beta2, eps, weight_decay, step (t >= 1), grad scale, max_norm}
// grad scale (0 reads as 1) multiplies the gradient before clipping: the DDP trainer
// sets 1/world so the summed all-reduce result is averaged here instead of in a pass
// of its own (exact for power-of-two world sizes: the norm scales by the same 2^-k).
#include "common.h"

namespace {

constexpr int kThreads = 256;

// `step` / `seed` (optional): the trainer's device step counter (hp[5]) and dropout
// seed word, advanced here so the captured step needs no launches of its own for them
__global__ __launch_bounds__(kThreads) void sumsq_kernel(const float* __restrict__ g, int64_t n,
                                                         float* __restrict__ part, float* __restrict__ step,
                                                         int64_t* __restrict__ seed) {
  __shared__ float red[kThreads / 64];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (step) step[0] += 1.f;
    if (seed) seed[0] += 1;
  }
  float s = 0.f;
  const int64_t n4 = n / 4;
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < n4; i += (int64_t)gridDim.x * kThreads) {
    const float4 v = g4[i];
    s = fmaf(v.x, v.x, s); s = fmaf(v.y, v.y, s); s = fmaf(v.z, v.z, s); s = fmaf(v.w, v.w, s);
  }
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)kThreads + threadIdx.x; i < n; i += (int64_t)gridDim.x * kThreads)
    s = fmaf(g[i], g[i], s);
  s = p6::wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(kThreads) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                         const float* __restrict__ part, int nparts,
                                                         const float* __restrict__ hp, float* __restrict__ norm_out) {
  __shared__ float s_coef;
  __shared__ double red[kThreads / 64];
  const float lr = hp[0], b1 = hp[1], b2 = hp[2], eps = hp[3], wd = hp[4], max_norm = hp[7];
  const float gs = hp[6] != 0.f ? hp[6] : 1.f;
  // bias corrections from the device step counter hp[5] (incremented in-stream, so
  // a captured step replays with the right t): 1 - beta^t as torch computes it
  const double t = (double)hp[5];
  const float bc1 = (float)(1.0 - pow((double)b1, t)), bc2 = (float)(1.0 - pow((double)b2, t));
  if (max_norm > 0.f) {
    double s = 0.0;
    for (int i = threadIdx.x; i < nparts; i += kThreads) s += (double)part[i];
    s = p6::wave_sum(s);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
      const float norm = gs * (float)sqrt(red[0] + red[1] + red[2] + red[3]);
      const float c = max_norm / (norm + 1e-6f);
      s_coef = c < 1.f ? c : 1.f;
      if (blockIdx.x == 0 && norm_out) norm_out[0] = norm;
    }
    __syncthreads();
  } else if (threadIdx.x == 0) {
    s_coef = 1.f;
  }
  // (the clip coefficient applies to the scaled gradient; fold both into one factor)
  __syncthreads();
  const float coef = s_coef * gs;
  const float step_size = lr / bc1;
  const float bc2s = sqrtf(bc2);
  const float decay = 1.f - lr * wd;
  auto upd = [&](float& pi, float& mi, float& vi, float graw) {
    const float gi = graw * coef;
    pi = pi * decay;
    mi = mi + (1.f - b1) * (gi - mi);                 // exp_avg.lerp_(grad, 1 - beta1)
    vi = vi * b2 + (1.f - b2) * gi * gi;              // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
    const float denom = sqrtf(vi) / bc2s + eps;
    pi = pi - step_size * (mi / denom);
  };
  // float4 chunks, U per trip with every load of the trip issued before the first
  // store: a load issued after a store is waited for with vmcnt(0), i.e. behind that
  // store's acknowledgement (one memory round trip per trip instead of per element)
  constexpr int U = 4;
  const int64_t n4 = n / 4, stride = (int64_t)gridDim.x * kThreads;
  float4* p4 = reinterpret_cast<float4*>(p);
  float4* m4 = reinterpret_cast<float4*>(m);
  float4* v4 = reinterpret_cast<float4*>(v);
  const float4* g4 = reinterpret_cast<const float4*>(g);
  for (int64_t i0 = blockIdx.x * (int64_t)kThreads + threadIdx.x; i0 < n4; i0 += U * stride) {
    float4 pv[U], mv[U], vv[U], gv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride < n4 ? i0 + u * stride : i0;
      gv[u] = g4[i]; pv[u] = p4[i]; mv[u] = m4[i]; vv[u] = v4[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      upd(pv[u].x, mv[u].x, vv[u].x, gv[u].x);
      upd(pv[u].y, mv[u].y, vv[u].y, gv[u].y);
      upd(pv[u].z, mv[u].z, vv[u].z, gv[u].z);
      upd(pv[u].w, mv[u].w, vv[u].w, gv[u].w);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t i = i0 + u * stride;
      if (i < n4) { p4[i] = pv[u]; m4[i] = mv[u]; v4[i] = vv[u]; }
    }
  }
  for (int64_t i = n4 * 4 + blockIdx.x * (int64_t)kThreads + threadIdx.x; i < n; i += stride) {
    float pi = p[i], mi = m[i], vi = v[i];
    upd(pi, mi, vi, g[i]);
    p[i] = pi; m[i] = mi; v[i] = vi;
  }
}

}  // namespace

extern "C" int pose6d_sumsq_partial(const float* g, int64_t n, float* partials, int32_t nparts, void* stream) {
  P6_CHECK_ARG(nparts > 0 && nparts <= 65535, "pose6d_sumsq_partial: bad nparts");
  sumsq_kernel<<<nparts, kThreads, 0, p6::stream_of(stream)>>>(g, n, partials, nullptr, nullptr);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_sumsq_partial_step(const float* g, int64_t n, float* partials, int32_t nparts, float* step,
                                         int64_t* seed, void* stream) {
  P6_CHECK_ARG(nparts > 0 && nparts <= 65535, "pose6d_sumsq_partial_step: bad nparts");
  sumsq_kernel<<<nparts, kThreads, 0, p6::stream_of(stream)>>>(g, n, partials, step, seed);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_adamw_step(float* param, const float* grad, float* exp_avg, float* exp_avg_sq, int64_t n,
                                 const float* partials, int32_t nparts, const float* hp, float* norm_out,
                                 void* stream) {
  if (n == 0) return POSE6D_OK;
  P6_CHECK_ARG(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
               "pose6d_adamw_step: buffers must be 16-byte aligned");
  // one trip of U = 4 float4 per thread for up to 64 M parameters (each block re-reads
  // the clip partials: a few KiB, L2-resident)
  int64_t blocks = (n + kThreads * 16 - 1) / (kThreads * 16);
  if (blocks > 16384) blocks = 16384;
  adamw_kernel<<<(unsigned)blocks, kThreads, 0, p6::stream_of(stream)>>>(param, grad, exp_avg, exp_avg_sq, n, partials,
                                                                        nparts, hp, norm_out);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

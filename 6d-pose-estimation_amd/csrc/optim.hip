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
#include <algorithm>
#include <utility>
#include <vector>

#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kJob = 4096;   // parameters per block of adamw_packed_kernel
using p6::PackDesc;

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

// The clip coefficient and the per-element AdamW update, shared by both update
// kernels (so the packed-output variant is bit-identical to adamw_kernel).  Every
// block re-reduces the NPART norm partials in fixed order: the same coefficient
// everywhere.  Contains barriers: construct from uniform control flow.
struct AdamW {
  float coef, step_size, bc2s, decay, b1, b2, eps;
  __device__ __forceinline__ AdamW(const float* __restrict__ part, int nparts, const float* __restrict__ hp,
                                   float* __restrict__ norm_out) {
#pragma clang fp contract(off)
    __shared__ float s_coef;
    __shared__ double red[kThreads / 64];
    const float lr = hp[0], wd = hp[4], max_norm = hp[7];
    b1 = hp[1]; b2 = hp[2]; eps = hp[3];
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
    coef = s_coef * gs;
    step_size = lr / bc1;
    bc2s = sqrtf(bc2);
    decay = 1.f - lr * wd;
  }
  // contraction off: every kernel that inlines this rounds identically (left to the
  // compiler, fma formation followed each kernel's own packed-math vectorisation)
  __device__ __forceinline__ void operator()(float& pi, float& mi, float& vi, float graw) const {
#pragma clang fp contract(off)
    const float gi = graw * coef;
    pi = pi * decay;
    mi = mi + (1.f - b1) * (gi - mi);                 // exp_avg.lerp_(grad, 1 - beta1)
    vi = vi * b2 + (1.f - b2) * gi * gi;              // exp_avg_sq.mul_(b2).addcmul_(g, g, 1 - b2)
    const float denom = sqrtf(vi) / bc2s + eps;
    pi = pi - step_size * (mi / denom);
  }
  __device__ __forceinline__ void operator()(float4& p, float4& m, float4& v, const float4& g) const {
    (*this)(p.x, m.x, v.x, g.x);
    (*this)(p.y, m.y, v.y, g.y);
    (*this)(p.z, m.z, v.z, g.z);
    (*this)(p.w, m.w, v.w, g.w);
  }
};

__global__ __launch_bounds__(kThreads) void adamw_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                         float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                         const float* __restrict__ part, int nparts,
                                                         const float* __restrict__ hp, float* __restrict__ norm_out) {
  const AdamW upd(part, nparts, hp, norm_out);
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
    for (int u = 0; u < U; ++u) upd(pv[u], mv[u], vv[u], gv[u]);
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

// Input channels per conv tile of adamw_packed_kernel: 64 x 64 tiles for 1x1 filters,
// else up to 8 channels x all taps (<= kTileCols columns of the [O][I*KH*KW] master),
// so that each (row, tap) of the tile is one run of channels in wp.
constexpr int kTileCols = 128;
__host__ __device__ constexpr int tile_channels(int taps) {
  return taps == 1 ? 64 : (kTileCols / taps >= 8 ? 8 : (kTileCols / taps > 0 ? kTileCols / taps : 1));
}

// AdamW that also writes the compute-dtype copies the convolutions read (the
// pose6d_pack_conv_weights layouts), so no launch re-reads the updated masters.
// One job per block, from a host-built table (int4 records):
//   {0, a, b, -}   plain update of p[a, b)  (<= 4096 parameters)
//   {1, k, o0, c0} conv descs[k]: filter rows o in [o0, o0+64) x input channels
//                  [c0, c0+cw) with every tap, i.e. the contiguous columns
//                  [c0*taps, (c0+cw)*taps) of the master viewed [O][I*KH*KW]:
//                  update those masters, then write wp[o][tap*Ip + ci] (1x1: straight
//                  from the registers; KxK: one cw-channel run per (o, tap) out of an
//                  LDS copy of the tile) and wt[(ci, tap)][o] (8 filters per store,
//                  transposed through the same LDS copy).  wp's channel / K padding is
//                  never written (zero since the initial pack).
template <typename T>
__device__ __forceinline__ void store_t(T* q, float x) { *q = p6::from_f<T>(x); }

// eight consecutive T from eight floats (16-B bf16 store, two float4 for fp32)
template <typename T>
__device__ __forceinline__ void store8(T* q, const float (&x)[8]) {
  if constexpr (sizeof(T) == 2) {
    const bf16x8 h = {(bf16)x[0], (bf16)x[1], (bf16)x[2], (bf16)x[3],
                      (bf16)x[4], (bf16)x[5], (bf16)x[6], (bf16)x[7]};
    *reinterpret_cast<bf16x8*>(q) = h;
  } else {
    reinterpret_cast<float4*>(q)[0] = make_float4(x[0], x[1], x[2], x[3]);
    reinterpret_cast<float4*>(q)[1] = make_float4(x[4], x[5], x[6], x[7]);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void adamw_packed_kernel(float* __restrict__ p, const float* __restrict__ g,
                                                                float* __restrict__ m, float* __restrict__ v,
                                                                const float* __restrict__ part, int nparts,
                                                                const float* __restrict__ hp,
                                                                float* __restrict__ norm_out,
                                                                const PackDesc* __restrict__ descs,
                                                                const int4* __restrict__ jobs) {
  __shared__ float tile[64 * (kTileCols + 1)];
  const AdamW upd(part, nparts, hp, norm_out);
  const int4 job = jobs[blockIdx.x];
  const int tid = threadIdx.x;
  if (job.x == 0) {
    const int a = job.y, b = job.z;
    if (((a | b) & 3) == 0) {   // float4 path: every load before the first store
      float4 pv[4], mv[4], vv[4], gv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        int i = a + (tid + u * kThreads) * 4;
        i = i < b ? i : a;
        gv[u] = *reinterpret_cast<const float4*>(g + i);
        pv[u] = *reinterpret_cast<const float4*>(p + i);
        mv[u] = *reinterpret_cast<const float4*>(m + i);
        vv[u] = *reinterpret_cast<const float4*>(v + i);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) upd(pv[u], mv[u], vv[u], gv[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = a + (tid + u * kThreads) * 4;
        if (i < b) {
          *reinterpret_cast<float4*>(p + i) = pv[u];
          *reinterpret_cast<float4*>(m + i) = mv[u];
          *reinterpret_cast<float4*>(v + i) = vv[u];
        }
      }
    } else {
      for (int i = a + tid; i < b; i += kThreads) {
        float pi = p[i], mi = m[i], vi = v[i];
        upd(pi, mi, vi, g[i]);
        p[i] = pi; m[i] = mi; v[i] = vi;
      }
    }
    return;
  }
  const PackDesc d = descs[job.y];
  const int o0 = job.z, c0 = job.w;
  const int taps = d.KH * d.KW, R = d.I * taps;
  const int cw = min(tile_channels(taps), d.I - c0), W = cw * taps, r0 = c0 * taps;
  const int rows = min(64, d.O - o0), LD = W + 1;
  const int64_t base = d.w - p + (int64_t)o0 * R + r0;   // the tile's first master in the flat buffer
  T* wp = reinterpret_cast<T*>(d.wp) + (int64_t)o0 * d.Kpad;
  if ((W & 3) == 0 && (R & 3) == 0) {
    // float4 chunks, four per thread per trip, every load of a trip before its first store
    const int w4 = W >> 2, nq = rows * w4;
    for (int q0 = 0; q0 < nq; q0 += 4 * kThreads) {
      float4 pv[4], mv[4], vv[4], gv[4];
      int64_t iv[4];
      int tv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int q = q0 + tid + u * kThreads;
        const int row = q / w4, col = (q - row * w4) * 4;
        tv[u] = q < nq ? row * LD + col : -1;
        iv[u] = q < nq ? base + (int64_t)row * R + col : base;
        gv[u] = *reinterpret_cast<const float4*>(g + iv[u]);
        pv[u] = *reinterpret_cast<const float4*>(p + iv[u]);
        mv[u] = *reinterpret_cast<const float4*>(m + iv[u]);
        vv[u] = *reinterpret_cast<const float4*>(v + iv[u]);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) upd(pv[u], mv[u], vv[u], gv[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (tv[u] < 0) continue;
        *reinterpret_cast<float4*>(p + iv[u]) = pv[u];
        *reinterpret_cast<float4*>(m + iv[u]) = mv[u];
        *reinterpret_cast<float4*>(v + iv[u]) = vv[u];
        const int row = tv[u] / LD, col = tv[u] - row * LD;
        if (taps == 1) {   // k == ci: four adjacent packed entries
          T* dst = wp + (int64_t)row * d.Kpad + c0 + col;
          if constexpr (sizeof(T) == 2) {
            const bf16x4 h = {(bf16)pv[u].x, (bf16)pv[u].y, (bf16)pv[u].z, (bf16)pv[u].w};
            *reinterpret_cast<bf16x4*>(dst) = h;
          } else {
            *reinterpret_cast<float4*>(dst) = pv[u];
          }
        }
        float* t = tile + tv[u];
        t[0] = pv[u].x; t[1] = pv[u].y; t[2] = pv[u].z; t[3] = pv[u].w;
      }
    }
  } else {
    for (int e = tid; e < rows * W; e += kThreads) {
      const int row = e / W, col = e - row * W;
      const int64_t i = base + (int64_t)row * R + col;
      float pi = p[i], mi = m[i], vi = v[i];
      upd(pi, mi, vi, g[i]);
      p[i] = pi; m[i] = mi; v[i] = vi;
      if (taps == 1) store_t(wp + (int64_t)row * d.Kpad + c0 + col, pi);
      tile[row * LD + col] = pi;
    }
  }
  if (taps == 1 && d.wt == nullptr) return;
  __syncthreads();
#ifndef POSE6D_ADAMW_NOWP   // (timing-only builds: tools/adamw_bench.py)
#define POSE6D_ADAMW_NOWP 0
#endif
#ifndef POSE6D_ADAMW_NOWT
#define POSE6D_ADAMW_NOWT 0
#endif
  if (taps > 1 && !POSE6D_ADAMW_NOWP) {
    // wp[o][ptap*Ip + c0 + ci], ci < cw: column ci*taps + tap of the tile, at packed tap
    // ptap = kh*KWp + kw + KWp - KW (KWp = KW but for the row-tap stems)
    const int kwp = d.KWp > 0 ? d.KWp : d.KW;
    for (int it = tid; it < rows * taps; it += kThreads) {
      const int row = it / taps, tap = it - row * taps;
      const int kh = tap / d.KW, ptap = tap + kh * (kwp - d.KW) + (kwp - d.KW);
      T* dst = wp + (int64_t)row * d.Kpad + ptap * d.Ip + c0;
      const float* src = tile + row * LD + tap;
      if (cw == 8 && ((uintptr_t)dst & 15) == 0) {
        float x[8];
#pragma unroll
        for (int ci = 0; ci < 8; ++ci) x[ci] = src[ci * taps];
        store8(dst, x);
      } else {
        for (int ci = 0; ci < cw; ++ci) store_t(dst + ci, src[ci * taps]);
      }
    }
  }
  if (d.wt == nullptr || POSE6D_ADAMW_NOWT) return;
  // wt[r][o] for the tile's columns r: eight filters per store
  T* wt = reinterpret_cast<T*>(d.wt) + (int64_t)r0 * d.O + o0;
  if ((rows & 7) == 0 && (d.O & 7) == 0) {
    const int r8 = rows >> 3;
    for (int it = tid; it < W * r8; it += kThreads) {
      const int rl = it / r8, o8 = (it - rl * r8) * 8;
      float x[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) x[k] = tile[(o8 + k) * LD + rl];
      store8(wt + (int64_t)rl * d.O + o8, x);
    }
  } else {
    for (int it = tid; it < W * rows; it += kThreads) {
      const int rl = it / rows, ol = it - rl * rows;
      store_t(wt + (int64_t)rl * d.O + ol, tile[ol * LD + rl]);
    }
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

static int packed_jobs(const void* descs, int32_t n_desc, const float* param, int64_t n, int32_t* jobs, int32_t cap,
                       int32_t* count) {
  P6_CHECK_ARG(n >= 0 && n <= INT32_MAX, "pose6d_adamw_packed_jobs: buffer too large for int32 offsets");
  P6_CHECK_ARG(n_desc >= 0 && (n_desc == 0 || descs), "pose6d_adamw_packed_jobs: bad descriptors");
  const PackDesc* d = reinterpret_cast<const PackDesc*>(descs);
  // the convs' masters, in buffer order
  std::vector<std::pair<int64_t, int>> reg;
  for (int k = 0; k < n_desc; ++k) {
    const int64_t off = d[k].w - param, len = (int64_t)d[k].O * d[k].I * d[k].KH * d[k].KW;
    P6_CHECK_ARG(d[k].w >= param && off + len <= n && (off & 3) == 0 && d[k].wp,
                 "pose6d_adamw_packed_jobs: conv %d's master is not a 16-B aligned slice of param", k);
    const int kwp = d[k].KWp > 0 ? d[k].KWp : d[k].KW;
    P6_CHECK_ARG(kwp >= d[k].KW && d[k].Kpad >= d[k].KH * kwp * d[k].Ip && d[k].Ip >= d[k].I && (d[k].Kpad & 3) == 0,
                 "pose6d_adamw_packed_jobs: conv %d: bad packed geometry", k);
    // a tile holds one channel's taps at least: KH * KW must fit the LDS tile's columns
    P6_CHECK_ARG(d[k].KH * d[k].KW <= kTileCols,
                 "pose6d_adamw_packed_jobs: conv %d: %d x %d filter taps exceed the %d-column packing tile", k,
                 d[k].KH, d[k].KW, kTileCols);
    reg.push_back({off, k});
  }
  std::sort(reg.begin(), reg.end());
  int32_t cnt = 0;
  auto put = [&](int a, int b, int c, int e) {
    if (cnt < cap && jobs) {
      jobs[4 * cnt] = a; jobs[4 * cnt + 1] = b; jobs[4 * cnt + 2] = c; jobs[4 * cnt + 3] = e;
    }
    ++cnt;
  };
  auto plain = [&](int64_t a, int64_t b) {
    for (; a < b; a += kJob) put(0, (int)a, (int)(a + kJob < b ? a + kJob : b), 0);
  };
  int64_t cur = 0;
  for (auto& [off, k] : reg) {
    P6_CHECK_ARG(off >= cur, "pose6d_adamw_packed_jobs: conv masters overlap");
    plain(cur, off);
    const int R = d[k].I * d[k].KH * d[k].KW, cw = tile_channels(d[k].KH * d[k].KW);
    for (int o0 = 0; o0 < d[k].O; o0 += 64)
      for (int c0 = 0; c0 < d[k].I; c0 += cw) put(1, k, o0, c0);
    cur = off + (int64_t)d[k].O * R;
  }
  plain(cur, n);
  *count = cnt;
  return POSE6D_OK;
}

// returns the job count, or minus the error code
extern "C" int pose6d_adamw_packed_jobs(const void* descs, int32_t n_desc, const float* param, int64_t n,
                                        int32_t* jobs, int32_t cap) {
  int32_t cnt = 0;
  const int rc = packed_jobs(descs, n_desc, param, n, jobs, cap, &cnt);
  return rc != POSE6D_OK ? -rc : cnt;
}

extern "C" int pose6d_adamw_step_packed(float* param, const float* grad, float* exp_avg, float* exp_avg_sq,
                                        const float* partials, int32_t nparts, const float* hp, float* norm_out,
                                        int32_t dtype, const void* descs, const int32_t* jobs, int32_t n_jobs,
                                        void* stream) {
  if (n_jobs == 0) return POSE6D_OK;
  P6_CHECK_ARG(((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) % 16 == 0,
               "pose6d_adamw_step_packed: buffers must be 16-byte aligned");
  P6_CHECK_ARG(dtype == POSE6D_DT_BF16 || dtype == POSE6D_DT_F32, "pose6d_adamw_step_packed: bad dtype");
  P6_CHECK_ARG(n_jobs > 0 && jobs && descs, "pose6d_adamw_step_packed: bad job table");
  hipStream_t s = p6::stream_of(stream);
  if (dtype == POSE6D_DT_BF16)
    adamw_packed_kernel<bf16><<<n_jobs, kThreads, 0, s>>>(param, grad, exp_avg, exp_avg_sq, partials, nparts, hp,
                                                          norm_out, (const PackDesc*)descs, (const int4*)jobs);
  else
    adamw_packed_kernel<float><<<n_jobs, kThreads, 0, s>>>(param, grad, exp_avg, exp_avg_sq, partials, nparts, hp,
                                                           norm_out, (const PackDesc*)descs, (const int4*)jobs);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

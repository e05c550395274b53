// BatchNorm2d (train/eval) + ReLU + residual for NHWC activations, forward and
// backward.  Replaces the nn.BatchNorm2d / ReLU / residual-add chain of every
// torchvision Bottleneck (53 BN layers per ResNet50 trunk).
//
// Forward statistics come from the producing convolution's epilogue (per-wave
// partial sums in a [rows][2][C] workspace); pose6d_bn_finalize reduces them in
// fixed order (fp64), produces per-channel scale/shift, the saved mean/invstd and
// the running-stat update (torch semantics: biased var to normalise, unbiased var
// into running_var, momentum 0.1, num_batches_tracked += 1).
// pose6d_bn_act_fwd then applies  out = act(y*scale + shift [+ res | + res*rs + rsh]).
// Backward: pose6d_bn_bwd_reduce -> partial (sum dz, sum dz*xhat) per block,
// pose6d_bn_bwd_finalize -> dgamma/dbeta + coefficients, pose6d_bn_bwd_apply ->
// dy = gamma*invstd*(dz - mean(dz) - xhat*mean(dz*xhat)), optionally emitting dz
// (the gradient of a residual identity branch).
#include <stdlib.h>

#include <type_traits>

#include "bn_fold.h"
#include "common.h"

#ifndef POSE6D_FIN_WAVE_ROWS
#define POSE6D_FIN_WAVE_ROWS 0     // build-time: the training finalize folds <= this many rows per channel on one wave
                                   // (round 6: 0 -- the whole-workgroup fold is faster at every row count)
#endif
namespace {

constexpr int kFinWaveRows = POSE6D_FIN_WAVE_ROWS;
#ifndef POSE6D_FIN_TIMING
#define POSE6D_FIN_TIMING 0   // timing-only builds (wrong results): 1 = finalize kernels return at entry, 2 = not launched
#endif

constexpr int kThreads = 256;

template <typename T> struct V;
template <> struct V<bf16> { static constexpr int E = 8; };
template <> struct V<float> { static constexpr int E = 4; };

template <typename T>
__device__ __forceinline__ void load_vec(const T* p, float* f) {
  constexpr int E = V<T>::E;
  T t[E];
  *reinterpret_cast<uint4*>(t) = *reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int e = 0; e < E; ++e) f[e] = p6::to_f(t[e]);
}
template <typename T>
__device__ __forceinline__ void store_vec(T* p, const float* f) {
  constexpr int E = V<T>::E;
  T t[E];
#pragma unroll
  for (int e = 0; e < E; ++e) t[e] = p6::from_f<T>(f[e]);
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(t);
}

// ---------------------------------------------------------------- finalize
// ONE launch (training): block = 256 / L channels x L lanes (L = 64 or 256 by the
// row count); lane l folds partial rows l, l + L, ... of its channel as shifted
// sums about K = row 0's mean:
//   S1 = sum_i (sum_i - n_i K),  S2 = sum_i (M2_i + n_i (mean_i - K)^2)
// (fp64, no divisions: n_i = 32 except the last row), the lanes combine by a
// fixed xor-shuffle tree (+ an LDS step across waves for L = 256:
// deterministic), and mean = K + S1/N, var = (S2 - S1^2/N)/N.  The shift keeps
// S1^2/N small against S2 (K is a mean of the same data): no E[x^2]-E[x]^2
// cancellation.
// lane l (of L on channel c) folds rows l, l + L, ...; after the call thread `lane == 0`
// of the channel holds (K, s1, s2) of the whole channel (L = 256: thread 0 of the block)
template <int L>
__device__ __forceinline__ void bn_stats_fold(const float* __restrict__ part, int rows, int C, int64_t M, int c,
                                              double& K, double& s1, double& s2) {
  __shared__ double red[2][kThreads / 64];
  const int lane = threadIdx.x % L;
  s1 = 0.0; s2 = 0.0; K = 0.0;
  if (c < C) {
    const float* ps = part + (int64_t)c * rows;          // channel-major partials: coalesced rows
    const float* pq = part + ((int64_t)C + c) * rows;
    K = (double)ps[0] / (double)min((int64_t)32, M);
    const double n_last = (double)(M - (int64_t)(rows - 1) * 32), inv_last = 1.0 / n_last;
    constexpr int U = 4;
    int r = lane;
    for (; r + (U - 1) * L < rows; r += U * L) {
      float sv[U], qv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        sv[u] = ps[r + u * L];
        qv[u] = pq[r + u * L];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const bool last = r + u * L == rows - 1;
        const double n = last ? n_last : 32.0, inv_n = last ? inv_last : 0.03125;
        const double d = (double)sv[u] - n * K;        // n_i (mean_i - K)
        s1 += d;
        s2 += (double)qv[u] + d * d * inv_n;
      }
    }
    for (; r < rows; r += L) {
      const bool last = r == rows - 1;
      const double n = last ? n_last : 32.0, inv_n = last ? inv_last : 0.03125;
      const double d = (double)ps[r] - n * K;
      s1 += d;
      s2 += (double)pq[r] + d * d * inv_n;
    }
  }
  s1 = p6::wave_sum(s1);
  s2 = p6::wave_sum(s2);
  if constexpr (L > 64) {
    const int w = threadIdx.x >> 6;
    __syncthreads();   // (red reused across calls)
    if ((threadIdx.x & 63) == 0) { red[0][w] = s1; red[1][w] = s2; }
    __syncthreads();
    if (threadIdx.x == 0) {
      s1 = 0.0; s2 = 0.0;
#pragma unroll
      for (int i = 0; i < kThreads / 64; ++i) { s1 += red[0][i]; s2 += red[1][i]; }
    }
  }
}

template <int L, bool SC1 = false>
__device__ __forceinline__ void bn_stats_finalize_body(
    int blk, const float* __restrict__ part, int rows, int C, int64_t M, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt,
    float momentum, float eps, float* __restrict__ scale, float* __restrict__ shift, float* __restrict__ smean,
    float* __restrict__ sinv) {
  const int lane = threadIdx.x % L;
  const int c = blk * (kThreads / L) + threadIdx.x / L;
  // the per-channel parameters and running statistics the tail needs, fetched now
  // so their round trip overlaps the partial-row reduction instead of following it
  float g_c = 0.f, b_c = 0.f, rm_c = 0.f, rv_c = 0.f;
  if (lane == 0 && c < C) {
    g_c = gamma[c];
    b_c = beta[c];
    rm_c = rmean[c];
    rv_c = rvar[c];
  }
  double K, s1, s2;
  bn_stats_fold<L>(part, rows, C, M, c, K, s1, s2);
  if (lane == 0 && c < C) {
    const p6::BnFoldOut o = p6::bn_fold_result(M, eps, K, s1, s2, g_c, b_c);
    const double N = (double)M;
    if constexpr (SC1) {
      p6::st_sc1(scale, c, o.sc);
      p6::st_sc1(shift, c, o.sh);
    } else {
      scale[c] = o.sc;
      shift[c] = o.sh;
    }
    smean[c] = (float)o.mean;
    sinv[c] = o.inv;
    const double unb = N > 1.0 ? o.var * N / (N - 1.0) : o.var;
    rmean[c] = (1.f - momentum) * rm_c + momentum * (float)o.mean;
    rvar[c] = (1.f - momentum) * rv_c + momentum * (float)unb;
    if (c == 0 && nbt) nbt[0] += 1;
  }
}

template <int L>
__global__ __launch_bounds__(kThreads) void bn_stats_finalize_kernel(
    const float* __restrict__ part, int rows, int C, int64_t M, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt,
    float momentum, float eps, float* __restrict__ scale, float* __restrict__ shift, float* __restrict__ smean,
    float* __restrict__ sinv) {

  if (POSE6D_FIN_TIMING == 1) return;
  if constexpr (L == 64) {
    // <= 512 rows: one channel per wave, the arithmetic the producing convolution's
    // in-launch finalize shares (bn_fold.h)
    const pose6d_bn_stats_t d{part, gamma, beta, rmean, rvar, nbt, scale, shift, smean, sinv, momentum, eps, C};
    p6::bn_fold_wave<1>(d, [&](int64_t i) { return part[i]; }, rows, M, blockIdx.x * 4 + (threadIdx.x >> 6), 1);
  } else {
    bn_stats_finalize_body<L>(blockIdx.x, part, rows, C, M, gamma, beta, rmean, rvar, nbt, momentum, eps, scale,
                              shift, smean, sinv);
  }
}

// two BatchNorms over the same output grid (a downsampling block's bn3 and its
// downsample BN: same rows and count) in one launch, blockIdx.y selecting the BN;
// each BN's arithmetic is bn_stats_finalize_kernel<L>'s, bit for bit
template <int L>
__global__ __launch_bounds__(kThreads) void bn_stats_finalize2_kernel(pose6d_bn_stats_t a, pose6d_bn_stats_t b,
                                                                      int rows, int64_t M) {

  if (POSE6D_FIN_TIMING == 1) return;
  const pose6d_bn_stats_t& d = blockIdx.y ? b : a;
  if ((int)blockIdx.x * (kThreads / L) >= d.C) return;
  if constexpr (L == 64) {
    const float* part = d.partial;
    p6::bn_fold_wave<1>(d, [&](int64_t i) { return part[i]; }, rows, M, blockIdx.x * 4 + (threadIdx.x >> 6), 1);
    return;
  }
  bn_stats_finalize_body<L>(blockIdx.x, d.partial, rows, d.C, M, d.gamma, d.beta, d.running_mean, d.running_var,
                            d.num_batches, d.momentum, d.eps, d.scale, d.shift, d.save_mean, d.save_invstd);
}

// eval: running statistics -> scale / shift / saved mean / invstd (no partials)
__global__ __launch_bounds__(kThreads) void bn_eval_finalize_kernel(const float* __restrict__ gamma,
                                                                    const float* __restrict__ beta,
                                                                    const float* __restrict__ rmean,
                                                                    const float* __restrict__ rvar, int C, float eps,
                                                                    float* __restrict__ scale,
                                                                    float* __restrict__ shift,
                                                                    float* __restrict__ smean,
                                                                    float* __restrict__ sinv) {
  const int c = blockIdx.x * kThreads + threadIdx.x;
  if (c >= C) return;
  const float inv = 1.0f / sqrtf(rvar[c] + eps);
  const float sc = gamma[c] * inv;
  scale[c] = sc;
  shift[c] = beta[c] - rmean[c] * sc;
  smean[c] = rmean[c];
  sinv[c] = inv;
}

// ---------------------------------------------------------------- eval fold (all BNs, one launch)
// bn_eval_finalize_kernel for a table of BatchNorms (pose6d_bn_eval_fold)
struct EvalFold {
  const float *gamma, *beta, *rmean, *rvar;
  float *scale, *shift, *smean, *sinv;
  float eps;
  int32_t C;
};
static_assert(sizeof(EvalFold) == 72, "pose6d_bn_fold_t layout");
__global__ __launch_bounds__(kThreads) void bn_eval_fold_kernel(const EvalFold* __restrict__ d) {
  const EvalFold f = d[blockIdx.y];
  for (int c = blockIdx.x * kThreads + threadIdx.x; c < f.C; c += gridDim.x * kThreads) {
    const float inv = 1.0f / sqrtf(f.rvar[c] + f.eps);
    const float sc = f.gamma[c] * inv;
    f.scale[c] = sc;
    f.shift[c] = f.beta[c] - f.rmean[c] * sc;
    f.smean[c] = f.rmean[c];
    f.sinv[c] = inv;
  }
}

// ---------------------------------------------------------------- apply fwd
template <typename T>
__global__ __launch_bounds__(kThreads) void bn_act_kernel(const T* __restrict__ y, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, const T* __restrict__ res,
                                                          const float* __restrict__ rscale,
                                                          const float* __restrict__ rshift, int relu,
                                                          T* __restrict__ out, int64_t M, int C,
                                                          uint8_t* __restrict__ mbits) {
  constexpr int E = V<T>::E;
  const int cpr = C / E;
  const int64_t total = M * cpr;
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kThreads) {
    const int c0 = (int)(i % cpr) * E;
    const int64_t off = i * E;
    float v[E], r[E];
    load_vec(y + off, v);
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = fmaf(v[e], scale[c0 + e], shift[c0 + e]);
    if (res) {
      load_vec(res + off, r);
      if (rscale) {
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] += fmaf(r[e], rscale[c0 + e], rshift[c0 + e]);
      } else {
#pragma unroll
        for (int e = 0; e < E; ++e) v[e] += r[e];
      }
    }
    if (relu) {
#pragma unroll
      for (int e = 0; e < E; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    store_vec(out + off, v);
    if (mbits) {
      // bit e = (stored out > 0): the backward's ReLU mask without re-reading `out`
      unsigned b = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) b |= (p6::to_f(p6::from_f<T>(v[e])) > 0.f ? 1u : 0u) << e;
      mbits[i] = (uint8_t)b;
    }
  }
}

// ---------------------------------------------------------------- finalize + apply, one launch
// pose6d_bn_finalize_act: the training finalize and bn_act_kernel's apply in ONE launch
// (the kernel boundary between them -- a launch gap plus the apply's ramp behind a
// ~5 us latency-bound finalize -- is what the separate launches cost).  Workgroups
// [0, nfin) are the finalize (bn_stats_finalize_kernel<L>'s blocks, same arithmetic),
// each storing scale / shift write-through and then ITS ready flag (= the launch's
// epoch).  Workgroups [nfin, ...) apply: one 64-channel column group x RPB rows each;
// they fetch their y / residual chunks first, then one wave polls the flags of the
// finalize workgroups that cover its 64 channels (sc1 loads, bounded), reads scale /
// shift write-through and stores bn_act_kernel's result bit for bit.  Nothing assumes
// a dispatch order: an apply workgroup that does not see its flags within kFinSpins
// polls folds its 64 channels itself (the finalize's arithmetic, same bits) -- slow,
// never wrong, never a hang.
constexpr int kFinGroup = 64;     // channels per apply column group
constexpr int kFinSpins = 4096;   // ~4096 x (poll + s_sleep 2) ~ 0.5 ms before the fallback

template <int L>
__device__ __forceinline__ int fin_blocks(int C) { return L == 64 ? (C + 3) / 4 : C; }

// the 64 channels' scale / shift into LDS for a workgroup that gave up waiting: the
// finalize's fold recomputed (rows <= 512: one wave per 16 channels, bn_fold.h; more
// rows: the whole workgroup per channel, bn_stats_fold<256>)
template <int L>
__device__ void fin_fallback(const pose6d_bn_stats_t& d, int rows, int64_t M, int c0, float* sc, float* sh) {
  if constexpr (L == 64) {
    const int w = threadIdx.x >> 6;
    p6::bn_fold_wave_compute(d, rows, M, c0 + 16 * w, 16, sc + 16 * w, sh + 16 * w);
  } else {
    for (int j = 0; j < kFinGroup; ++j) {
      double K, s1, s2;
      bn_stats_fold<256>(d.partial, rows, d.C, M, c0 + j, K, s1, s2);
      if (threadIdx.x == 0 && c0 + j < d.C) {
        const p6::BnFoldOut o = p6::bn_fold_result(M, d.eps, K, s1, s2, d.gamma[c0 + j], d.beta[c0 + j]);
        sc[j] = o.sc;
        sh[j] = o.sh;
      }
    }
  }
  __syncthreads();
}

template <typename T, int L>
__global__ __launch_bounds__(kThreads) void bn_fin_act_kernel(pose6d_bn_stats_t d, int rows, int64_t M, int nfin,
                                                              const T* __restrict__ y, const T* __restrict__ res,
                                                              int relu, T* __restrict__ out,
                                                              uint8_t* __restrict__ mbits, int* __restrict__ flags,
                                                              const int64_t* __restrict__ epoch) {
  __shared__ float csc[kFinGroup], csh[kFinGroup];
  __shared__ int fb;
  const int64_t e64 = epoch[0];
  const int ep = (int)(e64 & 0x3fffffff) + 1;   // flags start at 0; never equal to a fresh epoch's value
  const int b = blockIdx.x;
  const int C = d.C;
  if (b < nfin) {
    // ---- finalize: bn_stats_finalize_kernel<L>'s workgroup b, scale / shift written through
    if constexpr (L == 64) {
      const float* part = d.partial;
      p6::bn_fold_wave<1, p6::kBnFoldSlots, true>(d, [&](int64_t i) { return part[i]; }, rows, M,
                                                   b * 4 + (threadIdx.x >> 6), 1);
    } else {
      bn_stats_finalize_body<L, true>(b, d.partial, rows, C, M, d.gamma, d.beta, d.running_mean, d.running_var,
                                      d.num_batches, d.momentum, d.eps, d.scale, d.shift, d.save_mean,
                                      d.save_invstd);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave, before the barrier
    __syncthreads();
    if (threadIdx.x == 0) p6::st_sc1(flags, b, ep);
    return;
  }
  // ---- apply: column group g (64 channels), rows [rb * RPB, + RPB)
  constexpr int E = V<T>::E;
  constexpr int CPS = kFinGroup / E;     // 16-byte chunks per row of a group
  constexpr int RPB = kThreads / CPS;    // rows per workgroup
  const int ng = C / kFinGroup;
  const int a = b - nfin;
  const int g = a % ng, rb = a / ng;
  const int j = threadIdx.x % CPS;
  const int64_t r = (int64_t)rb * RPB + threadIdx.x / CPS;
  const bool ok = r < M;
  const int c0 = g * kFinGroup + j * E;
  const int64_t off = r * C + c0;
  float v[E], rv[E];
  if (ok) {
    load_vec(y + off, v);
    if (res) load_vec(res + off, rv);
  }
  // wait for the finalize workgroups of channels [64 g, 64 g + 64)
  constexpr int FPG = L == 64 ? kFinGroup / 4 : kFinGroup;   // finalize workgroups per group
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int f = g * FPG + lane;
    bool ready = false;
    int it = 0;
    for (; it < (e64 < 0 ? 0 : kFinSpins); ++it) {   // (a negative epoch: the fallback, for the tests)
      const bool mine = lane >= FPG || f >= nfin || p6::ld_sc1(flags, f) == ep;
      if (__all(mine)) { ready = true; break; }
      __builtin_amdgcn_s_sleep(2);
    }
    if (lane == 0) fb = ready ? 0 : 1;
  }
  __syncthreads();
  float sc[E], sh[E];
  if (fb) {
    fin_fallback<L>(d, rows, M, g * kFinGroup, csc, csh);
#pragma unroll
    for (int e = 0; e < E; ++e) { sc[e] = csc[j * E + e]; sh[e] = csh[j * E + e]; }
  } else {
#pragma unroll
    for (int e4 = 0; e4 < E; e4 += 4) {
      const f32x4 a4 = p6::ld_sc1_x4(d.scale, c0 + e4), b4 = p6::ld_sc1_x4(d.shift, c0 + e4);
#pragma unroll
      for (int k = 0; k < 4; ++k) { sc[e4 + k] = a4[k]; sh[e4 + k] = b4[k]; }
    }
  }
  if (!ok) return;
  // bn_act_kernel's arithmetic, term for term
#pragma unroll
  for (int e = 0; e < E; ++e) v[e] = fmaf(v[e], sc[e], sh[e]);
  if (res) {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] += rv[e];
  }
  if (relu) {
#pragma unroll
    for (int e = 0; e < E; ++e) v[e] = fmaxf(v[e], 0.f);
  }
  store_vec(out + off, v);
  if (mbits) {
    unsigned bits = 0;
#pragma unroll
    for (int e = 0; e < E; ++e) bits |= (p6::to_f(p6::from_f<T>(v[e])) > 0.f ? 1u : 0u) << e;
    mbits[off / E] = (uint8_t)bits;
  }
}

// ---------------------------------------------------------------- backward
// grid (channel-chunk groups, row blocks): block = CL chunk-lanes (consecutive 16-B
// chunks of a row: coalesced) x RL row-lanes; partial row = blockIdx.y.
// ReLU mask of the forward output: MK 0 none, 1 out > 0 (read), 2 recomputed from
// the raw conv output y as bf16-or-fp32(y * scale + shift) > 0 -- exactly the sign
// pose6d_bn_act_fwd stored, without reading its output (no residual on that BN)
template <int MK, typename T>
__device__ __forceinline__ void relu_mask(float (&d)[V<T>::E], const uint4& ov, const float (&yy)[V<T>::E],
                                          const float* __restrict__ rs, const float* __restrict__ rb, int c0) {
  constexpr int E = V<T>::E;
  if constexpr (MK == 1) {
    float o[E];
    load_vec(reinterpret_cast<const T*>(&ov), o);
#pragma unroll
    for (int e = 0; e < E; ++e) d[e] = o[e] > 0.f ? d[e] : 0.f;
  } else if constexpr (MK == 2) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float v = p6::to_f(p6::from_f<T>(fmaf(yy[e], rs[c0 + e], rb[c0 + e])));
      d[e] = v > 0.f ? d[e] : 0.f;
    }
  } else if constexpr (MK == 3) {   // one mask byte per chunk (bn_act_fwd's bits), in ov.x
#pragma unroll
    for (int e = 0; e < E; ++e) d[e] = (ov.x >> e) & 1u ? d[e] : 0.f;
  }
}

// DUAL: a second BatchNorm fed by the same dout + mask (a downsampling block's
// branch BN: y2 / mean2 / inv2 -> part2), summed in the same pass -- sum dz is shared,
// sum dz * xhat2 is its own; each BN's sums are the single-BN kernel's, bit for bit
template <typename T, int MK, bool DUAL = false>
__global__ __launch_bounds__(kThreads) void bn_bwd_reduce2_kernel(const T* __restrict__ dout, const T* __restrict__ out,
                                                                  const float* __restrict__ rs,
                                                                  const float* __restrict__ rb,
                                                                  const T* __restrict__ y,
                                                                  const float* __restrict__ mean,
                                                                  const float* __restrict__ inv,
                                                                  float* __restrict__ part, int64_t M, int C,
                                                                  int rows_per_block, const T* __restrict__ y2 = nullptr,
                                                                  const float* __restrict__ mean2 = nullptr,
                                                                  const float* __restrict__ inv2 = nullptr,
                                                                  float* __restrict__ part2 = nullptr) {
  constexpr int E = V<T>::E;
  __shared__ float sred[kThreads][(DUAL ? 3 : 2) * E + 1];
  const int cpr = C / E;
  const int CL = cpr < 64 ? cpr : 64, RL = kThreads / CL;
  const int cl = threadIdx.x % CL, rl = threadIdx.x / CL;
  const int ch = blockIdx.x * CL + cl;
  const int c0 = ch * E;
  float s[E], q[E], mu[E], iv[E];
  float q2[DUAL ? E : 1], mu2[DUAL ? E : 1], iv2[DUAL ? E : 1];
#pragma unroll
  for (int e = 0; e < E; ++e) { s[e] = q[e] = 0.f; mu[e] = mean[c0 + e]; iv[e] = inv[c0 + e]; }
  if constexpr (DUAL) {
#pragma unroll
    for (int e = 0; e < E; ++e) { q2[e] = 0.f; mu2[e] = mean2[c0 + e]; iv2[e] = inv2[c0 + e]; }
  }
  const int64_t r0 = (int64_t)blockIdx.y * rows_per_block;
  const int64_t r1 = min(M, r0 + rows_per_block);
  // U rows per trip with every load issued before any use: 3 * U 16-byte loads in
  // flight per lane (one row per trip left this kernel latency bound at ~25 % of HBM)
  constexpr int U = 4;
  int64_t r = r0 + rl;
  for (; r + (U - 1) * RL < r1; r += U * RL) {
    uint4 dv[U], ov[U], yv[U], y2v[DUAL ? U : 1];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t off = (r + u * RL) * C + c0;
      dv[u] = *reinterpret_cast<const uint4*>(dout + off);
      if constexpr (MK == 1) ov[u] = *reinterpret_cast<const uint4*>(out + off);
      if constexpr (MK == 3) ov[u].x = reinterpret_cast<const uint8_t*>(out)[off / E];
      yv[u] = *reinterpret_cast<const uint4*>(y + off);
      if constexpr (DUAL) y2v[u] = *reinterpret_cast<const uint4*>(y2 + off);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      float d[E], yy[E];
      load_vec(reinterpret_cast<const T*>(&dv[u]), d);
      load_vec(reinterpret_cast<const T*>(&yv[u]), yy);
      relu_mask<MK, T>(d, ov[u], yy, rs, rb, c0);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        s[e] += d[e];
        q[e] = fmaf(d[e], (yy[e] - mu[e]) * iv[e], q[e]);
      }
      if constexpr (DUAL) {
        float y2f[E];
        load_vec(reinterpret_cast<const T*>(&y2v[u]), y2f);
#pragma unroll
        for (int e = 0; e < E; ++e) q2[e] = fmaf(d[e], (y2f[e] - mu2[e]) * iv2[e], q2[e]);
      }
    }
  }
  for (; r < r1; r += RL) {
    const int64_t off = r * C + c0;
    float d[E], yy[E];
    uint4 ov{};
    load_vec(dout + off, d);
    if constexpr (MK == 1) ov = *reinterpret_cast<const uint4*>(out + off);
    if constexpr (MK == 3) ov.x = reinterpret_cast<const uint8_t*>(out)[off / E];
    load_vec(y + off, yy);
    relu_mask<MK, T>(d, ov, yy, rs, rb, c0);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      s[e] += d[e];
      q[e] = fmaf(d[e], (yy[e] - mu[e]) * iv[e], q[e]);
    }
    if constexpr (DUAL) {
      float y2f[E];
      load_vec(y2 + off, y2f);
#pragma unroll
      for (int e = 0; e < E; ++e) q2[e] = fmaf(d[e], (y2f[e] - mu2[e]) * iv2[e], q2[e]);
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) { sred[threadIdx.x][e] = s[e]; sred[threadIdx.x][E + e] = q[e]; }
  if constexpr (DUAL) {
#pragma unroll
    for (int e = 0; e < E; ++e) sred[threadIdx.x][2 * E + e] = q2[e];
  }
  __syncthreads();
  if (rl == 0) {
    for (int k = 1; k < RL; ++k) {
      const int t = k * CL + cl;
#pragma unroll
      for (int e = 0; e < E; ++e) { s[e] += sred[t][e]; q[e] += sred[t][E + e]; }
      if constexpr (DUAL) {
#pragma unroll
        for (int e = 0; e < E; ++e) q2[e] += sred[t][2 * E + e];
      }
    }
    // channel-major partials [2][C][row blocks] (coalesced reads in the finalize)
    const int64_t nrb = gridDim.y;
#pragma unroll
    for (int e = 0; e < E; ++e) {
      part[(int64_t)(c0 + e) * nrb + blockIdx.y] = s[e];
      part[((int64_t)C + c0 + e) * nrb + blockIdx.y] = q[e];
      if constexpr (DUAL) {
        part2[(int64_t)(c0 + e) * nrb + blockIdx.y] = s[e];
        part2[((int64_t)C + c0 + e) * nrb + blockIdx.y] = q2[e];
      }
    }
  }
}

struct BwdFin {   // one BatchNorm's finalize operands (grid.y picks one of two)
  const float* part;
  const float* gamma;
  const float* inv;
  float *dgamma, *dbeta, *coef;
};

__global__ __launch_bounds__(kThreads) void bn_bwd_finalize_kernel(const float* __restrict__ part, int rows, int C,
                                                                   double count, const float* __restrict__ gamma,
                                                                   const float* __restrict__ inv,
                                                                   float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                                   int accumulate, float* __restrict__ coef,
                                                                   BwdFin second_v = BwdFin{}) {
  if (blockIdx.y == 1) {   // the second BatchNorm of a dual backward
    part = second_v.part; gamma = second_v.gamma; inv = second_v.inv;
    dgamma = second_v.dgamma; dbeta = second_v.dbeta; coef = second_v.coef;
  }
  // one wave per channel: lanes read the channel's partial rows coalesced
  // (channel-major [2][C][rows]), fp64 sums combined by a fixed xor tree
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * (kThreads / 64) + (threadIdx.x >> 6);
  if (c >= C) return;
  const float* ps = part + (int64_t)c * rows;
  const float* pq = part + ((int64_t)C + c) * rows;
  // the tail's operands, fetched before the reduction (their round trip overlaps it)
  float g_c = 0.f, i_c = 0.f, db0 = 0.f, dg0 = 0.f;
  if (lane == 0) {
    g_c = gamma[c];
    i_c = inv[c];
    if (accumulate) {
      if (dbeta) db0 = dbeta[c];
      if (dgamma) dg0 = dgamma[c];
    }
  }
  double s = 0.0, q = 0.0;
  int r = lane;
  for (; r + 64 < rows; r += 128) {
    const float s0 = ps[r], s1 = ps[r + 64], q0 = pq[r], q1 = pq[r + 64];
    s += (double)s0 + (double)s1;
    q += (double)q0 + (double)q1;
  }
  for (; r < rows; r += 64) {
    s += (double)ps[r];
    q += (double)pq[r];
  }
  s = p6::wave_sum(s);
  q = p6::wave_sum(q);
  if (lane == 0) {
    if (dbeta) dbeta[c] = db0 + (float)s;
    if (dgamma) dgamma[c] = dg0 + (float)q;
    coef[c] = g_c * i_c;                    // c1
    coef[C + c] = (float)(s / count);       // c2 = mean(dz)
    coef[2 * C + c] = (float)(q / count);   // c3 = mean(dz * xhat)
  }
}

// the same finalize with one WORKGROUP per channel (grid.x = C): threads over rows, fp64
// sums combined by wave_sum and then across the four waves in order by thread 0 -- the
// one-wave form above is latency-bound on its shuffle / lane-0 tail (the training
// forward's finalize showed the same: tools/fin_bench.py, profiles/r06_fin_fold.txt)
__global__ __launch_bounds__(kThreads) void bn_bwd_finalize_wg_kernel(const float* __restrict__ part, int rows, int C,
                                                                      double count, const float* __restrict__ gamma,
                                                                      const float* __restrict__ inv,
                                                                      float* __restrict__ dgamma,
                                                                      float* __restrict__ dbeta, int accumulate,
                                                                      float* __restrict__ coef,
                                                                      BwdFin second_v = BwdFin{}) {

  if (POSE6D_FIN_TIMING == 1) return;
  __shared__ double red[2][kThreads / 64];
  if (blockIdx.y == 1) {
    part = second_v.part; gamma = second_v.gamma; inv = second_v.inv;
    dgamma = second_v.dgamma; dbeta = second_v.dbeta; coef = second_v.coef;
  }
  const int c = blockIdx.x;
  const int t = threadIdx.x;
  const float* ps = part + (int64_t)c * rows;
  const float* pq = part + ((int64_t)C + c) * rows;
  float g_c = 0.f, i_c = 0.f, db0 = 0.f, dg0 = 0.f;
  if (t == 0) {
    g_c = gamma[c];
    i_c = inv[c];
    if (accumulate) {
      if (dbeta) db0 = dbeta[c];
      if (dgamma) dg0 = dgamma[c];
    }
  }
  double s = 0.0, q = 0.0;
  int r = t;
  for (; r + kThreads < rows; r += 2 * kThreads) {
    const float s0 = ps[r], s1 = ps[r + kThreads], q0 = pq[r], q1 = pq[r + kThreads];
    s += (double)s0 + (double)s1;
    q += (double)q0 + (double)q1;
  }
  if (r < rows) {
    s += (double)ps[r];
    q += (double)pq[r];
  }
  s = p6::wave_sum(s);
  q = p6::wave_sum(q);
  if ((t & 63) == 0) { red[0][t >> 6] = s; red[1][t >> 6] = q; }
  __syncthreads();
  if (t != 0) return;
  s = 0.0; q = 0.0;
#pragma unroll
  for (int w = 0; w < kThreads / 64; ++w) { s += red[0][w]; q += red[1][w]; }
  if (dbeta) dbeta[c] = db0 + (float)s;
  if (dgamma) dgamma[c] = dg0 + (float)q;
  coef[c] = g_c * i_c;
  coef[C + c] = (float)(s / count);
  coef[2 * C + c] = (float)(q / count);
}

#ifndef POSE6D_BWD_FIN_WG
#define POSE6D_BWD_FIN_WG 1   // build-time: 0 = the one-wave-per-channel backward finalize
#endif
void launch_bwd_finalize(const float* part, int rows, int C, int64_t M, const float* gamma, const float* inv,
                         float* dgamma, float* dbeta, int accumulate, float* coef, const BwdFin& b2, int ny,
                         hipStream_t s) {
  if (POSE6D_FIN_TIMING == 2) return;
  if (POSE6D_BWD_FIN_WG)
    bn_bwd_finalize_wg_kernel<<<dim3(C, ny), kThreads, 0, s>>>(part, rows, C, (double)M, gamma, inv, dgamma, dbeta,
                                                               accumulate, coef, b2);
  else
    bn_bwd_finalize_kernel<<<dim3(p6::ceil_div(C, kThreads / 64), ny), kThreads, 0, s>>>(
        part, rows, C, (double)M, gamma, inv, dgamma, dbeta, accumulate, coef, b2);
}

template <typename T, int MK, bool DUAL = false>
__global__ __launch_bounds__(kThreads) void bn_bwd_apply_kernel(const T* __restrict__ dout, const T* __restrict__ out,
                                                                const float* __restrict__ rs,
                                                                const float* __restrict__ rb,
                                                                const T* __restrict__ y, const float* __restrict__ mean,
                                                                const float* __restrict__ inv,
                                                                const float* __restrict__ coef, T* __restrict__ dy,
                                                                T* __restrict__ dz_out, int64_t M, int C,
                                                                const T* __restrict__ y2 = nullptr,
                                                                const float* __restrict__ mean2 = nullptr,
                                                                const float* __restrict__ inv2 = nullptr,
                                                                const float* __restrict__ coef2 = nullptr,
                                                                T* __restrict__ dy2 = nullptr) {
  constexpr int E = V<T>::E;
  const int cpr = C / E;
  const int64_t total = M * cpr;
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kThreads) {
    const int c0 = (int)(i % cpr) * E;
    const int64_t off = i * E;
    float d[E], yy[E], r[E];
    uint4 ov{};
    load_vec(dout + off, d);
    if constexpr (MK == 1) ov = *reinterpret_cast<const uint4*>(out + off);
    if constexpr (MK == 3) ov.x = reinterpret_cast<const uint8_t*>(out)[off / E];
    load_vec(y + off, yy);
    relu_mask<MK, T>(d, ov, yy, rs, rb, c0);
    float y2f[DUAL ? E : 1];
    if constexpr (DUAL) load_vec(y2 + off, y2f);
    if (dz_out) store_vec(dz_out + off, d);
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int c = c0 + e;
      const float xh = (yy[e] - mean[c]) * inv[c];
      r[e] = coef[c] * (d[e] - coef[C + c] - xh * coef[2 * C + c]);
    }
    store_vec(dy + off, r);
    if constexpr (DUAL) {
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const int c = c0 + e;
        const float xh = (y2f[e] - mean2[c]) * inv2[c];
        r[e] = coef2[c] * (d[e] - coef2[C + c] - xh * coef2[2 * C + c]);
      }
      store_vec(dy2 + off, r);
    }
  }
}

// out[c] (+)= sum_m x[m][c]  (conv-bias gradient); one block per channel chunk of 64
template <typename T>
__global__ __launch_bounds__(kThreads) void channel_sum_kernel(const T* __restrict__ x, int64_t M, int C,
                                                               float* __restrict__ out, int accumulate) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, pr = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < C)
    for (int64_t m = pr; m < M; m += 4) s += p6::to_f(x[m * C + c]);
  red[pr][cl] = s;
  __syncthreads();
  if (pr == 0 && c < C) {
    s = red[0][cl] + red[1][cl] + red[2][cl] + red[3][cl];
    out[c] = accumulate ? out[c] + s : s;
  }
}

inline unsigned grid_for(int64_t chunks) {
  int64_t b = (chunks + kThreads - 1) / kThreads;
  // one chunk per thread for every ResNet50 activation at batch 32 (<= 12544 blocks): a
  // grid-stride trip after the first would wait for the previous trip's stores
  if (b > 65535) b = 65535;
  if (b < 1) b = 1;
  return (unsigned)b;
}

int rows_per_block(int64_t M) {
  // up to 256 row blocks (x the channel-chunk groups), at least 16 rows each
  int64_t r = (M + 255) / 256;
  if (r < 16) r = 16;
  return (int)r;
}

}  // namespace

extern "C" int pose6d_bn_fold_desc_size(void) { return (int)sizeof(EvalFold); }

extern "C" int pose6d_bn_eval_fold(const void* descs, int32_t n, int32_t max_c, void* stream) {
  P6_CHECK_ARG(n >= 0 && n <= 65535 && max_c >= 0, "pose6d_bn_eval_fold: bad table size");
  if (n == 0 || max_c == 0) return POSE6D_OK;
  bn_eval_fold_kernel<<<dim3(p6::ceil_div(max_c, kThreads), n), kThreads, 0, p6::stream_of(stream)>>>(
      (const EvalFold*)descs);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_bn_finalize(const float* partial, int32_t rows, int32_t C, int64_t count, const float* gamma,
                                  const float* beta, float* running_mean, float* running_var, int64_t* num_batches,
                                  float momentum, float eps, int32_t training, float* scale, float* shift,
                                  float* save_mean, float* save_invstd, double* workspace, void* stream) {
  (void)workspace;   // kept in the ABI; the single-launch finalize needs none
  P6_CHECK_ARG(C > 0 && (!training || (rows > 0 && count > 0)), "pose6d_bn_finalize: bad sizes");
  hipStream_t s = p6::stream_of(stream);
  if (POSE6D_FIN_TIMING == 2 && training) return POSE6D_OK;
  if (training) {
    if (rows > kFinWaveRows)
      bn_stats_finalize_kernel<256><<<C, kThreads, 0, s>>>(partial, rows, C, count, gamma, beta, running_mean,
                                                            running_var, num_batches, momentum, eps, scale, shift,
                                                            save_mean, save_invstd);
    else
      bn_stats_finalize_kernel<64><<<p6::ceil_div(C, 4), kThreads, 0, s>>>(partial, rows, C, count, gamma, beta,
                                                                          running_mean, running_var, num_batches,
                                                                          momentum, eps, scale, shift, save_mean,
                                                                          save_invstd);
  } else {
    bn_eval_finalize_kernel<<<p6::ceil_div(C, kThreads), kThreads, 0, s>>>(gamma, beta, running_mean, running_var, C,
                                                                          eps, scale, shift, save_mean, save_invstd);
  }
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_bn_finalize_dual(const pose6d_bn_stats_t* a, const pose6d_bn_stats_t* b, int32_t rows,
                                       int64_t count, void* stream) {
  P6_CHECK_ARG(a && b && a->C > 0 && b->C > 0 && rows > 0 && count > 0 && rows == p6::ceil_div(count, (int64_t)32),
               "pose6d_bn_finalize_dual: bad sizes");
  hipStream_t s = p6::stream_of(stream);
  if (POSE6D_FIN_TIMING == 2) return POSE6D_OK;
  const int cmax = a->C > b->C ? a->C : b->C;
  if (rows > kFinWaveRows)
    bn_stats_finalize2_kernel<256><<<dim3(cmax, 2), kThreads, 0, s>>>(*a, *b, rows, count);
  else
    bn_stats_finalize2_kernel<64><<<dim3(p6::ceil_div(cmax, 4), 2), kThreads, 0, s>>>(*a, *b, rows, count);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_bn_act_fwd_mask(int32_t dtype, const void* y, const float* scale, const float* shift,
                                      const void* res, const float* res_scale, const float* res_shift, int32_t relu,
                                      void* out, uint8_t* relu_mask, int64_t M, int32_t C, void* stream) {
  P6_CHECK_ARG(C % 8 == 0, "pose6d_bn_act_fwd: C %% 8 != 0");
  hipStream_t s = p6::stream_of(stream);
  if (dtype == POSE6D_DT_BF16)
    bn_act_kernel<bf16><<<grid_for(M * C / 8), kThreads, 0, s>>>((const bf16*)y, scale, shift, (const bf16*)res,
                                                                   res_scale, res_shift, relu, (bf16*)out, M, C,
                                                                   relu_mask);
  else
    bn_act_kernel<float><<<grid_for(M * C / 4), kThreads, 0, s>>>((const float*)y, scale, shift, (const float*)res,
                                                                    res_scale, res_shift, relu, (float*)out, M, C,
                                                                    relu_mask);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

// ready flags one pose6d_bn_finalize_act launch needs (int32, zeroed once by the caller)
extern "C" int32_t pose6d_bn_finalize_act_flags(int32_t rows, int32_t C) {
  return rows > kFinWaveRows ? C : (C + 3) / 4;
}

extern "C" int pose6d_bn_finalize_act(int32_t dtype, const pose6d_bn_stats_t* bn, int32_t rows, int64_t count,
                                      const void* y, const void* res, int32_t relu, void* out, uint8_t* relu_mask,
                                      int32_t* flags, const int64_t* epoch, void* stream) {
  P6_CHECK_ARG(bn && bn->C > 0 && bn->C % kFinGroup == 0 && rows > 0 && count > 0 &&
                   rows == p6::ceil_div(count, (int64_t)32),
               "pose6d_bn_finalize_act: bad sizes (C a multiple of 64, rows = ceil(count / 32))");
  P6_CHECK_ARG(bn->partial && bn->gamma && bn->beta && bn->running_mean && bn->running_var && bn->scale && bn->shift &&
                   bn->save_mean && bn->save_invstd && y && out && flags && epoch,
               "pose6d_bn_finalize_act: null argument");
  hipStream_t s = p6::stream_of(stream);
  const int C = bn->C;
  const int nfin = pose6d_bn_finalize_act_flags(rows, C);
  auto go = [&](auto* typed) {
    using TT = std::remove_pointer_t<decltype(typed)>;
    constexpr int RPB = kThreads / (kFinGroup / V<TT>::E);
    const int64_t napp = (int64_t)(C / kFinGroup) * p6::ceil_div(count, RPB);
    const unsigned grid = (unsigned)(nfin + napp);
    if (rows > kFinWaveRows)
      bn_fin_act_kernel<TT, 256><<<grid, kThreads, 0, s>>>(*bn, rows, count, nfin, (const TT*)y, (const TT*)res, relu,
                                                           (TT*)out, relu_mask, flags, epoch);
    else
      bn_fin_act_kernel<TT, 64><<<grid, kThreads, 0, s>>>(*bn, rows, count, nfin, (const TT*)y, (const TT*)res, relu,
                                                          (TT*)out, relu_mask, flags, epoch);
  };
  if (dtype == POSE6D_DT_BF16) go((bf16*)nullptr);
  else go((float*)nullptr);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_bn_act_fwd(int32_t dtype, const void* y, const float* scale, const float* shift,
                                 const void* res, const float* res_scale, const float* res_shift, int32_t relu,
                                 void* out, int64_t M, int32_t C, void* stream) {
  return pose6d_bn_act_fwd_mask(dtype, y, scale, shift, res, res_scale, res_shift, relu, out, nullptr, M, C, stream);
}

extern "C" int pose6d_bn_bwd_workspace_rows(int64_t M) { return p6::ceil_div(M, rows_per_block(M)); }

namespace {
int bn_bwd_impl(int mk, int32_t dtype, const void* dout, const void* out, const float* relu_scale,
                const float* relu_shift, const void* y, const float* mean, const float* invstd, const float* gamma,
                float* dgamma, float* dbeta, int32_t accumulate, void* dy, void* dz_out, float* workspace, int64_t M,
                int32_t C, void* stream);
}  // namespace

extern "C" int pose6d_bn_bwd(int32_t dtype, const void* dout, const void* out, const float* relu_scale,
                             const float* relu_shift, const void* y, const float* mean, const float* invstd,
                             const float* gamma, float* dgamma, float* dbeta, int32_t accumulate, void* dy,
                             void* dz_out, float* workspace, int64_t M, int32_t C, void* stream) {
  P6_CHECK_ARG(!relu_scale == !relu_shift, "pose6d_bn_bwd: relu_scale and relu_shift go together");
  return bn_bwd_impl(out ? 1 : relu_scale ? 2 : 0, dtype, dout, out, relu_scale, relu_shift, y, mean, invstd, gamma,
                     dgamma, dbeta, accumulate, dy, dz_out, workspace, M, C, stream);
}

extern "C" int pose6d_bn_bwd_mask(int32_t dtype, const void* dout, const uint8_t* relu_mask, const void* y,
                                  const float* mean, const float* invstd, const float* gamma, float* dgamma,
                                  float* dbeta, int32_t accumulate, void* dy, void* dz_out, float* workspace, int64_t M,
                                  int32_t C, void* stream) {
  P6_CHECK_ARG(relu_mask != nullptr, "pose6d_bn_bwd_mask: null mask");
  return bn_bwd_impl(3, dtype, dout, relu_mask, nullptr, nullptr, y, mean, invstd, gamma, dgamma, dbeta, accumulate,
                     dy, dz_out, workspace, M, C, stream);
}

namespace {
int bn_bwd_impl(int mk, int32_t dtype, const void* dout, const void* out, const float* relu_scale,
                const float* relu_shift, const void* y, const float* mean, const float* invstd, const float* gamma,
                float* dgamma, float* dbeta, int32_t accumulate, void* dy, void* dz_out, float* workspace, int64_t M,
                int32_t C, void* stream) {
  P6_CHECK_ARG(C % 8 == 0 && M > 0, "pose6d_bn_bwd: bad sizes");
  hipStream_t s = p6::stream_of(stream);
  const int rpb = rows_per_block(M);
  const int nb = p6::ceil_div(M, rpb);
  float* part = workspace;                          // [nb][2][C]
  float* coef = workspace + (int64_t)nb * 2 * C;    // [3][C]
  const int E = dtype == POSE6D_DT_BF16 ? 8 : 4;
  const int cpr = C / E;
  const int cl = cpr < 64 ? cpr : 64;
  P6_CHECK_ARG(cpr % cl == 0 && kThreads % cl == 0, "pose6d_bn_bwd: C / vector width must be a power of two");
  dim3 grid(cpr / cl, nb);
  auto reduce = [&](auto* typed) {
    using TT = std::remove_pointer_t<decltype(typed)>;
    auto k = mk == 1 ? bn_bwd_reduce2_kernel<TT, 1> : mk == 2 ? bn_bwd_reduce2_kernel<TT, 2>
           : mk == 3 ? bn_bwd_reduce2_kernel<TT, 3> : bn_bwd_reduce2_kernel<TT, 0>;
    k<<<grid, kThreads, 0, s>>>((const TT*)dout, (const TT*)out, relu_scale, relu_shift, (const TT*)y, mean, invstd,
                                part, M, C, rpb, nullptr, nullptr, nullptr, nullptr);
  };
  if (dtype == POSE6D_DT_BF16) reduce((bf16*)nullptr);
  else reduce((float*)nullptr);
  P6_LAUNCH_CHECK();
  launch_bwd_finalize(part, nb, C, M, gamma, invstd, dgamma, dbeta, accumulate, coef, BwdFin{}, 1, s);
  P6_LAUNCH_CHECK();
  auto apply = [&](auto* typed) {
    using TT = std::remove_pointer_t<decltype(typed)>;
    auto k = mk == 1 ? bn_bwd_apply_kernel<TT, 1> : mk == 2 ? bn_bwd_apply_kernel<TT, 2>
           : mk == 3 ? bn_bwd_apply_kernel<TT, 3> : bn_bwd_apply_kernel<TT, 0>;
    k<<<grid_for(M * C / V<TT>::E), kThreads, 0, s>>>((const TT*)dout, (const TT*)out, relu_scale, relu_shift,
                                                      (const TT*)y, mean, invstd, coef, (TT*)dy, (TT*)dz_out, M, C, nullptr, nullptr,
                                                      nullptr, nullptr, nullptr);
  };
  if (dtype == POSE6D_DT_BF16) apply((bf16*)nullptr);
  else apply((float*)nullptr);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}
}  // namespace

// The rest of a BatchNorm backward whose reduce pass ran in the data gradient that
// produced dout (pose6d_conv2d_backward_chain_bn, `partial` [2][C][rows]): finalize +
// apply, two launches; with partial2 / y2 / ... the dual branch BN too (grid.y = 2 in
// the finalize, both dy in one apply).  relu: relu_mask bits (needed for the dual) or
// relu_scale / relu_shift recomputed from y.  coef: 3 * C floats (6 * C dual).
extern "C" int pose6d_bn_bwd_partials(int32_t dtype, const float* partial, int32_t rows, const void* dout,
                                      const uint8_t* relu_mask, const float* relu_scale, const float* relu_shift,
                                      const void* y, const float* mean, const float* invstd, const float* gamma,
                                      float* dgamma, float* dbeta, void* dy, const float* partial2, const void* y2,
                                      const float* mean2, const float* invstd2, const float* gamma2, float* dgamma2,
                                      float* dbeta2, void* dy2, int32_t accumulate, float* coef, int64_t M, int32_t C,
                                      void* stream) {
  P6_CHECK_ARG(C % 8 == 0 && M > 0 && rows > 0 && partial && dout && y && dy && coef,
               "pose6d_bn_bwd_partials: bad arguments");
  P6_CHECK_ARG(relu_mask || (relu_scale && relu_shift), "pose6d_bn_bwd_partials: needs relu_mask or relu_scale/shift");
  const bool dual = partial2 != nullptr;
  P6_CHECK_ARG(!dual || (relu_mask && y2 && mean2 && invstd2 && gamma2 && dy2),
               "pose6d_bn_bwd_partials: the second BatchNorm needs relu_mask, y2, mean2, invstd2, gamma2, dy2");
  hipStream_t s = p6::stream_of(stream);
  float* coef2 = coef + 3 * (int64_t)C;
  const BwdFin b2{partial2, gamma2, invstd2, dgamma2, dbeta2, coef2};
  launch_bwd_finalize(partial, rows, C, M, gamma, invstd, dgamma, dbeta, accumulate, coef, b2, dual ? 2 : 1, s);
  P6_LAUNCH_CHECK();
  auto apply = [&](auto* typed) {
    using TT = std::remove_pointer_t<decltype(typed)>;
    const dim3 grid = grid_for(M * C / V<TT>::E);
    if (dual)
      bn_bwd_apply_kernel<TT, 3, true><<<grid, kThreads, 0, s>>>(
          (const TT*)dout, (const TT*)relu_mask, nullptr, nullptr, (const TT*)y, mean, invstd, coef, (TT*)dy, nullptr,
          M, C, (const TT*)y2, mean2, invstd2, coef2, (TT*)dy2);
    else if (relu_mask)
      bn_bwd_apply_kernel<TT, 3><<<grid, kThreads, 0, s>>>((const TT*)dout, (const TT*)relu_mask, nullptr, nullptr,
                                                           (const TT*)y, mean, invstd, coef, (TT*)dy, nullptr, M, C);
    else
      bn_bwd_apply_kernel<TT, 2><<<grid, kThreads, 0, s>>>((const TT*)dout, nullptr, relu_scale, relu_shift,
                                                           (const TT*)y, mean, invstd, coef, (TT*)dy, nullptr, M, C);
  };
  if (dtype == POSE6D_DT_BF16) apply((bf16*)nullptr);
  else apply((float*)nullptr);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

// Backward of a downsampling block's two BatchNorms at once: both are fed the same
// dout * mask (the block output's gradient through its ReLU bits); bn 1 = y / mean /
// invstd / gamma -> dy, bn 2 = y2 / ... -> dy2.  = pose6d_bn_bwd_mask(bn 1) then
// pose6d_bn_bwd_mask(bn 2), bit for bit, in three launches instead of six, dout and the
// mask read once per pass.  workspace: 2 * (pose6d_bn_bwd_workspace_rows(M) * 2 + 3) * C floats.
extern "C" int pose6d_bn_bwd_mask_dual(int32_t dtype, const void* dout, const uint8_t* relu_mask, const void* y,
                                       const float* mean, const float* invstd, const float* gamma, float* dgamma,
                                       float* dbeta, void* dy, const void* y2, const float* mean2,
                                       const float* invstd2, const float* gamma2, float* dgamma2, float* dbeta2,
                                       void* dy2, int32_t accumulate, float* workspace, int64_t M, int32_t C,
                                       void* stream) {
  P6_CHECK_ARG(C % 8 == 0 && M > 0 && relu_mask && y && y2 && dy && dy2, "pose6d_bn_bwd_mask_dual: bad arguments");
  hipStream_t s = p6::stream_of(stream);
  const int rpb = rows_per_block(M);
  const int nb = p6::ceil_div(M, rpb);
  const int64_t one = ((int64_t)nb * 2 + 3) * C;
  float* part = workspace;
  float* coef = workspace + (int64_t)nb * 2 * C;
  float* part2 = workspace + one;
  float* coef2 = part2 + (int64_t)nb * 2 * C;
  const int E = dtype == POSE6D_DT_BF16 ? 8 : 4;
  const int cpr = C / E;
  const int cl = cpr < 64 ? cpr : 64;
  P6_CHECK_ARG(cpr % cl == 0 && kThreads % cl == 0, "pose6d_bn_bwd_mask_dual: C / vector width must be a power of two");
  auto run = [&](auto* typed) {
    using TT = std::remove_pointer_t<decltype(typed)>;
    bn_bwd_reduce2_kernel<TT, 3, true><<<dim3(cpr / cl, nb), kThreads, 0, s>>>(
        (const TT*)dout, (const TT*)relu_mask, nullptr, nullptr, (const TT*)y, mean, invstd, part, M, C, rpb,
        (const TT*)y2, mean2, invstd2, part2);
  };
  if (dtype == POSE6D_DT_BF16) run((bf16*)nullptr);
  else run((float*)nullptr);
  P6_LAUNCH_CHECK();
  const BwdFin b2{part2, gamma2, invstd2, dgamma2, dbeta2, coef2};
  launch_bwd_finalize(part, nb, C, M, gamma, invstd, dgamma, dbeta, accumulate, coef, b2, 2, s);
  P6_LAUNCH_CHECK();
  auto apply = [&](auto* typed) {
    using TT = std::remove_pointer_t<decltype(typed)>;
    bn_bwd_apply_kernel<TT, 3, true><<<grid_for(M * C / V<TT>::E), kThreads, 0, s>>>(
        (const TT*)dout, (const TT*)relu_mask, nullptr, nullptr, (const TT*)y, mean, invstd, coef, (TT*)dy, nullptr,
        M, C, (const TT*)y2, mean2, invstd2, coef2, (TT*)dy2);
  };
  if (dtype == POSE6D_DT_BF16) apply((bf16*)nullptr);
  else apply((float*)nullptr);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_channel_sum(int32_t dtype, const void* x, int64_t M, int32_t C, float* out, int32_t accumulate,
                                  void* stream) {
  hipStream_t s = p6::stream_of(stream);
  if (dtype == POSE6D_DT_BF16)
    channel_sum_kernel<bf16><<<p6::ceil_div(C, 64), kThreads, 0, s>>>((const bf16*)x, M, C, out, accumulate);
  else
    channel_sum_kernel<float><<<p6::ceil_div(C, 64), kThreads, 0, s>>>((const float*)x, M, C, out, accumulate);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

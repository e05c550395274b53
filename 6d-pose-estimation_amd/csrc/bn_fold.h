// The BatchNorm2d training finalize of one channel on one wave: the arithmetic of
// pose6d_bn_finalize for statistics with <= 512 partial rows (bn.hip's single and dual
// finalize kernels).  Written so that any kernel can fold channels with the same bits:
// round 5 ran it inside the producing conv (the column's last workgroup folding its
// channels) -- bit-identical, but a serial tail of ~30 us per conv against the ~5 us
// launch it saved (profiles/r05f_bn_fold_rejected.txt), so only the finalize kernels
// use it.
//
// Partials are [2][C][rows] fp32 (row i: sum and M2 about the block mean of 32
// output pixels; the last row may hold fewer).  Lane l folds rows l, l + 64, ... in
// order as shifted sums about K = row 0's mean (fp64, no divisions):
//   S1 = sum_i (sum_i - n_i K),  S2 = sum_i (M2_i + n_i (mean_i - K)^2)
// the wave combines the lanes by the xor-shuffle tree of p6::wave_sum (every lane
// ends with the same value), and lane 0 forms mean = K + S1/N, var = (S2 - S1^2/N)/N
// (biased, to normalise; unbiased into running_var), torch's momentum update and
// num_batches_tracked += 1 (channel 0).  Contraction is off so that every kernel
// inlining this rounds identically.
#pragma once
#include "common.h"

namespace p6 {

constexpr int kBnFoldSlots = 8;   // partial rows per lane: rows <= 64 * 8

struct BnFoldLane {
  double s1 = 0.0, s2 = 0.0;
};

// lane's share: sv[u], qv[u] = (sum, M2) of row lane + 64 u (unused beyond rows;
// rows <= 64 * SL)
template <int SL>
__device__ __forceinline__ void bn_fold_rows(BnFoldLane& a, const float (&sv)[SL], const float (&qv)[SL], int lane,
                                             int rows, double K, double n_last, double inv_last) {
#pragma clang fp contract(off)
#pragma unroll
  for (int u = 0; u < SL; ++u) {
    const int r = lane + 64 * u;
    if (r < rows) {
      const bool last = r == rows - 1;
      const double n = last ? n_last : 32.0, inv_n = last ? inv_last : 0.03125;
      const double d = (double)sv[u] - n * K;   // n_i (mean_i - K)
      a.s1 += d;
      a.s2 += (double)qv[u] + d * d * inv_n;
    }
  }
}

// write-through (sc1) accesses through a buffer resource: scale / shift and the ready
// flags of a finalize that other workgroups of the SAME launch read (bn.hip
// pose6d_bn_finalize_act): the hand-off MI355X_MICROARCH.md measures valid with sc1
// stores and sc1 loads on both sides (the storing waves wait for their stores, one
// lane then stores the flag)
constexpr int kSc1 = 16;   // buffer cache-policy bits: sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ void st_sc1(float* p, int i, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rsrc_of(p), i * 4, 0, kSc1);
}
__device__ __forceinline__ void st_sc1(int* p, int i, int v) {
  __builtin_amdgcn_raw_buffer_store_b32((unsigned)v, rsrc_of(p), i * 4, 0, kSc1);
}
__device__ __forceinline__ int ld_sc1(const int* p, int i) {
  return (int)__builtin_amdgcn_raw_buffer_load_b32(rsrc_of(p), i * 4, 0, kSc1);
}
__device__ __forceinline__ f32x4 ld_sc1_x4(const float* p, int i) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsrc_of(p), i * 4, 0, kSc1));
}

// the channel's mean / biased var / invstd / scale / shift from its fold (fp64; the
// arithmetic of every finalize -- keep in one place so all of them round alike)
struct BnFoldOut {
  double mean, var;
  float inv, sc, sh;
};
__device__ __forceinline__ BnFoldOut bn_fold_result(int64_t M, float eps, double K, double s1, double s2, float g_c,
                                                    float b_c) {
#pragma clang fp contract(off)
  BnFoldOut o;
  const double N = (double)M;
  o.mean = K + s1 / N;
  o.var = (s2 - s1 * s1 / N) / N;
  if (o.var < 0.0) o.var = 0.0;
  o.inv = (float)(1.0 / sqrt(o.var + (double)eps));
  o.sc = g_c * o.inv;
  o.sh = b_c - (float)o.mean * o.sc;
  return o;
}

// lane 0 of the wave, after the wave sums: the channel's outputs (SC1: scale / shift
// written through for readers in the same launch)
template <bool SC1 = false>
__device__ __forceinline__ void bn_fold_tail(const pose6d_bn_stats_t& d, int c, int64_t M, double K, double s1,
                                             double s2, float g_c, float b_c, float rm_c, float rv_c) {
#pragma clang fp contract(off)
  const BnFoldOut o = bn_fold_result(M, d.eps, K, s1, s2, g_c, b_c);
  const double N = (double)M;
  if constexpr (SC1) {
    st_sc1(d.scale, c, o.sc);
    st_sc1(d.shift, c, o.sh);
  } else {
    d.scale[c] = o.sc;
    d.shift[c] = o.sh;
  }
  d.save_mean[c] = (float)o.mean;
  d.save_invstd[c] = o.inv;
  const double unb = N > 1.0 ? o.var * N / (N - 1.0) : o.var;
  d.running_mean[c] = (1.f - d.momentum) * rm_c + d.momentum * (float)o.mean;
  d.running_var[c] = (1.f - d.momentum) * rv_c + d.momentum * (float)unb;
  if (c == 0 && d.num_batches) d.num_batches[0] += 1;
}

// Channels c0 + j (j < nch <= 64, c < d.C) on this wave, G at a time with all of
// their partial loads in flight together; rows <= 64 * SL.  ld(i) returns partial[i]
// (plain loads, or sc1 loads when other workgroups of the same launch wrote the
// partials).  The per-channel parameters come in once, lane j holding channel j's,
// and reach lane 0 by a lane read.  The result does not depend on G or SL.
template <int G, int SL = kBnFoldSlots, bool SC1 = false, typename LD>
__device__ __forceinline__ void bn_fold_wave(const pose6d_bn_stats_t& d, LD ld, int rows, int64_t M, int c0,
                                             int nch) {
  const int lane = threadIdx.x & 63;
  const double n_last = (double)(M - (int64_t)(rows - 1) * 32), inv_last = 1.0 / n_last;
  const double k_div = (double)(M < 32 ? M : 32);
  const int nslot = (rows + 63) >> 6;
  float g_l = 0.f, b_l = 0.f, rm_l = 0.f, rv_l = 0.f;
  if (lane < nch && c0 + lane < d.C) {
    g_l = d.gamma[c0 + lane];
    b_l = d.beta[c0 + lane];
    rm_l = d.running_mean[c0 + lane];
    rv_l = d.running_var[c0 + lane];
  }
  for (int j0 = 0; j0 < nch; j0 += G) {
    float sv[G][SL], qv[G][SL], k0[G];
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const int c = c0 + j0 + gi;
      const bool ok = j0 + gi < nch && c < d.C;
      const int64_t ps = (int64_t)c * rows, pq = ((int64_t)d.C + c) * rows;
      k0[gi] = ok ? ld(ps) : 0.f;
#pragma unroll
      for (int u = 0; u < SL; ++u) {
        const int r = lane + 64 * u;
        const bool in = ok && u < nslot && r < rows;
        sv[gi][u] = in ? ld(ps + r) : 0.f;
        qv[gi][u] = in ? ld(pq + r) : 0.f;
      }
    }
#pragma unroll
    for (int gi = 0; gi < G; ++gi) {
      const int c = c0 + j0 + gi;
      if (j0 + gi >= nch || c >= d.C) break;   // wave-uniform
      const double K = (double)k0[gi] / k_div;
      BnFoldLane a;
      bn_fold_rows<SL>(a, sv[gi], qv[gi], lane, rows, K, n_last, inv_last);
      const double s1 = wave_sum(a.s1), s2 = wave_sum(a.s2);
      const int src = j0 + gi;
      const float g_c = __shfl(g_l, src, 64), b_c = __shfl(b_l, src, 64);
      const float rm_c = __shfl(rm_l, src, 64), rv_c = __shfl(rv_l, src, 64);
      if (lane == 0) bn_fold_tail<SC1>(d, c, M, K, s1, s2, g_c, b_c, rm_c, rv_c);
    }
  }
}

// The same fold, computing only scale / shift of channels c0 .. c0 + nch - 1 (nch <= 64)
// into sc[j] / sh[j] (any memory the caller reads after a barrier): the fallback of
// an apply workgroup that did not see the finalize's ready flags in time (bn.hip).
template <int SL = kBnFoldSlots>
__device__ __forceinline__ void bn_fold_wave_compute(const pose6d_bn_stats_t& d, int rows, int64_t M, int c0,
                                                     int nch, float* sc, float* sh) {
  const int lane = threadIdx.x & 63;
  const double n_last = (double)(M - (int64_t)(rows - 1) * 32), inv_last = 1.0 / n_last;
  const double k_div = (double)(M < 32 ? M : 32);
  const int nslot = (rows + 63) >> 6;
  for (int j = 0; j < nch; ++j) {
    const int c = c0 + j;
    if (c >= d.C) break;
    const int64_t ps = (int64_t)c * rows, pq = ((int64_t)d.C + c) * rows;
    float sv[SL], qv[SL];
#pragma unroll
    for (int u = 0; u < SL; ++u) {
      const int r = lane + 64 * u;
      const bool in = u < nslot && r < rows;
      sv[u] = in ? d.partial[ps + r] : 0.f;
      qv[u] = in ? d.partial[pq + r] : 0.f;
    }
    const double K = (double)d.partial[ps] / k_div;
    BnFoldLane a;
    bn_fold_rows<SL>(a, sv, qv, lane, rows, K, n_last, inv_last);
    const double s1 = wave_sum(a.s1), s2 = wave_sum(a.s2);
    if (lane == 0) {
      const BnFoldOut o = bn_fold_result(M, d.eps, K, s1, s2, d.gamma[c], d.beta[c]);
      sc[j] = o.sc;
      sh[j] = o.sh;
    }
  }
}

}  // namespace p6

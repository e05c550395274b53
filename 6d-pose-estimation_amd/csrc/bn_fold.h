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

// lane 0 of the wave, after the wave sums: the channel's outputs
__device__ __forceinline__ void bn_fold_tail(const pose6d_bn_stats_t& d, int c, int64_t M, double K, double s1,
                                             double s2, float g_c, float b_c, float rm_c, float rv_c) {
#pragma clang fp contract(off)
  const double N = (double)M;
  const double mean = K + s1 / N;
  double var = (s2 - s1 * s1 / N) / N;
  if (var < 0.0) var = 0.0;
  const float inv = (float)(1.0 / sqrt(var + (double)d.eps));
  const float sc = g_c * inv;
  d.scale[c] = sc;
  d.shift[c] = b_c - (float)mean * sc;
  d.save_mean[c] = (float)mean;
  d.save_invstd[c] = inv;
  const double unb = N > 1.0 ? var * N / (N - 1.0) : var;
  d.running_mean[c] = (1.f - d.momentum) * rm_c + d.momentum * (float)mean;
  d.running_var[c] = (1.f - d.momentum) * rv_c + d.momentum * (float)unb;
  if (c == 0 && d.num_batches) d.num_batches[0] += 1;
}

// Channels c0 + j (j < nch <= 64, c < d.C) on this wave, G at a time with all of
// their partial loads in flight together; rows <= 64 * SL.  ld(i) returns partial[i]
// (plain loads, or sc1 loads when other workgroups of the same launch wrote the
// partials).  The per-channel parameters come in once, lane j holding channel j's,
// and reach lane 0 by a lane read.  The result does not depend on G or SL.
template <int G, int SL = kBnFoldSlots, typename LD>
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
      if (lane == 0) bn_fold_tail(d, c, M, K, s1, s2, g_c, b_c, rm_c, rv_c);
    }
  }
}

}  // namespace p6

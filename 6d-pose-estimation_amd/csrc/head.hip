// Fully-connected pose heads (fp32): Linear fwd/bwd as one strided GEMM kernel,
// BatchNorm1d (+ReLU +Dropout) fused per column, bias gradients.
// Replaces the nn.Linear / nn.BatchNorm1d / nn.ReLU / nn.Dropout stacks of
// pose_net_rgb.py:23-50, pose_net_rgb_geometric.py:23-33,58-65,
// pose_net_rgbd_geometric.py:28-38.  M (batch) is 32 per GPU, so these are skinny
// GEMMs bound by reading the weight matrix once (8 MB for 2048x1024 fp32).
#include <stdlib.h>

#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int TBM = 32, TBN = 64, TBK = 32;

// C[m][n] = alpha * sum_k A(m,k) B(k,n) + (bias ? bias[n] : 0) + beta * C[m][n]
// A(m,k) = A[m*sam + k*sak], B(k,n) = B[k*sbk + n*sbn]
__global__ __launch_bounds__(kThreads) void gemm_f32_kernel(const float* __restrict__ A, int64_t sam, int64_t sak,
                                                            const float* __restrict__ B, int64_t sbk, int64_t sbn,
                                                            float* __restrict__ C, int64_t ldc,
                                                            const float* __restrict__ bias, int M, int N, int K,
                                                            float alpha, float beta, int kchunk,
                                                            float* __restrict__ part) {
  __shared__ float As[TBK][TBM + 1];
  __shared__ float Bs[TBK][TBN + 1];
  const int m0 = blockIdx.y * TBM, n0 = blockIdx.x * TBN;
  const int tid = threadIdx.x;
  const int tn = tid % 16, tm = tid / 16;  // each thread: rows tm*2..+1, cols tn*4..+3
  float acc[2][4] = {};
  // split-K: this block's K range (part != null -> raw partial sums to part[z])
  const int kbeg = blockIdx.z * kchunk, kend = min(K, kbeg + kchunk);
  for (int k0 = kbeg; k0 < kend; k0 += TBK) {
    for (int i = tid; i < TBK * TBM; i += kThreads) {
      // k fastest when A is k-contiguous, m fastest otherwise (coalescing)
      int kk, mm;
      if (sak == 1) { kk = i % TBK; mm = i / TBK; } else { mm = i % TBM; kk = i / TBM; }
      const int m = m0 + mm, k = k0 + kk;
      As[kk][mm] = (m < M && k < kend) ? A[m * sam + k * sak] : 0.f;
    }
    for (int i = tid; i < TBK * TBN; i += kThreads) {
      int kk, nn;
      if (sbk == 1) { kk = i % TBK; nn = i / TBK; } else { nn = i % TBN; kk = i / TBN; }
      const int n = n0 + nn, k = k0 + kk;
      Bs[kk][nn] = (n < N && k < kend) ? B[k * sbk + n * sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll 8
    for (int kk = 0; kk < TBK; ++kk) {
      const float a0 = As[kk][tm * 2], a1 = As[kk][tm * 2 + 1];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float b = Bs[kk][tn * 4 + j];
        acc[0][j] = fmaf(a0, b, acc[0][j]);
        acc[1][j] = fmaf(a1, b, acc[1][j]);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int m = m0 + tm * 2 + i, n = n0 + tn * 4 + j;
      if (m < M && n < N) {
        if (part) {
          part[((int64_t)blockIdx.z * M + m) * N + n] = acc[i][j];
          continue;
        }
        float v = alpha * acc[i][j];
        if (bias) v += bias[n];
        if (beta != 0.f) v += beta * C[m * ldc + n];
        C[m * ldc + n] = v;
      }
    }
}

// Skinny Linear GEMMs (the batch M <= 32 is the small side) on MFMA f32 16x16x4:
// C[M][N] = alpha * A B (+ bias) + beta * C with A(m, k) = A[m * sam + k] and
// B(k, n) = B[n * sbn + k] (BKC: the nn.Linear weight [N][K], forward) or
// B[k * sbk + n] (data gradient through the weight).  One workgroup per 16
// output columns; its 16 waves split K and meet in LDS (fixed wave order, no
// workspace, one launch): every weight byte is read once, by 4-byte-per-lane
// rows of 64 B.  Inside a 16-deep K chunk lane (r, q) feeds MFMA step s with
// k = 4 q + s, so A and (BKC) B fragments are single 16-byte loads; the
// reduction order differs from torch's but all products are exact fp32.
// eval BatchNorm1d (+ ReLU) applied to a Linear's output before it is stored
// (pose6d_gemm_f32_bn_eval): bn1d_fwd_kernel's eval arithmetic, term for term
struct BnEv {
  const float *gamma, *beta, *rmean, *rvar;
  float eps;
  int relu, on;
};
__device__ __forceinline__ float bn_eval_apply(float x, const BnEv& bn, int c) {
  const float mean = bn.rmean[c];
  const float inv = 1.0f / sqrtf(bn.rvar[c] + bn.eps);
  float v = (x - mean) * inv * bn.gamma[c] + bn.beta[c];
  if (bn.relu) v = fmaxf(v, 0.f);
  return v;
}

constexpr int kSkW = 16;                      // waves per workgroup
constexpr int kSkThreads = kSkW * 64;

// Split K across workgroups (grid.y = K slices of `kchunk`, `part` = [slices][M][N]
// partial sums, summed in slice order by gemm_splitk_reduce_kernel) when N / 16 column
// groups alone would leave most CUs idle: a 2048 x 1024 weight streamed by 64
// workgroups took ~15 us, i.e. ~0.5 TB/s.
template <bool BKC, bool VEC>
__global__ __launch_bounds__(kSkThreads) void skinny_gemm_kernel(
    const float* __restrict__ A, int64_t sam, const float* __restrict__ B, int64_t sbk, int64_t sbn,
    float* __restrict__ C, int64_t ldc, const float* __restrict__ bias, int M, int N, int K, float alpha, float beta,
    int kchunk, float* __restrict__ part, BnEv bn) {
  __shared__ float red[kSkW][32][17];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = lane & 15, q = lane >> 4;
  const int n0 = blockIdx.x * 16, n = n0 + r;
  const int ks0 = blockIdx.y * kchunk, ks1 = min(K, ks0 + kchunk);
  const int kc = ((ks1 - ks0 + kSkW - 1) / kSkW + 15) & ~15;
  const int kb = ks0 + w * kc, ke = min(ks1, kb + kc);
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
  const bool m0ok = r < M, m1ok = r + 16 < M, nok = n < N;
  for (int k = kb; k < ke; k += 16) {
    const int kq = k + 4 * q;
    float a0[4], a1[4], b[4];
    if (VEC && kq + 3 < ke) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const f32x4 va0 = m0ok ? *reinterpret_cast<const f32x4*>(A + r * sam + kq) : z;
      const f32x4 va1 = m1ok ? *reinterpret_cast<const f32x4*>(A + (r + 16) * sam + kq) : z;
#pragma unroll
      for (int s = 0; s < 4; ++s) { a0[s] = va0[s]; a1[s] = va1[s]; }
      if (BKC) {
        const f32x4 vb = nok ? *reinterpret_cast<const f32x4*>(B + n * sbn + kq) : z;
#pragma unroll
        for (int s = 0; s < 4; ++s) b[s] = vb[s];
      } else {
#pragma unroll
        for (int s = 0; s < 4; ++s) b[s] = nok ? B[(int64_t)(kq + s) * sbk + n] : 0.f;
      }
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int kk = kq + s;
        const bool kok = kk < ke;
        a0[s] = (kok && m0ok) ? A[r * sam + kk] : 0.f;
        a1[s] = (kok && m1ok) ? A[(r + 16) * sam + kk] : 0.f;
        b[s] = (kok && nok) ? (BKC ? B[n * sbn + kk] : B[(int64_t)kk * sbk + n]) : 0.f;
      }
    }
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], b[s], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s], b[s], acc1, 0, 0, 0);
    }
  }
  // lane holds rows 4q + i (+16) of column r
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    red[w][4 * q + i][r] = acc0[i];
    red[w][16 + 4 * q + i][r] = acc1[i];
  }
  __syncthreads();
  if (threadIdx.x < 32 * 16) {
    const int mm = threadIdx.x >> 4, cc = threadIdx.x & 15, nn = n0 + cc;
    if (mm < M && nn < N) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < kSkW; ++i) t += red[i][mm][cc];
      if (part) {
        part[((int64_t)blockIdx.y * M + mm) * N + nn] = t;
        return;
      }
      float v = alpha * t;
      if (bias) v += bias[nn];
      if (beta != 0.f) v += beta * C[mm * ldc + nn];
      if (bn.on) v = bn_eval_apply(v, bn, nn);
      C[mm * ldc + nn] = v;
    }
  }
}

// nn.Linear weight / bias gradient: dW[n][k] (+)= sum_b dy[b][n] x[b][k] and
// db[n] (+)= sum_b dy[b][n] (the batch, <= a few hundred rows, is the contraction).
// Block = 16 output rows n x 256 columns k; thread = 4 n x 4 k (one float4 of x and
// four broadcast dy values per batch row); the blocks of column tile 0 also write db.
__global__ __launch_bounds__(kThreads) void linear_wgrad_kernel(const float* __restrict__ dy, int64_t ldy,
                                                                const float* __restrict__ x, int64_t ldx,
                                                                float* __restrict__ dw, float* __restrict__ db, int N,
                                                                int K, int Bn, int accumulate, int xvec, int wvec) {
  const int kq = threadIdx.x & 63, ng = threadIdx.x >> 6;
  const int k0 = blockIdx.x * 256 + 4 * kq;
  const int nb = blockIdx.y * 16 + 4 * ng;
  float acc[4][4] = {};
  float bs[4] = {0.f, 0.f, 0.f, 0.f};
  const bool vec = xvec && k0 + 3 < K;
  // batch rows 8 at a time with every load issued first (one memory round trip per
  // 8 rows instead of per row); same per-element fma order as the row loop below
  constexpr int RB = 8;
  int b = 0;
  if (vec)
    for (; b + RB <= Bn; b += RB) {
      f32x4 xr[RB];
      float dr[RB][4];
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        xr[u] = *reinterpret_cast<const f32x4*>(x + (b + u) * ldx + k0);
#pragma unroll
        for (int i = 0; i < 4; ++i) dr[u][i] = nb + i < N ? dy[(b + u) * ldy + nb + i] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < RB; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          bs[i] += dr[u][i];
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(dr[u][i], xr[u][j], acc[i][j]);
        }
    }
  for (; b < Bn; ++b) {
    float xv[4];
    if (vec) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(x + b * ldx + k0);
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[j] = v[j];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) xv[j] = k0 + j < K ? x[b * ldx + k0 + j] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float d = nb + i < N ? dy[b * ldy + nb + i] : 0.f;
      bs[i] += d;
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(d, xv[j], acc[i][j]);
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int nn = nb + i;
    if (nn >= N) continue;
    float* o = dw + (int64_t)nn * K + k0;
    if (wvec && k0 + 3 < K) {
      f32x4 v = {acc[i][0], acc[i][1], acc[i][2], acc[i][3]};
      if (accumulate) v += *reinterpret_cast<const f32x4*>(o);
      *reinterpret_cast<f32x4*>(o) = v;
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (k0 + j < K) o[j] = accumulate ? o[j] + acc[i][j] : acc[i][j];
    }
    if (db && blockIdx.x == 0 && kq == 0) db[nn] = accumulate ? db[nn] + bs[i] : bs[i];
  }
}

// C[m][n] = alpha * sum_z part[z][m][n] (+ bias[n]) + beta * C[m][n]   (fixed order)
__global__ void gemm_splitk_reduce_kernel(const float* __restrict__ part, int splits, float* __restrict__ C,
                                          int64_t ldc, const float* __restrict__ bias, int M, int N, float alpha,
                                          float beta, BnEv bn = BnEv{}) {
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (i >= (int64_t)M * N) return;
  const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
  float s = 0.f;
  for (int z = 0; z < splits; ++z) s += part[(int64_t)z * M * N + i];
  float v = alpha * s;
  if (bias) v += bias[n];
  if (beta != 0.f) v += beta * C[m * ldc + n];
  if (bn.on) v = bn_eval_apply(v, bn, n);
  C[m * ldc + n] = v;
}

// db[n] (+)= sum_m dy[m * ldy + n]
__global__ void colsum_kernel(const float* __restrict__ dy, int64_t ldy, float* __restrict__ db, int M, int N,
                              int accumulate) {
  const int n = blockIdx.x * kThreads + threadIdx.x;
  if (n >= N) return;
  float s = 0.f;
  for (int m = 0; m < M; ++m) s += dy[m * ldy + n];
  db[n] = accumulate ? db[n] + s : s;
}

using p6::uniform01;

// BatchNorm1d over the batch + optional ReLU + Dropout.  Block = 64 columns (one
// per lane: coalesced rows) x 4 row groups (one per wave, rows g, g+4, ...); the
// per-group fp64 sums meet in LDS and are combined in group order (deterministic).
constexpr int kBnCols = 64, kBnGroups = kThreads / kBnCols;
constexpr int kRU = 8;   // rows per apply trip (batch 32 = one trip of 4 groups x 8)

__device__ __forceinline__ double group_total(double v, double (*red)[kBnCols], int g, int cl) {
  red[g][cl] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int i = 0; i < kBnGroups; ++i) t += red[i][cl];
  __syncthreads();
  return t;
}

__global__ __launch_bounds__(kThreads) void bn1d_fwd_kernel(
    const float* __restrict__ x, float* __restrict__ y, int M, int C, const float* __restrict__ gamma,
    const float* __restrict__ beta, float* __restrict__ rmean, float* __restrict__ rvar, int64_t* __restrict__ nbt,
    float momentum, float eps, int training, int relu, float p_drop, const uint64_t* __restrict__ seedp, uint64_t salt,
    uint8_t* __restrict__ mask, float* __restrict__ smean, float* __restrict__ sinv) {
  __shared__ double red[kBnGroups][kBnCols];
  const int cl = threadIdx.x % kBnCols, g = threadIdx.x / kBnCols;
  const int c = blockIdx.x * kBnCols + cl;
  const bool ok = c < C;
  float mean, inv;
  if (training) {
    double s = 0.0;
    if (ok)
      for (int m = g; m < M; m += kBnGroups) s += x[(int64_t)m * C + c];
    mean = (float)(group_total(s, red, g, cl) / M);
    double q = 0.0;
    if (ok)
      for (int m = g; m < M; m += kBnGroups) { const double d = x[(int64_t)m * C + c] - mean; q += d * d; }
    const double var = group_total(q, red, g, cl) / M;
    inv = (float)(1.0 / sqrt(var + eps));
    if (ok && g == 0) {
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * mean;
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)(M > 1 ? var * M / (M - 1) : var);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && nbt) nbt[0] += 1;
  } else {
    mean = ok ? rmean[c] : 0.f;
    inv = ok ? 1.0f / sqrtf(rvar[c] + eps) : 0.f;
  }
  if (!ok) return;
  if (g == 0) {
    smean[c] = mean;
    sinv[c] = inv;
  }
  const float gm = gamma[c], b = beta[c];
  const float keep_scale = p_drop > 0.f ? 1.0f / (1.0f - p_drop) : 1.0f;
  const uint64_t seed = p_drop > 0.f ? seedp[0] ^ salt : 0;
  // kRU rows per trip, every load before the trip's stores (a load issued behind a
  // store waits for the store's acknowledgement)
  for (int m0 = g; m0 < M; m0 += kRU * kBnGroups) {
    float v[kRU];
#pragma unroll
    for (int u = 0; u < kRU; ++u) {
      const int m = m0 + u * kBnGroups;
      v[u] = m < M ? x[(int64_t)m * C + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kRU; ++u) {
      const int m = m0 + u * kBnGroups;
      if (m >= M) break;
      const int64_t o = (int64_t)m * C + c;
      float t = (v[u] - mean) * inv * gm + b;
      if (relu) t = fmaxf(t, 0.f);
      if (p_drop > 0.f) {
        const bool keep = uniform01(seed, (uint64_t)o) >= p_drop;
        mask[o] = keep;
        t = keep ? t * keep_scale : 0.f;
      }
      y[o] = t;
    }
  }
}

// backward of bn1d_fwd (train mode: batch statistics), same block shape
__global__ __launch_bounds__(kThreads) void bn1d_bwd_kernel(
    const float* __restrict__ dy, const float* __restrict__ x, const float* __restrict__ y, int M, int C,
    const float* __restrict__ gamma, const float* __restrict__ smean, const float* __restrict__ sinv, int training,
    int relu, float p_drop, const uint8_t* __restrict__ mask, float* __restrict__ dx, float* __restrict__ dgamma,
    float* __restrict__ dbeta, int accumulate) {
  __shared__ double red[kBnGroups][kBnCols];
  const int cl = threadIdx.x % kBnCols, g = threadIdx.x / kBnCols;
  const int c = blockIdx.x * kBnCols + cl;
  const bool ok = c < C;
  const float mean = ok ? smean[c] : 0.f, inv = ok ? sinv[c] : 0.f, gm = ok ? gamma[c] : 0.f;
  const float keep_scale = p_drop > 0.f ? 1.0f / (1.0f - p_drop) : 1.0f;
  auto grad_in = [&](int64_t o) {
    float d = dy[o];
    if (p_drop > 0.f) d = mask[o] ? d * keep_scale : 0.f;
    if (relu && !(y[o] > 0.f)) d = 0.f;
    return d;
  };
  double sd = 0.0, sdx = 0.0;
  if (ok)
    for (int m = g; m < M; m += kBnGroups) {
      const int64_t o = (int64_t)m * C + c;
      const float d = grad_in(o);
      sd += d;
      sdx += (double)d * ((x[o] - mean) * inv);
    }
  sd = group_total(sd, red, g, cl);
  sdx = group_total(sdx, red, g, cl);
  if (!ok) return;
  if (g == 0) {
    if (dgamma) dgamma[c] = (accumulate ? dgamma[c] : 0.f) + (float)sdx;
    if (dbeta) dbeta[c] = (accumulate ? dbeta[c] : 0.f) + (float)sd;
  }
  const float c2 = (float)(sd / M), c3 = (float)(sdx / M);
  for (int m0 = g; m0 < M; m0 += kRU * kBnGroups) {   // loads of a trip before its stores
    float dv[kRU], xv[kRU];
#pragma unroll
    for (int u = 0; u < kRU; ++u) {
      const int m = m0 + u * kBnGroups;
      const int64_t o = (int64_t)(m < M ? m : m0) * C + c;
      dv[u] = grad_in(o);
      xv[u] = x[o];
    }
#pragma unroll
    for (int u = 0; u < kRU; ++u) {
      const int m = m0 + u * kBnGroups;
      if (m >= M) break;
      const float xh = (xv[u] - mean) * inv;
      dx[(int64_t)m * C + c] = training ? gm * inv * (dv[u] - c2 - xh * c3) : gm * inv * dv[u];
    }
  }
}

// elementwise act (+dropout) used by the plain Linear->ReLU->Dropout layers
__global__ void act_fwd_kernel(const float* __restrict__ x, float* __restrict__ y, int64_t n, int act, float p_drop,
                               const uint64_t* __restrict__ seedp, uint64_t salt, uint8_t* __restrict__ mask) {
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (i >= n) return;
  float v = x[i];
  if (act == 1) v = fmaxf(v, 0.f);
  else if (act == 2) v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));  // exact GELU
  if (p_drop > 0.f) {
    const bool keep = uniform01(seedp[0] ^ salt, (uint64_t)i) >= p_drop;
    mask[i] = keep;
    v = keep ? v / (1.0f - p_drop) : 0.f;
  }
  y[i] = v;
}

__global__ void act_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x, float* __restrict__ dx,
                               int64_t n, int act, float p_drop, const uint8_t* __restrict__ mask) {
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (i >= n) return;
  float d = dy[i];
  if (p_drop > 0.f) d = mask[i] ? d / (1.0f - p_drop) : 0.f;
  const float v = x[i];
  if (act == 1) d = v > 0.f ? d : 0.f;
  else if (act == 2) {
    const float cdf = 0.5f * (1.0f + erff(v * 0.70710678118654752f));
    const float pdf = 0.39894228040143268f * expf(-0.5f * v * v);
    d = d * (cdf + v * pdf);
  }
  dx[i] = d;
}

}  // namespace

namespace {
int gemm_f32_impl(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C,
                  int64_t ldc, const float* bias, int32_t M, int32_t N, int32_t K, float alpha, float beta,
                  float* workspace, int64_t ws_floats, const BnEv& bn, void* stream);
}  // namespace

extern "C" int pose6d_gemm_f32(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                               float* C, int64_t ldc, const float* bias, int32_t M, int32_t N, int32_t K, float alpha,
                               float beta, float* workspace, int64_t ws_floats, void* stream) {
  return gemm_f32_impl(A, sam, sak, B, sbk, sbn, C, ldc, bias, M, N, K, alpha, beta, workspace, ws_floats, BnEv{},
                       stream);
}

extern "C" int pose6d_gemm_f32_bn_eval(const float* A, int64_t sam, const float* W, float* C, int64_t ldc,
                                       const float* bias, int32_t M, int32_t N, int32_t K, const float* gamma,
                                       const float* beta, const float* running_mean, const float* running_var,
                                       float eps, int32_t relu, float* workspace, int64_t ws_floats, void* stream) {
  P6_CHECK_ARG(M > 0 && M <= 32 && N > 0 && K > 0, "pose6d_gemm_f32_bn_eval: batch must be 1..32 (skinny path)");
  P6_CHECK_ARG(gamma && beta && running_mean && running_var, "pose6d_gemm_f32_bn_eval: null BatchNorm1d operand");
  const BnEv bn{gamma, beta, running_mean, running_var, eps, relu != 0, 1};
  return gemm_f32_impl(A, sam, 1, W, 1, K, C, ldc, bias, M, N, K, 1.f, 0.f, workspace, ws_floats, bn, stream);
}

namespace {
int gemm_f32_impl(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn, float* C,
                  int64_t ldc, const float* bias, int32_t M, int32_t N, int32_t K, float alpha, float beta,
                  float* workspace, int64_t ws_floats, const BnEv& bn, void* stream) {
  P6_CHECK_ARG(M >= 0 && N >= 0 && K >= 0, "pose6d_gemm_f32: bad sizes");
  if (M == 0 || N == 0) return POSE6D_OK;
  hipStream_t s = p6::stream_of(stream);
  // batch-side skinny GEMMs (nn.Linear forward / data gradient): MFMA kernel
  const bool bkc = sbk == 1, bnc = sbn == 1;
  if (M <= 32 && sak == 1 && (bkc || bnc)) {
    const bool vec = ((uintptr_t)A & 15) == 0 && (sam & 3) == 0 && (K & 3) == 0 &&
                     (!bkc || (((uintptr_t)B & 15) == 0 && (sbn & 3) == 0));
    // K slices: ~256 workgroups, each wave of a slice >= 16 deep (kSkW x 16 per slice),
    // for weights of >= 4 MiB only: below that the reduce launch (~5 us) costs more than
    // the slices save (1024 x 512: 8.6 us in one launch)
    const int groups = p6::ceil_div(N, 16);
    int slices = 1;
    if (workspace && groups < 256 && (int64_t)N * K >= (1 << 20)) {
      slices = p6::ceil_div(256, groups);
      const int by_k = K / (kSkW * 16);
      if (slices > by_k) slices = by_k;
      const int64_t by_ws = ws_floats / ((int64_t)M * N);
      if (slices > by_ws) slices = (int)by_ws;
      if (slices < 1) slices = 1;
    }
    const int kchunk = slices > 1 ? p6::ceil_div(p6::ceil_div(K, slices), 16) * 16 : K;
    slices = slices > 1 ? p6::ceil_div(K, kchunk) : 1;
    float* part = slices > 1 ? workspace : nullptr;
    const dim3 grid(groups, slices);
    if (bkc) {
      if (vec) skinny_gemm_kernel<true, true><<<grid, kSkThreads, 0, s>>>(A, sam, B, sbk, sbn, C, ldc, bias, M, N, K,
                                                                          alpha, beta, kchunk, part, bn);
      else skinny_gemm_kernel<true, false><<<grid, kSkThreads, 0, s>>>(A, sam, B, sbk, sbn, C, ldc, bias, M, N, K,
                                                                        alpha, beta, kchunk, part, bn);
    } else {
      if (vec) skinny_gemm_kernel<false, true><<<grid, kSkThreads, 0, s>>>(A, sam, B, sbk, sbn, C, ldc, bias, M, N, K,
                                                                           alpha, beta, kchunk, part, bn);
      else skinny_gemm_kernel<false, false><<<grid, kSkThreads, 0, s>>>(A, sam, B, sbk, sbn, C, ldc, bias, M, N, K,
                                                                         alpha, beta, kchunk, part, bn);
    }
    P6_LAUNCH_CHECK();
    if (part) {
      gemm_splitk_reduce_kernel<<<(unsigned)(((int64_t)M * N + kThreads - 1) / kThreads), kThreads, 0, s>>>(
          part, slices, C, ldc, bias, M, N, alpha, beta, bn);
      P6_LAUNCH_CHECK();
    }
    return POSE6D_OK;
  }
  P6_CHECK_ARG(!bn.on, "pose6d_gemm_f32_bn_eval: operands outside the skinny MFMA path (aligned, batch <= 32)");
  const int tiles = p6::ceil_div(N, TBN) * p6::ceil_div(M, TBM);
  // skinny (batch-32) GEMMs: split K so that >= ~256 workgroups stream the weights
  int splits = 1;
  if (workspace && tiles < 256) {
    splits = p6::ceil_div(256, tiles);
    const int by_k = p6::ceil_div(K, 4 * TBK);
    if (splits > by_k) splits = by_k;
    const int64_t by_ws = ws_floats / ((int64_t)M * N);
    if (splits > by_ws) splits = (int)by_ws;
    if (splits < 1) splits = 1;
  }
  const int kchunk = splits > 1 ? p6::ceil_div(p6::ceil_div(K, splits), TBK) * TBK : K;
  splits = splits > 1 ? p6::ceil_div(K, kchunk) : 1;
  dim3 grid(p6::ceil_div(N, TBN), p6::ceil_div(M, TBM), splits);
  gemm_f32_kernel<<<grid, kThreads, 0, s>>>(A, sam, sak, B, sbk, sbn, C, ldc, bias, M, N, K, alpha, beta, kchunk,
                                            splits > 1 ? workspace : nullptr);
  P6_LAUNCH_CHECK();
  if (splits > 1) {
    gemm_splitk_reduce_kernel<<<(unsigned)(((int64_t)M * N + kThreads - 1) / kThreads), kThreads, 0, s>>>(
        workspace, splits, C, ldc, bias, M, N, alpha, beta);
    P6_LAUNCH_CHECK();
  }
  return POSE6D_OK;
}
}  // namespace

extern "C" int pose6d_colsum_f32(const float* dy, int64_t ldy, float* db, int32_t M, int32_t N, int32_t accumulate,
                                 void* stream) {
  P6_CHECK_ARG(M >= 0 && N >= 0 && ldy >= N, "pose6d_colsum_f32: bad shape");
  if (N == 0) return POSE6D_OK;
  colsum_kernel<<<p6::ceil_div(N, kThreads), kThreads, 0, p6::stream_of(stream)>>>(dy, ldy, db, M, N, accumulate);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_bn1d_fwd(const float* x, float* y, int32_t M, int32_t C, const float* gamma, const float* beta,
                               float* running_mean, float* running_var, int64_t* num_batches, float momentum, float eps,
                               int32_t training, int32_t relu, float p_drop, const uint64_t* seed, uint64_t salt,
                               uint8_t* mask, float* save_mean, float* save_invstd, void* stream) {
  P6_CHECK_ARG(M > 0 && C > 0, "pose6d_bn1d_fwd: bad sizes");
  P6_CHECK_ARG(!training || M > 1, "Expected more than 1 value per channel when training (BatchNorm1d)");
  P6_CHECK_ARG(p_drop == 0.f || (mask && seed), "pose6d_bn1d_fwd: dropout needs a mask buffer and a seed");
  bn1d_fwd_kernel<<<p6::ceil_div(C, kBnCols), kThreads, 0, p6::stream_of(stream)>>>(
      x, y, M, C, gamma, beta, running_mean, running_var, num_batches, momentum, eps, training, relu, p_drop, seed, salt,
      mask, save_mean, save_invstd);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_bn1d_bwd(const float* dy, const float* x, const float* y, int32_t M, int32_t C,
                               const float* gamma, const float* save_mean, const float* save_invstd, int32_t training,
                               int32_t relu, float p_drop, const uint8_t* mask, float* dx, float* dgamma, float* dbeta,
                               int32_t accumulate, void* stream) {
  bn1d_bwd_kernel<<<p6::ceil_div(C, kBnCols), kThreads, 0, p6::stream_of(stream)>>>(
      dy, x, y, M, C, gamma, save_mean, save_invstd, training, relu, p_drop, mask, dx, dgamma, dbeta, accumulate);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_act_fwd(const float* x, float* y, int64_t n, int32_t act, float p_drop, const uint64_t* seed,
                              uint64_t salt, uint8_t* mask, void* stream) {
  if (n == 0) return POSE6D_OK;
  P6_CHECK_ARG(p_drop == 0.f || (mask && seed), "pose6d_act_fwd: dropout needs a mask buffer and a seed");
  act_fwd_kernel<<<(unsigned)((n + kThreads - 1) / kThreads), kThreads, 0, p6::stream_of(stream)>>>(x, y, n, act, p_drop,
                                                                                                 seed, salt, mask);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_act_bwd(const float* dy, const float* x, float* dx, int64_t n, int32_t act, float p_drop,
                              const uint8_t* mask, void* stream) {
  if (n == 0) return POSE6D_OK;
  act_bwd_kernel<<<(unsigned)((n + kThreads - 1) / kThreads), kThreads, 0, p6::stream_of(stream)>>>(dy, x, dx, n, act,
                                                                                                 p_drop, mask);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_linear_wgrad(const float* dy, int64_t ldy, const float* x, int64_t ldx, float* dw, float* db,
                                   int32_t N, int32_t K, int32_t B, int32_t accumulate, void* stream) {
  P6_CHECK_ARG(N > 0 && K > 0 && B >= 0 && ldy >= N && ldx >= K, "pose6d_linear_wgrad: bad shape");
  const dim3 grid(p6::ceil_div(K, 256), p6::ceil_div(N, 16));
  const int xvec = ((uintptr_t)x & 15) == 0 && (ldx & 3) == 0;
  const int wvec = ((uintptr_t)dw & 15) == 0 && (K & 3) == 0;
  linear_wgrad_kernel<<<grid, kThreads, 0, p6::stream_of(stream)>>>(dy, ldy, x, ldx, dw, db, N, K, B, accumulate,
                                                                    xvec, wvec);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

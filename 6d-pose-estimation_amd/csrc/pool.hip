// Layout, packing and pooling kernels of the ResNet50 trunk (NHWC).
//   pose6d_nchw_to_nhwc      model input (B,C,H,W) fp32 -> NHWC dtype, channels padded
//   pose6d_pack_conv_weights OIHW fp32 masters -> packed [Cout][Kpad] (+ transposed
//                            [Cin][KH][KW][Cout] for dgrad), all convs in ONE launch
//                            (grid.y = conv, grid.z = which layout; writes coalesced)
//   pose6d_maxpool_fwd/bwd   nn.MaxPool2d (ResNet stem 3x3/s2/p1; z-CNN 2x2/s2);
//                            first max in window scan order wins (torch CPU), the
//                            backward gathers in output order (deterministic);
//                            one lane per (pixel, 16-byte channel chunk)
//   pose6d_avgpool_fwd/bwd   nn.AdaptiveAvgPool2d(1) + view(B, -1)
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace {

constexpr int kThreads = 256;

template <typename T> struct V;
template <> struct V<bf16> { static constexpr int E = 8; };
template <> struct V<float> { static constexpr int E = 4; };

template <typename T>
__device__ __forceinline__ void ld(const T* p, float* f) {
  constexpr int E = V<T>::E;
  T t[E];
  *reinterpret_cast<uint4*>(t) = *reinterpret_cast<const uint4*>(p);
#pragma unroll
  for (int e = 0; e < E; ++e) f[e] = p6::to_f(t[e]);
}
template <typename T>
__device__ __forceinline__ void st(T* p, const float* f) {
  constexpr int E = V<T>::E;
  T t[E];
#pragma unroll
  for (int e = 0; e < E; ++e) t[e] = p6::from_f<T>(f[e]);
  *reinterpret_cast<uint4*>(p) = *reinterpret_cast<const uint4*>(t);
}

template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ y, int N, int C, int HW, int Cp) {
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;  // pixel
  if (i >= (int64_t)N * HW) return;
  const int64_t n = i / HW, p = i - n * HW;
  for (int c = 0; c < Cp; ++c) y[i * Cp + c] = p6::from_f<T>(c < C ? x[(n * C + c) * HW + p] : 0.f);
}

// The model input (NCHW fp32, C <= 4 channels padded to 4) -> NHWC: four consecutive
// pixels per thread, one 16-byte load per channel plane and the 4 x 4 output
// elements as whole 16-byte stores (the per-element form issued a 2-byte store per
// element: 12.6 us for the bs32 batch in the training step, 18 us cold in eval).
template <typename T>
__global__ void nchw4_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ y, int N, int C, int HW) {
  const int64_t q = blockIdx.x * (int64_t)kThreads + threadIdx.x;   // pixel quad
  const int64_t nq = (int64_t)N * HW / 4;
  if (q >= nq) return;
  const int64_t i = q * 4;                    // first pixel (HW % 4 == 0: a quad stays in one image)
  const int64_t n = i / HW, p = i - n * HW;
  float4 v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
    v[c] = c < C ? *reinterpret_cast<const float4*>(x + (n * C + c) * HW + p) : make_float4(0.f, 0.f, 0.f, 0.f);
  const float px[4][4] = {{v[0].x, v[1].x, v[2].x, v[3].x}, {v[0].y, v[1].y, v[2].y, v[3].y},
                          {v[0].z, v[1].z, v[2].z, v[3].z}, {v[0].w, v[1].w, v[2].w, v[3].w}};
  if constexpr (sizeof(T) == 2) {
    T o[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) o[e] = p6::from_f<T>(px[e >> 2][e & 3]);
    uint4 w[2];
    __builtin_memcpy(w, o, 32);
    uint4* d = reinterpret_cast<uint4*>(y + i * 4);
    d[0] = w[0];
    d[1] = w[1];
  } else {
    float4* d = reinterpret_cast<float4*>(y + i * 4);
#pragma unroll
    for (int k = 0; k < 4; ++k) d[k] = make_float4(px[k][0], px[k][1], px[k][2], px[k][3]);
  }
}

using p6::PackDesc;

// z = 0: wp[o][k], k = (kh, kw, ci).  1x1 filters (k order == OIHW order): a straight
//        fp32 -> compute-dtype conversion, 8 elements per thread (two float4 loads, one
//        16-B store).  Larger filters: each OIHW row o is staged in LDS with float4
//        loads, then written in (kh, kw, ci) order two elements per store, with
//        channel / K padding.
// z = 1: wt[(ci, kh, kw)][o] is the transpose of w viewed as [O][I*KH*KW]: 64 x 64
//        tiles through LDS, float4 loads, two-element stores.
constexpr int kPackRow = 4608;   // largest staged row (512 x 3 x 3); longer rows gather directly

template <typename T>
__device__ __forceinline__ void store2(T* p, float a, float b) {
  if constexpr (sizeof(T) == 2) {
    const bf16 v[2] = {(bf16)a, (bf16)b};
    uint32_t u;
    __builtin_memcpy(&u, v, 4);
    *reinterpret_cast<uint32_t*>(p) = u;
  } else {
    *reinterpret_cast<float2*>(p) = make_float2(a, b);
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void pack_kernel(const PackDesc* __restrict__ descs) {
  __shared__ float sm[kPackRow > 64 * 65 ? kPackRow : 64 * 65];
  const PackDesc d = descs[blockIdx.y];
  const int taps = d.KH * d.KW;
  const int R = d.I * taps;
  const int tid = threadIdx.x;
  if (blockIdx.z == 0) {
    if (taps == 1 && d.Ip == d.I && d.Kpad == d.I && (d.I & 7) == 0) {
      const int64_t n8 = (int64_t)d.O * d.I / 8;
      for (int64_t q = blockIdx.x * (int64_t)kThreads + tid; q < n8; q += (int64_t)gridDim.x * kThreads) {
        const float4 a = *reinterpret_cast<const float4*>(d.w + q * 8);
        const float4 b = *reinterpret_cast<const float4*>(d.w + q * 8 + 4);
        T* dst = reinterpret_cast<T*>(d.wp) + q * 8;
        store2(dst, a.x, a.y);
        store2(dst + 2, a.z, a.w);
        store2(dst + 4, b.x, b.y);
        store2(dst + 6, b.z, b.w);
      }
      return;
    }
    const bool vec = (R & 3) == 0 && R <= kPackRow;
    const int kwp = d.KWp > 0 ? d.KWp : d.KW, shift = kwp - d.KW;   // packed taps per kernel row
    const int Kp = d.KH * kwp * d.Ip;
    for (int o = blockIdx.x; o < d.O; o += gridDim.x) {
      const float* row = d.w + (int64_t)o * R;
      const bool staged = R <= kPackRow;
      if (vec) {
        for (int r = tid * 4; r < R; r += kThreads * 4)
          *reinterpret_cast<float4*>(sm + r) = *reinterpret_cast<const float4*>(row + r);
        __syncthreads();
      } else if (staged) {
        for (int r = tid; r < R; r += kThreads) sm[r] = row[r];
        __syncthreads();
      }
      T* dst = reinterpret_cast<T*>(d.wp) + (int64_t)o * d.Kpad;
      for (int k = tid * 2; k < d.Kpad; k += kThreads * 2) {   // Kpad is even
        float v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int kk = k + h;
          v[h] = 0.f;
          if (kk < Kp) {
            const int pt = kk / d.Ip, c = kk - pt * d.Ip;
            const int kh = pt / kwp, kw = pt - kh * kwp - shift;
            const int tap = kh * d.KW + kw;
            if (c < d.I && kw >= 0) v[h] = staged ? sm[c * taps + tap] : row[c * taps + tap];
          }
        }
        store2(dst + k, v[0], v[1]);
      }
      __syncthreads();
    }
  } else if (d.wt) {
    const int tr = p6::ceil_div(R, 64), to = p6::ceil_div(d.O, 64);
    const bool vec = (R & 3) == 0 && (d.O & 1) == 0;
    const int tx4 = tid & 15, ty = tid >> 4;        // loads: 16 float4 columns x 16 rows per pass
    const int px = tid & 31, py = tid >> 5;         // stores: 32 element pairs x 8 rows per pass
    for (int t = blockIdx.x; t < tr * to; t += gridDim.x) {
      const int o0 = (t / tr) * 64, r0 = (t - (t / tr) * tr) * 64;
#pragma unroll
      for (int i = ty; i < 64; i += 16) {   // rows o0 + i of w, columns r0 + 4 tx4 ..
        const int o = o0 + i, r = r0 + 4 * tx4;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (o < d.O) {
          if (vec && r + 3 < R) {
            v = *reinterpret_cast<const float4*>(d.w + (int64_t)o * R + r);
          } else {
            const float* src = d.w + (int64_t)o * R;
            v.x = r < R ? src[r] : 0.f;
            v.y = r + 1 < R ? src[r + 1] : 0.f;
            v.z = r + 2 < R ? src[r + 2] : 0.f;
            v.w = r + 3 < R ? src[r + 3] : 0.f;
          }
        }
        float* q = sm + i * 65 + 4 * tx4;
        q[0] = v.x; q[1] = v.y; q[2] = v.z; q[3] = v.w;
      }
      __syncthreads();
      T* wt = reinterpret_cast<T*>(d.wt);
#pragma unroll
      for (int i = py; i < 64; i += 8) {   // rows r0 + i of wt, columns o0 + 2 px ..
        const int r = r0 + i, o = o0 + 2 * px;
        if (r >= R) continue;
        const float a = sm[(2 * px) * 65 + i], b = sm[(2 * px + 1) * 65 + i];
        if (vec && o + 1 < d.O) {
          store2(wt + (int64_t)r * d.O + o, a, b);
        } else {
          if (o < d.O) wt[(int64_t)r * d.O + o] = p6::from_f<T>(a);
          if (o + 1 < d.O) wt[(int64_t)r * d.O + o + 1] = p6::from_f<T>(b);
        }
      }
      __syncthreads();
    }
  }
}

// One lane per (output pixel, 16-byte channel chunk).  BN: the window
// element is T(max(y * scale + shift, 0)), exactly what pose6d_bn_act_fwd would have
// stored (the stem / z-CNN act -> pool pairs), so the pooled values and argmax equal
// bn_act_fwd followed by maxpool_fwd bit for bit -- without writing and re-reading the
// full-resolution activation (nothing else reads it: the backward recomputes the ReLU
// sign from y and routes the pool gradient by argmax).
template <typename T, bool BN>
__global__ __launch_bounds__(kThreads) void pool_fwd_kernel(const T* __restrict__ x, const float* __restrict__ scale,
                                                            const float* __restrict__ shift, T* __restrict__ y,
                                                            uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                            int Ho, int Wo, int k, int s, int p) {
  constexpr int E = V<T>::E;
  const int cpr = C / E;
  // grid (ceil(Wo * cpr / 256), N * Ho): one output row per blockIdx.y
  const int i = blockIdx.x * kThreads + threadIdx.x;  // (column, chunk) within the output row
  if (i >= Wo * cpr) return;
  const int n = blockIdx.y / Ho, oy = blockIdx.y - n * Ho;
  const int ox = i / cpr, c0 = (i - ox * cpr) * E;
  const int64_t pix = ((int64_t)n * Ho + oy) * Wo + ox;
  float sc[E], sh[E], best[E];
  uint8_t bi[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    if constexpr (BN) {
      sc[e] = scale[c0 + e];
      sh[e] = shift[c0 + e];
    }
    best[e] = -__builtin_inff();
    bi[e] = 0;
  }
  bool first = true;
  auto take = [&](const float* raw, int j) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float v = raw[e];
      if constexpr (BN) v = p6::to_f(p6::from_f<T>(fmaxf(fmaf(v, sc[e], sh[e]), 0.f)));
      if (first || v > best[e] || v != v) { best[e] = v; bi[e] = (uint8_t)j; }
    }
    first = false;
  };
  const T* xn = x + (int64_t)n * H * W * C + c0;
  for (int kh = 0; kh < k; ++kh) {
    const int iy = oy * s - p + kh;
    if (iy < 0 || iy >= H) continue;
    for (int kw = 0; kw < k; ++kw) {
      const int ix = ox * s - p + kw;
      if (ix < 0 || ix >= W) continue;
      float v[E];
      ld(xn + ((int64_t)iy * W + ix) * C, v);
      take(v, kh * k + kw);
    }
  }
  st(y + pix * C + c0, best);
  if (idx) {
    if constexpr (E == 8) {
      uint2 u;
      __builtin_memcpy(&u, bi, 8);
      *reinterpret_cast<uint2*>(idx + pix * C + c0) = u;
    } else {
      uint32_t u;
      __builtin_memcpy(&u, bi, 4);
      *reinterpret_cast<uint32_t*>(idx + pix * C + c0) = u;
    }
  }
}

template <typename T, bool BN>
void launch_pool_fwd(dim3 grid, hipStream_t st_, const T* x, const float* scale, const float* shift, T* y,
                     uint8_t* idx, int N, int H, int W, int C, int Ho, int Wo, int k, int s, int p) {
  pool_fwd_kernel<T, BN><<<grid, kThreads, 0, st_>>>(x, scale, shift, y, idx, N, H, W, C, Ho, Wo, k, s, p);
}

// NW > 0: at most NW windows per axis contain an input pixel (ceil(k / s) <= NW: 2 for
// the 3x3 / s2 stem pool, 1 for the z-CNN 2x2 / s2 pools); all NW * NW candidate dy / argmax
// loads are issued up front (out-of-range candidates read a clamped in-range window and
// are skipped), then summed in the same (oy, ox) order as the generic loop -- bit-identical.
template <typename T, int NW>
__global__ __launch_bounds__(kThreads) void maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ idx,
                                                               T* __restrict__ dx, int N, int H, int W, int C, int Ho,
                                                               int Wo, int k, int s, int p) {
  constexpr int E = V<T>::E;
  using IdxVec = typename std::conditional<E == 8, uint2, uint32_t>::type;
  const int cpr = C / E;
  // grid (ceil(W * cpr / 256), N * H): one input row per blockIdx.y
  const int i = blockIdx.x * kThreads + threadIdx.x;  // (column, chunk) within the row
  if (i >= W * cpr) return;
  const int n = blockIdx.y / H, iy = blockIdx.y - n * H;
  const int ix = i / cpr, c0 = (i - ix * cpr) * E;
  const int64_t pix = ((int64_t)n * H + iy) * W + ix;
  // windows containing (iy, ix): oy*s - p <= iy <= oy*s - p + k - 1
  const int oy0 = max(0, (iy + p - k + s) / s), oy1 = min(Ho - 1, (iy + p) / s);
  const int ox0 = max(0, (ix + p - k + s) / s), ox1 = min(Wo - 1, (ix + p) / s);
  float g[E];
#pragma unroll
  for (int e = 0; e < E; ++e) g[e] = 0.f;
  auto add = [&](const uint4& draw, IdxVec iraw, uint8_t me) {
    uint8_t bi[E];
    __builtin_memcpy(bi, &iraw, E);
    T t[E];
    __builtin_memcpy(t, &draw, 16);
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (bi[e] == me) g[e] += p6::to_f(t[e]);
  };
  const int64_t nbase = (int64_t)n * Ho * Wo * C + c0;
  if constexpr (NW > 0) {
    uint4 draw[NW * NW];
    IdxVec iraw[NW * NW];
    uint8_t me[NW * NW];
    bool ok[NW * NW];
#pragma unroll
    for (int a = 0; a < NW; ++a) {
      const int oy = oy0 + a;
      const int cy = oy < Ho ? oy : Ho - 1;
#pragma unroll
      for (int b = 0; b < NW; ++b) {
        const int ox = ox0 + b;
        const int cx = ox < Wo ? ox : Wo - 1;
        const int kh = iy - (oy * s - p), kw = ix - (ox * s - p);
        const int j = a * NW + b;
        ok[j] = oy <= oy1 && ox <= ox1 && kh >= 0 && kw >= 0 && kh < k && kw < k;
        me[j] = (uint8_t)(kh * k + kw);
        const int64_t o = nbase + ((int64_t)cy * Wo + cx) * C;
        draw[j] = *reinterpret_cast<const uint4*>(dy + o);
        iraw[j] = *reinterpret_cast<const IdxVec*>(idx + o);
      }
    }
#pragma unroll
    for (int j = 0; j < NW * NW; ++j)
      if (ok[j]) add(draw[j], iraw[j], me[j]);
  } else {
    for (int oy = oy0; oy <= oy1; ++oy)
      for (int ox = ox0; ox <= ox1; ++ox) {
        const int kh = iy - (oy * s - p), kw = ix - (ox * s - p);
        if (kh < 0 || kw < 0 || kh >= k || kw >= k) continue;
        const int64_t o = nbase + ((int64_t)oy * Wo + ox) * C;
        add(*reinterpret_cast<const uint4*>(dy + o), *reinterpret_cast<const IdxVec*>(idx + o),
            (uint8_t)(kh * k + kw));
      }
  }
  st(dx + pix * C + c0, g);
}

// the compile-time-window backward for RPT consecutive input rows per lane (grid.y =
// N * H / RPT): the candidate loads of all RPT rows are issued before the first sum,
// so each wave keeps RPT * NW * NW window loads in flight and the grid needs RPT times
// fewer waves (the stem pool's dx is 51 MB: one load round trip per wave, 7 rounds of
// waves per CU at RPT = 1)
template <typename T, int NW, int RPT>
__global__ __launch_bounds__(kThreads) void maxpool_bwd_rows_kernel(const T* __restrict__ dy,
                                                                    const uint8_t* __restrict__ idx,
                                                                    T* __restrict__ dx, int N, int H, int W, int C,
                                                                    int Ho, int Wo, int k, int s, int p) {
  constexpr int E = V<T>::E;
  using IdxVec = typename std::conditional<E == 8, uint2, uint32_t>::type;
  const int cpr = C / E;
  const int i = blockIdx.x * kThreads + threadIdx.x;  // (column, chunk) within the row
  if (i >= W * cpr) return;
  const int HG = H / RPT;
  const int n = blockIdx.y / HG, iyb = (blockIdx.y - n * HG) * RPT;
  const int ix = i / cpr, c0 = (i - ix * cpr) * E;
  const int ox0 = max(0, (ix + p - k + s) / s), ox1 = min(Wo - 1, (ix + p) / s);
  const int64_t nbase = (int64_t)n * Ho * Wo * C + c0;
  uint4 draw[RPT][NW * NW];
  IdxVec iraw[RPT][NW * NW];
  uint8_t me[RPT][NW * NW];
  bool ok[RPT][NW * NW];
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    const int iy = iyb + r;
    const int oy0 = max(0, (iy + p - k + s) / s), oy1 = min(Ho - 1, (iy + p) / s);
#pragma unroll
    for (int a = 0; a < NW; ++a) {
      const int oy = oy0 + a;
      const int cy = oy < Ho ? oy : Ho - 1;
#pragma unroll
      for (int b = 0; b < NW; ++b) {
        const int ox = ox0 + b;
        const int cx = ox < Wo ? ox : Wo - 1;
        const int kh = iy - (oy * s - p), kw = ix - (ox * s - p);
        const int j = a * NW + b;
        ok[r][j] = oy <= oy1 && ox <= ox1 && kh >= 0 && kw >= 0 && kh < k && kw < k;
        me[r][j] = (uint8_t)(kh * k + kw);
        const int64_t o = nbase + ((int64_t)cy * Wo + cx) * C;
        draw[r][j] = *reinterpret_cast<const uint4*>(dy + o);
        iraw[r][j] = *reinterpret_cast<const IdxVec*>(idx + o);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RPT; ++r) {
    float g[E];
#pragma unroll
    for (int e = 0; e < E; ++e) g[e] = 0.f;
#pragma unroll
    for (int j = 0; j < NW * NW; ++j) {
      if (!ok[r][j]) continue;
      uint8_t bi[E];
      __builtin_memcpy(bi, &iraw[r][j], E);
      T t[E];
      __builtin_memcpy(t, &draw[r][j], 16);
#pragma unroll
      for (int e = 0; e < E; ++e)
        if (bi[e] == me[r][j]) g[e] += p6::to_f(t[e]);
    }
    st(dx + (((int64_t)n * H + iyb + r) * W + ix) * C + c0, g);
  }
}

template <typename T>
void launch_pool_bwd(int nw, dim3 grid, hipStream_t st_, const T* dy, const uint8_t* idx, T* dx, int N, int H, int W,
                     int C, int Ho, int Wo, int k, int s, int p) {
  // two input rows per lane (1 and 4 measured slower: profiles/r02f_pool_bwd_rows.txt)
  if (nw == 2 && H % 2 == 0) {
    grid.y /= 2;
    maxpool_bwd_rows_kernel<T, 2, 2><<<grid, kThreads, 0, st_>>>(dy, idx, dx, N, H, W, C, Ho, Wo, k, s, p);
  } else if (nw <= 1) {
    maxpool_bwd_kernel<T, 1><<<grid, kThreads, 0, st_>>>(dy, idx, dx, N, H, W, C, Ho, Wo, k, s, p);
  } else if (nw == 2) {
    maxpool_bwd_kernel<T, 2><<<grid, kThreads, 0, st_>>>(dy, idx, dx, N, H, W, C, Ho, Wo, k, s, p);
  } else {
    maxpool_bwd_kernel<T, 0><<<grid, kThreads, 0, st_>>>(dy, idx, dx, N, H, W, C, Ho, Wo, k, s, p);
  }
}

// block = 64 channel chunks (lanes) x 4 pixel groups (waves), grid (chunk groups, N);
// the four group sums meet in LDS in fixed order
template <typename T>
__global__ __launch_bounds__(kThreads) void avgpool_fwd_kernel(const T* __restrict__ x, float* __restrict__ y, int N,
                                                               int HW, int C) {
  constexpr int E = V<T>::E;
  __shared__ float red[4][64][E + 1];
  const int cpr = C / E;
  const int cl = threadIdx.x & 63, pg = threadIdx.x >> 6;
  const int ch = blockIdx.x * 64 + cl;
  const int64_t n = blockIdx.y;
  float s[E];
#pragma unroll
  for (int e = 0; e < E; ++e) s[e] = 0.f;
  if (ch < cpr) {
    int p = pg;
    for (; p + 12 < HW; p += 16) {
      float v[4][E];
#pragma unroll
      for (int u = 0; u < 4; ++u) ld(x + (n * HW + p + 4 * u) * C + ch * E, v[u]);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int e = 0; e < E; ++e) s[e] += v[u][e];
    }
    for (; p < HW; p += 4) {
      float v[E];
      ld(x + (n * HW + p) * C + ch * E, v);
#pragma unroll
      for (int e = 0; e < E; ++e) s[e] += v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < E; ++e) red[pg][cl][e] = s[e];
  __syncthreads();
  if (pg == 0 && ch < cpr) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float t = ((red[0][cl][e] + red[1][cl][e]) + red[2][cl][e]) + red[3][cl][e];
      y[n * C + ch * E + e] = t / (float)HW;
    }
  }
}

template <typename T>
__global__ void avgpool_bwd_kernel(const float* __restrict__ dy, T* __restrict__ dx, int N, int HW, int C) {
  constexpr int E = V<T>::E;
  const int cpr = C / E;
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;   // (pixel, chunk)
  if (i >= (int64_t)N * HW * cpr) return;
  const int c0 = (int)(i % cpr) * E;
  const int64_t pix = i / cpr;
  const int64_t n = pix / HW;
  float v[E];
#pragma unroll
  for (int e = 0; e < E; ++e) v[e] = dy[n * C + c0 + e] / (float)HW;
  st(dx + pix * C + c0, v);
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

}  // namespace

extern "C" int pose6d_nchw_to_nhwc(int32_t dtype, const float* x, void* y, int32_t N, int32_t C, int32_t H, int32_t W,
                                   int32_t Cpad, void* stream) {
  P6_CHECK_ARG(Cpad >= C, "pose6d_nchw_to_nhwc: Cpad < C");
  const int64_t n = (int64_t)N * H * W;
  if (n == 0) return POSE6D_OK;
  hipStream_t s = p6::stream_of(stream);
  if (Cpad == 4 && C <= 4 && (H * W) % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)y & 15) == 0) {
    if (dtype == POSE6D_DT_BF16)
      nchw4_to_nhwc_kernel<bf16><<<blocks(n / 4), kThreads, 0, s>>>(x, (bf16*)y, N, C, H * W);
    else
      nchw4_to_nhwc_kernel<float><<<blocks(n / 4), kThreads, 0, s>>>(x, (float*)y, N, C, H * W);
  } else if (dtype == POSE6D_DT_BF16)
    nchw_to_nhwc_kernel<bf16><<<blocks(n), kThreads, 0, s>>>(x, (bf16*)y, N, C, H * W, Cpad);
  else
    nchw_to_nhwc_kernel<float><<<blocks(n), kThreads, 0, s>>>(x, (float*)y, N, C, H * W, Cpad);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

// descs: host-built table already copied to device memory (n_desc entries of
// pose6d_pack_desc_size() bytes each, see pose6d.h for the field order)
extern "C" int pose6d_pack_desc_size(void) { return (int)sizeof(PackDesc); }

extern "C" int pose6d_pack_conv_weights(int32_t dtype, const void* descs, int32_t n_desc, int64_t total,
                                        void* stream) {
  (void)total;
  if (n_desc == 0) return POSE6D_OK;
  P6_CHECK_ARG(n_desc <= 65535, "pose6d_pack_conv_weights: too many descriptors");
  hipStream_t s = p6::stream_of(stream);
  dim3 grid(256, n_desc, 2);
  if (dtype == POSE6D_DT_BF16) pack_kernel<bf16><<<grid, kThreads, 0, s>>>((const PackDesc*)descs);
  else pack_kernel<float><<<grid, kThreads, 0, s>>>((const PackDesc*)descs);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

#define P6_POOL_CHECK(C, dtype) \
  P6_CHECK_ARG((C) % ((dtype) == POSE6D_DT_BF16 ? 8 : 4) == 0, "%s: C %% vector width != 0", __func__)

extern "C" int pose6d_maxpool_fwd(int32_t dtype, const void* x, void* y, uint8_t* argmax, int32_t N, int32_t H,
                                  int32_t W, int32_t C, int32_t k, int32_t s, int32_t p, int32_t Ho, int32_t Wo,
                                  void* stream) {
  P6_CHECK_ARG(k * k <= 255, "pose6d_maxpool_fwd: window too large");
  P6_POOL_CHECK(C, dtype);
  hipStream_t st_ = p6::stream_of(stream);
  if ((int64_t)N * Ho * Wo == 0) return POSE6D_OK;
  const int E = dtype == POSE6D_DT_BF16 ? 8 : 4;
  const dim3 grid(p6::ceil_div((int64_t)Wo * (C / E), kThreads), N * Ho);
  if (dtype == POSE6D_DT_BF16)
    launch_pool_fwd<bf16, false>(grid, st_, (const bf16*)x, nullptr, nullptr, (bf16*)y, argmax, N, H, W, C, Ho, Wo, k,
                                 s, p);
  else
    launch_pool_fwd<float, false>(grid, st_, (const float*)x, nullptr, nullptr, (float*)y, argmax, N, H, W, C, Ho, Wo,
                                  k, s, p);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_bn_relu_maxpool_fwd(int32_t dtype, const void* x, const float* scale, const float* shift,
                                          void* y, uint8_t* argmax, int32_t N, int32_t H, int32_t W, int32_t C,
                                          int32_t k, int32_t s, int32_t p, int32_t Ho, int32_t Wo, void* stream) {
  P6_CHECK_ARG(k * k <= 255, "pose6d_bn_relu_maxpool_fwd: window too large");
  P6_CHECK_ARG(scale && shift, "pose6d_bn_relu_maxpool_fwd: null scale / shift");
  P6_POOL_CHECK(C, dtype);
  hipStream_t st_ = p6::stream_of(stream);
  if ((int64_t)N * Ho * Wo == 0) return POSE6D_OK;
  const int E = dtype == POSE6D_DT_BF16 ? 8 : 4;
  const dim3 grid(p6::ceil_div((int64_t)Wo * (C / E), kThreads), N * Ho);
  if (dtype == POSE6D_DT_BF16)
    launch_pool_fwd<bf16, true>(grid, st_, (const bf16*)x, scale, shift, (bf16*)y, argmax, N, H, W, C, Ho, Wo, k, s, p);
  else
    launch_pool_fwd<float, true>(grid, st_, (const float*)x, scale, shift, (float*)y, argmax, N, H, W, C, Ho, Wo, k, s,
                                 p);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_maxpool_bwd(int32_t dtype, const void* dy, const uint8_t* argmax, void* dx, int32_t N, int32_t H,
                                  int32_t W, int32_t C, int32_t k, int32_t s, int32_t p, int32_t Ho, int32_t Wo,
                                  void* stream) {
  P6_POOL_CHECK(C, dtype);
  hipStream_t st_ = p6::stream_of(stream);
  if ((int64_t)N * H * W == 0) return POSE6D_OK;
  const int E = dtype == POSE6D_DT_BF16 ? 8 : 4;
  const dim3 grid(p6::ceil_div((int64_t)W * (C / E), kThreads), N * H);
  const int nw = (k + s - 1) / s;   // windows per axis containing one input pixel, at most
  if (dtype == POSE6D_DT_BF16)
    launch_pool_bwd<bf16>(nw, grid, st_, (const bf16*)dy, argmax, (bf16*)dx, N, H, W, C, Ho, Wo, k, s, p);
  else
    launch_pool_bwd<float>(nw, grid, st_, (const float*)dy, argmax, (float*)dx, N, H, W, C, Ho, Wo, k, s, p);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_avgpool_fwd(int32_t dtype, const void* x, float* y, int32_t N, int32_t HW, int32_t C,
                                  void* stream) {
  P6_POOL_CHECK(C, dtype);
  hipStream_t st_ = p6::stream_of(stream);
  const int E = dtype == POSE6D_DT_BF16 ? 8 : 4;
  const int64_t n = (int64_t)N * (C / E);
  if (n == 0) return POSE6D_OK;
  const dim3 grid(p6::ceil_div(C / E, 64), N);
  if (dtype == POSE6D_DT_BF16) avgpool_fwd_kernel<bf16><<<grid, kThreads, 0, st_>>>((const bf16*)x, y, N, HW, C);
  else avgpool_fwd_kernel<float><<<grid, kThreads, 0, st_>>>((const float*)x, y, N, HW, C);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_avgpool_bwd(int32_t dtype, const float* dy, void* dx, int32_t N, int32_t HW, int32_t C,
                                  void* stream) {
  P6_POOL_CHECK(C, dtype);
  hipStream_t st_ = p6::stream_of(stream);
  const int E = dtype == POSE6D_DT_BF16 ? 8 : 4;
  const int64_t n = (int64_t)N * HW * (C / E);
  if (n == 0) return POSE6D_OK;
  if (dtype == POSE6D_DT_BF16) avgpool_bwd_kernel<bf16><<<blocks(n), kThreads, 0, st_>>>(dy, (bf16*)dx, N, HW, C);
  else avgpool_bwd_kernel<float><<<blocks(n), kThreads, 0, st_>>>(dy, (float*)dx, N, HW, C);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

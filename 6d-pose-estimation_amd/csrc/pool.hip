// Layout, packing and pooling kernels of the ResNet50 trunk (NHWC).
//   pose6d_nchw_to_nhwc      model input (B,C,H,W) fp32 -> NHWC dtype, channels padded
//   pose6d_pack_conv_weights OIHW fp32 masters -> packed [Cout][Kpad] (+ transposed
//                            [Cin][KH][KW][Cout] for dgrad), all convs in ONE launch
//   pose6d_maxpool_fwd/bwd   nn.MaxPool2d (ResNet stem 3x3/s2/p1; z-CNN 2x2/s2);
//                            first max in window scan order wins (torch CPU), the
//                            backward gathers in output order (deterministic)
//   pose6d_avgpool_fwd/bwd   nn.AdaptiveAvgPool2d(1) + view(B, -1)
#include "common.h"

namespace {

constexpr int kThreads = 256;

template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, T* __restrict__ y, int N, int C, int HW, int Cp) {
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;  // pixel
  if (i >= (int64_t)N * HW) return;
  const int64_t n = i / HW, p = i - n * HW;
  for (int c = 0; c < Cp; ++c) y[i * Cp + c] = p6::from_f<T>(c < C ? x[(n * C + c) * HW + p] : 0.f);
}

struct PackDesc {
  const float* w;   // OIHW fp32
  void* wp;         // [O][Kpad]
  void* wt;         // [I][KH][KW][O] or null
  int O, I, Ip, KH, KW, Kpad;
  int64_t start, count;  // element range of this conv in the flattened [O][Kpad] index space
};

template <typename T>
__global__ void pack_kernel(const PackDesc* __restrict__ descs, int nd, int64_t total) {
  for (int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kThreads) {
    int lo = 0, hi = nd - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (descs[mid].start <= i) lo = mid; else hi = mid - 1;
    }
    const PackDesc d = descs[lo];
    const int64_t j = i - d.start;
    const int o = (int)(j / d.Kpad), k = (int)(j - (int64_t)o * d.Kpad);
    const int K = d.KH * d.KW * d.Ip;
    float v = 0.f;
    int tap = 0, c = 0, kh = 0, kw = 0;
    if (k < K) {
      tap = k / d.Ip; c = k - tap * d.Ip; kh = tap / d.KW; kw = tap - kh * d.KW;
      if (c < d.I) v = d.w[(((int64_t)o * d.I + c) * d.KH + kh) * d.KW + kw];
    }
    reinterpret_cast<T*>(d.wp)[j] = p6::from_f<T>(v);
    if (d.wt && k < K && c < d.I)  // wt[c][kh][kw][o]
      reinterpret_cast<T*>(d.wt)[(((int64_t)c * d.KH + kh) * d.KW + kw) * d.O + o] = p6::from_f<T>(v);
  }
}

template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, uint8_t* __restrict__ idx, int N, int H,
                                   int W, int C, int Ho, int Wo, int k, int s, int p) {
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;  // output element
  const int64_t total = (int64_t)N * Ho * Wo * C;
  if (i >= total) return;
  const int c = i % C;
  const int64_t pix = i / C;
  const int ox = pix % Wo, oy = (pix / Wo) % Ho, n = pix / ((int64_t)Wo * Ho);
  float best = -__builtin_inff();
  int bi = 0;
  bool any = false;
  for (int kh = 0; kh < k; ++kh) {
    const int iy = oy * s - p + kh;
    if (iy < 0 || iy >= H) continue;
    for (int kw = 0; kw < k; ++kw) {
      const int ix = ox * s - p + kw;
      if (ix < 0 || ix >= W) continue;
      const float v = p6::to_f(x[(((int64_t)n * H + iy) * W + ix) * C + c]);
      if (!any || v > best || v != v) { best = v; bi = kh * k + kw; any = true; }
    }
  }
  y[i] = p6::from_f<T>(best);
  if (idx) idx[i] = (uint8_t)bi;
}

template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ idx, T* __restrict__ dx, int N,
                                   int H, int W, int C, int Ho, int Wo, int k, int s, int p) {
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;  // input element
  const int64_t total = (int64_t)N * H * W * C;
  if (i >= total) return;
  const int c = i % C;
  const int64_t pix = i / C;
  const int ix = pix % W, iy = (pix / W) % H, n = pix / ((int64_t)W * H);
  // windows containing (iy, ix): oy*s - p <= iy <= oy*s - p + k - 1
  const int oy0 = max(0, (iy + p - k + s) / s), oy1 = min(Ho - 1, (iy + p) / s);
  const int ox0 = max(0, (ix + p - k + s) / s), ox1 = min(Wo - 1, (ix + p) / s);
  float g = 0.f;
  for (int oy = oy0; oy <= oy1; ++oy)
    for (int ox = ox0; ox <= ox1; ++ox) {
      const int kh = iy - (oy * s - p), kw = ix - (ox * s - p);
      if (kh < 0 || kw < 0 || kh >= k || kw >= k) continue;
      const int64_t o = (((int64_t)n * Ho + oy) * Wo + ox) * C + c;
      if (idx[o] == kh * k + kw) g += p6::to_f(dy[o]);
    }
  dx[i] = p6::from_f<T>(g);
}

template <typename T>
__global__ void avgpool_fwd_kernel(const T* __restrict__ x, float* __restrict__ y, int N, int HW, int C) {
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (i >= (int64_t)N * C) return;
  const int64_t n = i / C;
  const int c = i % C;
  float s = 0.f;
  for (int p = 0; p < HW; ++p) s += p6::to_f(x[(n * HW + p) * C + c]);
  y[i] = s / (float)HW;
}

template <typename T>
__global__ void avgpool_bwd_kernel(const float* __restrict__ dy, T* __restrict__ dx, int N, int HW, int C) {
  const int64_t i = blockIdx.x * (int64_t)kThreads + threadIdx.x;
  if (i >= (int64_t)N * HW * C) return;
  const int c = i % C;
  const int64_t n = i / ((int64_t)HW * C);
  dx[i] = p6::from_f<T>(dy[n * C + c] / (float)HW);
}

inline unsigned blocks(int64_t n) { return (unsigned)((n + kThreads - 1) / kThreads); }

}  // namespace

extern "C" int pose6d_nchw_to_nhwc(int32_t dtype, const float* x, void* y, int32_t N, int32_t C, int32_t H, int32_t W,
                                   int32_t Cpad, void* stream) {
  P6_CHECK_ARG(Cpad >= C, "pose6d_nchw_to_nhwc: Cpad < C");
  const int64_t n = (int64_t)N * H * W;
  if (n == 0) return POSE6D_OK;
  hipStream_t s = p6::stream_of(stream);
  if (dtype == POSE6D_DT_BF16)
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
  if (total == 0 || n_desc == 0) return POSE6D_OK;
  hipStream_t s = p6::stream_of(stream);
  unsigned g = blocks(total);
  if (g > 8192) g = 8192;
  if (dtype == POSE6D_DT_BF16) pack_kernel<bf16><<<g, kThreads, 0, s>>>((const PackDesc*)descs, n_desc, total);
  else pack_kernel<float><<<g, kThreads, 0, s>>>((const PackDesc*)descs, n_desc, total);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_maxpool_fwd(int32_t dtype, const void* x, void* y, uint8_t* argmax, int32_t N, int32_t H,
                                  int32_t W, int32_t C, int32_t k, int32_t s, int32_t p, int32_t Ho, int32_t Wo,
                                  void* stream) {
  P6_CHECK_ARG(k * k <= 255, "pose6d_maxpool_fwd: window too large");
  const int64_t n = (int64_t)N * Ho * Wo * C;
  if (n == 0) return POSE6D_OK;
  hipStream_t st = p6::stream_of(stream);
  if (dtype == POSE6D_DT_BF16)
    maxpool_fwd_kernel<bf16><<<blocks(n), kThreads, 0, st>>>((const bf16*)x, (bf16*)y, argmax, N, H, W, C, Ho, Wo, k, s, p);
  else
    maxpool_fwd_kernel<float><<<blocks(n), kThreads, 0, st>>>((const float*)x, (float*)y, argmax, N, H, W, C, Ho, Wo, k, s,
                                                               p);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_maxpool_bwd(int32_t dtype, const void* dy, const uint8_t* argmax, void* dx, int32_t N, int32_t H,
                                  int32_t W, int32_t C, int32_t k, int32_t s, int32_t p, int32_t Ho, int32_t Wo,
                                  void* stream) {
  const int64_t n = (int64_t)N * H * W * C;
  if (n == 0) return POSE6D_OK;
  hipStream_t st = p6::stream_of(stream);
  if (dtype == POSE6D_DT_BF16)
    maxpool_bwd_kernel<bf16><<<blocks(n), kThreads, 0, st>>>((const bf16*)dy, argmax, (bf16*)dx, N, H, W, C, Ho, Wo, k, s,
                                                              p);
  else
    maxpool_bwd_kernel<float><<<blocks(n), kThreads, 0, st>>>((const float*)dy, argmax, (float*)dx, N, H, W, C, Ho, Wo, k,
                                                               s, p);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_avgpool_fwd(int32_t dtype, const void* x, float* y, int32_t N, int32_t HW, int32_t C,
                                  void* stream) {
  const int64_t n = (int64_t)N * C;
  if (n == 0) return POSE6D_OK;
  hipStream_t st = p6::stream_of(stream);
  if (dtype == POSE6D_DT_BF16) avgpool_fwd_kernel<bf16><<<blocks(n), kThreads, 0, st>>>((const bf16*)x, y, N, HW, C);
  else avgpool_fwd_kernel<float><<<blocks(n), kThreads, 0, st>>>((const float*)x, y, N, HW, C);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

extern "C" int pose6d_avgpool_bwd(int32_t dtype, const float* dy, void* dx, int32_t N, int32_t HW, int32_t C,
                                  void* stream) {
  const int64_t n = (int64_t)N * HW * C;
  if (n == 0) return POSE6D_OK;
  hipStream_t st = p6::stream_of(stream);
  if (dtype == POSE6D_DT_BF16) avgpool_bwd_kernel<bf16><<<blocks(n), kThreads, 0, st>>>(dy, (bf16*)dx, N, HW, C);
  else avgpool_bwd_kernel<float><<<blocks(n), kThreads, 0, st>>>(dy, (float*)dx, N, HW, C);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

// Shared helpers for the pose6d HIP library (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "pose6d.h"

typedef __bf16 bf16;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) short s16x4;

namespace p6 {

// error reporting: every entry point returns 0 / a POSE6D_E* code and leaves
// a message for pose6d_last_error() (thread-local: reentrant across threads).
int set_error(int code, const char* fmt, ...);

#define P6_CHECK_ARG(cond, ...)                                                   \
  do {                                                                            \
    if (!(cond)) return ::p6::set_error(POSE6D_EINVAL, __VA_ARGS__);              \
  } while (0)

#define P6_LAUNCH_CHECK()                                                         \
  do {                                                                            \
    hipError_t e_ = hipGetLastError();                                            \
    if (e_ != hipSuccess)                                                         \
      return ::p6::set_error(POSE6D_ELAUNCH, "%s: %s", __func__, hipGetErrorString(e_)); \
  } while (0)

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// counter-based uniform in [0,1): splitmix64 finaliser of (seed, index); the
// dropout masks of every kernel draw from it (mask = uniform >= p)
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t i) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return (float)(z >> 40) * (1.0f / 16777216.0f);
}

// sum over a workgroup of NT threads (NT / 64 waves); `red` holds NT / 64 floats.
// Every thread gets the total.  Contains barriers: call from uniform control flow.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) t += red[w];
  return t;
}

// Row-tap layout (the 4-channel 7x7 / stride-2 stems): K ordered (kernel row, kRowTaps
// taps, 4 channels) with the filter's KW taps at the END of each row of kRowTaps, so
// that the taps of one kernel row of one output pixel are kRowTaps consecutive input
// pixels starting at an even one (2 ox - pad - (kRowTaps - KW)): 64 / 128 contiguous
// bytes (bf16 / fp32) per (pixel, kernel row).  Forward filters (wp) and the bf16
// weight-gradient slabs use it for these convs.
constexpr int kRowTaps = 8;
__host__ __device__ inline bool rowtap_geom(int Cin, int KH, int KW, int stride, int pad) {
  return Cin == 4 && stride == 2 && KH > 1 && KW <= kRowTaps && ((pad + kRowTaps - KW) & 1) == 0;
}

// one conv's weight-packing record (pose6d_pack_conv_weights, pose6d_adamw_step_packed)
struct PackDesc {
  const float* w;   // OIHW fp32 master
  void* wp;         // [O][Kpad], K = (kh, kw', ci): ci padded to Ip, KWp taps kw' per kernel row
  void* wt;         // [I][KH][KW][O] or null
  int O, I, Ip, KH, KW, Kpad;
  int KWp;          // packed taps per kernel row (KW; the row-tap stems: 8, filter tap kw at kw + KWp - KW)
  int reserved;
  int64_t start;    // (host bookkeeping: running sum of O * Kpad)
};

inline hipStream_t stream_of(void* s) { return reinterpret_cast<hipStream_t>(s); }

__host__ __device__ inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

}  // namespace p6

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
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

inline hipStream_t stream_of(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline int ceil_div(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

}  // namespace p6

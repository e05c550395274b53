// LDS-DMA pipeline helpers shared by the MFMA conv kernels (gfx950).
//
// global_load_lds_dwordx4 moves 16 B per lane straight into LDS (wave-uniform
// base + lane * 16: the LDS image is lane-linear, swizzles go on the SOURCE
// address).  A K-loop keeps several such stages in flight and retires them with a
// counted `s_waitcnt vmcnt(N)` + raw `s_barrier` -- never __syncthreads(), whose
// fence would drain every DMA still in flight.
#pragma once
#include "common.h"

namespace {

__device__ uint4 g_zero_page[4];   // 64 zero bytes: the source of padding / out-of-range rows

typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__device__ __forceinline__ int swz8(int row) { return (row >> 1) & 7; }

__device__ __forceinline__ void glds16(const void* g, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)lds_wave_base, 16, 0, 0);
}


__device__ __forceinline__ unsigned lds_addr(const char* p) {
  return (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

template <int N>
__device__ __forceinline__ void vmcnt_barrier() {
  static_assert(N >= 0 && N < 64, "vmcnt is a 6-bit count");
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

// wait until at most `ahead` stages (LOADS DMA instructions each) are still in
// flight, then barrier; `ahead` is wave-uniform, J the largest value it takes
template <int LOADS, int J>
__device__ __forceinline__ void wait_ahead(int ahead) {
  if constexpr (J <= 0) {
    vmcnt_barrier<0>();
  } else {
    if (ahead >= J) vmcnt_barrier<J * LOADS>();
    else wait_ahead<LOADS, J - 1>(ahead);
  }
}

}  // namespace

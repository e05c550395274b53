// Register-staged streaming rate per CU vs the LDS-DMA ring (gfx950 calibration, no compute).
//
// The question: is a single workgroup's stream rate bounded by the LDS-DMA instruction issue
// (tools/ldsdma_bench.hip: ~66 GB/s per workgroup whatever the ring depth), and would
// staging through VGPRs (global_load_dwordx4 -> ds_write_b128, D stages of registers in
// flight) feed a workgroup faster?  Modes:
//   dma  : the ldsdma_bench ring (2 slots, one stage in flight), for the side-by-side number
//   reg  : every stage loaded to VGPRs D stages ahead, written to a 2-slot LDS ring
//   mix  : half of every stage by DMA (one stage ahead), half by VGPRs (D stages ahead)
// Each mode optionally reads every landed slot back (ds_read_b128), as the MFMA fragment
// reads would.  Rows are `stride` bytes apart, 8 rows x 128 B per 1 KiB piece.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/regstream_bench tools/regstream_bench.hip
// run:   tools/regstream_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // promotable to VGPRs, unlike uint4

__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)lds, 16, 0, 0);
}

// MODE 0 = dma, 1 = reg, 2 = mix.  NW waves, SLOT KiB stages, D register stages ahead.
template <int MODE, int NW, int SLOT, int D>
__global__ __launch_bounds__(64 * NW) void stream_kernel(const char* __restrict__ buf, size_t mask, int steps,
                                                         int stride, int consume, unsigned* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PER = SLOT / NW;                       // 1 KiB pieces per wave per stage
  constexpr int PREG = MODE == 0 ? 0 : (MODE == 1 ? PER : PER / 2);
  constexpr int PDMA = PER - PREG;
  static_assert(PER * NW == SLOT && PER >= 2, "slot must be >= 2 pieces per wave");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t wg_base = (size_t)blockIdx.x * steps * SLOT * 1024;
  const int rowoff = (lane >> 3) * stride + (lane & 7) * 16;
  auto gaddr = [&](int st, int i) {
    const int piece = i * NW + wave;
    return (wg_base + (size_t)st * SLOT * 1024 + (size_t)piece * 8 * stride + rowoff) & mask;
  };
  auto dma = [&](int st, int slot) {
    char* dst = smem + slot * SLOT * 1024;
#pragma unroll
    for (int i = 0; i < PDMA; ++i) glds16(buf + gaddr(st, PREG + i), dst + ((PREG + i) * NW + wave) * 1024);
  };
  // The register stages live in a plain array indexed with unrolled constants only (no
  // lambda captures it by reference, which would put it in scratch).
  u32x4 regs[D > 0 ? D : 1][PREG > 0 ? PREG : 1];
  unsigned acc = 0;
  if constexpr (PREG > 0) {
#pragma unroll
    for (int d = 0; d < D; ++d)
#pragma unroll
      for (int i = 0; i < PREG; ++i) regs[d][i] = *reinterpret_cast<const u32x4*>(buf + gaddr(d, i));
  }
  if constexpr (PDMA > 0) dma(0, 0);
  for (int st0 = 0; st0 < steps; st0 += (D > 0 ? D : 1)) {
#pragma unroll
    for (int d = 0; d < (D > 0 ? D : 1); ++d) {
      const int st = st0 + d, slot = st & 1;
      if constexpr (PREG > 0) {
        char* dst = smem + slot * SLOT * 1024;
#pragma unroll
        for (int i = 0; i < PREG; ++i)
          *reinterpret_cast<u32x4*>(dst + (i * NW + wave) * 1024 + lane * 16) = regs[d][i];
        // unconditional (the tail re-reads the last stage) so that the compiler's vmcnt
        // bookkeeping stays exact instead of falling back to vmcnt(0) at the loop head
        const int nx = st + D < steps ? st + D : steps - 1;
#pragma unroll
        for (int i = 0; i < PREG; ++i) regs[d][i] = *reinterpret_cast<const u32x4*>(buf + gaddr(nx, i));
      }
      // DMA of stage st was issued at the end of the previous iteration; only this
      // iteration's register loads are younger than it.
      if constexpr (PDMA > 0) {
        if constexpr (PREG > 0) {
          asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PREG) : "memory");
        } else {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
      }
      __syncthreads();
      if constexpr (PDMA > 0) {
        if (st + 1 < steps) dma(st + 1, slot ^ 1);
      }
      if (consume) {
        const char* src = smem + slot * SLOT * 1024;
#pragma unroll
        for (int i = 0; i < SLOT * 1024 / (64 * NW * 16); ++i) {
          const uint4 v = *reinterpret_cast<const uint4*>(src + (i * 64 * NW + threadIdx.x) * 16);
          acc ^= v.x ^ v.y ^ v.z ^ v.w;
        }
      }
      __syncthreads();
    }
  }
  if (acc == 0x12345678u) sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int MODE, int NW, int SLOT, int D>
void run(const char* buf, size_t foot, int wpc, int stride, int consume, unsigned* sink) {
  constexpr int lds = 2 * SLOT * 1024;
  if (lds * wpc > 160 * 1024) return;
  if ((64 * NW) * wpc > 2048) return;
  const int grid = 256 * wpc;
  const int steps = 96;
  auto k = stream_kernel<MODE, NW, SLOT, D>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) k<<<grid, 64 * NW, lds>>>(buf, foot - 1, steps, stride, consume, sink);
  CK(hipGetLastError());
  const int reps = 10;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) k<<<grid, 64 * NW, lds>>>(buf, foot - 1, steps, stride, consume, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double t = ms * 1e-3 / reps;
  const double bytes = (double)grid * steps * SLOT * 1024;
  static const char* names[] = {"dma", "reg", "mix"};
  printf("%s NW=%d slot=%2dK D=%d wpc=%d foot=%6zuM stride=%5d consume=%d : %7.2f us  %6.1f GB/s/CU  %5.1f TB/s\n",
         names[MODE], NW, SLOT, D, wpc, foot >> 20, stride, consume, t * 1e6, bytes / t / 256 / 1e9, bytes / t / 1e12);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int NW, int SLOT>
void sweep(const char* buf, size_t foot, int stride, int consume, unsigned* sink) {
  for (int wpc = 1; wpc <= 2; wpc *= 2) {
    run<0, NW, SLOT, 1>(buf, foot, wpc, stride, consume, sink);
    run<1, NW, SLOT, 1>(buf, foot, wpc, stride, consume, sink);
    run<1, NW, SLOT, 2>(buf, foot, wpc, stride, consume, sink);
    run<1, NW, SLOT, 3>(buf, foot, wpc, stride, consume, sink);
    run<1, NW, SLOT, 4>(buf, foot, wpc, stride, consume, sink);
    run<2, NW, SLOT, 1>(buf, foot, wpc, stride, consume, sink);
    run<2, NW, SLOT, 2>(buf, foot, wpc, stride, consume, sink);
    run<2, NW, SLOT, 3>(buf, foot, wpc, stride, consume, sink);
  }
}

int main() {
  const size_t big = (size_t)1 << 31;
  char* buf;
  unsigned* sink;
  CK(hipMalloc(&buf, big));
  CK(hipMemset(buf, 1, big));
  CK(hipMalloc(&sink, 1 << 24));
  const size_t foots[] = {(size_t)4 << 20, (size_t)64 << 20, big};
  for (int consume = 0; consume <= 1; ++consume) {
    for (size_t foot : foots) {
      sweep<4, 16>(buf, foot, 2048, consume, sink);
      sweep<8, 32>(buf, foot, 2048, consume, sink);
      fflush(stdout);
    }
  }
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}

// LDS-DMA streaming rate per CU vs bytes in flight (gfx950 calibration, no compute).
//
// Each workgroup streams `steps` stages of SLOT KiB through an S-slot LDS ring with
// global_load_lds_dwordx4 (1 KiB per wave-instruction: 8 rows x 128 B, rows `stride`
// bytes apart, as the conv kernels' operand images), counted vmcnt + s_barrier per
// stage, optionally reading every landed slot back with ds_read_b128 (as the MFMA
// fragment reads would).  The footprint (power of two) decides where the bytes are
// served from: a few MiB = the XCD L2, tens of MiB = the Infinity Cache, GiB = HBM.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/ldsdma_bench tools/ldsdma_bench.hip
// run:   tools/ldsdma_bench            (prints one line per configuration)
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

__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void vm_bar() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int PER, int J>
__device__ __forceinline__ void wait_j(int j) {
  if constexpr (J <= 0) {
    vm_bar<0>();
  } else {
    if (j >= J) vm_bar<J * PER>();
    else wait_j<PER, J - 1>(j);
  }
}

// NW waves, SLOT KiB per stage, S ring slots
template <int NW, int SLOT, int S>
__global__ __launch_bounds__(64 * NW) void stream_kernel(const char* __restrict__ buf, size_t mask, int steps,
                                                         int stride, int consume, unsigned* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PER = SLOT / NW;   // 1 KiB DMA instructions per wave per stage
  static_assert(PER >= 1 && PER * NW == SLOT, "slot must be a multiple of the wave count");
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const size_t wg_base = (size_t)blockIdx.x * steps * SLOT * 1024;
  const int rowoff = (lane >> 3) * stride + (lane & 7) * 16;
  auto issue = [&](int st, int slot) {
    char* dst = smem + slot * SLOT * 1024;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int piece = i * NW + wave;   // 1 KiB piece of the stage = 8 rows
      const size_t off = (wg_base + (size_t)st * SLOT * 1024 + (size_t)piece * 8 * stride + rowoff) & mask;
      glds16(buf + off, dst + piece * 1024);
    }
  };
  unsigned acc = 0;
  for (int s = 0; s < S - 1 && s < steps; ++s) issue(s, s);
  int cur = 0, wb = S - 1;
  for (int st = 0; st < steps; ++st) {
    const int left = steps - 1 - st;
    wait_j<PER, S - 2>(left < S - 2 ? left : S - 2);
    if (st + S - 1 < steps) issue(st + S - 1, wb);
    if (consume) {
      const char* src = smem + cur * SLOT * 1024;
#pragma unroll
      for (int i = 0; i < SLOT * 1024 / (64 * NW * 16); ++i) {
        const uint4 v = *reinterpret_cast<const uint4*>(src + (i * 64 * NW + threadIdx.x) * 16);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    cur = cur == S - 1 ? 0 : cur + 1;
    wb = wb == S - 1 ? 0 : wb + 1;
  }
  if (acc == 0x12345678u) sink[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int NW, int SLOT, int S>
void run(const char* buf, size_t foot, int wpc, int stride, int consume, unsigned* sink) {
  constexpr int lds = S * SLOT * 1024;
  if (lds * wpc > 160 * 1024) return;
  if ((64 * NW) * wpc > 2048) return;
  const int grid = 256 * wpc;
  const int steps = 64;
  auto k = stream_kernel<NW, SLOT, S>;
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
  printf("NW=%d slot=%2dK S=%d wpc=%d inflight/CU=%3dK foot=%6zuM stride=%5d consume=%d : %7.2f us  %6.1f GB/s/CU  %5.1f TB/s\n",
         NW, SLOT, S, wpc, (S - 1) * SLOT * wpc, foot >> 20, stride, consume, t * 1e6, bytes / t / 256 / 1e9,
         bytes / t / 1e12);
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int NW, int SLOT>
void sweep_s(const char* buf, size_t foot, int stride, int consume, unsigned* sink) {
  for (int wpc = 1; wpc <= 4; wpc *= 2) {
    run<NW, SLOT, 2>(buf, foot, wpc, stride, consume, sink);
    run<NW, SLOT, 3>(buf, foot, wpc, stride, consume, sink);
    run<NW, SLOT, 4>(buf, foot, wpc, stride, consume, sink);
    run<NW, SLOT, 5>(buf, foot, wpc, stride, consume, sink);
    run<NW, SLOT, 6>(buf, foot, wpc, stride, consume, sink);
    run<NW, SLOT, 8>(buf, foot, wpc, stride, consume, sink);
  }
}

int main(int argc, char** argv) {
  const size_t big = (size_t)1 << 31;
  char* buf;
  unsigned* sink;
  CK(hipMalloc(&buf, big));
  CK(hipMemset(buf, 1, big));
  CK(hipMalloc(&sink, 1 << 24));
  const size_t foots[] = {(size_t)4 << 20, (size_t)64 << 20, big};
  const int consume = argc > 1 ? atoi(argv[1]) : 0;
  for (size_t foot : foots) {
    for (int stride : {128, 2048}) {
      sweep_s<4, 16>(buf, foot, stride, consume, sink);
      sweep_s<4, 32>(buf, foot, stride, consume, sink);
      sweep_s<8, 32>(buf, foot, stride, consume, sink);
    }
    fflush(stdout);
  }
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}

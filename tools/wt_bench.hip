// Kernel-boundary cost of dirty L2 lines: a chain of dependent streaming kernels
// (read src, write dst, bf16-sized 16-B vectors) whose stores are plain, write-through
// (sc1) or non-temporal (nt), captured in a hipGraph and replayed.  Prints the
// per-kernel time of each form for several tensor sizes.
// build: hipcc -O3 --offload-arch=gfx950 -o tools/wt_bench tools/wt_bench.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); exit(1); } } while (0)

typedef unsigned u32x4v __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void stream_kernel(const u32x4v* __restrict__ src, u32x4v* __restrict__ dst, long n) {
  const int bytes = (int)(n * 16 > 0x7fffffffL ? 0x7fffffff : n * 16);
  __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, bytes, 0x00020000);
  for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) {
    u32x4v v = src[i];
    v.x += 1u;
    if (MODE == 0) dst[i] = v;
    else if (MODE == 1) __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(i * 16), 0, 16);   // sc1
    else if (MODE == 2) __builtin_nontemporal_store(v, dst + i);                                // nt
    else __builtin_amdgcn_raw_buffer_store_b128(v, rs, (int)(i * 16), 0, 0);                    // buffer, plain
  }
}

template <int MODE>
float run(u32x4v* a, u32x4v* b, long n, int chain, int reps) {
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipGraph_t g;
  hipGraphExec_t ge;
  const int grid = (int)((n + 255) / 256 < 4096 ? (n + 255) / 256 : 4096);
  CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
  for (int k = 0; k < chain; ++k) {
    if (k & 1) stream_kernel<MODE><<<grid, 256, 0, s>>>(b, a, n);
    else stream_kernel<MODE><<<grid, 256, 0, s>>>(a, b, n);
  }
  CK(hipStreamEndCapture(s, &g));
  CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  for (int w = 0; w < 3; ++w) CK(hipGraphLaunch(ge, s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  CK(hipEventRecord(e0, s));
  for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ge, s));
  CK(hipEventRecord(e1, s));
  CK(hipEventSynchronize(e1));
  float ms = 0.f;
  CK(hipEventElapsedTime(&ms, e0, e1));
  CK(hipGraphExecDestroy(ge));
  CK(hipGraphDestroy(g));
  CK(hipStreamDestroy(s));
  return ms * 1000.f / (reps * chain);
}

int main() {
  const long sizes_mb[] = {1, 4, 13, 26, 51, 102};
  const long maxn = 102L * 1024 * 1024 / 16;
  u32x4v *a, *b;
  CK(hipMalloc(&a, maxn * 16));
  CK(hipMalloc(&b, maxn * 16));
  CK(hipMemset(a, 0, maxn * 16));
  CK(hipMemset(b, 0, maxn * 16));
  printf("%8s %10s %10s %10s %10s   (us per kernel, chain of 40 dependent launches)\n", "MB", "plain", "buf-plain",
         "buf-sc1", "nt");
  for (long mb : sizes_mb) {
    const long n = mb * 1024 * 1024 / 16;
    const float p = run<0>(a, b, n, 40, 20), bp = run<3>(a, b, n, 40, 20), w = run<1>(a, b, n, 40, 20),
                t = run<2>(a, b, n, 40, 20);
    printf("%8ld %10.2f %10.2f %10.2f %10.2f\n", mb, p, bp, w, t);
  }
  return 0;
}

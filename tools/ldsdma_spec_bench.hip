// GEMM K-loop skeleton on gfx950: how fast can one workgroup stream operand stages
// through an LDS ring while MFMAs consume them?  (calibration for the conv kernels'
// structure, no real GEMM: the MFMA operands are the LDS bytes, the sums are kept.)
//
// Two structures per configuration:
//   uniform     -- every wave issues its share of each stage's LDS-DMA, then reads
//                  its fragments and runs its MFMAs (the structure of conv_lds_body)
//   specialised -- NP producer waves only issue LDS-DMA (and wait for it), NC consumer
//                  waves only read fragments and run MFMAs; one s_barrier per stage
// Per stage: SLOT KiB of operands (1 KiB per DMA wave-instruction, 8 rows x 128 B
// with rows `stride` bytes apart), every consumer wave RPW ds_read_b128 per lane and
// MF v_mfma_f32_16x16x32_bf16.  The footprint (4 MiB) keeps the operands L2-resident.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/ldsdma_spec_bench tools/ldsdma_spec_bench.hip
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

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned u32x4;

__device__ __forceinline__ void glds16(const void* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                   (void __attribute__((address_space(3)))*)lds, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
template <int PER, int J>
__device__ __forceinline__ void wait_j(int j) {
  if constexpr (J <= 0) {
    vm_wait<0>();
  } else {
    if (j >= J) vm_wait<J * PER>();
    else wait_j<PER, J - 1>(j);
  }
}

// NP producer waves (0 = uniform: every wave produces), NC consumer waves (uniform: NC = all)
template <int NP, int NC, int SLOT, int S, int RPW, int MF>
__global__ __launch_bounds__(64 * (NP + NC)) void loop_kernel(const char* __restrict__ buf, size_t mask, int steps,
                                                               int stride, float* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr bool UNI = NP == 0;
  constexpr int NW = UNI ? NC : NP + NC;
  constexpr int NPROD = UNI ? NC : NP;          // waves issuing DMA
  constexpr int PER = SLOT / NPROD;              // DMA instructions per producing wave per stage
  static_assert(PER * NPROD == SLOT, "slot must split over the producer waves");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool prod = UNI || wave < NP;
  const bool cons = UNI || wave >= NP;
  const int pw = UNI ? wave : wave;              // producer index
  const int cw = UNI ? wave : wave - NP;         // consumer index
  const size_t wg_base = (size_t)blockIdx.x * 977 * 1024;
  const int rowoff = (lane >> 3) * stride + (lane & 7) * 16;
  auto issue = [&](int st, int slot) {
    char* dst = smem + slot * SLOT * 1024;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int piece = i * NPROD + pw;
      const size_t off = (wg_base + (size_t)st * SLOT * 1024 + (size_t)piece * 8 * stride + rowoff) & mask;
      glds16(buf + off, dst + piece * 1024);
    }
  };
  f32x4 acc[4] = {};
  if (prod)
    for (int s = 0; s < S - 1 && s < steps; ++s) issue(s, s);
  int cur = 0, wb = S - 1;
  for (int st = 0; st < steps; ++st) {
    const int left = steps - 1 - st;
    if (prod) wait_j<PER, S - 2>(left < S - 2 ? left : S - 2);
    asm volatile("s_barrier" ::: "memory");
    if (prod && st + S - 1 < steps) issue(st + S - 1, wb);
    if (cons) {
      const char* src = smem + cur * SLOT * 1024;
      u32x4 f[RPW];
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const int chunk = (cw * RPW + r) * 64 + lane;   // 16-B chunk of the slot
        f[r] = *reinterpret_cast<const u32x4*>(src + (chunk % (SLOT * 64)) * 16);
      }
      if constexpr (MF >= 0) {
#pragma unroll
        for (int m = 0; m < MF; ++m)
          acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, f[m % RPW]),
                                                               __builtin_bit_cast(bf16x8, f[(m + 1) % RPW]),
                                                               acc[m & 3], 0, 0, 0);
      } else {   // fp32: -MF exact v_mfma_f32_16x16x4_f32 (32 cycles each)
#pragma unroll
        for (int m = 0; m < -MF; ++m)
          acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(__builtin_bit_cast(f32x4, f[m % RPW])[m & 3],
                                                            __builtin_bit_cast(f32x4, f[(m + 1) % RPW])[m & 3],
                                                            acc[m & 3], 0, 0, 0);
      }
    }
    cur = cur == S - 1 ? 0 : cur + 1;
    wb = wb == S - 1 ? 0 : wb + 1;
  }
  const float v = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
  if (v == 12345.f) sink[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

// lgkmcnt(0) that the compiler sees as redefining the fragment registers
// (and, named as operands too, after the MFMAs that produce `acc`: otherwise hipcc
// may sink those MFMAs below the wait and the reads stop overlapping them)
template <int N>
__device__ __forceinline__ void lgkm_wait(u32x4 (&f)[N], f32x4 (&acc)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3])::"memory");
#pragma unroll
  for (int i = 0; i < N; ++i) asm volatile("" : "+v"(f[i]));
}

// software-pipelined uniform loop: after the barrier that publishes stage st+1, every
// wave issues the fragment reads of stage st+1 and then the MFMAs of stage st (its
// fragments already in registers), so the LDS reads overlap the matrix work; the
// slot of stage st (read completely before that barrier) is refilled right away
template <int NW, int SLOT, int S, int RPW, int MF>
__global__ __launch_bounds__(64 * NW) void pipe_kernel(const char* __restrict__ buf, size_t mask, int steps, int stride,
                                                       float* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PER = SLOT / NW;
  static_assert(PER * NW == SLOT, "slot must split over the waves");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t wg_base = (size_t)blockIdx.x * 977 * 1024;
  const int rowoff = (lane >> 3) * stride + (lane & 7) * 16;
  auto issue = [&](int st, int slot) {
    char* dst = smem + slot * SLOT * 1024;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int piece = i * NW + wave;
      const size_t off = (wg_base + (size_t)st * SLOT * 1024 + (size_t)piece * 8 * stride + rowoff) & mask;
      glds16(buf + off, dst + piece * 1024);
    }
  };
  // fragment reads as inline asm (no wait): hipcc neither orders them behind the
  // in-flight LDS-DMA (vmcnt(0)) nor waits for them before unrelated MFMAs; the
  // explicit lgkm_wait below (operands named "+v") releases them
  const unsigned ring = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)smem;
  auto read = [&](u32x4 (&f)[RPW], int slot) {
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      const int chunk = (wave * RPW + r) * 64 + lane;
      const unsigned a = ring + slot * SLOT * 1024 + (chunk % (SLOT * 64)) * 16;
      asm volatile("ds_read_b128 %0, %1" : "=v"(f[r]) : "v"(a));
    }
  };
  f32x4 acc[4] = {};
  for (int s = 0; s < S - 1 && s < steps; ++s) issue(s, s);
  wait_j<PER, S - 2>(steps - 1 < S - 2 ? steps - 1 : S - 2);   // stage 0 landed
  asm volatile("s_barrier" ::: "memory");
  u32x4 fa[RPW], fb[RPW];
  read(fa, 0);
  lgkm_wait<RPW>(fa, acc);
  int slot = 0;
  for (int st = 0; st < steps; st += 2) {
    // two iterations per trip so the fragment buffers alternate without copies
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int s_ = st + h;
      if (s_ >= steps) break;
      u32x4 (&cur)[RPW] = h == 0 ? fa : fb;
      u32x4 (&nxt)[RPW] = h == 0 ? fb : fa;
      // issued so far: stages 0 .. min(s_+S-2, steps-1); stage s_+1 must have landed
      const int hi = s_ + S - 2 < steps - 1 ? s_ + S - 2 : steps - 1;
      const int left = hi - (s_ + 1);
      if (s_ + 1 < steps) wait_j<PER, (S >= 3 ? S - 3 : 0)>(left < 0 ? 0 : left);
      asm volatile("s_barrier" ::: "memory");
      const int nslot = slot == S - 1 ? 0 : slot + 1;
      if (s_ + S - 1 < steps) issue(s_ + S - 1, slot == 0 ? S - 1 : slot - 1);
      if (s_ + 1 < steps) read(nxt, nslot);
#pragma unroll
      for (int m = 0; m < MF; ++m)
        acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, cur[m % RPW]),
                                                             __builtin_bit_cast(bf16x8, cur[(m + 1) % RPW]),
                                                             acc[m & 3], 0, 0, 0);
      lgkm_wait<RPW>(nxt, acc);
      slot = nslot;
    }
  }
  const float v = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
  if (v == 12345.f) sink[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

// register-staged uniform loop (2 LDS slots): stage st+1 sits in VGPRs (global_load_dwordx4,
// issued D iterations earlier) and is written to the free slot with ds_write_b128 after the
// fragment reads of stage st are issued; no LDS-DMA at all
template <int NW, int SLOT, int RPW, int MF, int D>
__global__ __launch_bounds__(64 * NW) void reg_kernel(const char* __restrict__ buf, size_t mask, int steps, int stride,
                                                      float* __restrict__ sink) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int PER = SLOT / NW;
  static_assert(PER * NW == SLOT, "slot must split over the waves");
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const size_t wg_base = (size_t)blockIdx.x * 977 * 1024;
  const int rowoff = (lane >> 3) * stride + (lane & 7) * 16;
  auto src_of = [&](int st, int i) {
    const int piece = i * NW + wave;
    return reinterpret_cast<const u32x4*>(buf + ((wg_base + (size_t)st * SLOT * 1024 + (size_t)piece * 8 * stride +
                                                   rowoff) & mask));
  };
  auto dst_of = [&](int slot, int i) {
    return reinterpret_cast<u32x4*>(smem + slot * SLOT * 1024 + (i * NW + wave) * 1024 + lane * 16);
  };
  u32x4 regs[D][PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) regs[0][i] = *src_of(0, i);
#pragma unroll
  for (int i = 0; i < PER; ++i) *dst_of(0, i) = regs[0][i];
#pragma unroll
  for (int d = 0; d < D; ++d)
#pragma unroll
    for (int i = 0; i < PER; ++i) regs[d][i] = *src_of(1 + d < steps ? 1 + d : steps - 1, i);
  f32x4 acc[4] = {};
  for (int st0 = 0; st0 < steps; st0 += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int st = st0 + d;
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      const char* src = smem + (st & 1) * SLOT * 1024;
      u32x4 f[RPW];
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        const int chunk = (wave * RPW + r) * 64 + lane;
        f[r] = *reinterpret_cast<const u32x4*>(src + (chunk % (SLOT * 64)) * 16);
      }
#pragma unroll
      for (int i = 0; i < PER; ++i) *dst_of((st + 1) & 1, i) = regs[d][i];
      const int nx = st + 1 + D < steps ? st + 1 + D : steps - 1;
#pragma unroll
      for (int i = 0; i < PER; ++i) regs[d][i] = *src_of(nx, i);
      if constexpr (MF >= 0) {
#pragma unroll
        for (int m = 0; m < MF; ++m)
          acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, f[m % RPW]),
                                                               __builtin_bit_cast(bf16x8, f[(m + 1) % RPW]),
                                                               acc[m & 3], 0, 0, 0);
      } else {
#pragma unroll
        for (int m = 0; m < -MF; ++m)
          acc[m & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(__builtin_bit_cast(f32x4, f[m % RPW])[m & 3],
                                                            __builtin_bit_cast(f32x4, f[(m + 1) % RPW])[m & 3],
                                                            acc[m & 3], 0, 0, 0);
      }
    }
  }
  const float v = acc[0][0] + acc[1][1] + acc[2][2] + acc[3][3];
  if (v == 12345.f) sink[blockIdx.x * blockDim.x + threadIdx.x] = v;
}

template <int NW, int SLOT, int RPW, int MF, int D>
void run_reg(const char* buf, size_t foot, int wpc, float* sink, const char* name) {
  constexpr int lds = 2 * SLOT * 1024;
  if (lds * wpc > 160 * 1024 || 64 * NW * wpc > 2048) return;
  const int grid = 256 * wpc, steps = 60, stride = 2048;
  auto k = reg_kernel<NW, SLOT, RPW, MF, D>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) k<<<grid, 64 * NW, lds>>>(buf, foot - 1, steps, stride, sink);
  CK(hipGetLastError());
  const int reps = 10;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) k<<<grid, 64 * NW, lds>>>(buf, foot - 1, steps, stride, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double t = ms * 1e-3 / reps;
  const double per_step_ns = t / steps * 1e9;
  const double mfma_cyc = (MF >= 0 ? (double)MF * 16 : -(double)MF * 32) * NW * wpc / 4;
  printf("%-12s NW=%d slot=%2dK D=%d RPW=%2d MF=%2d wpc=%d : %7.2f us  %6.1f ns/stage  %6.1f GB/s/CU  "
         "MFMA %5.1f%% of the stage (2.4 GHz)\n",
         name, NW, SLOT, D, RPW, MF, wpc, t * 1e6, per_step_ns / wpc, (double)grid * steps * SLOT * 1024 / t / 256 / 1e9,
         100.0 * mfma_cyc / (per_step_ns * 2.4));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int NW, int SLOT, int S, int RPW, int MF>
void run_pipe(const char* buf, size_t foot, int wpc, float* sink, const char* name) {
  constexpr int lds = S * SLOT * 1024;
  if (lds * wpc > 160 * 1024 || 64 * NW * wpc > 2048) return;
  const int grid = 256 * wpc, steps = 64, stride = 2048;
  auto k = pipe_kernel<NW, SLOT, S, RPW, MF>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) k<<<grid, 64 * NW, lds>>>(buf, foot - 1, steps, stride, sink);
  CK(hipGetLastError());
  const int reps = 10;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) k<<<grid, 64 * NW, lds>>>(buf, foot - 1, steps, stride, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double t = ms * 1e-3 / reps;
  const double per_step_ns = t / steps * 1e9;
  const double mfma_cyc = (double)MF * 16 * NW * wpc / 4;
  printf("%-12s NW=%d slot=%2dK S=%d RPW=%2d MF=%2d wpc=%d : %7.2f us  %6.1f ns/stage  %6.1f GB/s/CU  "
         "MFMA %5.1f%% of the stage (2.4 GHz)\n",
         name, NW, SLOT, S, RPW, MF, wpc, t * 1e6, per_step_ns / wpc, (double)grid * steps * SLOT * 1024 / t / 256 / 1e9,
         100.0 * mfma_cyc / (per_step_ns * 2.4));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

template <int NP, int NC, int SLOT, int S, int RPW, int MF>
void run(const char* buf, size_t foot, int wpc, float* sink, const char* name) {
  constexpr int NW = NP == 0 ? NC : NP + NC;
  constexpr int lds = S * SLOT * 1024;
  if (lds * wpc > 160 * 1024 || 64 * NW * wpc > 2048) return;
  const int grid = 256 * wpc, steps = 64, stride = 2048;
  auto k = loop_kernel<NP, NC, SLOT, S, RPW, MF>;
  CK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) k<<<grid, 64 * NW, lds>>>(buf, foot - 1, steps, stride, sink);
  CK(hipGetLastError());
  const int reps = 10;
  CK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) k<<<grid, 64 * NW, lds>>>(buf, foot - 1, steps, stride, sink);
  CK(hipEventRecord(e1));
  CK(hipEventSynchronize(e1));
  float ms;
  CK(hipEventElapsedTime(&ms, e0, e1));
  const double t = ms * 1e-3 / reps;
  const double per_step_ns = t / steps * 1e9;
  const double mfma_cyc = (MF >= 0 ? (double)MF * 16 : -(double)MF * 32) * NC * wpc / 4;   // per SIMD per stage
  printf("%-12s NP=%d NC=%d slot=%2dK S=%d RPW=%2d MF=%2d wpc=%d : %7.2f us  %6.1f ns/stage  %6.1f GB/s/CU  "
         "MFMA %5.1f%% of the stage (2.4 GHz)\n",
         name, NP, NC, SLOT, S, RPW, MF, wpc, t * 1e6, per_step_ns / wpc, (double)grid * steps * SLOT * 1024 / t / 256 / 1e9,
         100.0 * mfma_cyc / (per_step_ns * 2.4));
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
  const size_t foot = (size_t)4 << 20;
  char* buf;
  float* sink;
  CK(hipMalloc(&buf, (size_t)64 << 20));
  CK(hipMemset(buf, 0, (size_t)64 << 20));
  CK(hipMalloc(&sink, 1 << 24));
  if (argc > 1 && argv[1][0] == 'r') {   // register-staged vs LDS-DMA, same tiles
    for (int wpc = 1; wpc <= 2; ++wpc) {
      run<0, 4, 16, 3, 8, 8>(buf, foot, wpc, sink, "uni64x64");
      run_reg<4, 16, 8, 8, 1>(buf, foot, wpc, sink, "reg64x64");
      run_reg<4, 16, 8, 8, 2>(buf, foot, wpc, sink, "reg64x64");
      run<0, 8, 32, 3, 12, 16>(buf, foot, wpc, sink, "uni128x128");
      run_reg<8, 32, 12, 16, 1>(buf, foot, wpc, sink, "reg128x128");
      run_reg<8, 32, 12, 16, 2>(buf, foot, wpc, sink, "reg128x128");
      run<0, 4, 16, 3, 8, -32>(buf, foot, wpc, sink, "f32uni64");
      run_reg<4, 16, 8, -32, 1>(buf, foot, wpc, sink, "f32reg64");
      run_reg<4, 16, 8, -32, 2>(buf, foot, wpc, sink, "f32reg64");
    }
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
  }
  // fp32 64x64 tile (4 waves of 32x32: 32 exact 16x16x4 MFMAs + 8 reads per wave per 16 KiB stage)
  run<0, 4, 16, 3, 8, -32>(buf, foot, 1, sink, "f32uni64");
  run<0, 4, 16, 3, 8, -32>(buf, foot, 2, sink, "f32uni64");
  run<4, 4, 16, 3, 8, -32>(buf, foot, 1, sink, "f32spec64");
  run<4, 4, 16, 4, 8, -32>(buf, foot, 1, sink, "f32spec64");
  run<2, 4, 16, 4, 8, -32>(buf, foot, 1, sink, "f32spec64");
  run<4, 4, 16, 3, 8, -32>(buf, foot, 2, sink, "f32spec64");
  run<4, 8, 32, 3, 12, -32>(buf, foot, 1, sink, "f32spec128");
  run<0, 8, 32, 3, 12, -32>(buf, foot, 1, sink, "f32uni128");
  run<0, 4, 16, 3, 8, -32>(buf, foot, 3, sink, "f32uni64");
  run<0, 4, 16, 3, 1, -32>(buf, foot, 1, sink, "f32uni64lowLDS");
  // two K-steps per barrier (32 KiB stages, 64 MFMAs + 16 reads per wave)
  run<0, 4, 32, 2, 16, -64>(buf, foot, 1, sink, "f32uni64x2");
  run<0, 4, 32, 2, 16, -64>(buf, foot, 2, sink, "f32uni64x2");
  run<0, 4, 32, 3, 16, -64>(buf, foot, 1, sink, "f32uni64x2");
  run<0, 4, 64, 2, 32, -128>(buf, foot, 1, sink, "f32uni64x4");
  run<0, 8, 64, 2, 24, -64>(buf, foot, 1, sink, "f32uni128x2");
  run<0, 4, 32, 2, 16, 16>(buf, foot, 1, sink, "bf16uni64x2");
  run<0, 4, 32, 2, 16, 16>(buf, foot, 2, sink, "bf16uni64x2");
  run<4, 4, 16, 3, 1, -32>(buf, foot, 1, sink, "f32spec64lowLDS");
  run_pipe<8, 32, 3, 12, 16>(buf, foot, 1, sink, "pipe128");
  run_pipe<8, 32, 4, 12, 16>(buf, foot, 1, sink, "pipe128");
  run_pipe<4, 32, 3, 16, 32>(buf, foot, 1, sink, "pipe128w4");
  run_pipe<4, 32, 4, 16, 32>(buf, foot, 1, sink, "pipe128w4");
  run_pipe<4, 16, 3, 8, 8>(buf, foot, 1, sink, "pipe64");
  run_pipe<4, 16, 3, 8, 8>(buf, foot, 2, sink, "pipe64");
  run_pipe<8, 48, 3, 16, 32>(buf, foot, 1, sink, "pipe256x128");
  run_pipe<8, 32, 3, 12, 0>(buf, foot, 1, sink, "pipe128noMF");
  run_pipe<8, 32, 3, 1, 16>(buf, foot, 1, sink, "pipe128lowLDS");
  // 64x64 tile, 4 waves of 32x32 (today's default): 16 KiB stages, 8 reads + 8 MFMAs per wave
  run<0, 4, 16, 2, 8, 8>(buf, foot, 1, sink, "uni64x64");
  run<0, 4, 16, 2, 8, 8>(buf, foot, 2, sink, "uni64x64");
  run<0, 4, 16, 3, 8, 8>(buf, foot, 2, sink, "uni64x64");
  run<0, 4, 16, 4, 8, 8>(buf, foot, 1, sink, "uni64x64");
  run<0, 4, 16, 2, 8, 8>(buf, foot, 4, sink, "uni64x64");
  // 128x128 tile, 8 waves of 32x64 (tile 4): 32 KiB stages, 12 reads + 16 MFMAs per wave
  run<0, 8, 32, 2, 12, 16>(buf, foot, 1, sink, "uni128x128");
  run<0, 8, 32, 3, 12, 16>(buf, foot, 1, sink, "uni128x128");
  run<0, 8, 32, 4, 12, 16>(buf, foot, 1, sink, "uni128x128");
  run<0, 8, 32, 2, 12, 16>(buf, foot, 2, sink, "uni128x128");
  // 128x128 tile, 4 waves of 64x64 (tile 0): 16 reads + 32 MFMAs per wave
  run<0, 4, 32, 3, 16, 32>(buf, foot, 1, sink, "uni128x128w4");
  run<0, 4, 32, 4, 16, 32>(buf, foot, 1, sink, "uni128x128w4");
  // specialised: producers + consumers, 128x128 tile
  run<4, 8, 32, 3, 12, 16>(buf, foot, 1, sink, "spec128");
  run<4, 8, 32, 4, 12, 16>(buf, foot, 1, sink, "spec128");
  run<8, 8, 32, 3, 12, 16>(buf, foot, 1, sink, "spec128");
  run<8, 8, 32, 4, 12, 16>(buf, foot, 1, sink, "spec128");
  run<4, 4, 32, 3, 16, 32>(buf, foot, 1, sink, "spec128w4");
  run<4, 4, 32, 4, 16, 32>(buf, foot, 1, sink, "spec128w4");
  run<8, 4, 32, 4, 16, 32>(buf, foot, 1, sink, "spec128w4");
  run<2, 4, 32, 4, 16, 32>(buf, foot, 1, sink, "spec128w4");
  // specialised 64x64
  run<4, 4, 16, 3, 8, 8>(buf, foot, 1, sink, "spec64");
  run<4, 4, 16, 4, 8, 8>(buf, foot, 1, sink, "spec64");
  run<4, 4, 16, 3, 8, 8>(buf, foot, 2, sink, "spec64");
  run<2, 4, 16, 4, 8, 8>(buf, foot, 1, sink, "spec64");
  run<2, 4, 16, 4, 8, 8>(buf, foot, 2, sink, "spec64");
  // MFMA-only reference (no DMA at all: NP waves idle, consumers read a fixed slot)
  run<0, 8, 32, 2, 12, 16>(buf, foot, 1, sink, "uni128x128");
  // 256x128 tile, 8 consumer waves of 64x64 (48 KiB stages)
  run<8, 8, 48, 3, 16, 32>(buf, foot, 1, sink, "spec256x128");
  run<4, 8, 48, 3, 16, 32>(buf, foot, 1, sink, "spec256x128");
  run<0, 8, 48, 3, 16, 32>(buf, foot, 1, sink, "uni256x128");
  CK(hipFree(buf));
  CK(hipFree(sink));
  return 0;
}

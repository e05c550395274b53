// Implicit-GEMM convolution (forward and data-gradient) on MFMA for gfx950.
//
// Replaces the cuDNN convolutions behind torchvision's ResNet50 trunk (used by
// every reference model, e.g. pose_net_rgbd_geometric.py:23-25) and the z-CNN of
// pose_net_rgb_geometric.py:36-55.
//
// GEMM view (NHWC activations, K ordered (kh, kw, c) with c fastest):
//   forward : Y[m = (n,oy,ox)][co] = sum_k A[m][k] * Wp[co][k],  A = im2col(X)
//   dgrad   : dX[m = (n,y,x)][ci]  = sum_k A[m][k] * Wt[ci][k],  A = col2im-gather(dY)
// One 256-thread workgroup = 4 waves (2 x 2) computes a BM x BN tile; K advances
// 64 bytes per step (BK = 32 bf16 / 16 fp32) through a double-buffered,
// XOR-swizzled LDS image (register staged so that padding taps load zeros).
// MFMA: v_mfma_f32_16x16x32_bf16 (bf16) or v_mfma_f32_16x16x4_f32 (fp32, exact
// fp32 products; used for the fp32 parity path).  Every lane reads its A and B
// fragments with one ds_read_b128 each; the swizzle makes those conflict-free.
// Epilogue: + bias, per-wave BatchNorm partial statistics (sum, sum of squares of
// the fp32 accumulators -> stats workspace, reduced by pose6d_bn_finalize), the
// tile goes through LDS so that global stores are whole 16-byte chunks of
// contiguous NHWC rows, optionally adding a residual tensor (dgrad: dX += dRes).
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "lds_dma.h"
#include "wgrad_body.h"

namespace {

constexpr int kThreads = 256;

template <typename T> struct KT;
template <> struct KT<bf16> { static constexpr int VEC = 8; static constexpr int BK = 32; };
template <> struct KT<float> { static constexpr int VEC = 4; static constexpr int BK = 16; };

// kDgradS2: stride-2 data gradient split into the four output parity classes
// (y & 1, x & 1); each class only gathers the taps that reach it, so no MAC is
// spent on the zeros a masked stride-2 gather would multiply.
// kGemmDual (eval only): a bottleneck's last 1x1 conv and its downsample branch in one
// launch -- K-steps [0, Kpad) are the block's 1x1 GEMM over src, the rest the 1x1
// (stride2) downsample over src2 with weights wts2, summed into a second accumulator
// set; the epilogue applies both BatchNorms exactly as the separate launches did.
enum Mode { kGemm = 0, kFwd = 1, kFwdNarrow = 2, kDgrad = 3, kDgradS2 = 4, kGemmDual = 5, kFwdRowTap = 6 };

// Row-tap forward (kFwdRowTap: the 4-channel stems, 7x7 / stride 2 / pad 3; layout in
// common.h): the filter packed with kRowTaps taps per kernel row and a zero tap in front
// (pose6d_conv_pack_geom), so the 8 taps x 4 channels of one kernel row of one output
// pixel are 8 consecutive input pixels -- 64 contiguous bytes (bf16) starting at an
// even pixel (2 ox - pad - 1): the LDS-DMA A tile fetches them as four aligned 16-B
// chunks (fp32: one kernel row per 128-B K-step row).  Replaces the register-staged
// 8-byte gather of kFwdNarrow for these convs.
using p6::kRowTaps;

struct Geom {
  int M, Ncols, K, Kpad;   // GEMM dims; Kpad = weight row length
  int SH, SW, SC, log2SC;  // gathered source tensor (NHWC)
  int RH, RW;              // row grid: m = (n * RH + y) * RW + x
  int KH, KW, stride, pad;
  int gm, gn;              // grid in tiles
  int s2one;               // kDgradS2: 0 = grid covers the four parity classes; c + 1 = only class c
  // forward with the BatchNorm already known (eval): the epilogue stores
  // act(T(y) * scale + shift [+ res | + res * res_scale + res_shift]) instead of y
  // (pose6d_conv2d_fwd_act); `res` is then the residual tensor
  const float *act_scale, *act_shift, *act_rscale, *act_rshift;
  int act, act_relu;
  // data gradient: the residual contribution is res * mask (one bit per element, one
  // byte per 16-byte chunk: pose6d_bn_act_fwd_mask's ReLU bits), i.e. the masked dout
  // of the block's last BN, instead of a materialised dz (null = res as is)
  const uint8_t* res_mask;
  // kGemmDual: the downsample operand [N][SH2][SW2][Kpad2], its packed weights
  // [Ncols][Kpad2], its stride (rows m = (n, oy, ox) of the RH x RW output grid)
  const void* src2;
  const void* wts2;
  int Kpad2, SH2, SW2, stride2;
  // data gradient that completes a BatchNorm's output gradient (pose6d_bn_reduce_t):
  // the epilogue also sums that BN's dz = dX * relu and dz * xhat per channel over its
  // tile into partial row bnr_rows-major [2][C][bnr_rows] (null bnr_part = off)
  const void* bnr_y;
  const float *bnr_mean, *bnr_inv, *bnr_rs, *bnr_rb;
  const uint8_t* bnr_mask;
  float* bnr_part;
  const void* bnr_y2;
  const float *bnr_mean2, *bnr_inv2;
  float* bnr_part2;
  int bnr_rows;
  // split-K (LDS-DMA path, kGemm / kFwd / kDgrad): each output tile's K-steps are
  // divided over `splits` workgroups (0 or 1 = none); see splitk_merge.  sk_cnt /
  // sk_part: the caller's split-K workspace (arrival counters, partial tiles)
  int splits;
  int* sk_cnt;
  float* sk_part;
};

// ---------------------------------------------------------------------------
// Split-K inside one launch.  The small-grid layers (layer3/4 at batch 32: a few
// hundred 64x64 tiles, 16-72 K-steps each) are bound by the operand bytes a CU
// keeps in flight, not by MFMA: bigger tiles move fewer bytes per MAC but leave CUs
// idle unless the K range of a tile is shared by several workgroups.  Each split
// writes its fp32 partial tile write-through (buffer stores with sc1), waits for
// them (vmcnt(0)), and after a workgroup barrier one lane adds 1 to the tile's
// arrival counter (agent scope); the workgroup whose add returns splits-1 is the
// last: it re-arms the counter, reads the other partials with sc1 buffer loads
// (after a barrier) and sums ALL partials in split order p0 + p1 + ... (its own from
// registers) -- one summation order per plan, whoever arrives last -- then runs the
// normal epilogue (bias, BN statistics, act, residual).  No workgroup waits for
// another, so residency does not matter.  This is the hand-off MI355X_MICROARCH.md
// measures valid with sc1 stores and loads in place of release / acquire fences.
// The partials and counters live in a CALLER-PROVIDED workspace (no library-owned
// state, so launches on different streams with different workspaces never meet):
// [kSkCntBytes of arrival counters, one int per output tile][partial tiles].  The
// counter block has a fixed size so that every plan run on one workspace finds its
// counters at the same words; the caller zeroes it once (every launch leaves it
// zero).  Size query: pose6d_conv_splitk_workspace.
constexpr int kSkMaxTiles = 8192;                       // plans with more tiles never split
constexpr int64_t kSkCntBytes = (int64_t)kSkMaxTiles * 4;   // 32 KiB

// TM x TN accumulator tiles per wave; PART = floats of one (tile, split) partial
template <int TM, int TN, int NW>
__device__ __forceinline__ bool splitk_merge(f32x4 (&acc)[TM][TN], char* smem, int tile, int split, int nsplit,
                                             int* cnt, float* part) {
  constexpr int PART = NW * TM * TN * 64 * 4;
  constexpr int SC1 = 16;   // buffer cache-policy bits: sc1
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  float* base = part + (int64_t)tile * nsplit * PART;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(base, 0, nsplit * PART * 4, 0x00020000);
  const int voff = (wave * TM * TN * 64 + lane) * 16;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs,
                                             voff + (i * TN + j) * 1024, split * PART * 4, SC1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave, before the barrier
  __syncthreads();
  int* flag = reinterpret_cast<int*>(smem);
  if (tid == 0) flag[0] = __hip_atomic_fetch_add(&cnt[tile], 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  const bool last = flag[0] == nsplit - 1;
  __syncthreads();   // flag read by every wave before the epilogue reuses the LDS
  if (!last) return false;
  if (tid == 0) __hip_atomic_store(&cnt[tile], 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  f32x4 mine[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) mine[i][j] = acc[i][j];
  for (int s = 0; s < nsplit; ++s) {
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const f32x4 v = s == split ? mine[i][j]
                                   : __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                                                   rs, voff + (i * TN + j) * 1024, s * PART * 4, SC1));
        acc[i][j] = s == 0 ? v : acc[i][j] + v;
      }
  }
  return true;
}

// LDS bytes the BN-reduce epilogue needs beyond the staged tile: per wave, per chunk
// column, (sum dz, sum dz xhat, sum dz xhat2) x 16-byte chunk = 12 bytes per column,
// + four per-channel constants
constexpr int bnr_lds(int nw, int bn) { return 12 * nw * bn + 16 * bn; }

// kDgradS2 launched in place (dres == dx) when a single parity class has taps
// (1x1 stride 2): the other classes' pixels are already final, so the grid covers
// that class alone instead of launching three workgroups per tile that only exit.
void s2_single_class(Geom& g, const void* res, const void* out) {
  g.s2one = 0;
  if (res != out) return;
  int n = 0, last = 0;
  for (int cls = 0; cls < 4; ++cls) {
    const int kh0 = ((cls >> 1) + g.pad) & 1, kw0 = ((cls & 1) + g.pad) & 1;
    if (((g.KH - kh0 + 1) >> 1) * ((g.KW - kw0 + 1) >> 1) > 0) { ++n; last = cls; }
  }
  if (n == 1) g.s2one = last + 1;
}
__host__ __device__ inline int s2_classes(const Geom& g) { return g.s2one ? 1 : 4; }


// ds_read_b128 fragment reads: lanes (row = l & 15, chunk = l >> 4) of a 16-row
// block; this XOR makes every 16-lane LDS group hit 16 distinct 16-byte slots.
__device__ __forceinline__ int swz(int row) { return (4 - ((row >> 2) & 3)) & 3; }

// Output row of GEMM row m: m itself, or for a kDgradS2 parity class cls = (py, px)
// the dX pixel (n, 2*yy + py, 2*xx + px) of class-local row m = (n, yy, xx).
__device__ __forceinline__ int64_t out_row(const Geom& g, int cls, int m) {
  if (cls < 0) return m;
  const int hw = g.RH * g.RW;
  const int n = m / hw, rem = m - n * hw;
  const int yy = rem / g.RW, xx = rem - yy * g.RW;
  return ((int64_t)n * 2 * g.RH + 2 * yy + (cls >> 1)) * (2 * g.RW) + 2 * xx + (cls & 1);
}

// Shared epilogue: + bias, BatchNorm partial statistics, LDS-staged 16-B stores
// (+ residual).  Must be entered after a barrier that ends all LDS reads.
// ACT: the eval BN-act store (Geom::act) compiled in (1) or out (0): the launchers
// instantiate both, so the training kernels carry no trace of it
// NW waves per workgroup: WM = NW / 2 along M times 2 along N, each wave owning a
// (BM / WM) x (BN / 2) block of 16x16 MFMA tiles (TM x TN of them)
// n consecutive floats (n = 4 or 8, 16-B aligned) as 16-B loads
template <int N>
__device__ __forceinline__ void load_f32s(const float* __restrict__ p, float (&f)[N]) {
  static_assert(N % 4 == 0, "16-byte loads");
#pragma unroll
  for (int i = 0; i < N / 4; ++i) {
    const float4 v = *reinterpret_cast<const float4*>(p + 4 * i);
    f[4 * i] = v.x; f[4 * i + 1] = v.y; f[4 * i + 2] = v.z; f[4 * i + 3] = v.w;
  }
}

template <int NW> struct WaveGrid { static constexpr int WM = NW / 2, WN = 2, NT = 64 * NW; };

// BatchNorm-backward partial sums of one tile (Geom::bnr_*): a thread's chunks share
// one chunk column (E channels); lanes of a column fold by xor shuffles, waves through
// LDS (`red`, past the staged tile), in a fixed order -- deterministic.  dz = dX as
// stored (T) times the BN's ReLU: the stored bits (bnr_mask) or T(y * rs + rb) > 0
// recomputed, exactly as pose6d_bn_bwd's reduce decides it.  The per-channel
// constants sit in LDS (`cst` [4][BN]: mean, invstd, then rs, rb or mean2, invstd2),
// read per 4-channel group where used: held in registers they cost the data-gradient
// kernels two waves of occupancy.
template <typename T, int BN, int NW, int IT>
__device__ __forceinline__ void bnr_partials(const Geom& g, const uint4 (&ov)[IT], const bool (&okv)[IT],
                                             const int64_t (&oidx)[IT], const uint4 (&yv)[IT],
                                             const unsigned (&mb)[IT], float* red, const float* cst, int prow,
                                             int n0) {
  constexpr int E = 16 / (int)sizeof(T), CPR = BN * (int)sizeof(T) / 16;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cl = (tid % CPR) * E;   // the chunk column's first channel within the tile
  const bool dual = g.bnr_y2 != nullptr, mk3 = g.bnr_mask != nullptr;
  float sd[E], sq[E], sq2[E];
#pragma unroll
  for (int e = 0; e < E; ++e) sd[e] = sq[e] = sq2[e] = 0.f;
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    if (!okv[it]) continue;
    T a[E], yy[E], y2[E];
    __builtin_memcpy(a, &ov[it], 16);
    __builtin_memcpy(yy, &yv[it], 16);
    // the dual branch's y: loaded here, not prefetched (registers; still before the stores)
    const uint4 y2v = dual ? *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(g.bnr_y2) + oidx[it])
                           : uint4{0, 0, 0, 0};
    __builtin_memcpy(y2, &y2v, 16);
#pragma unroll
    for (int e4 = 0; e4 < E; e4 += 4) {
      const float4 mu = *reinterpret_cast<const float4*>(cst + cl + e4);
      const float4 iv = *reinterpret_cast<const float4*>(cst + BN + cl + e4);
      const float4 ca = *reinterpret_cast<const float4*>(cst + 2 * BN + cl + e4);
      const float4 cb = *reinterpret_cast<const float4*>(cst + 3 * BN + cl + e4);
      const float m4[4] = {mu.x, mu.y, mu.z, mu.w}, i4[4] = {iv.x, iv.y, iv.z, iv.w};
      const float a4[4] = {ca.x, ca.y, ca.z, ca.w}, b4[4] = {cb.x, cb.y, cb.z, cb.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int e = e4 + k;
        const float y = p6::to_f(yy[e]);
        const bool on = mk3 ? ((mb[it] >> e) & 1u) != 0u : p6::to_f(p6::from_f<T>(fmaf(y, a4[k], b4[k]))) > 0.f;
        const float d = on ? p6::to_f(a[e]) : 0.f;
        sd[e] += d;
        sq[e] = fmaf(d, (y - m4[k]) * i4[k], sq[e]);
        if (dual) sq2[e] = fmaf(d, (p6::to_f(y2[e]) - a4[k]) * b4[k], sq2[e]);
      }
    }
    asm volatile("" ::: "memory");   // keep the constant reads per trip (not hoisted into registers)
  }
#pragma unroll
  for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
    for (int e = 0; e < E; ++e) {
      sd[e] += __shfl_xor(sd[e], o, 64);
      sq[e] += __shfl_xor(sq[e], o, 64);
      if (dual) sq2[e] += __shfl_xor(sq2[e], o, 64);
    }
  if (lane < CPR) {
    float* r = red + (wave * CPR + lane) * 3 * E;
#pragma unroll
    for (int e = 0; e < E; ++e) { r[e] = sd[e]; r[E + e] = sq[e]; r[2 * E + e] = sq2[e]; }
  }
  __syncthreads();
  if (tid < BN) {
    const int cc = tid / E, e = tid - cc * E, c = n0 + tid;
    float S = 0.f, Q = 0.f, Q2 = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float* r = red + (w * CPR + cc) * 3 * E;
      S += r[e];
      Q += r[E + e];
      Q2 += r[2 * E + e];
    }
    if (c < g.Ncols) {
      const int64_t rows = g.bnr_rows;
      g.bnr_part[(int64_t)c * rows + prow] = S;
      g.bnr_part[((int64_t)g.Ncols + c) * rows + prow] = Q;
      if (dual) {
        g.bnr_part2[(int64_t)c * rows + prow] = S;
        g.bnr_part2[((int64_t)g.Ncols + c) * rows + prow] = Q2;
      }
    }
  }
}

// What the epilogue's store loop reads from global memory besides the tile: the
// residual chunks and their mask bytes, and for the BN-reduce epilogue the BN's input
// y chunks, its ReLU bits and per-channel constants (epi_prefetch).  Kept apart from
// conv_epilogue so that a workgroup with one or two K-steps can issue these loads
// right behind its operand DMA (one memory round trip instead of two per workgroup:
// the 1x1 data gradients with K = Cout = 64 / 128 are a DMA wait, 8 MFMAs and this
// epilogue).
template <typename T, int BM, int BN, int NW, bool BNR>
struct EpiPre {
  static constexpr int CPR = BN * (int)sizeof(T) / 16;                 // 16-B chunks per tile row
  static constexpr int IT = (BM * CPR + 64 * NW - 1) / (64 * NW);      // store-loop trips per thread
  static constexpr int BI = BNR ? IT : 1;
  bool okv[IT];
  int64_t oidx[IT];    // element offset of the trip's chunk in `out` (0 when out of range)
  uint4 rv[IT];
  unsigned mbv[IT];
  uint4 byv[BI];       // BN reduce: the BN's input y chunks
  unsigned bmv[BI];    // and its ReLU bits
  float bcst[4];       // this thread's channel's BN-reduce constants (tid < BN)
};

template <typename T, int BM, int BN, int ACT, int NW, bool BNR>
__device__ __forceinline__ void epi_prefetch(EpiPre<T, BM, BN, NW, BNR>& p, const Geom& g,
                                             const T* __restrict__ res, int m0, int n0, int cls) {
  using P = EpiPre<T, BM, BN, NW, BNR>;
  constexpr int NT = WaveGrid<NW>::NT, CPR = P::CPR, IT = P::IT;
  constexpr int E = 16 / (int)sizeof(T);
  constexpr bool act = ACT == 1;
  const int tid = threadIdx.x;
  const bool bnr = BNR && g.bnr_part != nullptr;
  for (int k = 0; k < 4; ++k) p.bcst[k] = 0.f;
  if constexpr (BNR) {
    if (bnr && tid < BN) {
      const int c = n0 + tid < g.Ncols ? n0 + tid : 0;
      p.bcst[0] = g.bnr_mean[c];
      p.bcst[1] = g.bnr_inv[c];
      if (g.bnr_y2) {
        p.bcst[2] = g.bnr_mean2[c];
        p.bcst[3] = g.bnr_inv2[c];
      } else if (!g.bnr_mask) {
        p.bcst[2] = g.bnr_rs[c];
        p.bcst[3] = g.bnr_rb[c];
      }
    }
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = tid + it * NT;
    const int lr = idx / CPR, cc = idx - lr * CPR;
    const int m = m0 + lr, c = n0 + cc * E;
    p.okv[it] = idx < BM * CPR && m < g.M && c < g.Ncols;
    p.oidx[it] = p.okv[it] ? out_row(g, cls, m) * g.Ncols + c : 0;
    p.rv[it] = uint4{0, 0, 0, 0};
    p.mbv[it] = 0xFFu;
    if (res) {
      p.rv[it] = *reinterpret_cast<const uint4*>(res + p.oidx[it]);
      if (!act && g.res_mask) p.mbv[it] = g.res_mask[p.oidx[it] / E];
    }
    if constexpr (BNR) {
      p.byv[it] = uint4{0, 0, 0, 0};
      p.bmv[it] = 0u;
      if (bnr) {
        p.byv[it] = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(g.bnr_y) + p.oidx[it]);
        if (g.bnr_mask) p.bmv[it] = g.bnr_mask[p.oidx[it] / E];
      }
    }
  }
}

// BNR: the BN-reduce epilogue (Geom::bnr_*) compiled in -- the data-gradient instances.
// `pre`: the store loop's global operands, already fetched (epi_prefetch) when
// `pre_done`, else fetched here first.
template <typename T, int BM, int BN, int ACT = 0, int NW = 4, bool DUAL = false, bool BNR = false>
__device__ __forceinline__ void conv_epilogue(f32x4 (&acc)[BM / (16 * (NW / 2))][BN / 32], char* smem, const Geom& g,
                                              const float* __restrict__ bias, const T* __restrict__ res,
                                              T* __restrict__ out, float* __restrict__ stats, int m0, int n0,
                                              int cls, const f32x4 (*acc2)[BN / 32],
                                              EpiPre<T, BM, BN, NW, BNR>& pre, bool pre_done) {
  constexpr int WM = WaveGrid<NW>::WM, NT = WaveGrid<NW>::NT;
  constexpr int TM = BM / (16 * WM), TN = BN / 32;
  static_assert(TM % 2 == 0, "BatchNorm partials cover 32-row blocks of one wave");
  constexpr int CROW = BN * (int)sizeof(T) + 16;  // epilogue tile row stride (bytes)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr int CPR = BN * (int)sizeof(T) / 16;  // 16-B chunks per tile row
  constexpr int E = 16 / (int)sizeof(T);
  constexpr int IT = (BM * CPR + NT - 1) / NT;    // store-loop trips per thread
  static_assert(NT % CPR == 0, "store loop: fixed chunk column per thread");
  constexpr bool act = ACT == 1;
  // Everything the store loop reads from global memory (the residual chunks and their
  // mask bytes here, the eval BN-act constants once the tile is staged) is fetched
  // before the first store, and the stores are issued after the last use: a load
  // issued after a store can only be waited for with vmcnt(0), which waits for the
  // store's acknowledgement too -- a full memory round trip per trip of the store loop
  // (measured: the eval 1x1 convs took 1.2-2.2x their plain-store time that way).
  if (!pre_done) epi_prefetch<T, BM, BN, ACT, NW, BNR>(pre, g, res, m0, n0, cls);
  const bool (&okv)[IT] = pre.okv;
  const int64_t (&oidx)[IT] = pre.oidx;
  const uint4 (&rv)[IT] = pre.rv;
  const unsigned (&mbv)[IT] = pre.mbv;
  const auto& byv = pre.byv;
  const auto& bmv = pre.bmv;
  const float (&bcst)[4] = pre.bcst;
  const bool bnr = BNR && g.bnr_part != nullptr;
  const int wm = wave >> 1, wn = wave & 1;
  const int fr = lane & 15, fc = lane >> 4;
  const int row_base = m0 + wm * (BM / WM);
  const int col_base = n0 + wn * (BN / 2);
  if (bias) {
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int c = col_base + j * 16 + fr;
      const float bv = c < g.Ncols ? bias[c] : 0.f;
#pragma unroll
      for (int i = 0; i < TM; ++i) acc[i][j] += bv;
    }
  }
  if (stats) {
    // partials over blocks of 32 rows (two 16-row MFMA tiles), stats row r = m / 32,
    // stored channel-major: stats[c][r] (sum), stats[C + c][r] (M2):
    // (sum, M2 about the block-local mean) -- Chan-mergeable, free of the
    // E[x^2]-E[x]^2 cancellation; row counts follow from M (pose6d_bn_finalize).
#pragma unroll
    for (int h = 0; h < TM / 2; ++h) {
      const int rb = row_base + h * 32;
      const int nval = min(max(g.M - rb, 0), 32);
      const float inv_n = nval > 0 ? 1.0f / (float)nval : 0.f;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        float s = 0.f;
#pragma unroll
        for (int i = 2 * h; i < 2 * h + 2; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = row_base + i * 16 + fc * 4 + r;
            s += m < g.M ? acc[i][j][r] : 0.f;
          }
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        const float mu = s * inv_n;
        float q = 0.f;
#pragma unroll
        for (int i = 2 * h; i < 2 * h + 2; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int m = row_base + i * 16 + fc * 4 + r;
            const float d = acc[i][j][r] - mu;
            q = m < g.M ? fmaf(d, d, q) : q;
          }
        q += __shfl_xor(q, 16, 64);
        q += __shfl_xor(q, 32, 64);
        const int c = col_base + j * 16 + fr;
        if (lane < 16 && c < g.Ncols && nval > 0) {
          // channel-major [2][C][rows]: the finalize reads each channel's rows coalesced
          const int64_t rows = (g.M + 31) >> 5;
          stats[(int64_t)c * rows + (rb >> 5)] = s;
          stats[((int64_t)g.Ncols + c) * rows + (rb >> 5)] = q;
        }
      }
    }
  }
  // stage the tile through LDS (staging buffers are dead after the final barrier)
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int lr = wm * (BM / WM) + i * 16 + fc * 4 + r;
        const int lc = wn * (BN / 2) + j * 16 + fr;
        *reinterpret_cast<T*>(smem + lr * CROW + lc * (int)sizeof(T)) = p6::from_f<T>(acc[i][j][r]);
        // kGemmDual: the downsample branch's tile, rounded to T as its own launch stored it
        if constexpr (DUAL)
          *reinterpret_cast<T*>(smem + (BM + lr) * CROW + lc * (int)sizeof(T)) = p6::from_f<T>(acc2[i][j][r]);
      }
  float* bnr_cst = reinterpret_cast<float*>(smem + BM * CROW + 12 * NW * BN);
  if constexpr (BNR) {
    if (bnr && tid < BN) {
#pragma unroll
      for (int k = 0; k < 4; ++k) bnr_cst[k * BN + tid] = bcst[k];
    }
  }
  float asc[E], ash[E], arsc[E], arsh[E];
  // (issued after the accumulators are staged: their registers are free again)
  if (act) {
    // a thread's 16-B chunk column (tid % CPR) is the same on every trip: one set of
    // channel constants; Ncols % 8 == 0, so a chunk is wholly in range or out
    const int c = n0 + (tid % CPR) * E;
    const int cs = c < g.Ncols ? c : 0;
    load_f32s<E>(g.act_scale + cs, asc);
    load_f32s<E>(g.act_shift + cs, ash);
    if (g.act_rscale) {
      load_f32s<E>(g.act_rscale + cs, arsc);
      load_f32s<E>(g.act_rshift + cs, arsh);
    } else {
#pragma unroll
      for (int e = 0; e < E; ++e) arsc[e] = arsh[e] = 0.f;
    }
  }
  // raw barrier: LDS writes done (lgkmcnt), the prefetched global loads stay in flight
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  uint4 ov[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int idx = tid + it * NT;
    const int lr = idx < BM * CPR ? idx / CPR : 0, cc = idx - (idx / CPR) * CPR;
    uint4 v = *reinterpret_cast<const uint4*>(smem + lr * CROW + cc * 16);
    if (act) {
      // pose6d_bn_act_fwd's arithmetic on the stored (T-rounded) conv output
      T a[E], b[E];
      __builtin_memcpy(a, &v, 16);
      if constexpr (DUAL) {
        const uint4 dv = *reinterpret_cast<const uint4*>(smem + (BM + lr) * CROW + cc * 16);
        __builtin_memcpy(b, &dv, 16);
      } else {
        __builtin_memcpy(b, &rv[it], 16);
      }
#pragma unroll
      for (int e = 0; e < E; ++e) {
        float x = fmaf(p6::to_f(a[e]), asc[e], ash[e]);
        if (DUAL || res) x += g.act_rscale ? fmaf(p6::to_f(b[e]), arsc[e], arsh[e]) : p6::to_f(b[e]);
        if (g.act_relu) x = fmaxf(x, 0.f);
        a[e] = p6::from_f<T>(x);
      }
      __builtin_memcpy(&v, a, 16);
    } else if (res) {
      const unsigned mb = mbv[it];
      T a[E], b[E];
      __builtin_memcpy(a, &v, 16);
      __builtin_memcpy(b, &rv[it], 16);
#pragma unroll
      for (int e = 0; e < E; ++e)
        a[e] = p6::from_f<T>(p6::to_f(a[e]) + ((mb >> e) & 1u ? p6::to_f(b[e]) : 0.f));
      __builtin_memcpy(&v, a, 16);
    }
    ov[it] = v;
  }
  if constexpr (BNR) {
    if (bnr) {
      const int prow = ((cls >= 0 && !g.s2one) ? cls : 0) * g.gm + m0 / BM;
      bnr_partials<T, BN, NW, IT>(g, ov, okv, oidx, byv, bmv, reinterpret_cast<float*>(smem + BM * CROW), bnr_cst,
                                  prow, n0);
    }
  }
#pragma unroll
  for (int it = 0; it < IT; ++it)
    if (okv[it]) *reinterpret_cast<uint4*>(out + oidx[it]) = ov[it];
}

template <typename T, int BM, int BN, int MODE, bool ACT>
__global__ __launch_bounds__(kThreads) void conv_igemm_kernel(const T* __restrict__ src, const T* __restrict__ wts,
                                                              const float* __restrict__ bias, const T* __restrict__ res,
                                                              T* __restrict__ out, float* __restrict__ stats, Geom g) {
  constexpr int VEC = KT<T>::VEC;
  constexpr int BK = KT<T>::BK;
  constexpr int TM = BM / 32;            // 16x16 tiles per wave along M (waves 2 x 2)
  constexpr int TN = BN / 32;
  constexpr int A_PER = BM / 64;         // 16-B chunks per thread per A stage
  constexpr int B_PER = BN / 64;
  constexpr int STAGE = (BM + BN) * 64;  // bytes per LDS buffer
  extern __shared__ __attribute__((aligned(16))) char smem[];

  // XCD-aware remap: consecutive logical tiles (same M rows) share an XCD's L2.
  const int nwg = g.gm * g.gn;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int tm = bid / g.gn, tn = bid - tm * g.gn;
  const int m0 = tm * BM, n0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ck = tid & 3;  // this thread's 16-B chunk within a 64-B row segment

  // ---- per-thread A rows (fixed over K) ----
  int a_pix[A_PER], a_y[A_PER], a_x[A_PER];
  bool a_ok[A_PER];
#pragma unroll
  for (int i = 0; i < A_PER; ++i) {
    const int m = m0 + (tid >> 2) + 64 * i;
    a_ok[i] = m < g.M;
    const int mm = a_ok[i] ? m : 0;
    if (MODE == kGemm) {
      a_pix[i] = mm; a_y[i] = 0; a_x[i] = 0;
    } else {
      const int hw = g.RH * g.RW;
      const int n = mm / hw, rem = mm - n * hw;
      const int y = rem / g.RW, x = rem - y * g.RW;
      a_pix[i] = n * g.SH * g.SW;
      if (MODE == kDgrad) { a_y[i] = y + g.pad; a_x[i] = x + g.pad; }
      else { a_y[i] = y * g.stride - g.pad; a_x[i] = x * g.stride - g.pad; }
    }
  }
  // ---- per-thread B rows ----
  const T* b_ptr[B_PER];
  bool b_ok[B_PER];
#pragma unroll
  for (int i = 0; i < B_PER; ++i) {
    const int n = n0 + (tid >> 2) + 64 * i;
    b_ok[i] = n < g.Ncols;
    b_ptr[i] = wts + (int64_t)(b_ok[i] ? n : 0) * g.Kpad + ck * VEC;
  }

  const int nk = g.Kpad / BK;
  uint4 ra[A_PER], rb[B_PER];

  auto load_tile = [&](int kt) {
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < B_PER; ++i)
      rb[i] = b_ok[i] ? *reinterpret_cast<const uint4*>(b_ptr[i] + k0) : make_uint4(0, 0, 0, 0);
    if (MODE == kGemm) {
#pragma unroll
      for (int i = 0; i < A_PER; ++i)
        ra[i] = a_ok[i] ? *reinterpret_cast<const uint4*>(src + (int64_t)a_pix[i] * g.K + k0 + ck * VEC)
                        : make_uint4(0, 0, 0, 0);
    } else if (MODE == kFwd || MODE == kDgrad) {
      const int tap = k0 >> g.log2SC, c0 = k0 & (g.SC - 1);
      const int kh = tap / g.KW, kw = tap - kh * g.KW;
#pragma unroll
      for (int i = 0; i < A_PER; ++i) {
        int sy, sx;
        bool ok = a_ok[i] && k0 < g.K;
        if (MODE == kFwd) {
          sy = a_y[i] + kh; sx = a_x[i] + kw;
        } else {
          const int ty = a_y[i] - kh, tx = a_x[i] - kw;
          ok = ok && ty >= 0 && tx >= 0;
          if (g.stride == 2) { ok = ok && !(ty & 1) && !(tx & 1); sy = ty >> 1; sx = tx >> 1; }
          else { sy = ty; sx = tx; }
        }
        ok = ok && (unsigned)sy < (unsigned)g.SH && (unsigned)sx < (unsigned)g.SW;
        ra[i] = ok ? *reinterpret_cast<const uint4*>(src + ((int64_t)(a_pix[i] + sy * g.SW + sx) << g.log2SC) + c0 +
                                                     ck * VEC)
                   : make_uint4(0, 0, 0, 0);
      }
    } else {  // kFwdNarrow: SC == 4 channels per tap (stem, Cin padded 3 -> 4)
      constexpr int UNITS = VEC / 4;       // taps per 16-B chunk (bf16: 2, fp32: 1)
#pragma unroll
      for (int i = 0; i < A_PER; ++i) {
        uint32_t w[4];
#pragma unroll
        for (int u = 0; u < UNITS; ++u) {
          const int k = k0 + ck * VEC + u * 4;
          const int tap = k >> 2;
          const int kh = tap / g.KW, kw = tap - kh * g.KW;
          const int sy = a_y[i] + kh, sx = a_x[i] + kw;
          const bool ok = a_ok[i] && k < g.K && (unsigned)sy < (unsigned)g.SH && (unsigned)sx < (unsigned)g.SW;
          const T* p = src + ((int64_t)(a_pix[i] + sy * g.SW + sx) << 2);
          if (UNITS == 2) {
            uint2 v = ok ? *reinterpret_cast<const uint2*>(p) : make_uint2(0, 0);
            w[2 * u] = v.x; w[2 * u + 1] = v.y;
          } else {
            uint4 v = ok ? *reinterpret_cast<const uint4*>(p) : make_uint4(0, 0, 0, 0);
            w[0] = v.x; w[1] = v.y; w[2] = v.z; w[3] = v.w;
          }
        }
        ra[i] = make_uint4(w[0], w[1], w[2], w[3]);
      }
    }
  };

  auto store_tile = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + BM * 64;
#pragma unroll
    for (int i = 0; i < A_PER; ++i) {
      const int row = (tid >> 2) + 64 * i;
      *reinterpret_cast<uint4*>(As + row * 64 + ((ck ^ swz(row)) << 4)) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_PER; ++i) {
      const int row = (tid >> 2) + 64 * i;
      *reinterpret_cast<uint4*>(Bs + row * 64 + ((ck ^ swz(row)) << 4)) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fc = lane >> 4;
  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + BM * 64;
    uint4 af[TM], bfr[TN];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * (BM / 2) + i * 16 + fr;
      af[i] = *reinterpret_cast<const uint4*>(As + row * 64 + ((fc ^ swz(row)) << 4));
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wn * (BN / 2) + j * 16 + fr;
      bfr[j] = *reinterpret_cast<const uint4*>(Bs + row * 64 + ((fc ^ swz(row)) << 4));
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        if constexpr (sizeof(T) == 2) {
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, af[i]),
                                                              __builtin_bit_cast(bf16x8, bfr[j]), acc[i][j], 0, 0, 0);
        } else {
          const f32x4 a4 = __builtin_bit_cast(f32x4, af[i]);
          const f32x4 b4 = __builtin_bit_cast(f32x4, bfr[j]);
#pragma unroll
          for (int s = 0; s < 4; ++s) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[s], b4[s], acc[i][j], 0, 0, 0);
        }
      }
  };

  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile(kt + 1);
    compute(cur);
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  EpiPre<T, BM, BN, 4, false> pre;
  conv_epilogue<T, BM, BN, ACT ? 1 : 0>(acc, smem, g, bias, res, out, stats, m0, n0, -1, nullptr, pre, false);
}

// ============================================================================
// Fast path (bf16, K a multiple of 64 within one tap): BK = 64, an S-stage LDS
// ring filled by LDS-DMA (global_load_lds_dwordx4, 1 KiB = 8 rows x 128 B per
// wave instruction), S-1 stages in flight while one is computed; one raw
// s_barrier per K-step behind a counted vmcnt (never __syncthreads in the loop:
// its fence would drain the in-flight DMA).  Padding taps / rows past M read a
// zero page instead of being masked.  The XOR swizzle (row >> 1) & 7 is applied
// on the DMA SOURCE address (the LDS destination of LDS-DMA is lane-linear) and
// on the ds_read_b128 fragment reads: conflict-free for both 16-lane k-halves.
// S is picked per layer: deep rings for small, long-K grids (latency bound: one
// workgroup per CU, each K-step short), shallow ones for big grids (occupancy).
// ============================================================================
// Fragment reads of one k-half as ONE asm block: NR ds_read_b128 then
// lgkmcnt(0).  Written as plain C++ loads, hipcc cannot tell the ring slot being
// read from the slots the in-flight LDS-DMA is filling and emits vmcnt(0) before
// the first ds_read of every K-step, draining the whole prefetch ring (the .s
// showed it: deeper rings bought nothing).  The counted vmcnt + barrier in the
// K-loop is what orders these reads after the DMA that filled the slot.
template <int NR>
__device__ __forceinline__ void lds_read_frags(u32x4 (&f)[NR], const unsigned (&addr)[NR]) {
  static_assert(NR == 4 || NR == 6 || NR == 8, "fragment batch of 4, 6 or 8 reads");
  if constexpr (NR == 4) {
    asm volatile(
        "ds_read_b128 %0, %4\n\tds_read_b128 %1, %5\n\tds_read_b128 %2, %6\n\tds_read_b128 %3, %7\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3])
        : "v"(addr[0]), "v"(addr[1]), "v"(addr[2]), "v"(addr[3]));
  } else if constexpr (NR == 6) {
    asm volatile(
        "ds_read_b128 %0, %6\n\tds_read_b128 %1, %7\n\tds_read_b128 %2, %8\n\tds_read_b128 %3, %9\n\t"
        "ds_read_b128 %4, %10\n\tds_read_b128 %5, %11\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3]), "=&v"(f[4]), "=&v"(f[5])
        : "v"(addr[0]), "v"(addr[1]), "v"(addr[2]), "v"(addr[3]), "v"(addr[4]), "v"(addr[5]));
  } else {
    asm volatile(
        "ds_read_b128 %0, %8\n\tds_read_b128 %1, %9\n\tds_read_b128 %2, %10\n\tds_read_b128 %3, %11\n\t"
        "ds_read_b128 %4, %12\n\tds_read_b128 %5, %13\n\tds_read_b128 %6, %14\n\tds_read_b128 %7, %15\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3]), "=&v"(f[4]), "=&v"(f[5]), "=&v"(f[6]), "=&v"(f[7])
        : "v"(addr[0]), "v"(addr[1]), "v"(addr[2]), "v"(addr[3]), "v"(addr[4]), "v"(addr[5]), "v"(addr[6]),
          "v"(addr[7]));
  }
}

// Both k-halves of a 64x64 tile's fragments (2 x 4 ds_read_b128) issued as ONE asm
// batch without a wait; lds_wait_first / lds_wait_all then release them in two
// steps (counted lgkmcnt), so the second half's reads are in flight while the
// first half's MFMAs run.  The waits name the fragments as in-out operands: the
// compiler cannot hoist an MFMA that consumes them above the wait.
__device__ __forceinline__ void lds_issue_frags8(u32x4 (&f)[2][4], const unsigned (&a)[2][4]) {
  asm volatile(
      "ds_read_b128 %0, %8\n\tds_read_b128 %1, %9\n\tds_read_b128 %2, %10\n\tds_read_b128 %3, %11\n\t"
      "ds_read_b128 %4, %12\n\tds_read_b128 %5, %13\n\tds_read_b128 %6, %14\n\tds_read_b128 %7, %15"
      : "=&v"(f[0][0]), "=&v"(f[0][1]), "=&v"(f[0][2]), "=&v"(f[0][3]), "=&v"(f[1][0]), "=&v"(f[1][1]),
        "=&v"(f[1][2]), "=&v"(f[1][3])
      : "v"(a[0][0]), "v"(a[0][1]), "v"(a[0][2]), "v"(a[0][3]), "v"(a[1][0]), "v"(a[1][1]), "v"(a[1][2]),
        "v"(a[1][3]));
}
__device__ __forceinline__ void lds_wait_first(u32x4 (&f)[4]) {
  asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
}
__device__ __forceinline__ void lds_wait_all(u32x4 (&f)[4]) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
}

// one 16-byte fragment pair -> the 16x16 accumulator: bf16 = one 16x16x32 MFMA,
// fp32 = four exact 16x16x4 MFMAs (component s of every lane's chunk)
template <typename T>
__device__ __forceinline__ void mma_frag(f32x4& acc, const u32x4& a, const u32x4& b) {
  if constexpr (sizeof(T) == 2) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc, 0,
                                                  0, 0);
  } else {
    const f32x4 a4 = __builtin_bit_cast(f32x4, a), b4 = __builtin_bit_cast(f32x4, b);
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a4[s], b4[s], acc, 0, 0, 0);
  }
}

#ifndef POSE6D_PAIRED_FRAGS
#define POSE6D_PAIRED_FRAGS 1
#endif
constexpr bool kPairedFrags = POSE6D_PAIRED_FRAGS;

// Element geometry of the LDS-DMA path: a 16-byte chunk holds CH elements, a K-step
// (one 128-byte LDS row per GEMM row) KS = 8 CH: 64 bf16 or 32 fp32.  bf16 feeds
// v_mfma_f32_16x16x32_bf16 (one per 16x16 tile and k-half); fp32 feeds the exact
// v_mfma_f32_16x16x4_f32, four per tile and k-half -- a lane's 16-byte chunk holds
// k = 4 (fc + 4 kk) + s, s = 0..3, for A and B alike, so MFMA s sums the same k.
template <typename T> struct LK { static constexpr int CH = 16 / (int)sizeof(T), KS = 8 * CH; };

// one workgroup's work; `bid_in` = its index in this conv's sub-grid (the whole grid,
// or the leading part of a fused backward launch), `smem` = the kernel's dynamic LDS
// PRE: a workgroup with at most two K-steps fetches its epilogue's global operands
// (epi_prefetch) right after issuing its operand DMA (build-time switch for A/B
// timing: -DPOSE6D_EPI_PRE=0 builds the fetch-after-the-loop form)
#ifndef POSE6D_EPI_PRE
#define POSE6D_EPI_PRE 1
#endif
#ifndef POSE6D_S2_ROTATE
#define POSE6D_S2_ROTATE 1   // build-time (A/B): 0 = the fixed class order (profiles/r05rot_s2_class_order_ab.txt)
#endif
template <typename T, int BM, int BN, int MODE, int S, bool ACT = false, int NW = 4, bool BNR = false,
          bool PRE = false>
__device__ __forceinline__ void conv_lds_body(char* smem, int bid_in, const T* __restrict__ src,
                                              const T* __restrict__ wts, const float* __restrict__ bias,
                                              const T* __restrict__ res, T* __restrict__ out,
                                              float* __restrict__ stats, const Geom& g) {
  constexpr int CH = LK<T>::CH, KS = LK<T>::KS;
  static_assert(KS == 64 || KS == 32, "bf16 or fp32");
  constexpr int LOG_KS = KS == 64 ? 6 : 5;
  constexpr int WM = WaveGrid<NW>::WM;
  constexpr int TM = BM / (16 * WM), TN = BN / 32;
  constexpr int RW = 8 * NW;                        // rows one DMA instruction of every wave covers
  constexpr int A_INS = BM / RW, B_INS = BN / RW;   // DMA instructions per thread per stage
  static_assert(A_INS * RW == BM && B_INS * RW == BN, "tile rows must be a multiple of 8 x waves");
  constexpr int LOADS = A_INS + B_INS;
  constexpr int SA = BM * 128, STAGE = (BM + BN) * 128;
  static_assert(S >= 2, "ring needs two stages");

  constexpr bool SK = MODE == kGemm || MODE == kFwd || MODE == kDgrad;   // split-K capable modes
  const int nsplit = SK && g.splits > 1 ? g.splits : 1;
  const int per = g.gm * g.gn;
  const int nwg = (MODE == kDgradS2 ? s2_classes(g) * per : per) * nsplit;
  int bid = bid_in;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  // split-K: the splits of one tile are consecutive logical ids (one XCD, mostly)
  int split = 0;
  if (nsplit > 1) {
    split = bid % nsplit;
    bid /= nsplit;
  }
  const int tile_id = bid;
  // parity class (kDgradS2): the four classes of one tile are consecutive logical
  // ids, so every XCD gets an even share of the heavy and the empty classes and the
  // four blocks that gather the same dY rows run on the same L2
  constexpr bool DUAL = MODE == kGemmDual;
  int cls = -1, py = 0, px = 0, kh0 = 0, kw0 = 0, ntx = 1, nk = g.Kpad >> LOG_KS;
  const int nk1 = nk;   // kGemmDual: K-steps of the first (block) GEMM
  if (DUAL) nk += g.Kpad2 >> LOG_KS;
  if (MODE == kDgradS2) {
    if (g.s2one) {
      cls = g.s2one - 1;
    } else {
#if POSE6D_S2_ROTATE
      // the four classes of tile t are logical ids 4t .. 4t+3 (one XCD, one L2), in an
      // order that rotates with t: the dispatcher deals an XCD's workgroups out to its
      // shader engines in turn, so a fixed order would give each engine one class (the
      // 4-tap class's engine doing 4/9 of the work; a 1x1's tap class on one engine)
      cls = 3 - ((bid + (bid >> 2)) & 3);
#else
      cls = 3 - (bid & 3);
#endif
      bid >>= 2;
    }
    py = cls >> 1; px = cls & 1;
    kh0 = (py + g.pad) & 1; kw0 = (px + g.pad) & 1;   // first tap of this parity, then every 2nd
    const int nty = (g.KH - kh0 + 1) >> 1;
    ntx = (g.KW - kw0 + 1) >> 1;
    nk = (nty * ntx) << (g.log2SC - LOG_KS);
    // a class no tap reaches (1x1 stride 2: three of four) contributes zeros: with
    // the residual accumulated in place (res == out) its pixels are already final
    if (nk == 0 && res == out) return;
  }
  // consecutive logical tiles share an XCD (remap above): M-major keeps a few A row
  // blocks + all of B in that XCD's L2
  const int tm = bid / g.gn, tn = bid - tm * g.gn;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int r8 = lane >> 3, pch = lane & 7;
  const char* zp = reinterpret_cast<const char*>(g_zero_page);

  // rows this lane DMAs: row = i*RW + wave*8 + r8; it fetches logical chunk pch ^ swz8(row)
  int a_pix[A_INS], a_y[A_INS], a_x[A_INS], a_ck[A_INS];
  int a_pix2[DUAL ? A_INS : 1];   // kGemmDual: the row's pixel in the downsample operand
  bool a_ok[A_INS];
#pragma unroll
  for (int i = 0; i < A_INS; ++i) {
    const int row = i * RW + wave * 8 + r8;
    const int m = m0 + row;
    a_ok[i] = m < g.M;
    a_ck[i] = (pch ^ swz8(row)) * CH;
    const int mm = a_ok[i] ? m : 0;
    if (MODE == kGemm || DUAL) {
      a_pix[i] = mm; a_y[i] = 0; a_x[i] = 0;
      if constexpr (DUAL) {
        const int hw = g.RH * g.RW;
        const int n = mm / hw, rem = mm - n * hw;
        const int y = rem / g.RW, x = rem - y * g.RW;
        a_pix2[i] = (n * g.SH2 + y * g.stride2) * g.SW2 + x * g.stride2;
      }
    } else {
      const int hw = g.RH * g.RW;
      const int n = mm / hw, rem = mm - n * hw;
      const int y = rem / g.RW, x = rem - y * g.RW;
      a_pix[i] = n * g.SH * g.SW;
      if (MODE == kDgrad) { a_y[i] = y + g.pad; a_x[i] = x + g.pad; }
      else if (MODE == kDgradS2) { a_y[i] = y; a_x[i] = x; }
      else if (MODE == kFwdRowTap) { a_y[i] = y * g.stride - g.pad; a_x[i] = x * g.stride - g.pad - (kRowTaps - g.KW); }
      else { a_y[i] = y * g.stride - g.pad; a_x[i] = x * g.stride - g.pad; }
    }
  }
  // B rows: n >= Ncols read the zero page (offset masked to 0)
  const T* b_base[B_INS];
  unsigned b_mask[B_INS];
#pragma unroll
  for (int j = 0; j < B_INS; ++j) {
    const int row = j * RW + wave * 8 + r8;
    const int n = n0 + row;
    const bool ok = n < g.Ncols;
    b_base[j] = ok ? wts + (int64_t)n * g.Kpad + (pch ^ swz8(row)) * CH : reinterpret_cast<const T*>(zp);
    b_mask[j] = ok ? ~0u : 0u;
  }
  // kGemmDual: the downsample weights' rows, switched to after the first GEMM's K-steps
  const T* b_base2[DUAL ? B_INS : 1];
  if constexpr (DUAL) {
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const int row = j * RW + wave * 8 + r8;
      const int n = n0 + row;
      b_base2[j] = n < g.Ncols ? reinterpret_cast<const T*>(g.wts2) + (int64_t)n * g.Kpad2 + (pch ^ swz8(row)) * CH
                               : reinterpret_cast<const T*>(zp);
    }
  }
  int phase = 0;   // kGemmDual: 0 = block GEMM, 1 = downsample GEMM

  // The K loop walks filter taps in order; inside a tap the 64-deep slices are
  // contiguous channels.  Row source pointers (and their validity: padding, rows
  // past M, stride-2 holes) change only at a tap boundary, so they are rebuilt
  // there (uniform branch) and each K-step only adds the channel offset c0 --
  // the per-step address arithmetic that made these kernels issue-bound at one
  // workgroup per CU.  issue() is called with consecutive kt.
  int tap_len = (MODE == kGemm || DUAL) ? g.Kpad : (MODE == kFwdRowTap ? KS : g.SC);   // row-tap: one K-step
  int c0 = 0, kh = kh0, kw = kw0, tw = 0, tap_koff = MODE == kDgradS2 ? (kh0 * g.KW + kw0) * g.SC : 0;
  const T* a_base[A_INS];
  unsigned a_mask[A_INS];
  auto set_tap = [&]() {
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
      bool ok = a_ok[i];
      int64_t off = 0;
      if (MODE == kGemm || DUAL) {
        off = (int64_t)a_pix[i] * g.K;
        if constexpr (DUAL) {
          if (phase) {
            off = (int64_t)a_pix2[i] * g.Kpad2;
            a_base[i] = ok ? reinterpret_cast<const T*>(g.src2) + off + a_ck[i] : reinterpret_cast<const T*>(zp);
            a_mask[i] = ok ? ~0u : 0u;
            continue;
          }
        }
      } else if (MODE == kFwdRowTap) {
        // K-step kh: this lane's 16-B chunk (logical chunk a_ck / CH) is kernel row kr,
        // taps 4 x2 .. (8 elements = 2 pixels bf16, 4 = 1 pixel fp32) of that row
        const int ke = kh * KS + a_ck[i];
        const int kr = ke >> 5, sy = a_y[i] + kr, sx = a_x[i] + ((ke & 31) >> 2);
        ok = ok && kr < g.KH && (unsigned)sy < (unsigned)g.SH && (unsigned)sx < (unsigned)g.SW;
        a_base[i] = ok ? src + ((int64_t)(a_pix[i] + sy * g.SW + sx) << 2) : reinterpret_cast<const T*>(zp);
        a_mask[i] = ok ? ~0u : 0u;
        continue;
      } else {
        int sy, sx;
        if (MODE == kFwd) {
          sy = a_y[i] + kh; sx = a_x[i] + kw;
        } else if (MODE == kDgradS2) {
          // dX(2yy+py) <- dY((2yy + py + pad - kh) / 2); the numerator is even by construction
          sy = a_y[i] + ((py + g.pad - kh) >> 1);
          sx = a_x[i] + ((px + g.pad - kw) >> 1);
        } else {
          const int ty = a_y[i] - kh, tx = a_x[i] - kw;
          ok = ok && ty >= 0 && tx >= 0;
          if (g.stride == 2) { ok = ok && !(ty & 1) && !(tx & 1); sy = ty >> 1; sx = tx >> 1; }
          else { sy = ty; sx = tx; }
        }
        ok = ok && (unsigned)sy < (unsigned)g.SH && (unsigned)sx < (unsigned)g.SW;
        off = (int64_t)(a_pix[i] + sy * g.SW + sx) << g.log2SC;
      }
      a_base[i] = ok ? src + off + a_ck[i] : reinterpret_cast<const T*>(zp);
      a_mask[i] = ok ? ~0u : 0u;
    }
  };

  // one stage's DMA as (source, LDS destination) pairs, then the tap walk advanced;
  // issue() fires them back to back, the interleaved compute (POSE6D_ILV) one per MFMA
  const T* dsrc[LOADS];
  char* ddst[LOADS];
  auto prep = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + SA;
    if (c0 == 0) set_tap();
    const unsigned boff = (unsigned)(tap_koff + c0);
#pragma unroll
    for (int j = 0; j < B_INS; ++j) {
      const T* bb = b_base[j];
      if constexpr (DUAL) bb = phase ? b_base2[j] : b_base[j];
      dsrc[j] = bb + (boff & b_mask[j]);
      ddst[j] = Bs + (j * RW + wave * 8) * 128;
    }
#pragma unroll
    for (int i = 0; i < A_INS; ++i) {
      dsrc[B_INS + i] = a_base[i] + ((unsigned)c0 & a_mask[i]);
      ddst[B_INS + i] = As + (i * RW + wave * 8) * 128;
    }
    c0 += KS;
    if (c0 == tap_len) {
      c0 = 0;
      if constexpr (DUAL) {
        phase = 1;
        tap_len = g.Kpad2;
        return;
      }
      if (MODE == kDgradS2) {
        kw += 2;
        if (++tw == ntx) { tw = 0; kw = kw0; kh += 2; }
        tap_koff = (kh * g.KW + kw) * g.SC;
      } else if (MODE == kFwdRowTap) {   // kh counts K-steps
        ++kh;
        tap_koff += KS;
      } else {
        if (++kw == g.KW) { kw = 0; ++kh; }
        tap_koff += g.SC;
      }
    }
  };
  auto issue = [&](int kt, int buf) {
    (void)kt;
    prep(buf);
#pragma unroll
    for (int q = 0; q < LOADS; ++q) glds16(dsrc[q], ddst[q]);
  };

  // split-K: this workgroup's K-steps [kb, ke) of the tile; the tap walk starts at kb
  if (SK && nsplit > 1) {
    const int kb = (int)((int64_t)split * nk / nsplit), ke = (int)((int64_t)(split + 1) * nk / nsplit);
    nk = ke - kb;
    if (MODE == kGemm) {
      c0 = kb << LOG_KS;
    } else {
      const int spt = g.SC >> LOG_KS;   // K-steps per filter tap
      const int tap = kb / spt;
      c0 = (kb - tap * spt) << LOG_KS;
      kh = tap / g.KW;
      kw = tap - kh * g.KW;
      tap_koff = tap * g.SC;
    }
    if (c0 != 0) set_tap();   // issue() rebuilds the row pointers only at a tap start
  }

  f32x4 acc[TM][TN];
  f32x4 acc2[DUAL ? TM : 1][DUAL ? TN : 1];   // kGemmDual: the block GEMM's sums, parked
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // per-lane fragment byte offsets inside a ring slot (row-dependent swizzle), per k-half
  const int fr = lane & 15, fc = lane >> 4;
  unsigned frag_off[2][TM + TN];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int row = wm * (BM / WM) + i * 16 + fr;
      frag_off[kk][i] = row * 128 + (((fc + 4 * kk) ^ swz8(row)) << 4);
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wn * (BN / 2) + j * 16 + fr;
      frag_off[kk][TM + j] = SA + row * 128 + (((fc + 4 * kk) ^ swz8(row)) << 4);
    }
  }
  const unsigned ring_base = lds_addr(smem);
  // mid(): issued between the fragment reads and their wait, so the next stage's
  // LDS-DMA issue (tens of cycles per instruction) overlaps the LDS read latency
  // POSE6D_ILV: the next stage's DMA instructions issued one after each first-k-half
  // MFMA instead of as one burst before them (a DMA wave-instruction costs the wave
  // ~60-185 issue cycles, an MFMA 16 of pipe time: interleaved, the issue cost hides
  // behind the matrix pipe)
  auto compute_ilv = [&](int buf, bool has, auto& acc) {
    const unsigned slot = ring_base + buf * STAGE;
    constexpr int NM = TM * TN;   // MFMAs per k-half
    constexpr int GAP = NM / LOADS > 0 ? NM / LOADS : 1;
    if constexpr (TM + TN == 4 && kPairedFrags) {
      unsigned addr[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int r = 0; r < 4; ++r) addr[kk][r] = slot + frag_off[kk][r];
      u32x4 f[2][4];
      lds_issue_frags8(f, addr);
      lds_wait_first(f[0]);
#pragma unroll
      for (int q = 0; q < NM; ++q) {
        mma_frag<T>(acc[q / TN][q % TN], f[0][q / TN], f[0][TM + q % TN]);
        if (q % GAP == GAP - 1 && q / GAP < LOADS && has) glds16(dsrc[q / GAP], ddst[q / GAP]);
      }
#pragma unroll
      for (int q = NM / GAP; q < LOADS; ++q)
        if (has) glds16(dsrc[q], ddst[q]);
      lds_wait_all(f[1]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mma_frag<T>(acc[i][j], f[1][i], f[1][TM + j]);
      return;
    }
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      unsigned addr[TM + TN];
#pragma unroll
      for (int r = 0; r < TM + TN; ++r) addr[r] = slot + frag_off[kk][r];
      u32x4 f[TM + TN];
      lds_read_frags<TM + TN>(f, addr);
#pragma unroll
      for (int q = 0; q < NM; ++q) {
        mma_frag<T>(acc[q / TN][q % TN], f[q / TN], f[TM + q % TN]);
        if (kk == 0 && q % GAP == GAP - 1 && q / GAP < LOADS && has) glds16(dsrc[q / GAP], ddst[q / GAP]);
      }
      if (kk == 0) {
#pragma unroll
        for (int q = NM / GAP; q < LOADS; ++q)
          if (has) glds16(dsrc[q], ddst[q]);
      }
    }
  };
  auto compute = [&](int buf, auto&& mid, auto& acc) {
    const unsigned slot = ring_base + buf * STAGE;
    if constexpr (TM + TN == 4 && kPairedFrags) {
      unsigned addr[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int r = 0; r < 4; ++r) addr[kk][r] = slot + frag_off[kk][r];
      u32x4 f[2][4];
      lds_issue_frags8(f, addr);
      mid();
      lds_wait_first(f[0]);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        if (kk == 1) lds_wait_all(f[1]);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) mma_frag<T>(acc[i][j], f[kk][i], f[kk][TM + j]);
      }
      return;
    }
    mid();
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      unsigned addr[TM + TN];
#pragma unroll
      for (int r = 0; r < TM + TN; ++r) addr[r] = slot + frag_off[kk][r];
      u32x4 f[TM + TN];
      lds_read_frags<TM + TN>(f, addr);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mma_frag<T>(acc[i][j], f[i], f[TM + j]);
    }
  };

  // prologue: stages 0 .. S-2 in flight; step kt refills the buffer step kt-1 read
  for (int s = 0; s < S - 1 && s < nk; ++s) issue(s, s);
  // early epilogue fetch (PRE): younger than the prologue DMA, so the loop's counted
  // waits (which count DMA only) over-wait it on the first step -- correct, and with
  // one or two K-steps the two sets of loads are in flight together
  EpiPre<T, BM, BN, NW, BNR> pre;
  const bool early = POSE6D_EPI_PRE && PRE && !DUAL && nk <= 2;
  if (early) epi_prefetch<T, BM, BN, ACT ? 1 : 0, NW, BNR>(pre, g, res, m0, n0, cls);
  int cur = 0, wbuf = S - 1;
  for (int kt = 0; kt < nk; ++kt) {
    const int left = nk - 1 - kt;
    wait_ahead<LOADS, S - 2>(left < S - 2 ? left : S - 2);   // stage kt landed, for every wave
    auto mid = [&]() {
      if (kt + S - 1 < nk) issue(kt + S - 1, wbuf);
    };
    if constexpr (DUAL) {
      // the block GEMM is complete: park its sums, accumulate the downsample afresh
      // (one accumulator set in the loop keeps the register budget of the plain kernel)
      if (kt == nk1) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) {
            acc2[i][j] = acc[i][j];
            acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
          }
      }
    }
#ifndef POSE6D_ILV
#define POSE6D_ILV 0
#endif
    if constexpr (POSE6D_ILV && !DUAL) {
      const bool has = kt + S - 1 < nk;
      if (has) prep(wbuf);
      compute_ilv(cur, has, acc);
    } else {
      compute(cur, mid, acc);
    }
    cur = cur == S - 1 ? 0 : cur + 1;
    wbuf = wbuf == S - 1 ? 0 : wbuf + 1;
  }
  asm volatile("s_barrier" ::: "memory");   // every wave done reading the ring before the epilogue reuses it
  if constexpr (SK) {
    if (nsplit > 1 && !splitk_merge<TM, TN, NW>(acc, smem, tile_id, split, nsplit, g.sk_cnt, g.sk_part)) return;
  }
  if constexpr (DUAL)   // acc2 = the block GEMM, acc = the downsample branch
    conv_epilogue<T, BM, BN, 1, NW, true>(acc2, smem, g, bias, nullptr, out, nullptr, m0, n0, -1, acc, pre, false);
  else
    conv_epilogue<T, BM, BN, ACT ? 1 : 0, NW, false, BNR>(acc, smem, g, bias, res, out, stats, m0, n0, cls, nullptr,
                                                          pre, early);
}

// BNR: data gradient with the BatchNorm-reduce epilogue (its own instance: the
// forward 1x1 kernels, kGemm too, keep their register budget)
template <typename T, int BM, int BN, int MODE, int S, bool ACT, int NW, bool BNR = false>
__global__ __launch_bounds__(64 * NW) void conv_lds_kernel(const T* __restrict__ src, const T* __restrict__ wts,
                                                           const float* __restrict__ bias, const T* __restrict__ res,
                                                           T* __restrict__ out, float* __restrict__ stats, Geom g) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  conv_lds_body<T, BM, BN, MODE, S, ACT, NW, BNR>(smem, blockIdx.x, src, wts, bias, res, out, stats, g);
}

#include "conv_patch.h"

// Fused backward of one conv.  Both passes read the same dY, and the weight-
// gradient workgroups fill the CUs the (often small) data-gradient grid leaves idle
// -- one launch instead of two.  Workgroup order = the order the dispatcher starts
// them, longest work first (`wfirst`, chosen per conv by launch_bwd): with wfirst,
// [0, nw) the weight gradient, [nw_pad, nw_pad + nd) the data gradient, else the data
// gradient [0, nd) and the weight gradient [nd_pad, nd_pad + nw); the carried slab
// reduce last.  (nw_pad / nd_pad round up to 8 so each part's XCD remap stays intact;
// the padding workgroups exit at once.)  The weight-gradient workgroups of a 1x1
// conv run ~10 K-steps; dispatched behind thousands of one- to four-step data-
// gradient workgroups they were the launch's tail.
// T = float: the same launch for the reference-precision (fp32) step -- the fp32
// LDS-DMA data gradient and the fp32 LDS-DMA weight gradient (wgrad_body.h).
#ifndef POSE6D_BWD_F32_MS
#define POSE6D_BWD_F32_MS 32   // build-time (A/B): pixels per fp32 weight-gradient stage in the fused launch
#endif
constexpr int kBwdF32MS = POSE6D_BWD_F32_MS;
// WBT (fp32 only): the weight-gradient tile, 64 or 128 (the wider KxK convs' plans: 128x128
// on 32-pixel stages, conv_wgrad_lds_body_f32)
template <int DMODE, int DS, int WS, typename T = bf16, int WBT = 64>
__global__ __launch_bounds__(kThreads) void conv_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ wt,
                                                            const T* __restrict__ dres, T* __restrict__ dx,
                                                            Geom gd, int nd, int nd_pad, int wfirst,
                                                            const T* __restrict__ x, float* __restrict__ ws,
                                                            p6::WGeom gw, ReduceJob rj) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  const int nw = gw.gm * gw.gn * gw.splits;
  const int nw_pad = (nw + 7) & ~7;
  const int d0 = wfirst ? nw_pad : 0;                  // first data-gradient workgroup
  const int w0 = wfirst ? 0 : nd_pad;                  // first weight-gradient workgroup
  const int r0 = wfirst ? nw_pad + nd : nd_pad + nw;   // first reduce workgroup (last: they fill the tail)
  if (b >= d0 && b < d0 + nd) {
    conv_lds_body<T, 64, 64, DMODE, DS, false, 4, true, true>(smem, b - d0, dy, wt, nullptr, dres, dx, nullptr, gd);
  } else if (b >= w0 && b < w0 + nw) {
    // kGemm data gradient <=> pointwise conv: the weight gradient takes the pointwise body
    if constexpr (sizeof(T) == 2)
      conv_wgrad_lds_body<64, 64, WS, DMODE == kGemm>(smem, b - w0, x, dy, ws, gw);
    else if constexpr (WBT == 128)
      conv_wgrad_lds_body_f32<32, WS, DMODE == kGemm, 128>(smem, b - w0, x, dy, ws, gw);
    else
      conv_wgrad_lds_body_f32<kBwdF32MS, WS, DMODE == kGemm>(smem, b - w0, x, dy, ws, gw);
  } else if (b >= r0) {
    // the previous conv's weight-gradient slabs (another workspace), reduced here
    // instead of in a launch of their own
    run_reduce_job(smem, b - r0, rj);
  }
}

// The 8-wave form of the fused backward for the bf16 weight gradients on 128x128 tiles
// (wgrad_body.h, NW = 8: twice the MACs per staged byte of the 64x64 tile; the KxK
// convs' plans, conv_wgrad.hip): the data gradient runs on 128x64 tiles of 8 waves in
// the same launch, the carried slab reduce on the first four waves of its workgroups
// (the other four only meet its one barrier).
template <int DMODE, int DS, int WS>
__global__ __launch_bounds__(2 * kThreads) void conv_bwd8_kernel(const bf16* __restrict__ dy,
                                                                  const bf16* __restrict__ wt,
                                                                  const bf16* __restrict__ dres, bf16* __restrict__ dx,
                                                                  Geom gd, int nd, int nd_pad, int wfirst,
                                                                  const bf16* __restrict__ x, float* __restrict__ ws,
                                                                  p6::WGeom gw, ReduceJob rj) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int b = blockIdx.x;
  const int nw = gw.gm * gw.gn * gw.splits;
  const int nw_pad = (nw + 7) & ~7;
  const int d0 = wfirst ? nw_pad : 0;
  const int w0 = wfirst ? 0 : nd_pad;
  const int r0 = wfirst ? nw_pad + nd : nd_pad + nw;
  if (b >= d0 && b < d0 + nd) {
    conv_lds_body<bf16, 128, 64, DMODE, DS, false, 8, true, true>(smem, b - d0, dy, wt, nullptr, dres, dx, nullptr,
                                                                  gd);
  } else if (b >= w0 && b < w0 + nw) {
    conv_wgrad_lds_body<128, 128, WS, DMODE == kGemm, false, 8>(smem, b - w0, x, dy, ws, gw);
  } else if (b >= r0) {
    if (threadIdx.x < kThreads) run_reduce_job(smem, b - r0, rj);
    else __syncthreads();   // the reduce body's one workgroup barrier
  }
}

// K-steps of the longest work item (kDgradS2: the class with the most taps);
// ks = elements per K-step (64 bf16, 32 fp32)
int fast_nk(int mode, const Geom& g, int ks = 64) {
  if (mode == kGemmDual) return (g.Kpad + g.Kpad2) / ks;
  if (mode != kDgradS2) return g.Kpad / ks;
  int best = 0;
  for (int cls = 0; cls < 4; ++cls) {
    const int kh0 = ((cls >> 1) + g.pad) & 1, kw0 = ((cls & 1) + g.pad) & 1;
    const int t = ((g.KH - kh0 + 1) >> 1) * ((g.KW - kw0 + 1) >> 1);
    best = t > best ? t : best;
  }
  return best * g.SC / ks;
}

int stage_bytes(int tile) {
  static const int bm[4] = {128, 128, 64, 64}, bn[4] = {128, 64, 128, 64};
  return (bm[tile] + bn[tile]) * 128;
}

template <typename T, int BM, int BN, int MODE, int S, int NW = 4>
int launch_fast(const Geom& g0, const void* src, const void* w, const float* bias, const void* res, void* out,
                float* stats, hipStream_t s) {
  Geom g = g0;
  g.gm = p6::ceil_div(g.M, BM);
  g.gn = p6::ceil_div(g.Ncols, BN);
  const int nk = fast_nk(MODE, g, LK<T>::KS);
  const int ring = (nk < S ? (nk > 0 ? nk : 1) : S) * (BM + BN) * 128;
  // kGemmDual stages both branches' tiles for its epilogue
  const int epi = (MODE == kGemmDual ? 2 : 1) * BM * (BN * (int)sizeof(T) + 16) + (g.bnr_part ? bnr_lds(NW, BN) : 0);
  const int lds = ring > epi ? ring : epi;
  if (MODE == kDgradS2) s2_single_class(g, res, out);
  constexpr bool SK = MODE == kGemm || MODE == kFwd || MODE == kDgrad;
  // the plan's split count (choose / splitk_need: <= nk, <= kSkMaxTiles tiles, the
  // workspace checked by run_conv)
  if (!SK || g.splits < 1 || !g.sk_cnt) g.splits = 1;
  const int grid = g.gm * g.gn * (MODE == kDgradS2 ? s2_classes(g) : 1) * (g.splits > 1 ? g.splits : 1);
  if constexpr (MODE == kGemm || MODE == kFwd || MODE == kGemmDual) {
    if (g.act) {   // eval BN-act epilogue (pose6d_conv2d_fwd_act)
      conv_lds_kernel<T, BM, BN, MODE, S, true, NW><<<grid, 64 * NW, lds, s>>>(
          (const T*)src, (const T*)w, bias, (const T*)res, (T*)out, stats, g);
      P6_LAUNCH_CHECK();
      return POSE6D_OK;
    }
  }
  if constexpr (MODE == kGemm || MODE == kDgrad || MODE == kDgradS2) {
    if (g.bnr_part) {   // data gradient + BatchNorm reduce
      conv_lds_kernel<T, BM, BN, MODE, S, false, NW, true><<<grid, 64 * NW, lds, s>>>(
          (const T*)src, (const T*)w, bias, (const T*)res, (T*)out, stats, g);
      P6_LAUNCH_CHECK();
      return POSE6D_OK;
    }
  }
  conv_lds_kernel<T, BM, BN, MODE, S, false, NW><<<grid, 64 * NW, lds, s>>>(
      (const T*)src, (const T*)w, bias, (const T*)res, (T*)out, stats, g);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

template <typename T, int BM, int BN, int MODE, int NW = 4>
int launch_fast_s(const Geom& g, int stages, const void* src, const void* w, const float* bias, const void* res,
                  void* out, float* stats, hipStream_t s) {
  switch (stages) {
    case 2: return launch_fast<T, BM, BN, MODE, 2, NW>(g, src, w, bias, res, out, stats, s);
    case 3: return launch_fast<T, BM, BN, MODE, 3, NW>(g, src, w, bias, res, out, stats, s);
    case 4: return launch_fast<T, BM, BN, MODE, 4, NW>(g, src, w, bias, res, out, stats, s);
    default:
      if constexpr ((BM + BN) * 128 * 6 <= 160 * 1024) return launch_fast<T, BM, BN, MODE, 6, NW>(g, src, w, bias,
                                                                                                  res, out, stats, s);
      else return launch_fast<T, BM, BN, MODE, 4, NW>(g, src, w, bias, res, out, stats, s);
  }
}

template <typename T, int MODE>
int launch_fast_mode(const Geom& g, int tile, int stages, const void* src, const void* w, const float* bias,
                     const void* res, void* out, float* stats, hipStream_t s) {
  switch (tile) {
    case 0: return launch_fast_s<T, 128, 128, MODE>(g, stages, src, w, bias, res, out, stats, s);
    case 1: return launch_fast_s<T, 128, 64, MODE>(g, stages, src, w, bias, res, out, stats, s);
    case 4: return launch_fast_s<T, 128, 128, MODE, 8>(g, stages, src, w, bias, res, out, stats, s);
    case 5: return launch_fast_s<T, 128, 64, MODE, 8>(g, stages, src, w, bias, res, out, stats, s);
    default: return launch_fast_s<T, 64, 64, MODE>(g, stages, src, w, bias, res, out, stats, s);
  }
}

template <typename T>
int dispatch_fast_t(int mode, const Geom& g, int tile, int stages, const void* src, const void* w, const float* bias,
                    const void* res, void* out, float* stats, hipStream_t s) {
  switch (mode) {
    case kGemm: return launch_fast_mode<T, kGemm>(g, tile, stages, src, w, bias, res, out, stats, s);
    case kFwd: return launch_fast_mode<T, kFwd>(g, tile, stages, src, w, bias, res, out, stats, s);
    case kFwdRowTap:   // (few instances: 64x64 or 128x64 tiles, 2 / 3 / 4 slots)
      if (tile == 1 || tile == 5) {
        if (stages >= 4) return launch_fast<T, 128, 64, kFwdRowTap, 4, 4>(g, src, w, bias, res, out, stats, s);
        if (stages == 3) return launch_fast<T, 128, 64, kFwdRowTap, 3, 4>(g, src, w, bias, res, out, stats, s);
        return launch_fast<T, 128, 64, kFwdRowTap, 2, 4>(g, src, w, bias, res, out, stats, s);
      }
      if (stages >= 4) return launch_fast<T, 64, 64, kFwdRowTap, 4, 4>(g, src, w, bias, res, out, stats, s);
      if (stages == 3) return launch_fast<T, 64, 64, kFwdRowTap, 3, 4>(g, src, w, bias, res, out, stats, s);
      return launch_fast<T, 64, 64, kFwdRowTap, 2, 4>(g, src, w, bias, res, out, stats, s);
    case kDgradS2: return launch_fast_mode<T, kDgradS2>(g, tile, stages, src, w, bias, res, out, stats, s);
    case kGemmDual: return launch_fast_s<T, 64, 64, kGemmDual>(g, stages, src, w, bias, res, out, stats, s);
    default: return launch_fast_mode<T, kDgrad>(g, tile, stages, src, w, bias, res, out, stats, s);
  }
}

int dispatch_fast(int dtype, int mode, const Geom& g, int tile, int stages, const void* src, const void* w,
                  const float* bias, const void* res, void* out, float* stats, hipStream_t s) {
  return dtype == POSE6D_DT_BF16 ? dispatch_fast_t<bf16>(mode, g, tile, stages, src, w, bias, res, out, stats, s)
                                 : dispatch_fast_t<float>(mode, g, tile, stages, src, w, bias, res, out, stats, s);
}

template <typename T, int BM, int BN, int MODE>
int launch_t(const Geom& g0, const void* src, const void* w, const float* bias, const void* res, void* out,
             float* stats, hipStream_t s) {
  Geom g = g0;
  g.gm = p6::ceil_div(g.M, BM);
  g.gn = p6::ceil_div(g.Ncols, BN);
  const int stage = 2 * (BM + BN) * 64;
  const int epi = BM * (BN * (int)sizeof(T) + 16);
  const int lds = stage > epi ? stage : epi;
  if constexpr (MODE != kDgrad) {
    if (g.act) {   // eval BN-act epilogue (pose6d_conv2d_fwd_act)
      conv_igemm_kernel<T, BM, BN, MODE, true><<<g.gm * g.gn, kThreads, lds, s>>>(
          (const T*)src, (const T*)w, bias, (const T*)res, (T*)out, stats, g);
      P6_LAUNCH_CHECK();
      return POSE6D_OK;
    }
  }
  conv_igemm_kernel<T, BM, BN, MODE, false><<<g.gm * g.gn, kThreads, lds, s>>>(
      (const T*)src, (const T*)w, bias, (const T*)res, (T*)out, stats, g);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

template <typename T, int MODE>
int launch_mode(const Geom& g, int tile, const void* src, const void* w, const float* bias, const void* res,
                void* out, float* stats, hipStream_t s) {
  switch (tile) {
    case 0: return launch_t<T, 128, 128, MODE>(g, src, w, bias, res, out, stats, s);
    case 1: return launch_t<T, 128, 64, MODE>(g, src, w, bias, res, out, stats, s);
    case 2: return launch_t<T, 64, 128, MODE>(g, src, w, bias, res, out, stats, s);
    default: return launch_t<T, 64, 64, MODE>(g, src, w, bias, res, out, stats, s);
  }
}

// tile choice: the biggest tile that still gives >= 2 waves of workgroups per CU-pass
int pick_tile(int M, int N) {
  auto blocks = [&](int bm, int bn) { return (int64_t)p6::ceil_div(M, bm) * p6::ceil_div(N, bn); };
  if (N <= 64) return blocks(128, 64) >= 512 ? 1 : 3;
  if (blocks(128, 128) >= 512) return 0;
  if (blocks(128, 64) >= 512) return 1;
  if (blocks(64, 128) >= 512) return 2;
  return 3;
}

int ilog2(int v) {
  int r = 0;
  while ((1 << r) < v) ++r;
  return (1 << r) == v ? r : -1;
}

template <typename T>
int dispatch(int mode, const Geom& g, int tile, const void* src, const void* w, const float* bias, const void* res,
             void* out, float* stats, hipStream_t s) {
  switch (mode) {
    case kGemm: return launch_mode<T, kGemm>(g, tile, src, w, bias, res, out, stats, s);
    case kFwd: return launch_mode<T, kFwd>(g, tile, src, w, bias, res, out, stats, s);
    case kFwdNarrow: return launch_mode<T, kFwdNarrow>(g, tile, src, w, bias, res, out, stats, s);
    default: return launch_mode<T, kDgrad>(g, tile, src, w, bias, res, out, stats, s);
  }
}



// statistics rows: one per 32 output pixels (the last may cover fewer)
extern "C" int pose6d_conv_stats_rows(int32_t N, int32_t Ho, int32_t Wo, int32_t Cout) {
  (void)Cout;
  return p6::ceil_div((int64_t)N * Ho * Wo, 32);
}

// implementation choice: the LDS-DMA fast path whenever each 128-byte K slice (64
// bf16 / 32 fp32 channels) lies inside one filter tap; the register-staged kernel
// otherwise (the Cin-4 stem, the 3- and 32-channel z-CNN layers).  A pose6d_tuning_t
// (the *_tuned entry points: tests and tools/conv_bench.py only) can force the
// register-staged kernel, a tile, a ring depth or the masked stride-2 gather; the
// product entry points never take one, so each conv has one plan (one summation order).
bool fast_ok(int dtype, int mode, const Geom& g) {
  if (mode == kFwdNarrow) return false;
  if (mode == kFwdRowTap) return true;   // its only path (fwd_geom checked the geometry)
  if (mode == kGemmDual) {
    const int ks2 = dtype == POSE6D_DT_BF16 ? 64 : 32;
    return g.K % ks2 == 0 && g.Kpad == g.K && g.Kpad2 % ks2 == 0;
  }
  const int ks = dtype == POSE6D_DT_BF16 ? 64 : 32;   // elements per 128-byte K-step
  if (g.K % ks != 0 || g.Kpad != g.K) return false;
  return mode == kGemm || g.SC % ks == 0;
}

// Tile per GEMM shape.  The 64x64 / 4-wave tile keeps the most workgroups resident
// and wins while K is short or the grid would get thin; a 128x128 tile on 8 waves
// (tile 4) halves the LDS-DMA bytes per MFMA (each 32 KiB stage feeds four times
// the MACs of a 16 KiB one), which wins inside the training step once K >= 256 and
// the grid keeps >= 384 workgroups (layer2.0 ds / conv1, layer3.0 ds / conv1,
// layer3 conv3: 1-3 us each).  128x64 on 8 waves (tile 5) won standalone sweeps
// (tools/conv_bench.py) but lost in the step, so bf16 never picks it.  fp32
// (MFMA-bound: 4x the MFMAs per byte) takes 128x128 on long K at about one
// workgroup per CU (profiles/r02_conv_tiles.txt).
#ifndef POSE6D_TILE4_MIN_K
#define POSE6D_TILE4_MIN_K 128   // build-time (A/B): the bf16 128x128 tile's minimum K (round 4:
                                 // 256 -> 128 moved layer2's 128 -> 512 convs onto it, step 4.608 -> 4.601 ms)
#endif
int pick_tile_fast(int dtype, int64_t M, int N, int K) {
  const int64_t wg4 = p6::ceil_div(M, 128) * (int64_t)p6::ceil_div(N, 128);
#ifndef POSE6D_F32_TILE_RULE
#define POSE6D_F32_TILE_RULE 0   // build-time (A/B): 1 = 128x128 from K >= 256 on >= 96 tiles, 2 = from K >= 128, N >= 128
#endif
  if (dtype == POSE6D_DT_F32 && POSE6D_F32_TILE_RULE == 1) return (K >= 256 && N >= 128 && wg4 >= 96) ? 4 : 3;
  if (dtype == POSE6D_DT_F32 && POSE6D_F32_TILE_RULE == 2) return (K >= 128 && N >= 128) ? 4 : 3;
  if (dtype == POSE6D_DT_F32) return (K >= 512 && N >= 128 && wg4 >= 192 && wg4 < 384) ? 4 : 3;
  return (N >= 128 && K >= POSE6D_TILE4_MIN_K && wg4 >= 384) ? 4 : 3;
}

// an override field of a pose6d_tuning_t, or the default (-1 / no struct)
int tune(const pose6d_tuning_t* t, int32_t pose6d_tuning_t::*f, int dflt) {
  return (t && t->*f >= 0) ? (int)(t->*f) : dflt;
}

struct Plan {
  bool fast;
  int mode, tile, stages;
  Geom g;
};

// stride-2 data gradient as four parity classes: needs every dX pixel's class to
// have the same extent (H, W even; Ho = H / 2, Wo = W / 2)
bool s2_ok(const Geom& g) {
  return g.stride == 2 && (g.RH & 1) == 0 && (g.RW & 1) == 0 && g.SH == g.RH / 2 && g.SW == g.RW / 2;
}

// Default split-K count of a FORWARD conv (data gradients keep one split, so the fused
// backward launch and the separate data-gradient launch stay bit-identical): a function
// of the geometry only (never of a tuned tile or
// ring depth, so every tile / ring variant of a plan keeps one summation order).
// Split-K pays where a long K loop runs on a grid of at most one 64x64 workgroup per
// CU: layer4's 3x3 convs (72 K-steps, 200 tiles at batch 32: 23.2 -> 18.6 us forward,
// 23.5 -> 18.6 us data gradient, graph-replayed) and its 2048->512 1x1 (32 K-steps:
// 12.7 -> 11.9 us); fp32 the same shapes (32-channel K-steps): 90.1 -> 84.8, 43.7 -> 40.9
// and 95.2 -> 83.7 us (profiles/r04_f32_conv_sweep.txt).  Everywhere else the merge (write-through partial stores, the
// arrival atomic, the partial reads: ~3-5 us on the last arriver's critical path)
// costs more than the shorter K loop saves (profiles/r04_splitk_sweep.txt).
#ifndef POSE6D_SPLITK_SMALL_TILES
#define POSE6D_SPLITK_SMALL_TILES 64   // build-time (A/B): 0 = the batch-32 rule only
#endif
int default_splits(int dtype, int mode, const Geom& g, bool fused) {
  if (fused || !(mode == kGemm || mode == kFwd || mode == kDgrad)) return 1;
  (void)dtype;
  const int ks = dtype == POSE6D_DT_BF16 ? 64 : 32;
  const int nk = fast_nk(mode, g, ks);
  const int64_t tiles64 = (int64_t)p6::ceil_div(g.M, 64) * p6::ceil_div(g.Ncols, 64);
  // small grids (batch 1-2: at most a quarter of the CUs busy) with >= 16 K-steps: four
  // shorter K walks per tile (B = 1 eval forwards 7.7 -> 7.1 us on 14x14 1024->256, 14.4 ->
  // 10.6 us on layer4's 3x3; profiles/r06_b1_splitk.txt); no batch-32 conv has <= 64 tiles
  if (nk >= 16 && tiles64 <= POSE6D_SPLITK_SMALL_TILES) return 4;
  if (nk >= 32 && tiles64 <= 256) return 2;
  return 1;
}

// fused = the data-gradient half of conv_bwd_kernel (its workgroups are 64x64 / 4 waves)
Plan choose(int dtype, int mode, const Geom& g, bool fused = false, const pose6d_tuning_t* tn = nullptr,
            bool fwd = false) {
  Plan p{};
  p.fast = fast_ok(dtype, mode, g) && tune(tn, &pose6d_tuning_t::conv_base, 0) == 0;
  p.mode = mode;
  p.g = g;
  if (!p.fast) {
    p.tile = tune(tn, &pose6d_tuning_t::conv_tile, pick_tile(g.M, g.Ncols));
    if (p.tile > 3) p.tile = 3;
    return p;
  }
  if (mode == kDgrad && s2_ok(g) && tune(tn, &pose6d_tuning_t::conv_s2, 1)) {
    p.mode = kDgradS2;
    p.g.M = g.M / 4;
    p.g.RH = g.RH / 2;
    p.g.RW = g.RW / 2;
  }
  // build-time forward-plan overrides (A/B variant builds only: tools/build_variant.sh);
  // they apply to bf16 forward convs with M <= POSE6D_FWD_OVR_MAXM
#ifndef POSE6D_FWD_OVR_MAXM
#define POSE6D_FWD_OVR_MAXM 0
#endif
#ifndef POSE6D_FWD_TILE
#define POSE6D_FWD_TILE -1
#endif
#ifndef POSE6D_FWD_STAGES
#define POSE6D_FWD_STAGES 0
#endif
  const bool ovr = fwd && dtype == POSE6D_DT_BF16 && p.g.M <= POSE6D_FWD_OVR_MAXM;
  int dflt_tile = pick_tile_fast(dtype, p.g.M, g.Ncols, g.K);
  // long-K 1x1 forwards on the small grids (layer3 / layer4 at batch 32, M <= 6272): 8-wave
  // tiles on a 4-slot ring -- 128x128 where that still gives >= 96 workgroups, else
  // 128x64.  In-graph eval times (profiles/r05b_eval_variants.txt): 1024->256 16.0 ->
  // 11.0 us, 1024->512 18.9 -> 15.9, 1024->2048/s2 17.5 -> 15.2, 2048->512 12.9 -> 12.3
#ifndef POSE6D_LONG1X1
#define POSE6D_LONG1X1 1   // build-time (A/B): 0 = the round-4 tile / ring rules for these convs
#endif
  const bool long1x1 = POSE6D_LONG1X1 && fwd && dtype == POSE6D_DT_BF16 && g.KH == 1 && g.KW == 1 && g.K >= 1024 &&
                       p.g.M <= 6272;
  if (long1x1) {
    const int64_t wg4 = (int64_t)p6::ceil_div(p.g.M, 128) * p6::ceil_div(g.Ncols, 128);
    dflt_tile = (g.Ncols >= 512 && wg4 >= 96) ? 4 : 5;
  }
  if (ovr && POSE6D_FWD_TILE >= 0) dflt_tile = POSE6D_FWD_TILE;
  // fp32 KxK stride-2 data gradients (four parity classes of 1-4 taps): 64x64 tiles on a
  // 4-slot ring -- graph-timed 56x56 128->128 114.6 -> 94.1, 28x28 256->256 97.1 -> 92.0,
  // 14x14 512->512 165.0 -> 111.7 us (profiles/r05s2st_f32_s2_dgrad_plan.txt)
#ifndef POSE6D_F32_S2_PLAN
#define POSE6D_F32_S2_PLAN 1   // build-time (A/B): 0 = the generic tile / ring rules
#endif
  const bool f32s2 = POSE6D_F32_S2_PLAN && dtype == POSE6D_DT_F32 && p.mode == kDgradS2 && !fused &&
                     (g.KH > 1 || g.KW > 1);
  if (f32s2) dflt_tile = 3;
  p.tile = (fused || mode == kGemmDual) ? 3 : tune(tn, &pose6d_tuning_t::conv_tile, dflt_tile);
  if (p.tile == 2 || p.tile < 0 || p.tile > 5) p.tile = 3;   // no 64x128 instance on the fast path
  // two slots (32 KiB at 64x64) keep several workgroups per CU resident, which hides
  // the DMA latency better than a deeper ring; only long-K grids that leave CUs
  // idle (one wave of workgroups) take a 4-deep ring
  // tiles: 0 = 128x128, 1 = 128x64, 3 = 64x64 (4 waves); 4 = 128x128, 5 = 128x64 (8 waves)
  const bool rows128 = p.tile <= 1 || p.tile == 4 || p.tile == 5;
  const bool cols128 = p.tile == 0 || p.tile == 4;
  const int64_t grid = (int64_t)p6::ceil_div(p.g.M, rows128 ? 128 : 64) * p6::ceil_div(g.Ncols, cols128 ? 128 : 64) *
                       (p.mode == kDgradS2 ? 4 : 1);
  int dflt = (fast_nk(p.mode, p.g, dtype == POSE6D_DT_BF16 ? 64 : 32) > 24 && grid <= 512) ? 4 : 2;
  // fp32 forward (MFMA-bound: 4 exact 16x16x4 MFMAs per 16-byte chunk): 3 slots for
  // 1x1 filters, 2 for the rest (tools/conv_bench.py --graph --dtype f32 sweep, round 2)
  if (dtype == POSE6D_DT_F32 && (p.mode == kGemm || p.mode == kFwd)) dflt = (g.KH == 1 && g.KW == 1) ? 3 : 2;
  if (long1x1 || f32s2) dflt = 4;
  if (ovr && POSE6D_FWD_STAGES > 0) dflt = POSE6D_FWD_STAGES;
  p.stages = tune(tn, &pose6d_tuning_t::conv_stages, dflt);
  if (p.stages < 2) p.stages = 2;
  if (p.stages > 6) p.stages = 6;
  if (p.stages == 5) p.stages = 4;
  if (cols128 && rows128 && p.stages > 4) p.stages = 4;   // 6 x 32 KiB exceeds the 160 KiB LDS
  if (fused && p.stages == 3) p.stages = 4;   // the fused backward instantiates 2- and 4-slot data gradients
  // forwards split by default; data gradients only under an explicit tuning (tests, tools):
  // the backward entry points take no split-K workspace, and the fused and separate data
  // gradients stay one plan (one summation order)
  p.g.splits = tune(tn, &pose6d_tuning_t::conv_splitk, fwd ? default_splits(dtype, p.mode, p.g, fused) : 1);
  if (fused || !(p.mode == kGemm || p.mode == kFwd || p.mode == kDgrad) || p.g.splits < 1) p.g.splits = 1;
  {
    const int64_t tiles = (int64_t)p6::ceil_div(p.g.M, rows128 ? 128 : 64) * p6::ceil_div(g.Ncols, cols128 ? 128 : 64);
    const int nk = fast_nk(p.mode, p.g, dtype == POSE6D_DT_BF16 ? 64 : 32);
    if (tiles > kSkMaxTiles) p.g.splits = 1;
    if (p.g.splits > nk) p.g.splits = nk > 0 ? nk : 1;
  }
  // split-K plans keep their long-K ring depth (the sweep's fastest: 4 slots) unless tuned
  if (p.g.splits > 1 && tune(tn, &pose6d_tuning_t::conv_stages, -1) < 0 && p.stages < 4 && !(cols128 && rows128))
    p.stages = 4;
  return p;
}

#ifndef POSE6D_PATCH
#define POSE6D_PATCH 1   // build-time (A/B): 0 = 3x3 forwards always on the implicit GEMM
#endif
// 2 ring slots: deeper rings measured slower (graph-timed, profiles/r05d_patch_sweep.txt:
// 56x56 64->64 17.8 / 23.5 / 25.1 us at 2 / 3 / 6 slots)
constexpr int kPatchStages = 2;
// the patch plan applies to bf16 3x3 / stride 1 / pad 1 forwards with 64-channel
// slices and no BatchNorm statistics, unless a tuning forces an implicit-GEMM plan
// (tile / ring / kernel / split-K) or turns it off (conv_patch = 0)
bool patch_eligible(int dtype, int mode, const Geom& g, const float* stats, const pose6d_tuning_t* tn,
                    PatchPlan* pp) {
  if (!POSE6D_PATCH || dtype != POSE6D_DT_BF16 || mode != kFwd || stats != nullptr) return false;
  if (g.KH != 3 || g.KW != 3 || g.stride != 1 || g.pad != 1 || g.SH != g.RH || g.SW != g.RW) return false;
  if (g.SC % 64 != 0 || g.Ncols % kPatchBN != 0 || g.Kpad != g.K || g.act_rscale != nullptr) return false;
  if (tn) {
    if (tn->conv_patch == 0) return false;
    if (tn->conv_patch < 0 && (tn->conv_tile >= 0 || tn->conv_stages >= 0 || tn->conv_base >= 0 ||
                               tn->conv_splitk >= 0))
      return false;
    if (tn->conv_patch == 1 && (tn->conv_tile >= 0 || tn->conv_base >= 0 || tn->conv_splitk >= 0))
      return false;
  }
  // the 56x56 stage only: in the eval graph the layer1 3x3 convs gain 1.7-2.5 us each,
  // the 28x28 ones lose 0.5-0.7 us (profiles/r05e_eval_layers.txt), and on 14x14 / 7x7
  // (few tiles per image, long K) the implicit GEMM is faster (profiles/r05d_patch_sweep.txt:
  // 17.7 vs 18.3 us, 19.1 vs 48.2 us)
  if (g.RH * g.RW < 3136 && !(tn && tn->conv_patch == 1)) return false;
  *pp = patch_plan(g.M / (g.RH * g.RW), g.RH, g.RW, g.SC, g.Ncols, kPatchStages);
  return pp->ok;
}

// bytes of split-K workspace a plan needs (0: it does not split K)
int64_t splitk_need(const Plan& p) {
  if (!p.fast || p.g.splits <= 1) return 0;
  const bool rows128 = p.tile <= 1 || p.tile == 4 || p.tile == 5;
  const bool cols128 = p.tile == 0 || p.tile == 4;
  const int bm = rows128 ? 128 : 64, bn = cols128 ? 128 : 64;
  const int64_t tiles = (int64_t)p6::ceil_div(p.g.M, bm) * p6::ceil_div(p.g.Ncols, bn);
  return kSkCntBytes + tiles * p.g.splits * bm * bn * 4;
}

int run_conv(int dtype, int mode, const Geom& g, const void* src, const void* w, const float* bias, const void* res,
             void* out, float* stats, hipStream_t s, const pose6d_tuning_t* tn = nullptr, bool fwd = false,
             void* sk_ws = nullptr, int64_t sk_bytes = 0) {
  // 3x3 stride-1 bf16 forwards without BatchNorm statistics (eval; conv_patch.h: the
  // input patch staged once per 64-channel slice instead of once per filter tap) are
  // decided first -- the patch kernel never splits K, so it needs no split-K workspace
  // even where the implicit-GEMM plan of the same geometry would
  {
    PatchPlan pp{};
    if (patch_eligible(dtype, mode, g, stats, tn, &pp)) {
      const int st = tn && tn->conv_patch == 1 && tn->conv_stages > 0 ? tn->conv_stages : kPatchStages;
      if (st != kPatchStages) pp = patch_plan(g.M / (g.RH * g.RW), g.RH, g.RW, g.SC, g.Ncols, st);
      P6_CHECK_ARG(pp.ok, "conv: patch plan with %d ring slots exceeds the LDS", st);
      const int N = g.M / (g.RH * g.RW);
      switch (st) {
        case 3: return launch_patch<3>(g, pp, N, src, w, bias, res, out, s);
        case 4: return launch_patch<4>(g, pp, N, src, w, bias, res, out, s);
        case 6: return launch_patch<6>(g, pp, N, src, w, bias, res, out, s);
        case 8: return launch_patch<8>(g, pp, N, src, w, bias, res, out, s);
        default: return launch_patch<kPatchStages>(g, pp, N, src, w, bias, res, out, s);
      }
    }
  }
  Plan p = choose(dtype, mode, g, false, tn, fwd);
  const int64_t need = splitk_need(p);
  if (need > 0) {
    P6_CHECK_ARG(sk_ws != nullptr && sk_bytes >= need,
                 "conv: this plan splits K over %d workgroups per tile (pose6d_conv_variant >> 16) and needs a split-K "
                 "workspace of %lld bytes (pose6d_conv_splitk_workspace), got %lld",
                 p.g.splits, (long long)need, (long long)(sk_ws ? sk_bytes : 0));
    P6_CHECK_ARG(((uintptr_t)sk_ws & 255) == 0, "conv: the split-K workspace must be 256-byte aligned");
    p.g.sk_cnt = (int*)sk_ws;
    p.g.sk_part = (float*)((char*)sk_ws + kSkCntBytes);
  }
  if (p.fast) return dispatch_fast(dtype, p.mode, p.g, p.tile, p.stages, src, w, bias, res, out, stats, s);
  return dtype == POSE6D_DT_BF16 ? dispatch<bf16>(mode, g, p.tile, src, w, bias, res, out, stats, s)
                                 : dispatch<float>(mode, g, p.tile, src, w, bias, res, out, stats, s);
}

// Packed filter layout of a forward conv (the wp operand): taps per kernel row (KW, or
// kRowTaps for the row-tap stems) and the padded K, a multiple of the K-step of every
// kernel that reads it.  pose6d_conv_pack_geom exports it.
int pack_geom(int dtype, int Cin, int KH, int KW, int stride, int pad, int* kwp) {
  const bool rowtap = p6::rowtap_geom(Cin, KH, KW, stride, pad);
  *kwp = rowtap ? kRowTaps : KW;
  const int ks = dtype == POSE6D_DT_BF16 ? 64 : 32;   // LDS-DMA K-step
  const int bk = rowtap ? ks : (dtype == POSE6D_DT_BF16 ? 32 : 16);
  return p6::ceil_div(KH * *kwp * Cin, bk) * bk;
}

Geom fwd_geom(int dtype, int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad, int Ho, int Wo,
              int* mode) {
  Geom g{};
  int kwp = 0;
  g.M = N * Ho * Wo; g.Ncols = Cout;
  g.Kpad = pack_geom(dtype, Cin, KH, KW, stride, pad, &kwp);
  g.K = kwp == kRowTaps ? g.Kpad : KH * KW * Cin;
  g.SH = H; g.SW = W; g.SC = Cin; g.log2SC = ilog2(Cin); g.RH = Ho; g.RW = Wo;
  g.KH = KH; g.KW = KW; g.stride = stride; g.pad = pad;
  if (KH == 1 && KW == 1 && stride == 1 && pad == 0) *mode = kGemm;
  else if (kwp == kRowTaps) *mode = kFwdRowTap;
  else if (Cin == 4) *mode = kFwdNarrow;
  else *mode = kFwd;
  return g;
}

Geom dgrad_geom(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad, int Ho, int Wo,
                int* mode) {
  Geom g{};
  g.M = N * H * W; g.Ncols = Cin; g.K = KH * KW * Cout; g.Kpad = g.K;
  g.SH = Ho; g.SW = Wo; g.SC = Cout; g.log2SC = ilog2(Cout); g.RH = H; g.RW = W;
  g.KH = KH; g.KW = KW; g.stride = stride; g.pad = pad;
  *mode = (KH == 1 && KW == 1 && stride == 1 && pad == 0) ? kGemm : kDgrad;
  return g;
}

}  // namespace

extern "C" int pose6d_conv2d_fwd(int32_t dtype, const void* x, const void* w, const float* bias, void* y,
                                 float* stats, int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH,
                                 int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo, void* splitk_ws,
                                 int64_t splitk_ws_bytes, void* stream) {
  return pose6d_conv2d_fwd_tuned(dtype, x, w, bias, y, stats, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo,
                                 nullptr, splitk_ws, splitk_ws_bytes, stream);
}

extern "C" int pose6d_conv2d_fwd_tuned(int32_t dtype, const void* x, const void* w, const float* bias, void* y,
                                       float* stats, int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout,
                                       int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo,
                                       const pose6d_tuning_t* tuning, void* splitk_ws, int64_t splitk_ws_bytes,
                                       void* stream) {
  P6_CHECK_ARG(dtype == POSE6D_DT_F32 || dtype == POSE6D_DT_BF16, "pose6d_conv2d_fwd: bad dtype %d", dtype);
  P6_CHECK_ARG(N > 0 && H > 0 && W > 0 && Cout > 0 && Cout % 8 == 0, "pose6d_conv2d_fwd: bad shape (Cout %% 8)");
  P6_CHECK_ARG(Ho == (H + 2 * pad - KH) / stride + 1 && Wo == (W + 2 * pad - KW) / stride + 1,
               "pose6d_conv2d_fwd: Ho/Wo inconsistent");
  const int bk = dtype == POSE6D_DT_BF16 ? 32 : 16;
  int mode;
  const Geom g = fwd_geom(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &mode);
  if (mode == kFwd)
    P6_CHECK_ARG(g.log2SC >= 0 && Cin % bk == 0, "pose6d_conv2d_fwd: Cin must be 4 or a power of two >= %d (got %d)",
                 bk, Cin);
  if (mode == kGemm) P6_CHECK_ARG(Cin % bk == 0, "pose6d_conv2d_fwd: 1x1 Cin %% %d != 0", bk);
  if (mode == kFwdRowTap)
    P6_CHECK_ARG(dtype == POSE6D_DT_F32 || W % 2 == 0, "pose6d_conv2d_fwd: the bf16 row-tap stem needs an even W");
  return run_conv(dtype, mode, g, x, w, bias, nullptr, y, stats, p6::stream_of(stream), tuning, true, splitk_ws,
                  splitk_ws_bytes);
}

extern "C" int pose6d_conv_pack_geom(int32_t dtype, int32_t Cin, int32_t KH, int32_t KW, int32_t stride, int32_t pad,
                                     int32_t* kw_packed, int32_t* Kpad) {
  P6_CHECK_ARG(kw_packed && Kpad && Cin > 0 && KH > 0 && KW > 0, "pose6d_conv_pack_geom: bad arguments");
  *Kpad = pack_geom(dtype, Cin, KH, KW, stride, pad, kw_packed);
  return POSE6D_OK;
}

// eval-mode conv + BatchNorm apply (+ residual, + ReLU) in one launch: the store of
// pose6d_conv2d_fwd followed by pose6d_bn_act_fwd, bit for bit, without the raw output
extern "C" int pose6d_conv2d_fwd_act(int32_t dtype, const void* x, const void* w, const float* bias, void* out,
                                     int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH, int32_t KW,
                                     int32_t stride, int32_t pad, int32_t Ho, int32_t Wo, const float* scale,
                                     const float* shift, const void* res, const float* res_scale,
                                     const float* res_shift, int32_t relu, void* splitk_ws, int64_t splitk_ws_bytes,
                                     void* stream) {
  P6_CHECK_ARG(dtype == POSE6D_DT_F32 || dtype == POSE6D_DT_BF16, "pose6d_conv2d_fwd_act: bad dtype %d", dtype);
  P6_CHECK_ARG(N > 0 && H > 0 && W > 0 && Cout > 0 && Cout % 8 == 0, "pose6d_conv2d_fwd_act: bad shape (Cout %% 8)");
  P6_CHECK_ARG(Ho == (H + 2 * pad - KH) / stride + 1 && Wo == (W + 2 * pad - KW) / stride + 1,
               "pose6d_conv2d_fwd_act: Ho/Wo inconsistent");
  P6_CHECK_ARG(scale && shift, "pose6d_conv2d_fwd_act: null scale / shift");
  P6_CHECK_ARG(!res_scale == !res_shift && (!res_scale || res), "pose6d_conv2d_fwd_act: bad residual BN args");
  const int bk = dtype == POSE6D_DT_BF16 ? 32 : 16;
  int mode;
  Geom g = fwd_geom(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &mode);
  if (mode == kFwd)
    P6_CHECK_ARG(g.log2SC >= 0 && Cin % bk == 0,
                 "pose6d_conv2d_fwd_act: Cin must be 4 or a power of two >= %d (got %d)", bk, Cin);
  if (mode == kGemm) P6_CHECK_ARG(Cin % bk == 0, "pose6d_conv2d_fwd_act: 1x1 Cin %% %d != 0", bk);
  P6_CHECK_ARG(mode != kFwdRowTap && mode != kFwdNarrow,
               "pose6d_conv2d_fwd_act: 4-channel convs have no BN-act epilogue (pose6d_conv2d_fwd, then the BN)");
  g.act = 1;
  g.act_relu = relu != 0;
  g.act_scale = scale;
  g.act_shift = shift;
  g.act_rscale = res_scale;
  g.act_rshift = res_shift;
  return run_conv(dtype, mode, g, x, w, bias, res, out, nullptr, p6::stream_of(stream), nullptr, true, splitk_ws,
                  splitk_ws_bytes);
}

extern "C" int pose6d_conv2d_fwd_act_dual(int32_t dtype, const void* x, const void* w, const void* xd, const void* wd,
                                          void* out, int32_t N, int32_t Ho, int32_t Wo, int32_t Cin, int32_t Cout,
                                          int32_t Hd, int32_t Wd, int32_t Cind, int32_t stride_d, const float* scale,
                                          const float* shift, const float* scale_d, const float* shift_d,
                                          int32_t relu, void* stream) {
  P6_CHECK_ARG(dtype == POSE6D_DT_F32 || dtype == POSE6D_DT_BF16, "pose6d_conv2d_fwd_act_dual: bad dtype %d", dtype);
  P6_CHECK_ARG(N > 0 && Ho > 0 && Wo > 0 && Cout > 0 && Cout % 8 == 0, "pose6d_conv2d_fwd_act_dual: bad shape");
  P6_CHECK_ARG(stride_d >= 1 && Ho == (Hd - 1) / stride_d + 1 && Wo == (Wd - 1) / stride_d + 1,
               "pose6d_conv2d_fwd_act_dual: downsample geometry inconsistent");
  P6_CHECK_ARG(scale && shift && scale_d && shift_d, "pose6d_conv2d_fwd_act_dual: null BatchNorm scale / shift");
  const int ks = dtype == POSE6D_DT_BF16 ? 64 : 32;
  P6_CHECK_ARG(Cin % ks == 0 && Cind % ks == 0, "pose6d_conv2d_fwd_act_dual: Cin and Cind must be multiples of %d",
               ks);
  int mode;
  Geom g = fwd_geom(dtype, N, Ho, Wo, Cin, Cout, 1, 1, 1, 0, Ho, Wo, &mode);
  g.src2 = xd;
  g.wts2 = wd;
  g.Kpad2 = Cind;
  g.SH2 = Hd;
  g.SW2 = Wd;
  g.stride2 = stride_d;
  g.act = 1;
  g.act_relu = relu != 0;
  g.act_scale = scale;
  g.act_shift = shift;
  g.act_rscale = scale_d;
  g.act_rshift = shift_d;
  const Plan p = choose(dtype, kGemmDual, g);
  P6_CHECK_ARG(p.fast, "pose6d_conv2d_fwd_act_dual: shape outside the LDS-DMA path");
  // bit identity with the separate launches needs their K loops unsplit (the dual
  // kernel has no split-K); pose6d_conv_variant reports the separate plans' splits
  {
    int m3, md;
    const Geom g3 = fwd_geom(dtype, N, Ho, Wo, Cin, Cout, 1, 1, 1, 0, Ho, Wo, &m3);
    const Geom gd = fwd_geom(dtype, N, Hd, Wd, Cind, Cout, 1, 1, stride_d, 0, Ho, Wo, &md);
    P6_CHECK_ARG(choose(dtype, m3, g3, false, nullptr, true).g.splits == 1 &&
                     choose(dtype, md, gd, false, nullptr, true).g.splits == 1,
                 "pose6d_conv2d_fwd_act_dual: the separate launches of this pair split K (pose6d_conv_variant >> 16); "
                 "run them separately");
  }
  return dispatch_fast(dtype, kGemmDual, p.g, p.tile, p.stages, x, w, nullptr, nullptr, out, nullptr,
                       p6::stream_of(stream));
}

namespace {
// BatchNorm-reduce partial rows of a data-gradient plan: one per output tile (x the four
// parity classes of kDgradS2)
// (0: a register-staged plan, which has no BN-reduce epilogue)
int bnr_plan_rows(const Plan& p) {
  if (!p.fast) return 0;
  const int bm = (p.tile <= 1 || p.tile == 4 || p.tile == 5) ? 128 : 64;
  return p6::ceil_div(p.g.M, bm) * (p.mode == kDgradS2 ? 4 : 1);
}

void set_bnr(Geom& g, const pose6d_bn_reduce_t* b) {
  if (!b) return;
  g.bnr_y = b->y; g.bnr_mean = b->mean; g.bnr_inv = b->invstd;
  g.bnr_rs = b->relu_scale; g.bnr_rb = b->relu_shift; g.bnr_mask = b->relu_mask;
  g.bnr_part = b->partial; g.bnr_rows = b->rows;
  g.bnr_y2 = b->y2; g.bnr_mean2 = b->mean2; g.bnr_inv2 = b->invstd2; g.bnr_part2 = b->partial2;
}

int check_bnr(const pose6d_bn_reduce_t* b, const Plan& p, const void* dres, const void* dx) {
  if (!b) return POSE6D_OK;
  P6_CHECK_ARG(b->y && b->mean && b->invstd && b->partial, "pose6d_bn_reduce_t: null y / mean / invstd / partial");
  P6_CHECK_ARG(b->relu_mask || (b->relu_scale && b->relu_shift),
               "pose6d_bn_reduce_t: needs relu_mask or relu_scale + relu_shift");
  P6_CHECK_ARG(!b->y2 || (b->relu_mask && b->mean2 && b->invstd2 && b->partial2),
               "pose6d_bn_reduce_t: a second BatchNorm needs relu_mask, mean2, invstd2, partial2");
  P6_CHECK_ARG(dres != dx, "pose6d_bn_reduce_t: the data gradient must be written whole (no in-place residual)");
  P6_CHECK_ARG(p.fast, "pose6d_bn_reduce_t: this data gradient runs the register-staged kernel (no BN reduce)");
  P6_CHECK_ARG(b->rows == bnr_plan_rows(p), "pose6d_bn_reduce_t: rows %d != %d (pose6d_conv2d_backward_bn_rows)",
               b->rows, bnr_plan_rows(p));
  return POSE6D_OK;
}

int dgrad_impl(int32_t dtype, const void* dy, const void* wt, const void* dres, const uint8_t* dres_mask, void* dx,
               int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
               int32_t pad, int32_t Ho, int32_t Wo, void* stream, const pose6d_tuning_t* tn = nullptr,
               const pose6d_bn_reduce_t* bnr = nullptr, void* sk_ws = nullptr, int64_t sk_bytes = 0) {
  P6_CHECK_ARG(dtype == POSE6D_DT_F32 || dtype == POSE6D_DT_BF16, "pose6d_conv2d_dgrad: bad dtype %d", dtype);
  P6_CHECK_ARG(stride == 1 || stride == 2, "pose6d_conv2d_dgrad: stride must be 1 or 2");
  P6_CHECK_ARG(Cin % 8 == 0, "pose6d_conv2d_dgrad: Cin %% 8 != 0 (no data gradient for the stem)");
  P6_CHECK_ARG(!dres_mask || (dres && dres != dx), "pose6d_conv2d_dgrad: a residual mask needs a separate dres");
  const int bk = dtype == POSE6D_DT_BF16 ? 32 : 16;
  int mode;
  Geom g = dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &mode);
  g.res_mask = dres_mask;
  P6_CHECK_ARG(g.log2SC >= 0 && Cout % bk == 0, "pose6d_conv2d_dgrad: Cout must be a power of two >= %d", bk);
  if (bnr) {
    const int rc = check_bnr(bnr, choose(dtype, mode, g, false, tn), dres, dx);
    if (rc) return rc;
    set_bnr(g, bnr);
  }
  return run_conv(dtype, mode, g, dy, wt, nullptr, dres, dx, nullptr, p6::stream_of(stream), tn, false, sk_ws,
                  sk_bytes);
}
}  // namespace

extern "C" int pose6d_conv2d_dgrad(int32_t dtype, const void* dy, const void* wt, const void* dres, void* dx,
                                   int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH, int32_t KW,
                                   int32_t stride, int32_t pad, int32_t Ho, int32_t Wo, void* stream) {
  return dgrad_impl(dtype, dy, wt, dres, nullptr, dx, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, stream);
}

extern "C" int pose6d_conv2d_dgrad_tuned(int32_t dtype, const void* dy, const void* wt, const void* dres, void* dx,
                                         int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout, int32_t KH,
                                         int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo,
                                         const pose6d_tuning_t* tuning, void* splitk_ws, int64_t splitk_ws_bytes,
                                         void* stream) {
  return dgrad_impl(dtype, dy, wt, dres, nullptr, dx, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, stream,
                    tuning, nullptr, splitk_ws, splitk_ws_bytes);
}

namespace {

template <int DMODE, int DS, int WS, typename T = bf16, int WBT = 64>
int launch_bwd(const Geom& gd0, const p6::WGeom& gw, const void* dy, const void* wt, const void* dres, void* dx,
               const void* x, float* ws, const ReduceJob& rj, hipStream_t s, int order) {
  Geom gd = gd0;
  gd.gm = p6::ceil_div(gd.M, 64);
  gd.gn = p6::ceil_div(gd.Ncols, 64);
  if (DMODE == kDgradS2) s2_single_class(gd, dres, dx);
  const int nd = gd.gm * gd.gn * (DMODE == kDgradS2 ? s2_classes(gd) : 1);
  const int nd_pad = (nd + 7) & ~7;
  const int nw = gw.gm * gw.gn * gw.splits;
  const int nk = fast_nk(DMODE, gd, LK<T>::KS);
  const int ring_d = (nk < DS ? (nk > 0 ? nk : 1) : DS) * 128 * 128;
  const int epi = 64 * (64 * (int)sizeof(T) + 16) + (gd.bnr_part ? bnr_lds(4, 64) : 0);
  const int ring_w = sizeof(T) == 2 ? WS * 128 * 128
                                    : (WBT == 128 ? WS * WgF32<32, 128>::STAGE : WS * WgF32<kBwdF32MS>::STAGE);
  int lds = ring_d > epi ? ring_d : epi;
  lds = lds > ring_w ? lds : ring_w;
  if (sizeof(T) == 4 && WBT == 128 && lds < acc_stage_bytes<128, 128>()) lds = acc_stage_bytes<128, 128>();
  // longest workgroups first: the weight gradient's K-steps per split against the
  // data gradient's K-steps per tile.  fp32: a 64-pixel weight-gradient stage is twice
  // the MACs of a 32-channel data-gradient K-step (28x28 128->512 fp32: 79.5 -> 72.5 us
  // with the weight gradient first, profiles/r04_bwd_plan_sweep.txt)
#ifndef POSE6D_BWD_WSTEP_F32
#define POSE6D_BWD_WSTEP_F32 2   // build-time (A/B): 1 = compare stages and K-steps 1:1 for fp32 too
#endif
  constexpr int WSTEP = sizeof(T) == 4 ? POSE6D_BWD_WSTEP_F32 : 1;
#ifndef POSE6D_BWD_ORDER
#define POSE6D_BWD_ORDER 1   // build-time (A/B): 0 = the data gradient always first, 2 = the weight gradient
#endif
  const int wfirst = order >= 0 ? order
                                : (POSE6D_BWD_ORDER == 2 || (POSE6D_BWD_ORDER && WSTEP * p6::ceil_div(gw.mps, 64) >= nk));
  const int grid = wfirst ? ((nw + 7) & ~7) + nd + rj.nblk : nd_pad + nw + rj.nblk;
  conv_bwd_kernel<DMODE, DS, WS, T, WBT><<<grid, kThreads, lds, s>>>(
      (const T*)dy, (const T*)wt, (const T*)dres, (T*)dx, gd, nd, nd_pad, wfirst, (const T*)x, ws, gw, rj);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

// the 8-wave fused launch (conv_bwd8_kernel): 128x64 data-gradient tiles, the 128x128
// weight-gradient body on a WS-slot ring; LDS = the larger of the two roles' rings and
// epilogue staging (the 128x128 fp32 tile staged for 16-byte slab stores: 72 KiB)
template <int DMODE, int DS, int WS>
int launch_bwd8(const Geom& gd0, const p6::WGeom& gw, const void* dy, const void* wt, const void* dres, void* dx,
                const void* x, float* ws, const ReduceJob& rj, hipStream_t s, int order) {
  Geom gd = gd0;
  gd.gm = p6::ceil_div(gd.M, 128);
  gd.gn = p6::ceil_div(gd.Ncols, 64);
  if (DMODE == kDgradS2) s2_single_class(gd, dres, dx);
  const int nd = gd.gm * gd.gn * (DMODE == kDgradS2 ? s2_classes(gd) : 1);
  const int nd_pad = (nd + 7) & ~7;
  const int nw = gw.gm * gw.gn * gw.splits;
  const int nk = fast_nk(DMODE, gd, 64);
  const int ring_d = (nk < DS ? (nk > 0 ? nk : 1) : DS) * (128 + 64) * 128;
  const int epi = 128 * (64 * 2 + 16) + (gd.bnr_part ? bnr_lds(8, 64) : 0);
  const int ring_w = WS * (128 + 128) * 128;
  int lds = ring_d > epi ? ring_d : epi;
  lds = lds > ring_w ? lds : ring_w;
  lds = lds > acc_stage_bytes<128, 128>() ? lds : acc_stage_bytes<128, 128>();
#ifndef POSE6D_BWD8_ORDER
#define POSE6D_BWD8_ORDER POSE6D_BWD_ORDER   // build-time (A/B): the 8-wave launch's order rule (as POSE6D_BWD_ORDER)
#endif
  const int wfirst = order >= 0 ? order : (POSE6D_BWD8_ORDER == 2 || (POSE6D_BWD8_ORDER && p6::ceil_div(gw.mps, 64) >= nk));
  const int grid = wfirst ? ((nw + 7) & ~7) + nd + rj.nblk : nd_pad + nw + rj.nblk;
  conv_bwd8_kernel<DMODE, DS, WS><<<grid, 2 * kThreads, lds, s>>>(
      (const bf16*)dy, (const bf16*)wt, (const bf16*)dres, (bf16*)dx, gd, nd, nd_pad, wfirst, (const bf16*)x, ws, gw,
      rj);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

template <int DMODE>
int launch_bwd8_mode(int ds, int ws_stages, const Geom& gd, const p6::WGeom& gw, const void* dy, const void* wt,
                     const void* dres, void* dx, const void* x, float* ws, const ReduceJob& rj, hipStream_t s,
                     int order) {
#ifdef POSE6D_BWD8_DS   // build-time (A/B): force the 8-wave fused launch's data-gradient ring depth
  ds = POSE6D_BWD8_DS;
#endif
  if (ws_stages >= 3)
    return ds == 2 ? launch_bwd8<DMODE, 2, 3>(gd, gw, dy, wt, dres, dx, x, ws, rj, s, order)
                   : launch_bwd8<DMODE, 4, 3>(gd, gw, dy, wt, dres, dx, x, ws, rj, s, order);
  return ds == 2 ? launch_bwd8<DMODE, 2, 2>(gd, gw, dy, wt, dres, dx, x, ws, rj, s, order)
                 : launch_bwd8<DMODE, 4, 2>(gd, gw, dy, wt, dres, dx, x, ws, rj, s, order);
}

// data-gradient ring depth of the fused launch for a plan of `stages` slots: fp32 plans
// of 4 run 3, so that with the 32-pixel weight-gradient stages (kBwdF32MS) the launch
// fits 48 KiB of LDS and three workgroups per CU (its VGPR budget allows three) -- the
// fp32 step 12.19 -> 11.94 ms against 4 slots and 64-pixel stages (64 KiB, two per CU;
// profiles/r05f32r_bwd_ring_ab.txt)
#ifndef POSE6D_BWD_BF16_DS4
#define POSE6D_BWD_BF16_DS4 4   // build-time (A/B): the bf16 fused data-gradient ring for 4-slot plans
#endif
int fused_ds(int dtype, int stages) {
  if (stages <= 2) return stages;
  return dtype == POSE6D_DT_F32 ? 3 : POSE6D_BWD_BF16_DS4;
}

template <int DMODE>
int launch_bwd_mode(int dtype, int ds, const Geom& gd, const p6::WGeom& gw, const void* dy, const void* wt,
                    const void* dres, void* dx, const void* x, float* ws, const ReduceJob& rj, hipStream_t s,
                    int order, int wbt = 64) {
  if (dtype == POSE6D_DT_F32 && wbt == 128)
    return fused_ds(dtype, ds) == 2
               ? launch_bwd<DMODE, 2, POSE6D_WGRAD_STAGES_F32, float, 128>(gd, gw, dy, wt, dres, dx, x, ws, rj, s, order)
               : launch_bwd<DMODE, 3, POSE6D_WGRAD_STAGES_F32, float, 128>(gd, gw, dy, wt, dres, dx, x, ws, rj, s,
                                                                          order);
  if (dtype == POSE6D_DT_F32)
    return fused_ds(dtype, ds) == 2
               ? launch_bwd<DMODE, 2, POSE6D_WGRAD_STAGES_F32, float>(gd, gw, dy, wt, dres, dx, x, ws, rj, s, order)
               : launch_bwd<DMODE, 3, POSE6D_WGRAD_STAGES_F32, float>(gd, gw, dy, wt, dres, dx, x, ws, rj, s, order);
  return ds == 2 ? launch_bwd<DMODE, 2, POSE6D_WGRAD_STAGES>(gd, gw, dy, wt, dres, dx, x, ws, rj, s, order)
                 : launch_bwd<DMODE, POSE6D_BWD_BF16_DS4, POSE6D_WGRAD_STAGES>(gd, gw, dy, wt, dres, dx, x, ws, rj, s,
                                                                               order);
}

}  // namespace

// Data + weight gradient of one conv.  When both passes take the bf16 LDS-DMA
// kernels (64x64 tiles, data-gradient ring of 2 or 4 slots, weight-gradient ring
// of 3) they run as ONE launch of conv_bwd_kernel, followed by the slab reduce;
// otherwise as the separate pose6d_conv2d_dgrad + pose6d_conv2d_wgrad launches.
// dx == NULL: weight gradient only.
namespace {
#ifndef POSE6D_BWD_F32_FUSE128
#define POSE6D_BWD_F32_FUSE128 1   // build-time (A/B): 0 = the fp32 128x128 weight gradients as launches of their own
#endif
bool bwd_fused(int dtype, const Plan& pd, const p6::WgradPlan& pw, const pose6d_tuning_t* tn) {
  // the fused kernels carry the 64x64 weight-gradient bodies (conv_bwd_kernel) and the
  // bf16 128x128 one (conv_bwd8_kernel: its data gradient on 128x64 tiles of 8 waves)
  if (!pd.fast || pd.tile != 3 || !(pd.stages == 2 || pd.stages == 4) || !pw.fast) return false;
  if (tune(tn, &pose6d_tuning_t::bwd_separate, 0) != 0) return false;
  if (pw.bm == 128 && dtype == POSE6D_DT_BF16) return pw.stages == 2 || pw.stages == 3;
  if (pw.bm == 128) return POSE6D_BWD_F32_FUSE128 && pw.stages == POSE6D_WGRAD_STAGES_F32;   // fp32 KxK, 128x128
  return pw.bm == 64 && pw.stages == (dtype == POSE6D_DT_BF16 ? POSE6D_WGRAD_STAGES : POSE6D_WGRAD_STAGES_F32);
}

// the data-gradient plan a fused launch runs: the bf16 8-wave launch (128x128 weight-
// gradient tiles) takes 128x64 data-gradient tiles of 8 waves (tile 5), which also sets
// the BatchNorm-reduce partial rows (bnr_plan_rows); the fp32 launch keeps the plan's tile
Plan fused_dplan(int dtype, const Plan& pd, const p6::WgradPlan& pw) {
  Plan q = pd;
  if (dtype == POSE6D_DT_BF16 && pw.bm == 128) q.tile = 5;
  return q;
}

int conv_backward_impl(int32_t dtype, const void* x, const void* dy, const void* wt, const void* dres, void* dx,
                       float* dw, int32_t accumulate, float* workspace, int64_t ws_bytes, int32_t N, int32_t H,
                       int32_t W, int32_t Cin, int32_t Cin_real, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
                       int32_t pad, int32_t Ho, int32_t Wo, int32_t phases, void* stream,
                       const ReduceJob* rj = nullptr, int32_t* deferred = nullptr,
                       const uint8_t* dres_mask = nullptr, const pose6d_tuning_t* tn = nullptr,
                       const pose6d_bn_reduce_t* bnr = nullptr) {
  P6_CHECK_ARG(dtype == POSE6D_DT_F32 || dtype == POSE6D_DT_BF16, "pose6d_conv2d_backward: bad dtype %d", dtype);
  if (deferred) *deferred = 0;
  const ReduceJob none{};
  auto flush_prev = [&]() -> int {   // the carried reduce as a launch of its own
    if (!rj || rj->nblk == 0) return POSE6D_OK;
    return p6::wgrad_reduce_launch(rj->ws, rj->dw, rj->Cout, rj->Kpad, rj->SC, rj->Cin, rj->KH, rj->KW, rj->KWp,
                                   rj->splits, rj->accumulate, p6::stream_of(stream));
  };
  P6_CHECK_ARG(phases >= 1 && phases <= 3, "pose6d_conv2d_backward_ex: phases must be 1, 2 or 3");
  P6_CHECK_ARG(!bnr || (dx && phases == 3), "pose6d_conv2d_backward: a BatchNorm reduce needs the data gradient");
  // chain mode with a register-staged weight gradient (fp32, the bf16 stem): that launch
  // carries the previous conv's slab reduce as trailing workgroups and leaves its own
  // reduce pending, as the fused bf16 launch does -- one launch per conv fewer
  auto carry_wgrad = [&](bool& carried) -> int {
    carried = false;
    if (!deferred || phases != 3) return POSE6D_OK;
    p6::WgradPlan pw;
    const p6::WGeom gw = p6::wgrad_geom(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &pw, tn);
    // bf16 LDS-DMA plans go through the fused launch -- except a weight gradient alone
    // (no data gradient: the row-tap stems), whose LDS-DMA kernel carries the reduce too
    if (pw.fast && dtype == POSE6D_DT_BF16 && dx != nullptr) return POSE6D_OK;
    P6_CHECK_ARG((int64_t)pw.splits * Cout * gw.Kpad * 4 <= ws_bytes,
                 "pose6d_conv2d_backward: workspace %lld bytes < %lld needed", (long long)ws_bytes,
                 (long long)pw.splits * Cout * gw.Kpad * 4);
    const int rc = p6::wgrad_launch_carry(dtype, gw, pw, x, dy, workspace, rj ? *rj : none, p6::stream_of(stream));
    carried = rc == POSE6D_OK;
    *deferred = carried;
    return rc;
  };
  if (dx == nullptr) {
    if (!(phases & 1)) return POSE6D_OK;
    bool carried;
    int rc = carry_wgrad(carried);
    if (rc || carried) return rc;
    rc = flush_prev();
    if (rc) return rc;
    return pose6d_conv2d_wgrad_tuned(dtype, x, dy, dw, accumulate, workspace, ws_bytes, N, H, W, Cin, Cin_real, Cout,
                                     KH, KW, stride, pad, Ho, Wo, tn, stream);
  }
  P6_CHECK_ARG(stride == 1 || stride == 2, "pose6d_conv2d_backward: stride must be 1 or 2");
  P6_CHECK_ARG(Cin % 8 == 0 && Cin_real <= Cin && ilog2(Cin) >= 3,
               "pose6d_conv2d_backward: Cin must be a power of two >= 8 for the data gradient");
  P6_CHECK_ARG(!dres_mask || (dres && dres != dx), "pose6d_conv2d_backward: a residual mask needs a separate dres");
  int mode;
  Geom gd0 = dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &mode);
  gd0.res_mask = dres_mask;
  const Plan pd = choose(dtype, mode, gd0, true, tn);
  p6::WgradPlan pw;
  const p6::WGeom gw = p6::wgrad_geom(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &pw, tn);
  const bool fused = bwd_fused(dtype, pd, pw, tn);
  if (!fused) {
    if (!(phases & 1)) return POSE6D_OK;
    const bool carry = deferred && phases == 3 && (!pw.fast || dtype == POSE6D_DT_F32);
    int rc = carry ? POSE6D_OK : flush_prev();
    if (rc) return rc;
    rc = dgrad_impl(dtype, dy, wt, dres, dres_mask, dx, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, stream, tn,
                    bnr);
    if (rc) return rc;
    if (carry) {
      bool carried;
      rc = carry_wgrad(carried);
      if (rc || carried) return rc;
      rc = flush_prev();
      if (rc) return rc;
    }
    return pose6d_conv2d_wgrad_tuned(dtype, x, dy, dw, accumulate, workspace, ws_bytes, N, H, W, Cin, Cin_real, Cout,
                                     KH, KW, stride, pad, Ho, Wo, tn, stream);
  }
  P6_CHECK_ARG((int64_t)pw.splits * Cout * gw.Kpad * 4 <= ws_bytes,
               "pose6d_conv2d_backward: workspace %lld bytes < %lld needed", (long long)ws_bytes,
               (long long)pw.splits * Cout * gw.Kpad * 4);
  hipStream_t s = p6::stream_of(stream);
  int rc = check_bnr(bnr, fused_dplan(dtype, pd, pw), dres, dx);
  if (rc) return rc;
  Geom gd = pd.g;
  set_bnr(gd, bnr);
  const ReduceJob& carried = rj ? *rj : none;
  const int order = tune(tn, &pose6d_tuning_t::bwd_order, -1);
  // one weight-gradient split of a 1x1 conv whose K is exactly Cin (layer4's 1x1 convs):
  // the slab [Cout][Cin] IS the OIHW dW, so the launch writes dW itself and no reduce
  // follows (the reduce would only have copied it)
#ifndef POSE6D_WGRAD_DIRECT
#define POSE6D_WGRAD_DIRECT 1   // build-time (A/B): 0 = every plan through the slab reduce
#endif
  const bool direct = POSE6D_WGRAD_DIRECT && gw.splits == 1 && KH == 1 && KW == 1 && gw.Kpad == Cin &&
                      Cin_real == Cin && !accumulate;
  float* slab = direct ? dw : workspace;
  if ((phases & 1) && pw.bm == 128 && dtype == POSE6D_DT_BF16) {
    switch (pd.mode) {
      case kGemm:
        rc = launch_bwd8_mode<kGemm>(pd.stages, pw.stages, gd, gw, dy, wt, dres, dx, x, slab, carried, s, order);
        break;
      case kDgradS2:
        rc = launch_bwd8_mode<kDgradS2>(pd.stages, pw.stages, gd, gw, dy, wt, dres, dx, x, slab, carried, s, order);
        break;
      default:
        rc = launch_bwd8_mode<kDgrad>(pd.stages, pw.stages, gd, gw, dy, wt, dres, dx, x, slab, carried, s, order);
        break;
    }
  } else if (phases & 1) {
    switch (pd.mode) {
      case kGemm:
        rc = launch_bwd_mode<kGemm>(dtype, pd.stages, gd, gw, dy, wt, dres, dx, x, slab, carried, s, order, pw.bm);
        break;
      case kDgradS2:
        rc = launch_bwd_mode<kDgradS2>(dtype, pd.stages, gd, gw, dy, wt, dres, dx, x, slab, carried, s, order,
                                       pw.bm);
        break;
      default:
        rc = launch_bwd_mode<kDgrad>(dtype, pd.stages, gd, gw, dy, wt, dres, dx, x, slab, carried, s, order, pw.bm);
        break;
    }
  }
  if (direct) {
    if (deferred) *deferred = 0;
    return rc;
  }
  if (deferred) {   // chain mode: this conv's slab reduce rides on the next launch
    *deferred = rc == POSE6D_OK;
    return rc;
  }
  if (rc || !(phases & 2)) return rc;
  return p6::wgrad_reduce_launch(workspace, dw, Cout, gw.Kpad, Cin, Cin_real, KH, KW, gw.kwp, gw.splits, accumulate,
                                 s);
}
}  // namespace

extern "C" int pose6d_conv2d_backward(int32_t dtype, const void* x, const void* dy, const void* wt, const void* dres,
                                      void* dx, float* dw, int32_t accumulate, float* workspace, int64_t ws_bytes,
                                      int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cin_real, int32_t Cout,
                                      int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo,
                                      void* stream) {
  return conv_backward_impl(dtype, x, dy, wt, dres, dx, dw, accumulate, workspace, ws_bytes, N, H, W, Cin, Cin_real,
                            Cout, KH, KW, stride, pad, Ho, Wo, 3, stream);
}

extern "C" int pose6d_conv2d_backward_tuned(int32_t dtype, const void* x, const void* dy, const void* wt,
                                            const void* dres, void* dx, float* dw, int32_t accumulate,
                                            float* workspace, int64_t ws_bytes, int32_t N, int32_t H, int32_t W,
                                            int32_t Cin, int32_t Cin_real, int32_t Cout, int32_t KH, int32_t KW,
                                            int32_t stride, int32_t pad, int32_t Ho, int32_t Wo,
                                            const pose6d_tuning_t* tuning, void* stream) {
  return conv_backward_impl(dtype, x, dy, wt, dres, dx, dw, accumulate, workspace, ws_bytes, N, H, W, Cin, Cin_real,
                            Cout, KH, KW, stride, pad, Ho, Wo, 3, stream, nullptr, nullptr, nullptr, tuning);
}

extern "C" int pose6d_conv2d_backward_ex(int32_t dtype, const void* x, const void* dy, const void* wt,
                                         const void* dres, void* dx, float* dw, int32_t accumulate, float* workspace,
                                         int64_t ws_bytes, int32_t N, int32_t H, int32_t W, int32_t Cin,
                                         int32_t Cin_real, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
                                         int32_t pad, int32_t Ho, int32_t Wo, int32_t phases, void* stream) {
  return conv_backward_impl(dtype, x, dy, wt, dres, dx, dw, accumulate, workspace, ws_bytes, N, H, W, Cin, Cin_real,
                            Cout, KH, KW, stride, pad, Ho, Wo, phases, stream);
}

// launch variant of a forward / data-gradient conv, for profiling joins:
// (stages << 12) | (fast << 8) | (mode << 4) | tile, tile 0 = 128x128, 1 = 128x64,
// 2 = 64x128, 3 = 64x64 (stages 0 on the register-staged path)
extern "C" int pose6d_conv_variant(int32_t dtype, int32_t pass, int32_t N, int32_t H, int32_t W, int32_t Cin,
                                   int32_t Cout, int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho,
                                   int32_t Wo) {
  int mode;
  const Geom g = pass == 0 ? fwd_geom(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &mode)
                           : dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &mode);
  const Plan p = choose(dtype, mode, g, false, nullptr, pass == 0);
  return (p.g.splits << 16) | (p.stages << 12) | ((int)p.fast << 8) | (p.mode << 4) | p.tile;
}

// workgroups of the patch plan a stats-free forward of this geometry runs (0 = the
// implicit-GEMM plans of pose6d_conv_variant)
extern "C" int pose6d_conv_patch_plan(int32_t dtype, int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout,
                                      int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo) {
  int mode;
  const Geom g = fwd_geom(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &mode);
  PatchPlan pp{};
  return patch_eligible(dtype, mode, g, nullptr, nullptr, &pp) ? pp.tiles * (Cout / kPatchBN) : 0;
}

// split-K workspace bytes of a forward (pass 0) / data-gradient (pass 1) conv's plan:
// 0 when the plan does not split K (then the workspace arguments may be NULL / 0)
extern "C" int64_t pose6d_conv_splitk_workspace_tuned(int32_t dtype, int32_t pass, int32_t N, int32_t H, int32_t W,
                                                      int32_t Cin, int32_t Cout, int32_t KH, int32_t KW,
                                                      int32_t stride, int32_t pad, int32_t Ho, int32_t Wo,
                                                      const pose6d_tuning_t* tuning) {
  int mode;
  const Geom g = pass == 0 ? fwd_geom(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &mode)
                           : dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &mode);
  return splitk_need(choose(dtype, mode, g, false, tuning, pass == 0));
}

extern "C" int64_t pose6d_conv_splitk_workspace(int32_t dtype, int32_t pass, int32_t N, int32_t H, int32_t W,
                                                int32_t Cin, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
                                                int32_t pad, int32_t Ho, int32_t Wo) {
  return pose6d_conv_splitk_workspace_tuned(dtype, pass, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, nullptr);
}

// fused backward variant (profiling joins): (1 << 16) | (dgrad mode << 4) | data-gradient
// ring stages when pose6d_conv2d_backward runs ONE conv_bwd_kernel launch, else 0
extern "C" int pose6d_bwd_variant(int32_t dtype, int32_t N, int32_t H, int32_t W, int32_t Cin, int32_t Cout,
                                  int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho, int32_t Wo) {
  if (Cin % 8 != 0 || ilog2(Cin) < 3) return 0;
  int mode;
  const Geom gd0 = dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &mode);
  const Plan pd = choose(dtype, mode, gd0, true);
  p6::WgradPlan pw;
  p6::wgrad_geom(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &pw);
  return bwd_fused(dtype, pd, pw, nullptr) ? (1 << 16) | (pd.mode << 4) | fused_ds(dtype, pd.stages) : 0;
}

namespace {
ReduceJob make_job(const pose6d_wgrad_reduce_t& j) {
  p6::WgradPlan pw;
  const p6::WGeom g = p6::wgrad_geom(j.dtype, j.N, j.H, j.W, j.Cin, j.Cout, j.KH, j.KW, j.stride, j.pad, j.Ho, j.Wo,
                                     &pw);
  ReduceJob r{};
  r.ws = j.ws; r.dw = j.dw; r.Cout = j.Cout; r.Kpad = g.Kpad; r.SC = j.Cin; r.Cin = j.Cin_real;
  r.KH = j.KH; r.KW = j.KW; r.KWp = g.kwp; r.splits = g.splits; r.accumulate = j.accumulate;
  r.G = reduce_group(g.splits);
  r.nblk = reduce_blocks(j.Cout, g.Kpad, r.G);
  return r;
}
}  // namespace

extern "C" int pose6d_wgrad_reduce(const pose6d_wgrad_reduce_t* job, void* stream) {
  P6_CHECK_ARG(job != nullptr, "pose6d_wgrad_reduce: null job");
  const ReduceJob r = make_job(*job);
  return p6::wgrad_reduce_launch(r.ws, r.dw, r.Cout, r.Kpad, r.SC, r.Cin, r.KH, r.KW, r.KWp, r.splits, r.accumulate,
                                 p6::stream_of(stream));
}

extern "C" int pose6d_conv2d_backward_chain(int32_t dtype, const void* x, const void* dy, const void* wt,
                                            const void* dres, void* dx, float* dw, int32_t accumulate,
                                            float* workspace, int64_t ws_bytes, int32_t N, int32_t H, int32_t W,
                                            int32_t Cin, int32_t Cin_real, int32_t Cout, int32_t KH, int32_t KW,
                                            int32_t stride, int32_t pad, int32_t Ho, int32_t Wo,
                                            const pose6d_wgrad_reduce_t* prev, int32_t* deferred, void* stream) {
  P6_CHECK_ARG(deferred != nullptr, "pose6d_conv2d_backward_chain: deferred must point to an int32");
  ReduceJob r{};
  if (prev) {
    P6_CHECK_ARG(prev->ws != workspace, "pose6d_conv2d_backward_chain: prev slabs must live in another workspace");
    r = make_job(*prev);
  }
  return conv_backward_impl(dtype, x, dy, wt, dres, dx, dw, accumulate, workspace, ws_bytes, N, H, W, Cin, Cin_real,
                            Cout, KH, KW, stride, pad, Ho, Wo, 3, stream, prev ? &r : nullptr, deferred);
}

extern "C" int pose6d_conv2d_backward_chain_masked(int32_t dtype, const void* x, const void* dy, const void* wt,
                                                   const void* dres, const uint8_t* dres_mask, void* dx, float* dw,
                                                   int32_t accumulate, float* workspace, int64_t ws_bytes, int32_t N,
                                                   int32_t H, int32_t W, int32_t Cin, int32_t Cin_real, int32_t Cout,
                                                   int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho,
                                                   int32_t Wo, const pose6d_wgrad_reduce_t* prev, int32_t* deferred,
                                                   void* stream) {
  P6_CHECK_ARG(deferred != nullptr, "pose6d_conv2d_backward_chain_masked: deferred must point to an int32");
  P6_CHECK_ARG(dres_mask != nullptr, "pose6d_conv2d_backward_chain_masked: null mask");
  ReduceJob r{};
  if (prev) {
    P6_CHECK_ARG(prev->ws != workspace, "pose6d_conv2d_backward_chain: prev slabs must live in another workspace");
    r = make_job(*prev);
  }
  return conv_backward_impl(dtype, x, dy, wt, dres, dx, dw, accumulate, workspace, ws_bytes, N, H, W, Cin, Cin_real,
                            Cout, KH, KW, stride, pad, Ho, Wo, 3, stream, prev ? &r : nullptr, deferred, dres_mask);
}

// BatchNorm-reduce partial rows of this conv's data gradient (pose6d_bn_reduce_t::rows):
// the plan pose6d_conv2d_backward_chain_bn will run, one row per output tile
extern "C" int pose6d_conv2d_backward_bn_rows(int32_t dtype, int32_t N, int32_t H, int32_t W, int32_t Cin,
                                              int32_t Cout, int32_t KH, int32_t KW, int32_t stride, int32_t pad,
                                              int32_t Ho, int32_t Wo) {
  if (Cin % 8 != 0 || ilog2(Cin) < 3) return 0;
  int mode;
  const Geom gd0 = dgrad_geom(N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &mode);
  const Plan pd = choose(dtype, mode, gd0, true);
  p6::WgradPlan pw;
  p6::wgrad_geom(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &pw);
  return bnr_plan_rows(bwd_fused(dtype, pd, pw, nullptr) ? fused_dplan(dtype, pd, pw) : choose(dtype, mode, gd0, false));
}

extern "C" int pose6d_conv2d_backward_chain_bn(int32_t dtype, const void* x, const void* dy, const void* wt,
                                               const void* dres, const uint8_t* dres_mask, void* dx, float* dw,
                                               int32_t accumulate, float* workspace, int64_t ws_bytes, int32_t N,
                                               int32_t H, int32_t W, int32_t Cin, int32_t Cin_real, int32_t Cout,
                                               int32_t KH, int32_t KW, int32_t stride, int32_t pad, int32_t Ho,
                                               int32_t Wo, const pose6d_wgrad_reduce_t* prev, int32_t* deferred,
                                               const pose6d_bn_reduce_t* bn, void* stream) {
  P6_CHECK_ARG(deferred != nullptr, "pose6d_conv2d_backward_chain_bn: deferred must point to an int32");
  P6_CHECK_ARG(!dres_mask || dres, "pose6d_conv2d_backward_chain_bn: a mask needs dres");
  ReduceJob r{};
  if (prev) {
    P6_CHECK_ARG(prev->ws != workspace, "pose6d_conv2d_backward_chain: prev slabs must live in another workspace");
    r = make_job(*prev);
  }
  return conv_backward_impl(dtype, x, dy, wt, dres, dx, dw, accumulate, workspace, ws_bytes, N, H, W, Cin, Cin_real,
                            Cout, KH, KW, stride, pad, Ho, Wo, 3, stream, prev ? &r : nullptr, deferred, dres_mask,
                            nullptr, bn);
}

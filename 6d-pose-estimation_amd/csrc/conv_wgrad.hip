// Convolution weight gradient on MFMA (split-K over output pixels) for gfx950.
//
//   dW[co][k] = sum_m dY[m][co] * im2col(X)[m][k],   k = (kh, kw, ci), m = (n, oy, ox)
//
// Both operands are m-major in HBM (NHWC), so each LDS stage holds a [32 m][cols]
// image of dY and of the gathered X, written as 16-byte rows; the MFMA operands
// need 8 consecutive m per lane and come out of LDS through the gfx950 hardware
// transpose read (ds_read_b64_tr_b16: 4 m x 1 column per lane per read).  The
// XOR swizzle puts the 8 rows one 32-lane half reads on 8 distinct bank octets.
// The reduction over m (up to 100k pixels) is split over workgroups; each split
// writes an fp32 slab [S][Cout][Kpad] and pose6d_conv2d_wgrad_reduce sums the
// slabs in fixed order into the OIHW fp32 gradient (deterministic, no atomics).
#include <stdlib.h>
#include <string.h>

#include "common.h"
#include "lds_dma.h"
#include "wgrad_body.h"

namespace {

using p6::WGeom;
constexpr int kThreads = 256;
constexpr int MT = 32;  // m rows per reduction step

template <typename T> struct WT;
template <> struct WT<bf16> { static constexpr int VEC = 8; };
template <> struct WT<float> { static constexpr int VEC = 4; };


// XOR (in 16-B chunk units, always even: keeps 32-B pairs together) for a row of
// `pairs` 32-byte pairs, such that rows {0..3, 8..11} (and {4..7, 12..15}) of a
// transposed read land on distinct bank octets.
template <int PAIRS>
__device__ __forceinline__ int swz_tr(int m) {
  if constexpr (PAIRS >= 8) return ((m & 3) | (((m >> 3) & 1) << 2)) << 1;
  else if constexpr (PAIRS == 4) return (((m >> 1) & 1) | (((m >> 3) & 1) << 1)) << 1;
  else return 0;
}

// 8 consecutive m (8*grp .. 8*grp+7) of one LDS column, as an MFMA bf16 operand:
// two ds_read_b64_tr_b16, lane 4q+p of each 16-lane group addressing row q, cols 4p..4p+3.
template <int ROWB>
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int col, int grp, int q) {
  bf16x8 f;
  const int cchunk = col >> 3, cin = (col & 7) * 2;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int r = 8 * grp + 4 * h + q;
    const char* a = img + r * ROWB + ((cchunk ^ swz_tr<ROWB / 32>(r)) << 4) + cin;
    const s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)a);
    const bf16x4 bv = __builtin_bit_cast(bf16x4, v);
#pragma unroll
    for (int e = 0; e < 4; ++e) f[4 * h + e] = bv[e];
  }
  return f;
}

template <typename T, int BM, int BN>
__global__ __launch_bounds__(kThreads) void conv_wgrad_kernel(const T* __restrict__ x, const T* __restrict__ dy,
                                                              float* __restrict__ ws, WGeom g, ReduceJob rj) {
  constexpr int VEC = WT<T>::VEC;
  constexpr bool BF = sizeof(T) == 2;
  constexpr int YROW = BM * (int)sizeof(T);   // bytes per LDS row of the dY image
  constexpr int XROW = BN * (int)sizeof(T);
  constexpr int YCPR = YROW / 16, XCPR = XROW / 16;  // 16-B chunks per row
  constexpr int YPER = MT * YCPR / kThreads, XPER = MT * XCPR / kThreads;
  constexpr int YRSTEP = kThreads / YCPR, XRSTEP = kThreads / XCPR;
  constexpr int STAGE = MT * (YROW + XROW);
  constexpr int TM = BM / 32, TN = BN / 32;
  static_assert(YPER >= 1 && XPER >= 1, "tile too small");
  extern __shared__ __attribute__((aligned(16))) char smem[];

  const int tiles = g.gm * g.gn;
  if ((int)blockIdx.x >= tiles * g.splits) {   // trailing workgroups: the carried reduce
    run_reduce_job(smem, blockIdx.x - tiles * g.splits, rj);
    return;
  }
  const int split = blockIdx.x / tiles;
  int t2 = blockIdx.x - split * tiles;
  const int tm = t2 / g.gn, tn = t2 - tm * g.gn;
  const int co0 = tm * BM, k0 = tn * BN;
  const int mbeg = split * g.mps;
  const int mend = min(g.M, mbeg + g.mps);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;

  // dY loads: row yr + i*YRSTEP, chunk yc
  const int yc = tid % YCPR, yr = tid / YCPR;
  const bool y_ok = co0 + yc * VEC < g.Cout;
  // X loads: chunk xc fixed -> its tap and channel are fixed for the whole loop
  const int xc = tid % XCPR, xr = tid / XCPR;
  const int kx = k0 + xc * VEC;
  const bool x_kok = kx < g.K;
  const int tap = x_kok ? (kx >> g.log2SC) : 0;
  const int ci = kx & (g.SC - 1);
  const int kh = tap / g.KW, kw = tap - kh * g.KW;
  // incremental (n, oy, ox) of this thread's X rows
  int xn[XPER], xy[XPER], xx[XPER];
#pragma unroll
  for (int i = 0; i < XPER; ++i) {
    const int m = mbeg + xr + i * XRSTEP;
    const int hw = g.RH * g.RW;
    xn[i] = m / hw;
    const int rem = m - xn[i] * hw;
    xy[i] = rem / g.RW;
    xx[i] = rem - xy[i] * g.RW;
  }

  uint4 ry[YPER], rx[XPER];
  auto load = [&](int mstep) {
#pragma unroll
    for (int i = 0; i < YPER; ++i) {
      const int m = mstep + yr + i * YRSTEP;
      ry[i] = (y_ok && m < mend) ? *reinterpret_cast<const uint4*>(dy + (int64_t)m * g.Cout + co0 + yc * VEC)
                                 : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < XPER; ++i) {
      const int m = mstep + xr + i * XRSTEP;
      const int sy = xy[i] * g.stride - g.pad + kh, sx = xx[i] * g.stride - g.pad + kw;
      const bool ok = x_kok && m < mend && (unsigned)sy < (unsigned)g.SH && (unsigned)sx < (unsigned)g.SW;
      const int64_t off = (((int64_t)xn[i] * g.SH + sy) * g.SW + sx) * g.SC + ci;
      if (VEC * (int)sizeof(T) == 16 && g.SC >= VEC) {
        rx[i] = ok ? *reinterpret_cast<const uint4*>(x + off) : make_uint4(0, 0, 0, 0);
      } else {  // stem (SC == 4, bf16): two 4-channel taps per chunk
        uint32_t w[4] = {0, 0, 0, 0};
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          const int k = kx + 4 * u, tp = k >> 2;
          const int h2 = tp / g.KW, w2 = tp - h2 * g.KW;
          const int sy2 = xy[i] * g.stride - g.pad + h2, sx2 = xx[i] * g.stride - g.pad + w2;
          if (m < mend && k < g.K && (unsigned)sy2 < (unsigned)g.SH && (unsigned)sx2 < (unsigned)g.SW) {
            const uint2 v = *reinterpret_cast<const uint2*>(x + (((int64_t)xn[i] * g.SH + sy2) * g.SW + sx2) * 4);
            w[2 * u] = v.x; w[2 * u + 1] = v.y;
          }
        }
        rx[i] = make_uint4(w[0], w[1], w[2], w[3]);
      }
      // advance this row by MT pixels
      xx[i] += MT;
      while (xx[i] >= g.RW) { xx[i] -= g.RW; if (++xy[i] == g.RH) { xy[i] = 0; ++xn[i]; } }
    }
  };
  auto store = [&](int buf) {
    char* Ys = smem + buf * STAGE;
    char* Xs = Ys + MT * YROW;
#pragma unroll
    for (int i = 0; i < YPER; ++i) {
      const int r = yr + i * YRSTEP;
      const int pc = BF ? (yc ^ swz_tr<YROW / 32>(r)) : yc;
      *reinterpret_cast<uint4*>(Ys + r * YROW + pc * 16) = ry[i];
    }
#pragma unroll
    for (int i = 0; i < XPER; ++i) {
      const int r = xr + i * XRSTEP;
      const int pc = BF ? (xc ^ swz_tr<XROW / 32>(r)) : xc;
      *reinterpret_cast<uint4*>(Xs + r * XROW + pc * 16) = rx[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  auto compute = [&](int buf) {
    const char* Ys = smem + buf * STAGE;
    const char* Xs = Ys + MT * YROW;
    if constexpr (BF) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) af[i] = tr_frag<YROW>(Ys, wm * (BM / 2) + i * 16 + 4 * p, grp, q);
#pragma unroll
      for (int j = 0; j < TN; ++j) bfr[j] = tr_frag<XROW>(Xs, wn * (BN / 2) + j * 16 + 4 * p, grp, q);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int s = 0; s < MT / 4; ++s) {
        const int r = 4 * s + grp;
        float a[TM], b[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
          a[i] = *reinterpret_cast<const float*>(Ys + r * YROW + (wm * (BM / 2) + i * 16 + li) * 4);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          b[j] = *reinterpret_cast<const float*>(Xs + r * XROW + (wn * (BN / 2) + j * 16 + li) * 4);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  const int nsteps = (mend - mbeg + MT - 1) / MT;
  if (nsteps > 0) {
    load(mbeg);
    store(0);
    __syncthreads();
    for (int st = 0; st < nsteps; ++st) {
      const int cur = st & 1;
      if (st + 1 < nsteps) load(mbeg + (st + 1) * MT);
      compute(cur);
      if (st + 1 < nsteps) store(cur ^ 1);
      __syncthreads();
    }
  }
  // slab write: rows co, cols k, staged through LDS as 16-byte row vectors (the
  // loop's last __syncthreads ended every read of the staging buffers)
  float* slab = ws + (int64_t)split * g.Cout * g.Kpad;
  store_acc_tile<BM, BN, true>(acc, smem, slab + (int64_t)co0 * g.Kpad + k0, g.Kpad, g.Cout - co0, g.Kpad - k0);
}


// standalone slab reduce (the body lives in wgrad_body.h: the fused backward of the
// next conv also runs it as extra workgroups)
template <int G>
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ ws, float* __restrict__ dw,
                                                           int Cout, int Kpad, int SC, int Cin, int KH, int KW,
                                                           int KWp, int splits, int accumulate) {
  __shared__ float4 red[256];
  wgrad_reduce_body<G>(red, blockIdx.x, ws, dw, Cout, Kpad, SC, Cin, KH, KW, KWp, splits, accumulate);
}

int launch_reduce(const float* ws, float* dw, int Cout, int Kpad, int SC, int Cin, int KH, int KW, int KWp,
                  int splits, int accumulate, hipStream_t s) {
  const int64_t quads = (int64_t)Cout * Kpad / 4;
  auto go = [&](auto kern, int L) {
    kern<<<(unsigned)((quads + L - 1) / L), 256, 0, s>>>(ws, dw, Cout, Kpad, SC, Cin, KH, KW, KWp, splits,
                                                         accumulate);
  };
  if (splits >= 64) go(wgrad_reduce_kernel<16>, 16);
  else if (splits >= 16) go(wgrad_reduce_kernel<4>, 64);
  else go(wgrad_reduce_kernel<1>, 256);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

using Plan = p6::WgradPlan;

// trailing workgroups (rj.nblk) run a carried slab reduce of the previous conv.
// BT = 64: 64x64 tiles on 4 waves; BT = 128: 128x128 tiles on 8 waves
template <int S, bool PW, bool RT, int BT = 64>
__global__ __launch_bounds__(BT == 128 ? 512 : kThreads) void conv_wgrad_lds_kernel(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, float* __restrict__ ws, WGeom g, ReduceJob rj) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles = g.gm * g.gn;
  if ((int)blockIdx.x >= tiles * g.splits) {
    if (threadIdx.x < kThreads) run_reduce_job(smem, blockIdx.x - tiles * g.splits, rj);
    return;
  }
  conv_wgrad_lds_body<BT, BT, S, PW, RT, BT == 128 ? 8 : 4>(smem, blockIdx.x, x, dy, ws, g);
}

// fp32 LDS-DMA weight gradient (wgrad_body.h conv_wgrad_lds_body_f32); trailing
// workgroups run a carried slab reduce of the previous conv (`rj`), as the
// register-staged kernel does.  64x64 tiles take 64-pixel stages, 128x128 tiles
// 32-pixel stages (32 KiB either way)
template <int BT>
constexpr int f32_ms() { return BT == 128 ? 32 : 64; }
template <int S, bool PW, int BT, bool RT = false>
__global__ __launch_bounds__(kThreads) void conv_wgrad_lds_f32_kernel(const float* __restrict__ x,
                                                                      const float* __restrict__ dy,
                                                                      float* __restrict__ ws, WGeom g, ReduceJob rj) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tiles = g.gm * g.gn;
  if ((int)blockIdx.x >= tiles * g.splits) {
    run_reduce_job(smem, blockIdx.x - tiles * g.splits, rj);
    return;
  }
  conv_wgrad_lds_body_f32<f32_ms<BT>(), S, PW, BT, RT>(smem, blockIdx.x, x, dy, ws, g);
}

template <int S, int BT>
int launch_fast_f32(const WGeom& g, const void* x, const void* dy, float* ws, hipStream_t s, const ReduceJob& rj) {
  int lds = S * WgF32<f32_ms<BT>(), BT>::STAGE;
  if (lds < acc_stage_bytes<BT, BT>()) lds = acc_stage_bytes<BT, BT>();
  const int grid = g.gm * g.gn * g.splits + rj.nblk;
  if constexpr (BT == 64) {
    if (g.kwp == p6::kRowTaps && g.SC == 4) {
      conv_wgrad_lds_f32_kernel<S, false, 64, true><<<grid, kThreads, lds, s>>>((const float*)x, (const float*)dy, ws,
                                                                               g, rj);
      P6_LAUNCH_CHECK();
      return POSE6D_OK;
    }
  }
  if (g.KH == 1 && g.KW == 1 && g.stride == 1 && g.pad == 0)
    conv_wgrad_lds_f32_kernel<S, true, BT><<<grid, kThreads, lds, s>>>((const float*)x, (const float*)dy, ws, g, rj);
  else
    conv_wgrad_lds_f32_kernel<S, false, BT><<<grid, kThreads, lds, s>>>((const float*)x, (const float*)dy, ws, g, rj);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

int launch_fast_f32_any(const Plan& p, const WGeom& g, const void* x, const void* dy, float* ws, hipStream_t s,
                        const ReduceJob& rj) {
  if (p.bm == 128) return p.stages == 3 ? launch_fast_f32<3, 128>(g, x, dy, ws, s, rj)
                                        : launch_fast_f32<2, 128>(g, x, dy, ws, s, rj);
  return p.stages == 3 ? launch_fast_f32<3, 64>(g, x, dy, ws, s, rj) : launch_fast_f32<2, 64>(g, x, dy, ws, s, rj);
}

int tuned(const pose6d_tuning_t* t, int32_t pose6d_tuning_t::*f, int dflt) {
  return (t && t->*f >= 0) ? (int)(t->*f) : dflt;
}

// build-time (A/B sweeps): workgroups the bf16 / register-staged (fp32, stem) split
// plans aim for, and the bf16 LDS ring depth
#ifndef POSE6D_WGRAD_TARGET
#define POSE6D_WGRAD_TARGET 256
#endif
#ifndef POSE6D_WGRAD_TARGET_KXK
#define POSE6D_WGRAD_TARGET_KXK 256
#endif
#ifndef POSE6D_WGRAD_TARGET_BASE
#define POSE6D_WGRAD_TARGET_BASE 1024
#endif
#ifndef POSE6D_WGRAD_TARGET_F32
#define POSE6D_WGRAD_TARGET_F32 512
#endif
#ifndef POSE6D_WGRAD_TARGET_F32_FAST
#define POSE6D_WGRAD_TARGET_F32_FAST 512
#endif


#ifndef POSE6D_WGRAD_F32_KXK_BT
#define POSE6D_WGRAD_F32_KXK_BT 128
#endif

// bf16 weight gradients take the LDS-DMA kernel (64x64 tiles, 3-slot ring) unless a
// pose6d_tuning_t (tests / tools only) asks for the register-staged kernel or another ring
// rowtap: the row-tap stems (wgrad_geom): SC is passed as 64 (its X image rows are
// 64 K-elements by construction); it aims for ~4 workgroups per CU on a 2-slot ring --
// its 4 K-tiles x 64 splits (one workgroup per CU, 98 64-pixel stages each) left each
// workgroup waiting on its DMA: 56 -> 34 us graph-timed (profiles/r05w_stem_wgrad_sweep.txt).
// The fp32 row-tap stem keeps the fp32 default (512 -> 128 splits of its 4 tiles: 147 us
// against 156 at 256 splits and 160 register-staged, profiles/r05w32_f32_stem_wgrad.txt)
#ifndef POSE6D_WGRAD_BF128
#define POSE6D_WGRAD_BF128 1   // build-time (A/B): 0 = the bf16 weight gradients on 64x64 tiles only, 2 = 128x128 wherever eligible
#endif
// wide: the geometry prefers the bf16 128x128 / 8-wave tile (KxK filters and stride-2 1x1
// convs: graph-timed alone 24-35 % faster than 64x64 on the 3x3 convs and the 28x28
// 512 -> 1024 downsample, slower on most stride-1 1x1 convs; profiles/r06_wgrad128_sweep.txt)
Plan plan(int dtype, int M, int Cout, int Kpad, int SC, const pose6d_tuning_t* tn = nullptr, bool rowtap = false,
          bool wide = false) {
  Plan p{};
  // wgrad_base: 0 = default, 1 = register-staged; fp32 only: 2 = LDS-DMA 64x64 tiles,
  // 3 = LDS-DMA 128x128 tiles (each where the channel counts allow it, else the default)
  const int wb = tuned(tn, &pose6d_tuning_t::wgrad_base, 0);
  const bool ok64 = SC % 64 == 0 && Cout % 64 == 0, ok128 = SC % 128 == 0 && Cout % 128 == 0;
  int f32_bt = 0;
  if (dtype == POSE6D_DT_F32 && wb != 1) {
    // default: 64x64 tiles for 1x1 filters and for Cout = 64, 128x128 for wider KxK
    // convs (the 64x64 body lost to the register-staged 128x128 tile there: 28x28
    // 128->128 3x3 85 vs 131 us, profiles/r04_f32_conv_sweep.txt)
    if (wb == 2 && ok64) f32_bt = 64;
    else if (wb == 3 && ok128) f32_bt = 128;
    else if (ok64 && (Kpad == SC || Cout == 64)) f32_bt = 64;
    else if (ok128) f32_bt = POSE6D_WGRAD_F32_KXK_BT;
  }
  // bf16: wgrad_base 4 = the 128x128 / 8-wave LDS-DMA tile (Cout and the padded K multiples
  // of 128; a 128-wide K tile may span two filter taps of 64 channels)
  // (wgrad_base 5: the 64x64 tile wherever the default would take 128x128; tools)
  const bool bf128 = dtype == POSE6D_DT_BF16 &&
                     (wb == 4 || (wb == 0 && (POSE6D_WGRAD_BF128 == 2 || (wide && POSE6D_WGRAD_BF128)))) && ok64 &&
                     Cout % 128 == 0 && Kpad % 128 == 0 && !rowtap;
  p.fast = dtype == POSE6D_DT_F32 ? f32_bt != 0 : ok64 && (wb == 0 || wb == 5 || bf128);
  int target, min_rows, step;
  int64_t max_bytes;
  if (p.fast && dtype == POSE6D_DT_F32) {
    // fp32 LDS-DMA body: 32 KiB stages, 2 slots (two workgroups per CU), ~2
    // workgroups per CU of splits
    p.bm = f32_bt;
    p.bn = f32_bt;
    p.stages = tuned(tn, &pose6d_tuning_t::wgrad_stages, POSE6D_WGRAD_STAGES_F32);
    if (p.stages < 2) p.stages = 2;
    if (p.stages > 3) p.stages = 3;
    target = POSE6D_WGRAD_TARGET_F32_FAST;
    min_rows = 256;
    step = f32_bt == 128 ? f32_ms<128>() : f32_ms<64>();
    max_bytes = 64ll << 20;
  } else if (p.fast) {
    p.bm = bf128 ? 128 : 64;
    p.bn = bf128 ? 128 : 64;
#ifndef POSE6D_WGRAD_STAGES_BF128
#define POSE6D_WGRAD_STAGES_BF128 2   // build-time (A/B): ring slots of the bf16 128x128 weight gradient
#endif
    p.stages = tuned(tn, &pose6d_tuning_t::wgrad_stages, bf128 ? POSE6D_WGRAD_STAGES_BF128 : POSE6D_WGRAD_STAGES);
    if (p.stages < 2) p.stages = 2;
    if (p.stages > (bf128 ? 3 : 4)) p.stages = bf128 ? 3 : 4;
    // ~256 workgroups (one per CU): with the fused launch dispatching its longest
    // workgroups first, long weight-gradient splits no longer form its tail, and
    // fewer splits write and reduce fewer fp32 slabs.  End-to-end A/B on one box
    // (profiles/r03w_wgrad_target_ab.txt): 256 / 384 / 448 / 512 / 640 / 896 / 1280 ->
    // 4.64 / 4.70 / 4.65 / 4.65 / 4.71 / 4.81 / 4.89 ms per step (640 was the best
    // target while the data gradient went first: 5.14 ms then, 384 -> 5.24)
    target = Kpad == SC ? POSE6D_WGRAD_TARGET : POSE6D_WGRAD_TARGET_KXK;   // 1x1 / larger filters
    if (rowtap) {
      target = 1024;
      p.stages = tuned(tn, &pose6d_tuning_t::wgrad_stages, 2);
      if (p.stages < 2) p.stages = 2;
      if (p.stages > 4) p.stages = 4;
    }
    min_rows = 256;
    step = 64;
    max_bytes = 48ll << 20;
  } else {
    p.bm = Cout >= 128 ? 128 : 64;
    p.bn = Kpad >= 128 ? 128 : 64;
    // fp32 (all convs) / the bf16 stem; sweeps in profiles/r03x_wgrad_base_target_ab.txt:
    // fp32 step 256 / 384 / 512 / 1024 / 2048 -> 13.73 / 13.63 / 13.04 / 13.36 / 13.38 ms,
    // the bf16 step with 512 for its stem 4.665 vs 4.636 ms at 1024
    target = dtype == POSE6D_DT_F32 ? POSE6D_WGRAD_TARGET_F32 : POSE6D_WGRAD_TARGET_BASE;
    min_rows = 256;
    step = MT;
    max_bytes = 64ll << 20;   // stem: 16 -> 64 MiB of slabs, 90 -> 65 us
  }
  const int tiles = p6::ceil_div(Cout, p.bm) * p6::ceil_div(Kpad, p.bn);
  // fp32 128x128 plans with many tiles (layer4's 3x3 convs: 144 tiles over 1568 pixels)
  // take twice the workgroups: 8 splits of 196 pixels, 207 -> 184 us on 7x7 512->512;
  // the few-tile KxK shapes keep the default target (profiles/r04_fp32_kxk_splits.txt)
#ifndef POSE6D_WGRAD_F32_MANY_TILES
#define POSE6D_WGRAD_F32_MANY_TILES 100000   // build-time (A/B): tiles from which the target doubles (round 6: off -- neutral to -0.2 %
                                           // the doubled slabs are read back by the next launch; profiles/r06_f32_split.txt)
#endif
  if (p.fast && dtype == POSE6D_DT_F32 && p.bm == 128 && tiles >= POSE6D_WGRAD_F32_MANY_TILES) target *= 2;
  // fp32 64x64 plans with >= 256 tiles (layer4's 512 -> 2048 / 2048 -> 512 1x1 convs): one
  // split -- a tile's 1568 pixels in one workgroup, 93 -> 78 us on 7x7 512->2048
  // (profiles/r04_bwd_plan_sweep.txt)
#ifndef POSE6D_WGRAD_F32_ONE_SPLIT_TILES
#define POSE6D_WGRAD_F32_ONE_SPLIT_TILES 256   // build-time (A/B)
#endif
  if (p.fast && dtype == POSE6D_DT_F32 && p.bm == 64 && tiles >= POSE6D_WGRAD_F32_ONE_SPLIT_TILES) target = tiles;
#ifndef POSE6D_WGRAD_BF128_ONE_SPLIT_TILES
#define POSE6D_WGRAD_BF128_ONE_SPLIT_TILES 128   // bf16 128x128 plans with >= this many tiles (layer4 3x3): one split
                                                 // (no slab round trip in the next launch: 4.532 -> 4.515 ms, profiles/r06_l4_onesplit.txt)
#endif
#ifndef POSE6D_WGRAD_F32_128_ONE_SPLIT_TILES
#define POSE6D_WGRAD_F32_128_ONE_SPLIT_TILES 0   // build-time (A/B): fp32 128x128 plans with >= this many tiles: one split
#endif
  if (POSE6D_WGRAD_F32_128_ONE_SPLIT_TILES > 0 && p.fast && dtype == POSE6D_DT_F32 && p.bm == 128 &&
      tiles >= POSE6D_WGRAD_F32_128_ONE_SPLIT_TILES)
    target = tiles;
#ifndef POSE6D_WGRAD_F32_128_TARGET
#define POSE6D_WGRAD_F32_128_TARGET 0   // build-time (A/B): workgroup target of the fp32 128x128 plans (0 = default)
#endif
  if (POSE6D_WGRAD_F32_128_TARGET > 0 && p.fast && dtype == POSE6D_DT_F32 && p.bm == 128)
    target = POSE6D_WGRAD_F32_128_TARGET;
#ifndef POSE6D_WGRAD_BF128_TARGET
#define POSE6D_WGRAD_BF128_TARGET 192   // workgroup target of the bf16 128x128 plans (0 = the KxK target, 256): fewer
                                        // slabs for the next launch to read back (profiles/r06_bf128_target.txt)
#endif
  if (POSE6D_WGRAD_BF128_TARGET > 0 && p.fast && dtype == POSE6D_DT_BF16 && p.bm == 128)
    target = POSE6D_WGRAD_BF128_TARGET;
  if (POSE6D_WGRAD_BF128_ONE_SPLIT_TILES > 0 && p.fast && dtype == POSE6D_DT_BF16 && p.bm == 128 &&
      tiles >= POSE6D_WGRAD_BF128_ONE_SPLIT_TILES)
    target = tiles;
#ifndef POSE6D_WGRAD_NARROW1X1_TARGET
#define POSE6D_WGRAD_NARROW1X1_TARGET 0   // build-time (A/B): target of the bf16 1x1 256 -> 64 weight gradients (layer1's
                                          // residual-junction convs; 0 = the 1x1 target)
#endif
  if (POSE6D_WGRAD_NARROW1X1_TARGET > 0 && p.fast && dtype == POSE6D_DT_BF16 && Kpad == SC && Cout == 64 &&
      Kpad >= 4 * Cout)
    target = POSE6D_WGRAD_NARROW1X1_TARGET;
  // aim for ~`target` workgroups, each reducing >= min_rows pixels, slabs capped in bytes
  int splits = p6::ceil_div(target, tiles);
  const int max_splits = p6::ceil_div(M, min_rows);
  if (splits > max_splits) splits = max_splits;
  const int64_t slab = (int64_t)Cout * Kpad * 4;
  const int max_by_bytes = (int)(max_bytes / slab);
  if (splits > max_by_bytes) splits = max_by_bytes;
  if (splits < 1) splits = 1;
  const int forced = tuned(tn, &pose6d_tuning_t::wgrad_splits, 0);   // tools: an explicit split count
  if (forced >= 1) splits = forced;
  int mps = p6::ceil_div(p6::ceil_div(M, splits), step) * step;
  splits = p6::ceil_div(M, mps);
  p.splits = splits;
  p.mps = mps;
  return p;
}

template <int S>
int launch_fast128(const WGeom& g, const void* x, const void* dy, float* ws, hipStream_t s, const ReduceJob& rj) {
  int lds = S * (128 + 128) * 128;
  if (lds < acc_stage_bytes<128, 128>()) lds = acc_stage_bytes<128, 128>();
  const int grid = g.gm * g.gn * g.splits + rj.nblk;
  if (g.KH == 1 && g.KW == 1 && g.stride == 1 && g.pad == 0)
    conv_wgrad_lds_kernel<S, true, false, 128><<<grid, 512, lds, s>>>((const bf16*)x, (const bf16*)dy, ws, g, rj);
  else
    conv_wgrad_lds_kernel<S, false, false, 128><<<grid, 512, lds, s>>>((const bf16*)x, (const bf16*)dy, ws, g, rj);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

template <int S>
int launch_fast(const WGeom& g, const void* x, const void* dy, float* ws, hipStream_t s,
                const ReduceJob& rj = ReduceJob{}) {
  static_assert(S * (64 + 64) * 128 >= acc_stage_bytes<64, 64>(), "ring too small to stage the tile");
  const int lds = S * (64 + 64) * 128;
  const int grid = g.gm * g.gn * g.splits + rj.nblk;
  if (g.kwp == p6::kRowTaps && g.SC == 4)
    conv_wgrad_lds_kernel<S, false, true><<<grid, kThreads, lds, s>>>((const bf16*)x, (const bf16*)dy, ws, g, rj);
  else if (g.KH == 1 && g.KW == 1 && g.stride == 1 && g.pad == 0)
    conv_wgrad_lds_kernel<S, true, false><<<grid, kThreads, lds, s>>>((const bf16*)x, (const bf16*)dy, ws, g, rj);
  else
    conv_wgrad_lds_kernel<S, false, false><<<grid, kThreads, lds, s>>>((const bf16*)x, (const bf16*)dy, ws, g, rj);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

int launch_fast_any(const Plan& p, const WGeom& g, const void* x, const void* dy, float* ws, hipStream_t s,
                    const ReduceJob& rj = ReduceJob{}) {
  if (p.bm == 128) return p.stages == 3 ? launch_fast128<3>(g, x, dy, ws, s, rj) : launch_fast128<2>(g, x, dy, ws, s, rj);
  return p.stages == 2 ? launch_fast<2>(g, x, dy, ws, s, rj)
       : p.stages == 3 ? launch_fast<3>(g, x, dy, ws, s, rj)
                       : launch_fast<4>(g, x, dy, ws, s, rj);
}

template <typename T, int BM, int BN>
int launch(const WGeom& g, const void* x, const void* dy, float* ws, hipStream_t s, const ReduceJob& rj) {
  const int ring = 2 * MT * (BM + BN) * (int)sizeof(T);
  int lds = ring > acc_stage_bytes<BM, BN>() ? ring : acc_stage_bytes<BM, BN>();
  if (lds < 256 * 16) lds = 256 * 16;   // the carried reduce's 256 float4
  conv_wgrad_kernel<T, BM, BN><<<g.gm * g.gn * g.splits + rj.nblk, kThreads, lds, s>>>((const T*)x, (const T*)dy,
                                                                                        ws, g, rj);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

template <typename T>
int launch_any(const WGeom& g, int bm, int bn, const void* x, const void* dy, float* ws, hipStream_t s,
               const ReduceJob& rj = ReduceJob{}) {
  if (bm == 128 && bn == 128) return launch<T, 128, 128>(g, x, dy, ws, s, rj);
  if (bm == 128) return launch<T, 128, 64>(g, x, dy, ws, s, rj);
  if (bn == 128) return launch<T, 64, 128>(g, x, dy, ws, s, rj);
  return launch<T, 64, 64>(g, x, dy, ws, s, rj);
}

int ilog2(int v) {
  int r = 0;
  while ((1 << r) < v) ++r;
  return (1 << r) == v ? r : -1;
}

}  // namespace

extern "C" int64_t pose6d_conv2d_wgrad_workspace_tuned(int32_t dtype, int32_t N, int32_t Ho, int32_t Wo, int32_t Cin,
                                                       int32_t Cout, int32_t KH, int32_t KW,
                                                       const pose6d_tuning_t* tuning) {
  const int bk = dtype == POSE6D_DT_BF16 ? 32 : 16;
  const int K = KH * KW * Cin;
  int64_t need = 0;
  {
    // (the stride is not an argument: a 1x1 conv may take the wide plan too (stride 2) --
    // report the larger of the two)
    const int Kpad = p6::ceil_div(K, bk) * bk;
    for (int wide = 0; wide < 2; ++wide) {
      const Plan p = plan(dtype, N * Ho * Wo, Cout, Kpad, Cin, tuning, false, wide != 0);
      const int64_t b = (int64_t)p.splits * Cout * Kpad * 4;
      if (b > need) need = b;
    }
  }
  // (the stride / padding are not arguments: a 4-channel stem may take the row-tap plan,
  // whose slabs are wider -- report the larger of the two)
  if (Cin == 4 && KH > 1 && KW <= p6::kRowTaps && Cout % 64 == 0) {
    const int Kpad = p6::ceil_div(KH * p6::kRowTaps * 4, 64) * 64;
    const Plan p = plan(dtype, N * Ho * Wo, Cout, Kpad, 64, tuning, true);
    const int64_t rt = (int64_t)p.splits * Cout * Kpad * 4;
    if (rt > need) need = rt;
  }
  return need;
}

extern "C" int64_t pose6d_conv2d_wgrad_workspace(int32_t dtype, int32_t N, int32_t Ho, int32_t Wo, int32_t Cin,
                                                 int32_t Cout, int32_t KH, int32_t KW) {
  return pose6d_conv2d_wgrad_workspace_tuned(dtype, N, Ho, Wo, Cin, Cout, KH, KW, nullptr);
}

namespace p6 {

WGeom wgrad_geom(int dtype, int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad, int Ho,
                 int Wo, WgradPlan* plan_out, const pose6d_tuning_t* tuning) {
  const int bk = dtype == POSE6D_DT_BF16 ? 32 : 16;
  WGeom g{};
  g.M = N * Ho * Wo; g.Cout = Cout; g.K = KH * KW * Cin; g.Kpad = ceil_div(g.K, bk) * bk;
  g.SH = H; g.SW = W; g.SC = Cin; g.log2SC = ilog2(Cin); g.RH = Ho; g.RW = Wo;
  g.KH = KH; g.KW = KW; g.stride = stride; g.pad = pad;
  g.kwp = KW;
  // the 4-channel stems: the LDS-DMA body on the row-tap X image (common.h), slabs in
  // row-tap K order (64-column blocks = two kernel rows); the reduce maps them to OIHW.
  // (bf16 fetches two pixels per 16-byte chunk: even W; fp32 one pixel per chunk)
  if (rowtap_geom(Cin, KH, KW, stride, pad) && Cout % 64 == 0 && (dtype == POSE6D_DT_F32 || (W & 1) == 0)) {
    const int Kpad = ceil_div(KH * kRowTaps * 4, 64) * 64;
    const Plan p = plan(dtype, g.M, Cout, Kpad, 64, tuning, true);   // (64: the LDS-DMA channel rule holds)
    if (p.fast) {
      g.kwp = kRowTaps;
      g.K = g.Kpad = Kpad;
      g.gm = ceil_div(Cout, p.bm); g.gn = ceil_div(g.Kpad, p.bn);
      g.splits = p.splits; g.mps = p.mps;
      if (plan_out) *plan_out = p;
      return g;
    }
  }
  const Plan p = plan(dtype, g.M, Cout, g.Kpad, Cin, tuning, false, KH * KW > 1 || stride > 1);
  g.gm = ceil_div(Cout, p.bm); g.gn = ceil_div(g.Kpad, p.bn);
  g.splits = p.splits; g.mps = p.mps;
  if (plan_out) *plan_out = p;
  return g;
}

int wgrad_reduce_launch(const float* ws, float* dw, int Cout, int Kpad, int SC, int Cin, int KH, int KW, int KWp,
                        int splits, int accumulate, hipStream_t s) {
  return launch_reduce(ws, dw, Cout, Kpad, SC, Cin, KH, KW, KWp, splits, accumulate, s);
}

int wgrad_launch_carry(int dtype, const WGeom& g, const WgradPlan& p, const void* x, const void* dy, float* ws,
                       const ReduceJob& rj, hipStream_t s) {
  if (p.fast && dtype == POSE6D_DT_BF16) return launch_fast_any(p, g, x, dy, ws, s, rj);
  if (p.fast) return launch_fast_f32_any(p, g, x, dy, ws, s, rj);
  return dtype == POSE6D_DT_BF16 ? launch_any<bf16>(g, p.bm, p.bn, x, dy, ws, s, rj)
                                 : launch_any<float>(g, p.bm, p.bn, x, dy, ws, s, rj);
}

}  // namespace p6

extern "C" int pose6d_conv2d_wgrad(int32_t dtype, const void* x, const void* dy, float* dw, int32_t accumulate,
                                   float* workspace, int64_t ws_bytes, int32_t N, int32_t H, int32_t W, int32_t Cin,
                                   int32_t Cin_real, int32_t Cout, int32_t KH, int32_t KW, int32_t stride,
                                   int32_t pad, int32_t Ho, int32_t Wo, void* stream) {
  return pose6d_conv2d_wgrad_tuned(dtype, x, dy, dw, accumulate, workspace, ws_bytes, N, H, W, Cin, Cin_real, Cout, KH,
                                   KW, stride, pad, Ho, Wo, nullptr, stream);
}

extern "C" int pose6d_conv2d_wgrad_tuned(int32_t dtype, const void* x, const void* dy, float* dw, int32_t accumulate,
                                         float* workspace, int64_t ws_bytes, int32_t N, int32_t H, int32_t W,
                                         int32_t Cin, int32_t Cin_real, int32_t Cout, int32_t KH, int32_t KW,
                                         int32_t stride, int32_t pad, int32_t Ho, int32_t Wo,
                                         const pose6d_tuning_t* tuning, void* stream) {
  P6_CHECK_ARG(dtype == POSE6D_DT_F32 || dtype == POSE6D_DT_BF16, "pose6d_conv2d_wgrad: bad dtype %d", dtype);
  P6_CHECK_ARG(ilog2(Cin) >= 2 && Cout % 8 == 0 && Cin_real <= Cin,
               "pose6d_conv2d_wgrad: Cin must be a power of two >= 4");
  Plan p;
  const WGeom g = p6::wgrad_geom(dtype, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, &p, tuning);
  P6_CHECK_ARG((int64_t)p.splits * Cout * g.Kpad * 4 <= ws_bytes,
               "pose6d_conv2d_wgrad: workspace %lld bytes < %lld needed (query pose6d_conv2d_wgrad_workspace[_tuned] "
               "with the same tuning)", (long long)ws_bytes, (long long)p.splits * Cout * g.Kpad * 4);
  hipStream_t s = p6::stream_of(stream);
  int rc;
  if (p.fast && dtype == POSE6D_DT_F32) {
    rc = launch_fast_f32_any(p, g, x, dy, workspace, s, ReduceJob{});
  } else if (p.fast) {
    rc = launch_fast_any(p, g, x, dy, workspace, s);
  } else {
    rc = dtype == POSE6D_DT_BF16 ? launch_any<bf16>(g, p.bm, p.bn, x, dy, workspace, s)
                                 : launch_any<float>(g, p.bm, p.bn, x, dy, workspace, s);
  }
  if (rc) return rc;
  return launch_reduce(workspace, dw, Cout, g.Kpad, Cin, Cin_real, KH, KW, g.kwp, g.splits, accumulate, s);
}

// weight-gradient kernel variant: (stages << 12) | (fast << 8) | (BM == 128) << 1 | (BN == 128)
extern "C" int pose6d_wgrad_variant(int32_t dtype, int32_t M, int32_t Cout, int32_t K, int32_t Cin) {
  const int bk = dtype == POSE6D_DT_BF16 ? 32 : 16;
  const Plan p = plan(dtype, M, Cout, p6::ceil_div(K, bk) * bk, Cin);
  return (p.stages << 12) | ((int)p.fast << 8) | ((p.bm == 128) << 1) | (p.bn == 128);
}

// Weight-gradient LDS-DMA body (bf16) shared by the standalone weight-gradient
// kernel (conv_wgrad.hip) and the fused data+weight gradient launch
// (conv_igemm.hip, pose6d_conv2d_backward).
#pragma once
#include "common.h"
#include "lds_dma.h"

// LDS ring depth of the bf16 weight-gradient kernel (standalone and inside the fused
// backward launch); build-time only, for A/B timing
#ifndef POSE6D_WGRAD_STAGES
#define POSE6D_WGRAD_STAGES 3
#endif
// LDS ring depth of the fp32 weight-gradient body (32 KiB stages): two slots keep two
// workgroups per CU resident
#ifndef POSE6D_WGRAD_STAGES_F32
#define POSE6D_WGRAD_STAGES_F32 2
#endif

namespace p6 {

struct WGeom {
  int M, Cout, K, Kpad;
  int SH, SW, SC, log2SC;
  int RH, RW;
  int KH, KW, stride, pad;
  int gm, gn, splits, mps;  // tiles over Cout, over K; splits; m per split (multiple of the step)
  int kwp;                  // taps per kernel row of the slab's K order: KW, or kRowTaps (bf16 row-tap stems)
};

struct WgradPlan {
  bool fast;
  int bm, bn, splits, mps, stages;
};

// a slab reduce carried by another launch (the next conv's backward: the fused bf16
// launch or the register-staged weight gradient), nblk extra workgroups
struct ReduceJob {
  const float* ws;
  float* dw;
  int Cout, Kpad, SC, Cin, KH, KW, KWp, splits, accumulate, G, nblk;
};

// defined in conv_wgrad.hip
WGeom wgrad_geom(int dtype, int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad, int Ho,
                 int Wo, WgradPlan* plan, const pose6d_tuning_t* tuning = nullptr);
int wgrad_reduce_launch(const float* ws, float* dw, int Cout, int Kpad, int SC, int Cin, int KH, int KW, int KWp,
                        int splits,
                        int accumulate, hipStream_t s);
// the register-staged weight gradient of plan `p` (not p.fast) with the carried
// reduce `rj` as its trailing workgroups; its own slabs are left for the caller to
// reduce (carried by the next launch or pose6d_wgrad_reduce)
int wgrad_launch_carry(int dtype, const WGeom& g, const WgradPlan& p, const void* x, const void* dy, float* ws,
                       const ReduceJob& rj, hipStream_t s);

}  // namespace p6

namespace {

// fp32 accumulator tile (4 waves as 2 x 2, each BM/2 x BN/2 of 16x16 MFMA tiles:
// lane (li, grp) holds rows 4 grp + r, column li) -> dst rows [0, BM) x cols [0, BN)
// (row stride ld), through LDS so the global stores are whole 16-byte vectors of
// contiguous columns: 4 (64x64) instead of 64 scattered dword stores per lane --
// the dword form made the weight-gradient slab epilogue store-issue bound.
// Entered after a barrier that ends every read of `smem`; needs BM * (BN + 16) * 4
// bytes of it.  CHECK: clip rows >= rows / cols >= cols (partial tiles).
template <int BM, int BN>
constexpr int acc_stage_bytes() { return BM * (BN + 16) * 4; }

template <int BM, int BN, bool CHECK, int NW = 4>
__device__ __forceinline__ void store_acc_tile(const f32x4 (&acc)[BM / 32][BN / (8 * NW)],
                                               char* smem, float* dst, int64_t ld, int rows, int cols) {
  // wave grid WM x WN = 2 x (NW / 2): each wave holds BM / WM rows x BN / WN columns
  constexpr int WM = 2, WN = NW / 2, NT = 64 * NW;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  constexpr int LDT = BN + 16;              // floats per LDS row: rows alternate 16-bank halves
  float* t = reinterpret_cast<float*>(smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int grp = lane >> 4, li = lane & 15;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        t[(wm * (BM / WM) + i * 16 + grp * 4 + r) * LDT + wn * (BN / WN) + j * 16 + li] = acc[i][j][r];
  __syncthreads();
  constexpr int CPR = BN / 4;               // float4 per row
  constexpr int RPP = NT / CPR;             // rows per pass
  const int c4 = tid % CPR, r0 = tid / CPR;
#pragma unroll
  for (int pass = 0; pass < BM / RPP; ++pass) {
    const int row = pass * RPP + r0;
    const float4 v = *reinterpret_cast<const float4*>(t + row * LDT + c4 * 4);
    if (CHECK && (row >= rows || c4 * 4 >= cols)) continue;
    *reinterpret_cast<float4*>(dst + (int64_t)row * ld + c4 * 4) = v;
  }
}

// ============================================================================
// Fast path (bf16, Cin a multiple of 64, Cout a multiple of 64): each stage is
// 64 pixels deep; dY [64 m][64 co] and X [64 m][64 k] sub-images (one filter tap,
// 64 contiguous channels per X row) are filled by LDS-DMA (8 rows x 128 B per
// wave instruction, XOR swizzle on the source chunk) through an S-slot ring with
// counted vmcnt + raw barriers, and read back transposed with ds_read_b64_tr_b16
// in one asm block per k-half (see lds_read_frags in conv_igemm.hip for why the
// reads are asm).  Rows past the split's end read the zero page.
// ============================================================================
__device__ __forceinline__ int swz_tr4(int r) { return ((((r >> 1) & 1) | (((r >> 3) & 1) << 1)) << 1); }

typedef __attribute__((ext_vector_type(2))) unsigned u32x2;

// 2 * NF transposed reads (NF operands of 8 m each) + lgkmcnt(0), as one asm block
template <int NF>
__device__ __forceinline__ void lds_read_tr_frags(u32x2 (&f)[2 * NF], const unsigned (&a)[2 * NF]) {
  static_assert(NF == 2 || NF == 4, "2 or 4 operands per batch");
  if constexpr (NF == 2) {
    asm volatile(
        "ds_read_b64_tr_b16 %0, %4\n\tds_read_b64_tr_b16 %1, %5\n\tds_read_b64_tr_b16 %2, %6\n\t"
        "ds_read_b64_tr_b16 %3, %7\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3])
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]));
  } else {
    asm volatile(
        "ds_read_b64_tr_b16 %0, %8\n\tds_read_b64_tr_b16 %1, %9\n\tds_read_b64_tr_b16 %2, %10\n\t"
        "ds_read_b64_tr_b16 %3, %11\n\tds_read_b64_tr_b16 %4, %12\n\tds_read_b64_tr_b16 %5, %13\n\t"
        "ds_read_b64_tr_b16 %6, %14\n\tds_read_b64_tr_b16 %7, %15\n\ts_waitcnt lgkmcnt(0)"
        : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3]), "=&v"(f[4]), "=&v"(f[5]), "=&v"(f[6]), "=&v"(f[7])
        : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]));
  }
}

// the 4-operand batch without its wait (lds_wait_tr8 releases it), so other work
// can be issued while the reads are in flight
__device__ __forceinline__ void lds_issue_tr8(u32x2 (&f)[8], const unsigned (&a)[8]) {
  asm volatile(
      "ds_read_b64_tr_b16 %0, %8\n\tds_read_b64_tr_b16 %1, %9\n\tds_read_b64_tr_b16 %2, %10\n\t"
      "ds_read_b64_tr_b16 %3, %11\n\tds_read_b64_tr_b16 %4, %12\n\tds_read_b64_tr_b16 %5, %13\n\t"
      "ds_read_b64_tr_b16 %6, %14\n\tds_read_b64_tr_b16 %7, %15"
      : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3]), "=&v"(f[4]), "=&v"(f[5]), "=&v"(f[6]), "=&v"(f[7])
      : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]), "v"(a[4]), "v"(a[5]), "v"(a[6]), "v"(a[7]));
}
__device__ __forceinline__ void lds_wait_tr8(u32x2 (&f)[8]) {
  asm volatile("s_waitcnt lgkmcnt(0)"
               : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7]));
}

// one workgroup's work; `bid` = its index in the weight-gradient sub-grid (whose
// size is a multiple of 8 or the whole grid, so bid & 7 is its XCD), `smem` = the
// kernel's dynamic LDS
// PW: pointwise conv (1x1, stride 1, no padding) -- X rows are the output pixels
// themselves, so every operand row advances by a constant stride per 64-pixel stage
// and only the split's last stage can run past its end: the per-stage issue is a
// pointer increment and one compare per row instead of the general (n, oy, ox)
// walk with per-row padding checks (which left the 1x1 weight gradients issue
// bound: ~1200 issue cycles per wave per K-step against 128 of MFMA)
// RT: the row-tap X image (the 4-channel 7x7 / stride-2 stems, common.h): sub-image
// s of a stage is the slab's K columns [k0 + 64 s, + 64) = two kernel rows x 8 taps x 4
// channels, i.e. each X row is two 64-byte runs of 8 input pixels
// NW: waves per workgroup, as a 2 x NW/2 grid over the (BM co) x (BN k) tile -- 4 (64x64
// tiles: 32 x 32 per wave) or 8 (128x128 tiles: 64 x 32 per wave, twice the MACs per
// staged byte of the 64x64 tile and half the DMA instructions per wave per byte)
template <int BM, int BN, int S, bool PW = false, bool RT = false, int NW = 4>
__device__ __forceinline__ void conv_wgrad_lds_body(char* smem, int bid, const bf16* __restrict__ x,
                                                    const bf16* __restrict__ dy, float* __restrict__ ws,
                                                    const p6::WGeom& g) {
  constexpr int MS = 64;                          // pixels per stage
  constexpr int YS = BM / 64, XS = BN / 64;       // 64-column sub-images per operand
  constexpr int RI = 64 / (8 * NW);               // DMA rows of a sub-image per thread (8 rows per wave instruction)
  constexpr int LOADS = RI * (YS + XS);           // DMA instructions per thread per stage
  constexpr int SUB = MS * 128;                   // bytes per sub-image
  constexpr int STAGE = (YS + XS) * SUB;
  constexpr int WM = 2, WN = NW / 2;
  constexpr int TM = BM / (16 * WM), TN = BN / (16 * WN);
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert((TM + TN) % 2 == 0 && TM + TN <= 8, "fragment batches of 2 or 4 operands");

  const int tiles = g.gm * g.gn;
  const int nwg = tiles * g.splits;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int split = bid / tiles;   // all tiles of one pixel range share an XCD's L2
  const int t2 = bid - split * tiles;
  const int tm = t2 / g.gn, tn = t2 - tm * g.gn;
  const int co0 = tm * BM, k0 = tn * BN;
  const int mbeg = split * g.mps;
  const int mend = min(g.M, mbeg + g.mps);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave / WN, wn = wave % WN;
  const int r8 = lane >> 3, pch = lane & 7;
  const char* zp = reinterpret_cast<const char*>(g_zero_page);
  constexpr bool pointwise = PW;

  // each thread DMAs rows R = i * 8 NW + wave * 8 + r8 (i < RI) of every sub-image;
  // the logical chunk it fetches carries the row's swizzle
  int ck[RI];
#pragma unroll
  for (int i = 0; i < RI; ++i) ck[i] = (pch ^ swz_tr4(i * 8 * NW + wave * 8 + r8)) * 8;
  int tap_h[XS], tap_w[XS], ci0[XS];
#pragma unroll
  for (int s = 0; s < XS; ++s) {
    const int kk0 = k0 + s * 64;
    const int tap = kk0 >> g.log2SC;
    ci0[s] = kk0 & (g.SC - 1);
    tap_h[s] = tap / g.KW;
    tap_w[s] = tap - tap_h[s] * g.KW;
  }
  // output-pixel coordinates of this lane's two DMA rows, advanced by 64 pixels per
  // stage without divisions (issue() is called with consecutive st)
  const int hw = g.RH * g.RW;
  const int step_y = MS / g.RW, step_x = MS - step_y * g.RW;
  int rn[RI], roy[RI], rox[RI];
  if (!pointwise) {
#pragma unroll
    for (int i = 0; i < RI; ++i) {
      const int m = mbeg + i * 8 * NW + wave * 8 + r8;
      rn[i] = m / hw;
      const int rem = m - rn[i] * hw;
      roy[i] = rem / g.RW;
      rox[i] = rem - roy[i] * g.RW;
    }
  }

  // pointwise: per-row operand pointers advanced by a stage each issue
  const bf16* pw_y[RI][YS];
  const bf16* pw_x[RI][XS];
  int pw_m[RI];
  if constexpr (PW) {
#pragma unroll
    for (int i = 0; i < RI; ++i) {
      const int m = mbeg + i * 8 * NW + wave * 8 + r8;
      pw_m[i] = m;
#pragma unroll
      for (int s_ = 0; s_ < YS; ++s_) pw_y[i][s_] = dy + (int64_t)m * g.Cout + co0 + s_ * 64 + ck[i];
#pragma unroll
      for (int s_ = 0; s_ < XS; ++s_) pw_x[i][s_] = x + ((int64_t)m << g.log2SC) + ci0[s_] + ck[i];
    }
  }
  const int64_t y_step = (int64_t)MS * g.Cout, x_step = (int64_t)MS << g.log2SC;

  auto issue = [&](int st, int buf) {
    char* base = smem + buf * STAGE;
    if constexpr (PW) {
#pragma unroll
      for (int i = 0; i < RI; ++i) {
        const bool ok = pw_m[i] < mend;
#pragma unroll
        for (int s_ = 0; s_ < YS; ++s_)
          glds16(ok ? (const void*)pw_y[i][s_] : (const void*)zp, base + s_ * SUB + (i * 8 * NW + wave * 8) * 128);
#pragma unroll
        for (int s_ = 0; s_ < XS; ++s_)
          glds16(ok ? (const void*)pw_x[i][s_] : (const void*)zp,
                 base + (YS + s_) * SUB + (i * 8 * NW + wave * 8) * 128);
        pw_m[i] += MS;
#pragma unroll
        for (int s_ = 0; s_ < YS; ++s_) pw_y[i][s_] += y_step;
#pragma unroll
        for (int s_ = 0; s_ < XS; ++s_) pw_x[i][s_] += x_step;
      }
      (void)st;
      return;
    }
#pragma unroll
    for (int i = 0; i < RI; ++i) {
      const int R = i * 8 * NW + wave * 8 + r8;
      const int m = mbeg + st * MS + R;
      const bool ok = m < mend;
#pragma unroll
      for (int s = 0; s < YS; ++s) {
        const void* p = ok ? (const void*)(dy + (int64_t)m * g.Cout + co0 + s * 64 + ck[i]) : (const void*)zp;
        glds16(p, base + s * SUB + (i * 8 * NW + wave * 8) * 128);
      }
      int sy = 0, sx = 0;
      if (!pointwise) {
        sy = roy[i] * g.stride - g.pad;
        sx = rox[i] * g.stride - g.pad;
      }
#pragma unroll
      for (int s = 0; s < XS; ++s) {
        const void* p = zp;
        if constexpr (RT) {
          // this lane's chunk (8 elements = 2 taps x 4 channels) of K column block s
          const int ke = k0 + s * 64 + ck[i];
          const int kr = ke >> 5, yy = sy + kr, xx = sx - (p6::kRowTaps - g.KW) + ((ke & 31) >> 2);
          if (ok && kr < g.KH && (unsigned)yy < (unsigned)g.SH && (unsigned)xx < (unsigned)g.SW)
            p = x + ((((int64_t)rn[i] * g.SH + yy) * g.SW + xx) << 2);
        } else if (pointwise) {
          if (ok) p = x + ((int64_t)m << g.log2SC) + ci0[s] + ck[i];
        } else {
          const int yy = sy + tap_h[s], xx = sx + tap_w[s];
          if (ok && (unsigned)yy < (unsigned)g.SH && (unsigned)xx < (unsigned)g.SW)
            p = x + ((((int64_t)rn[i] * g.SH + yy) * g.SW + xx) << g.log2SC) + ci0[s] + ck[i];
        }
        glds16(p, base + (YS + s) * SUB + (i * 8 * NW + wave * 8) * 128);
      }
      if (!pointwise) {
        rox[i] += step_x;
        roy[i] += step_y;
        if (rox[i] >= g.RW) { rox[i] -= g.RW; ++roy[i]; }
        while (roy[i] >= g.RH) { roy[i] -= g.RH; ++rn[i]; }
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // transposed-read byte offsets in a slot: operand o, half h, k-half kk
  const int grp = lane >> 4, li = lane & 15, q = li >> 2, p = li & 3;
  unsigned off[2][2 * (TM + TN)];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int o = 0; o < TM + TN; ++o)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bool isy = o < TM;
        const int col = isy ? wm * (BM / WM) + o * 16 + 4 * p : wn * (BN / WN) + (o - TM) * 16 + 4 * p;
        const int sub = (isy ? 0 : YS) + (col >> 6), lc = col & 63;
        const int r = 32 * kk + 8 * grp + 4 * h + q;
        off[kk][2 * o + h] = sub * SUB + r * 128 + (((lc >> 3) ^ swz_tr4(r)) << 4) + (lc & 7) * 2;
      }
  const unsigned ring = lds_addr(smem);
  // mid(): the next stage's LDS-DMA issue, placed while the first fragment batch is in flight
  auto compute = [&](int buf, auto&& mid) {
    const unsigned slot = ring + buf * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      u32x2 f[2 * (TM + TN)];
      constexpr int NB = (TM + TN) % 4 == 0 ? 4 : 2;   // operands per asm batch
#pragma unroll
      for (int b0 = 0; b0 < TM + TN; b0 += NB) {
        unsigned a[2 * NB];
        u32x2 t[2 * NB];
#pragma unroll
        for (int u = 0; u < 2 * NB; ++u) a[u] = slot + off[kk][2 * b0 + u];
        if (kk == 0 && b0 == 0) {
          if constexpr (NB == 4) {
            lds_issue_tr8(t, a);
            mid();
            lds_wait_tr8(t);
          } else {
            mid();
            lds_read_tr_frags<2>(t, a);
          }
        } else if constexpr (NB == 4) {
          lds_read_tr_frags<4>(t, a);
        } else {
          lds_read_tr_frags<2>(t, a);
        }
#pragma unroll
        for (int u = 0; u < 2 * NB; ++u) f[2 * b0 + u] = t[u];
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const u32x4 av = {f[2 * i].x, f[2 * i].y, f[2 * i + 1].x, f[2 * i + 1].y};
          const u32x4 bv = {f[2 * (TM + j)].x, f[2 * (TM + j)].y, f[2 * (TM + j) + 1].x, f[2 * (TM + j) + 1].y};
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, av),
                                                              __builtin_bit_cast(bf16x8, bv), acc[i][j], 0, 0, 0);
        }
    }
  };

  const int nk = (mend - mbeg + MS - 1) / MS;
  for (int s = 0; s < S - 1 && s < nk; ++s) issue(s, s);
  int cur = 0, wbuf = S - 1;
  for (int kt = 0; kt < nk; ++kt) {
    const int left = nk - 1 - kt;
    wait_ahead<LOADS, S - 2>(left < S - 2 ? left : S - 2);
    compute(cur, [&]() {
      if (kt + S - 1 < nk) issue(kt + S - 1, wbuf);
    });
    cur = cur == S - 1 ? 0 : cur + 1;
    wbuf = wbuf == S - 1 ? 0 : wbuf + 1;
  }

  // every wave is done reading the ring (and every DMA has landed: the last
  // wait_ahead waited for all of them) before the tile is staged over it
  asm volatile("s_barrier" ::: "memory");
  float* slab = ws + (int64_t)split * g.Cout * g.Kpad;
  store_acc_tile<BM, BN, false, NW>(acc, smem, slab + (int64_t)co0 * g.Kpad + k0, g.Kpad, BM, BN);
}


// ============================================================================
// fp32 weight gradient on the LDS-DMA path (exact v_mfma_f32_16x16x4_f32): the
// reference-precision training step's weight gradients (train_rgbd_geometric.py:106-112
// trains in fp32).  64 (co) x 64 (k) tile on 4 waves (2 x 2, each 32 x 32 = 2 x 2
// MFMA tiles); a stage is MS output pixels deep: dY [MS m][64 co] and X [MS m][64 k]
// fp32 images, 256-byte rows, filled by LDS-DMA (one wave instruction = 4 rows), the
// 16-byte chunk of odd rows XOR 4 (applied on the source address: the LDS side of
// LDS-DMA is lane-linear).  The contraction runs over m, which is the ROW index of
// both images, so an MFMA operand is one float per lane: A[i][k] = dY[m0 + k][co + i]
// (lane i = l % 16, k = l / 16) -- four rows per 32-lane LDS group, conflict-free
// under the swizzle (ds_read_b32 banks are (a / 4) mod 32).  The reads are inline asm
// (hipcc would otherwise wait for the whole DMA ring before every LDS read), issued a
// group of 4 m ahead of the MFMAs that consume them with counted lgkmcnt waits.
// Replaces the register-staged conv_wgrad_kernel<float> (global loads -> VGPRs ->
// ds_write -> __syncthreads per stage) on every fp32 conv with Cin, Cout multiples of 64.
// ============================================================================
template <int MS, int BT = 64>
struct WgF32 {
  static constexpr int ROWB = BT * 4;                // bytes per image row (BT fp32)
  static constexpr int CPR = ROWB / 16;              // 16-byte chunks per row
  static constexpr int RPI = 1024 / ROWB;            // rows per DMA wave instruction
  static constexpr int IMG = MS * ROWB;              // bytes per image
  static constexpr int STAGE = 2 * IMG;              // dY image, then X image
  static constexpr int INS = MS / RPI;               // DMA instructions per image per stage
  static constexpr int PER = INS / 4;                // ... per wave (4 waves)
  static constexpr int LOADS = 2 * PER;              // DMA instructions per wave per stage
  static constexpr int TT = BT / 32;                 // 16x16 MFMA tiles per wave and dimension
  static_assert(BT == 64 || BT == 128, "BT: 64 or 128");
  static_assert(PER * 4 == INS && MS % 16 == 0, "MS: a multiple of 16 pixels");
};

// the 8 operand reads (2 A + 2 B floats for each of two m-groups) of one MFMA group
// pair, as one asm batch without a wait
__device__ __forceinline__ void lds_read_b32x4(float (&f)[4], const unsigned (&a)[4]) {
  asm volatile("ds_read_b32 %0, %4\n\tds_read_b32 %1, %5\n\tds_read_b32 %2, %6\n\tds_read_b32 %3, %7"
               : "=&v"(f[0]), "=&v"(f[1]), "=&v"(f[2]), "=&v"(f[3])
               : "v"(a[0]), "v"(a[1]), "v"(a[2]), "v"(a[3]));
}
// wait until at most N LDS reads are outstanding; the operands of the group just
// landed are redefined after the wait (no MFMA consuming them moves above it)
template <int N>
__device__ __forceinline__ void lds_wait_b32x4(float (&f)[4]) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]) : "n"(N));
}

// RT: the fp32 row-tap stem (Cin = 4, 7x7 / stride 2): the 64-wide k tile is two kernel
// rows of 8 taps x 4 channels (common.h rowtap_geom), one fetched chunk = one pixel
template <int MS, int S, bool PW, int BT = 64, bool RT = false>
__device__ __forceinline__ void conv_wgrad_lds_body_f32(char* smem, int bid, const float* __restrict__ x,
                                                        const float* __restrict__ dy, float* __restrict__ ws,
                                                        const p6::WGeom& g) {
  using C = WgF32<MS, BT>;
  constexpr int PER = C::PER, LOADS = C::LOADS, STAGE = C::STAGE, IMG = C::IMG, TT = C::TT;
  const int tiles = g.gm * g.gn;
  const int nwg = tiles * g.splits;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  const int split = bid / tiles;   // all tiles of one pixel range share an XCD's L2
  const int t2 = bid - split * tiles;
  const int tm = t2 / g.gn, tn = t2 - tm * g.gn;
  const int co0 = tm * BT, k0 = tn * BT;
  const int mbeg = split * g.mps;
  const int mend = min(g.M, mbeg + g.mps);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const char* zp = reinterpret_cast<const char*>(g_zero_page);
  // the BT-wide k tile lies in one filter tap (SC % BT == 0)
  const int tap = k0 >> g.log2SC, ci0 = k0 & (g.SC - 1);
  const int tkh = tap / g.KW, tkw = tap - tkh * g.KW;
  // DMA rows of this lane: instruction j (j = i * 4 + wave) covers rows RPI j .. RPI j +
  // RPI - 1, the lane row RPI j + lane / CPR, chunk (lane % CPR) ^ (4 * odd row) of the row
  const int rsub = lane / C::CPR;
  const int ck = ((lane % C::CPR) ^ ((rsub & 1) << 2)) * 4;   // element offset of the fetched chunk
  static_assert(!RT || (BT == 64 && !PW), "row-tap: 64-wide tiles");
  // row-tap: kernel row and x offset of this lane's chunk (tap kw' = kw + 8 - KW)
  const int rt_kr = (k0 + ck) >> 5, rt_dx = (((k0 + ck) & 31) >> 2) - (p6::kRowTaps - g.KW);
  int rm[PER], rn[PER], roy[PER], rox[PER];
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int m = mbeg + C::RPI * (i * 4 + wave) + rsub;
    rm[i] = m;
    const int hw = g.RH * g.RW;
    rn[i] = m / hw;
    const int rem = m - rn[i] * hw;
    roy[i] = rem / g.RW;
    rox[i] = rem - roy[i] * g.RW;
  }
  const int step_y = MS / g.RW, step_x = MS - step_y * g.RW;
  auto issue = [&](int buf) {
    char* base = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int j = i * 4 + wave;
      const bool ok = rm[i] < mend;
      const void* py = ok ? (const void*)(dy + (int64_t)rm[i] * g.Cout + co0 + ck) : (const void*)zp;
      glds16(py, base + j * 1024);
      const void* px = zp;
      if (PW) {
        if (ok) px = x + ((int64_t)rm[i] << g.log2SC) + ci0 + ck;
      } else if (RT) {
        const int yy = roy[i] * g.stride - g.pad + rt_kr, xx = rox[i] * g.stride - g.pad + rt_dx;
        if (ok && rt_kr < g.KH && (unsigned)yy < (unsigned)g.SH && (unsigned)xx < (unsigned)g.SW)
          px = x + ((((int64_t)rn[i] * g.SH + yy) * g.SW + xx) << 2);
      } else {
        const int yy = roy[i] * g.stride - g.pad + tkh, xx = rox[i] * g.stride - g.pad + tkw;
        if (ok && (unsigned)yy < (unsigned)g.SH && (unsigned)xx < (unsigned)g.SW)
          px = x + ((((int64_t)rn[i] * g.SH + yy) * g.SW + xx) << g.log2SC) + ci0 + ck;
      }
      glds16(px, base + IMG + j * 1024);
      rm[i] += MS;
      if (!PW) {
        rox[i] += step_x;
        roy[i] += step_y;
        if (rox[i] >= g.RW) { rox[i] -= g.RW; ++roy[i]; }
        while (roy[i] >= g.RH) { roy[i] -= g.RH; ++rn[i]; }
      }
    }
  };

  f32x4 acc[TT][TT];
#pragma unroll
  for (int i = 0; i < TT; ++i)
#pragma unroll
    for (int j = 0; j < TT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // operand addresses: m-group q (rows 4q .. 4q+3), lane row 4q + (lane >> 4), column c
  // of the image at chunk (c >> 2) ^ (4 * odd row)
  const int li = lane & 15, kq = lane >> 4;
  // NB = 4-float read batches per group: TT A floats, then TT B floats
  constexpr int NB = TT / 2;
  unsigned off[2 * TT];
#pragma unroll
  for (int t = 0; t < TT; ++t) {
    const int ca = wm * (BT / 2) + t * 16 + li, cb = wn * (BT / 2) + t * 16 + li;
    off[t] = kq * C::ROWB + ((((ca >> 2) ^ ((kq & 1) << 2)) << 2) + (ca & 3)) * 4;
    off[TT + t] = IMG + kq * C::ROWB + ((((cb >> 2) ^ ((kq & 1) << 2)) << 2) + (cb & 3)) * 4;
  }
  const unsigned ring = lds_addr(smem);
  // one stage: MS / 4 m-groups of TT x TT MFMAs; operands of group q + 1 read while
  // group q's MFMAs run (counted waits)
  auto compute = [&](int buf, auto&& mid) {
    const unsigned slot = ring + buf * STAGE;
    constexpr int NQ = MS / 4;
    // three register sets: a set is refilled two groups after its last use
    float f[3][NB][4];
    auto rd = [&](int q, float (&d)[NB][4]) {
      const unsigned rq = slot + q * 4 * C::ROWB;
#pragma unroll
      for (int b = 0; b < NB; ++b) {
        const unsigned a[4] = {rq + off[4 * b], rq + off[4 * b + 1], rq + off[4 * b + 2], rq + off[4 * b + 3]};
        lds_read_b32x4(d[b], a);
      }
    };
    rd(0, f[0]);
    mid();   // the next stage's DMA issue overlaps the first reads' latency
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      float (&cur)[NB][4] = f[q % 3];
      if (q + 1 < NQ) {
        rd(q + 1, f[(q + 1) % 3]);
#pragma unroll
        for (int b = 0; b < NB; ++b) lds_wait_b32x4<4 * NB>(cur[b]);
      } else {
#pragma unroll
        for (int b = 0; b < NB; ++b) lds_wait_b32x4<0>(cur[b]);
      }
#pragma unroll
      for (int i = 0; i < TT; ++i)
#pragma unroll
        for (int j = 0; j < TT; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(cur[i >> 2][i & 3], cur[(TT + j) >> 2][(TT + j) & 3],
                                                          acc[i][j], 0, 0, 0);
    }
  };

  const int nk = (mend - mbeg + MS - 1) / MS;
  for (int s = 0; s < S - 1 && s < nk; ++s) issue(s);
  int cur = 0, wbuf = S - 1;
  for (int kt = 0; kt < nk; ++kt) {
    const int left = nk - 1 - kt;
    wait_ahead<LOADS, S - 2>(left < S - 2 ? left : S - 2);
    compute(cur, [&]() {
      if (kt + S - 1 < nk) issue(wbuf);
    });
    cur = cur == S - 1 ? 0 : cur + 1;
    wbuf = wbuf == S - 1 ? 0 : wbuf + 1;
  }
  asm volatile("s_barrier" ::: "memory");
  float* slab = ws + (int64_t)split * g.Cout * g.Kpad;
  store_acc_tile<BT, BT, false>(acc, smem, slab + (int64_t)co0 * g.Kpad + k0, g.Kpad, BT, BT);
}

// sum the split slabs (fixed order) into the OIHW fp32 gradient; k = (kh, kw, ci).
// Block = L float4 lanes (4 consecutive k each) x G split groups: group g sums
// slabs g, g + G, ... with U loads in flight, then the G partials are combined in
// LDS in group order (deterministic).  G is picked so that small gradients with
// hundreds of splits still spread their reads over many lanes.  `blk` = this
// workgroup's index among the reduce's workgroups; `red` = 256 float4 of LDS.
template <int G>
__device__ __forceinline__ void wgrad_reduce_body(float4* red, int blk, const float* __restrict__ ws,
                                                  float* __restrict__ dw, int Cout, int Kpad, int SC, int Cin, int KH,
                                                  int KW, int KWp, int splits, int accumulate) {
  constexpr int L = 256 / G;
  constexpr int U = 4;
  const int lane = threadIdx.x % L, grp = threadIdx.x / L;
  const int64_t e0 = ((int64_t)blk * L + lane) * 4;   // first of 4 consecutive (co, k) elements
  const int64_t total = (int64_t)Cout * Kpad;
  const bool ok = e0 < total;
  const int64_t slab = total;
  float4 acc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ok) {
    const float* p = ws + e0;
    int i = grp;
    for (; i + (U - 1) * G < splits; i += U * G) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = *reinterpret_cast<const float4*>(p + (int64_t)(i + u * G) * slab);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        acc[u].x += v[u].x; acc[u].y += v[u].y; acc[u].z += v[u].z; acc[u].w += v[u].w;
      }
    }
    for (; i < splits; i += G) {
      const float4 v = *reinterpret_cast<const float4*>(p + (int64_t)i * slab);
      acc[0].x += v.x; acc[0].y += v.y; acc[0].z += v.z; acc[0].w += v.w;
    }
  }
  float4 t = acc[0];
#pragma unroll
  for (int u = 1; u < U; ++u) { t.x += acc[u].x; t.y += acc[u].y; t.z += acc[u].z; t.w += acc[u].w; }
  red[grp * L + lane] = t;
  __syncthreads();
  if (grp == 0 && ok) {
#pragma unroll
    for (int g = 1; g < G; ++g) { const float4 v = red[g * L + lane]; t.x += v.x; t.y += v.y; t.z += v.z; t.w += v.w; }
    const float tv[4] = {t.x, t.y, t.z, t.w};
    const int co = (int)(e0 / Kpad), k0 = (int)(e0 - (int64_t)co * Kpad);
    // slab K order (kh, kw', ci) with KWp taps kw' per kernel row, filter tap kw = kw' - (KWp - KW)
    const int kwp = KWp > 0 ? KWp : KW;
    const int K = KH * kwp * SC;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int k = k0 + j;
      if (k >= K) continue;
      const int tap = k / SC, ci = k - tap * SC;
      if (ci >= Cin) continue;
      const int kh = tap / kwp, kw = tap - kh * kwp - (kwp - KW);
      if (kw < 0) continue;
      float* d = dw + (((int64_t)co * Cin + ci) * KH + kh) * KW + kw;
      *d = accumulate ? *d + tv[j] : tv[j];
    }
  }
}

using p6::ReduceJob;

__host__ __device__ inline int reduce_group(int splits) { return splits >= 64 ? 16 : splits >= 16 ? 4 : 1; }
__host__ __device__ inline int reduce_blocks(int Cout, int Kpad, int G) {
  const int64_t quads = (int64_t)Cout * Kpad / 4;
  const int L = 256 / G;
  return (int)((quads + L - 1) / L);
}

__device__ __forceinline__ void run_reduce_job(char* smem, int blk, const ReduceJob& j) {
  float4* red = reinterpret_cast<float4*>(smem);
  if (j.G == 16) wgrad_reduce_body<16>(red, blk, j.ws, j.dw, j.Cout, j.Kpad, j.SC, j.Cin, j.KH, j.KW, j.KWp, j.splits,
                                       j.accumulate);
  else if (j.G == 4) wgrad_reduce_body<4>(red, blk, j.ws, j.dw, j.Cout, j.Kpad, j.SC, j.Cin, j.KH, j.KW, j.KWp,
                                          j.splits, j.accumulate);
  else wgrad_reduce_body<1>(red, blk, j.ws, j.dw, j.Cout, j.Kpad, j.SC, j.Cin, j.KH, j.KW, j.KWp, j.splits,
                            j.accumulate);
}

}  // namespace

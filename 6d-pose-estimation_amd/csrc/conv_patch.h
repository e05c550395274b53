// 3x3 stride-1 convolution with the input patch staged ONCE per 64-channel slice
// (included by conv_igemm.hip inside its anonymous namespace; uses its Geom,
// conv_epilogue, lds_issue_frags8 and the LDS-DMA helpers of lds_dma.h).
//
// The implicit-GEMM kernel (conv_lds_body) streams the A operand once per filter
// tap: every input pixel crosses L2 -> LDS nine times, so a layer3 3x3 conv at
// batch 32 moves 231 MB through the CUs' load path for 3.2 MB of input and runs
// at ~15 % of the MFMA peak, bound by that stream.  Here a workgroup owns whole
// image rows (a tile = R full output rows of one image, or IPT whole images), so
// the input pixels its nine taps read form one rectangular patch with a one-pixel
// halo: per 64-channel slice the patch is DMA'd once into LDS and every tap reads
// its A fragments from it at a pixel offset (kh * PW + kw).  Only the weights are
// still streamed per tap (one 64 x 64 slice = 8 KiB per K-step).  Traffic per
// 64-channel slice of a 128 x 64 tile: 24-32 KiB patch + 72 KiB weights, against
// 9 x (16 + 8) KiB for the implicit GEMM's 128-row A images + weights.
//
// Tile: BM = 128 GEMM rows (tile-local output pixels; rows past the tile's BM_eff
// compute garbage that the epilogue masks), BN = 64 output channels, 8 waves
// (4 x 2, each 32 x 32 = 2 x 2 MFMA 16x16x32 tiles, the paired-fragment reads of
// conv_lds_body).  K order: slice-major (for each 64-channel slice: taps 0..8) --
// its own summation order, used for every call of a patch-eligible geometry
// without BatchNorm statistics (pose6d_conv2d_fwd with stats == NULL and
// pose6d_conv2d_fwd_act), so the fused eval epilogue stays bit-identical to the
// separate launches.
//
// Pipeline: K-step s = (slice c, tap t); unit U(s) = the weight slice of step s
// (one DMA instruction per wave) plus, when t == 8 and a next slice exists, the
// next slice's patch (PI instructions per wave) into the other patch buffer.  U(s)
// is issued S-1 steps ahead; the counted wait before step s leaves exactly the
// younger units in flight (their per-wave counts are known: 1 or 1 + PI), then a
// raw s_barrier publishes the landed bytes to every wave.  The next slice's patch
// lands one step before its first use; its buffer was last read 9 - S + 1 steps
// before the DMA is issued (S <= 9).

constexpr int kPatchBM = 128, kPatchBN = 64, kPatchNW = 8, kPatchPIMax = 4;

// patch plan of one forward conv (host): tile rows R (IPT == 1) or images per tile
struct PatchPlan {
  bool ok;
  int R, IPT, tpi, tiles, PW, P, PI, bufs, lds;
};

inline PatchPlan patch_plan(int N, int H, int W, int C, int Cout, int S) {
  PatchPlan p{};
  if (W < 1 || W > kPatchBM || C % 64 != 0 || Cout % kPatchBN != 0) return p;
  p.PW = W + 2;
  if (H * W * 2 <= kPatchBM) {   // whole images per tile
    p.IPT = kPatchBM / (H * W);
    p.R = H;
    p.tpi = 1;
    p.tiles = p6::ceil_div(N, p.IPT);
    p.P = p.IPT * (H + 2) * p.PW;
  } else {
    p.IPT = 1;
    p.R = kPatchBM / W < H ? kPatchBM / W : H;
    p.tpi = p6::ceil_div(H, p.R);
    p.tiles = N * p.tpi;
    p.P = (p.R + 2) * p.PW;
  }
  p.PI = p6::ceil_div(p6::ceil_div(p.P, 8), kPatchNW);
  if (p.PI > kPatchPIMax) return p;
  p.bufs = C / 64 > 1 ? 2 : 1;
  p.lds = p.bufs * p.PI * kPatchNW * 1024 + S * kPatchBN * 128;
  const int epi = kPatchBM * (kPatchBN * 2 + 16);
  if (p.lds < epi) p.lds = epi;
  p.ok = p.lds <= 160 * 1024;
  return p;
}

struct PatchGeom {
  int N, H, W, C, R, IPT, tpi, PW, P, PI, bufs, nslices;
};

// wait until at most n DMA instructions of this wave are in flight, then barrier
// (n is wave-uniform: a scalar switch over immediates)
__device__ __forceinline__ void vm_wait_barrier(int n) {
  switch (n) {
    case 0: vmcnt_barrier<0>(); break;
    case 1: vmcnt_barrier<1>(); break;
    case 2: vmcnt_barrier<2>(); break;
    case 3: vmcnt_barrier<3>(); break;
    case 4: vmcnt_barrier<4>(); break;
    case 5: vmcnt_barrier<5>(); break;
    case 6: vmcnt_barrier<6>(); break;
    case 7: vmcnt_barrier<7>(); break;
    case 8: vmcnt_barrier<8>(); break;
    case 9: vmcnt_barrier<9>(); break;
    case 10: vmcnt_barrier<10>(); break;
    case 11: vmcnt_barrier<11>(); break;
    case 12: vmcnt_barrier<12>(); break;
    case 13: vmcnt_barrier<13>(); break;
    case 14: vmcnt_barrier<14>(); break;
    case 15: vmcnt_barrier<15>(); break;
    case 16: vmcnt_barrier<16>(); break;
    case 17: vmcnt_barrier<17>(); break;
    case 18: vmcnt_barrier<18>(); break;
    case 19: vmcnt_barrier<19>(); break;
    case 20: vmcnt_barrier<20>(); break;
    case 21: vmcnt_barrier<21>(); break;
    case 22: vmcnt_barrier<22>(); break;
    case 23: vmcnt_barrier<23>(); break;
    case 24: vmcnt_barrier<24>(); break;
    case 25: vmcnt_barrier<25>(); break;
    case 26: vmcnt_barrier<26>(); break;
    case 27: vmcnt_barrier<27>(); break;
    case 28: vmcnt_barrier<28>(); break;
    case 29: vmcnt_barrier<29>(); break;
    case 30: vmcnt_barrier<30>(); break;
    case 31: vmcnt_barrier<31>(); break;
    case 32: vmcnt_barrier<32>(); break;
    case 33: vmcnt_barrier<33>(); break;
    case 34: vmcnt_barrier<34>(); break;
    case 35: vmcnt_barrier<35>(); break;
    case 36: vmcnt_barrier<36>(); break;
    case 37: vmcnt_barrier<37>(); break;
    case 38: vmcnt_barrier<38>(); break;
    case 39: vmcnt_barrier<39>(); break;
    case 40: vmcnt_barrier<40>(); break;
    case 41: vmcnt_barrier<41>(); break;
    case 42: vmcnt_barrier<42>(); break;
    case 43: vmcnt_barrier<43>(); break;
    case 44: vmcnt_barrier<44>(); break;
    case 45: vmcnt_barrier<45>(); break;
    case 46: vmcnt_barrier<46>(); break;
    case 47: vmcnt_barrier<47>(); break;
    default: vmcnt_barrier<0>(); break;
  }
}

template <int S, bool ACT>
__global__ __launch_bounds__(64 * kPatchNW) void conv3x3_patch_kernel(const bf16* __restrict__ src,
                                                                      const bf16* __restrict__ wts,
                                                                      const float* __restrict__ bias,
                                                                      const bf16* __restrict__ res,
                                                                      bf16* __restrict__ out, Geom g, PatchGeom pg) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  constexpr int BM = kPatchBM, BN = kPatchBN, NW = kPatchNW, TM = 2, TN = 2, CH = 8;
  static_assert(S >= 2 && S <= 9, "ring depth");
  const int gn = g.Ncols / BN;
  const int nwg = g.gm * gn;
  int bid = blockIdx.x;
  {
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  }
  // the N-tiles of one pixel block are consecutive logical ids: one XCD shares the patch
  const int tile = bid / gn, tn = bid - tile * gn;
  const int n0 = tn * BN;
  const int HW = pg.H * pg.W;
  int m0, meff, img0, y0;
  if (pg.IPT > 1) {
    img0 = tile * pg.IPT;
    y0 = 0;
    const int ni = pg.N - img0 < pg.IPT ? pg.N - img0 : pg.IPT;
    m0 = img0 * HW;
    meff = ni * HW;
  } else {
    img0 = tile / pg.tpi;
    y0 = (tile - img0 * pg.tpi) * pg.R;
    const int rows = pg.H - y0 < pg.R ? pg.H - y0 : pg.R;
    m0 = (img0 * pg.H + y0) * pg.W;
    meff = rows * pg.W;
  }
  const int prow = pg.IPT > 1 ? pg.H + 2 : pg.R + 2;   // patch rows per image block
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int r8 = lane >> 3, pch = lane & 7;
  const char* zp = reinterpret_cast<const char*>(g_zero_page);

  // patch DMA: instruction i of this wave covers patch pixels (i * NW + wave) * 8 + 0..7
  const bf16* pa_base[kPatchPIMax];
  unsigned pa_mask[kPatchPIMax];
#pragma unroll
  for (int i = 0; i < kPatchPIMax; ++i) {
    const int pp = (i * NW + wave) * 8 + r8;
    const int prr = pp / pg.PW, px = pp - prr * pg.PW;
    int img, iy;
    if (pg.IPT > 1) {
      const int bi = prr / prow;
      img = img0 + bi;
      iy = prr - bi * prow - 1;
    } else {
      img = img0;
      iy = y0 - 1 + prr;
    }
    const int ix = px - 1;
    const bool ok = i < pg.PI && pp < pg.P && img < pg.N && (unsigned)iy < (unsigned)pg.H &&
                    (unsigned)ix < (unsigned)pg.W;
    pa_base[i] = ok ? src + ((int64_t)(img * pg.H + iy) * pg.W + ix) * pg.C + (pch ^ swz8(pp)) * CH
                    : reinterpret_cast<const bf16*>(zp);
    pa_mask[i] = ok ? ~0u : 0u;
  }
  // weight DMA: one instruction per wave, rows wave * 8 + r8 of the 64-row slice
  const int brow = wave * 8 + r8;
  const bool bok = n0 + brow < g.Ncols;
  const bf16* b_base = bok ? wts + (int64_t)(n0 + brow) * g.Kpad + (pch ^ swz8(brow)) * CH
                           : reinterpret_cast<const bf16*>(zp);
  const unsigned b_mask = bok ? ~0u : 0u;

  const int PBYTES = pg.PI * NW * 1024;              // one patch buffer
  const int BOFF = pg.bufs * PBYTES;                  // weight ring after the patch buffers
  const int NS = pg.nslices * 9;
  auto issue_patch = [&](int c) {
    char* dst = smem + (c & 1) * PBYTES;
    const unsigned coff = (unsigned)(c * 64);
#pragma unroll
    for (int i = 0; i < kPatchPIMax; ++i)
      if (i < pg.PI) glds16(pa_base[i] + (coff & pa_mask[i]), dst + (i * NW + wave) * 1024);
  };
  auto issue_unit = [&](int s) {
    const int c = s / 9, t = s - c * 9;
    const unsigned boff = (unsigned)(t * pg.C + c * 64);
    glds16(b_base + (boff & b_mask), smem + BOFF + (s % S) * (BN * 128) + wave * 1024);
    if (t == 8 && c + 1 < pg.nslices) issue_patch(c + 1);
  };
  auto unit_cnt = [&](int s) -> int {
    if (s >= NS) return 0;
    const int c = s / 9, t = s - c * 9;
    return 1 + ((t == 8 && c + 1 < pg.nslices) ? pg.PI : 0);
  };

  // A fragment rows of this lane: tile-local output pixel -> its tap-(0,0) patch pixel
  const int fr = lane & 15, fc = lane >> 4;
  int pbase[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int lr = wm * 32 + i * 16 + fr;
    int pb = 0;
    if (lr < meff) {
      if (pg.IPT > 1) {
        const int bi = lr / HW, rem = lr - bi * HW;
        const int y = rem / pg.W, x = rem - y * pg.W;
        pb = (bi * prow + y) * pg.PW + x;
      } else {
        const int y = lr / pg.W, x = lr - y * pg.W;
        pb = y * pg.PW + x;
      }
    }
    pbase[i] = pb;
  }
  unsigned boffs[2][TN];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int row = wn * 32 + j * 16 + fr;
      boffs[kk][j] = row * 128 + (((fc + 4 * kk) ^ swz8(row)) << 4);
    }
  const unsigned lds0 = lds_addr(smem);

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  issue_patch(0);
  for (int s = 0; s < S - 1 && s < NS; ++s) issue_unit(s);
  for (int s = 0; s < NS; ++s) {
    int inflight = 0;
#pragma unroll
    for (int u = 1; u <= S - 2; ++u) inflight += unit_cnt(s + u);
    vm_wait_barrier(inflight);   // unit s (and the patch it completes) landed, for every wave
    const int c = s / 9, t = s - c * 9;
    const int kh = t / 3, kw = t - kh * 3;
    const int toff = kh * pg.PW + kw;
    const unsigned pbuf = lds0 + (c & 1) * PBYTES;
    const unsigned bslot = lds0 + BOFF + (s % S) * (BN * 128);
    unsigned addr[2][4];
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int pp = pbase[i] + toff;
        addr[kk][i] = pbuf + pp * 128 + (((fc + 4 * kk) ^ swz8(pp)) << 4);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) addr[kk][TM + j] = bslot + boffs[kk][j];
    }
    u32x4 f[2][4];
    lds_issue_frags8(f, addr);
    if (s + S - 1 < NS) issue_unit(s + S - 1);
    lds_wait_first(f[0]);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      if (kk == 1) lds_wait_all(f[1]);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) mma_frag<bf16>(acc[i][j], f[kk][i], f[kk][TM + j]);
    }
  }
  asm volatile("s_barrier" ::: "memory");   // every wave done reading before the epilogue reuses the LDS
  Geom ge = g;
  ge.M = m0 + meff;   // rows past the tile's pixels are masked
  EpiPre<bf16, BM, BN, NW, false> pre;
  conv_epilogue<bf16, BM, BN, ACT ? 1 : 0, NW, false, false>(acc, smem, ge, bias, res, out, nullptr, m0, n0, -1,
                                                              nullptr, pre, false);
}

template <int S>
int launch_patch(const Geom& g0, const PatchPlan& pp, int N, const void* src, const void* w, const float* bias,
                 const void* res, void* out, hipStream_t s) {
  Geom g = g0;
  g.gm = pp.tiles;
  g.gn = g.Ncols / kPatchBN;
  g.splits = 1;
  PatchGeom pg{};
  pg.N = N; pg.H = g.RH; pg.W = g.RW; pg.C = g.SC; pg.R = pp.R; pg.IPT = pp.IPT; pg.tpi = pp.tpi;
  pg.PW = pp.PW; pg.P = pp.P; pg.PI = pp.PI; pg.bufs = pp.bufs; pg.nslices = g.SC / 64;
  const int grid = g.gm * g.gn;
  if (g.act)
    conv3x3_patch_kernel<S, true><<<grid, 64 * kPatchNW, pp.lds, s>>>((const bf16*)src, (const bf16*)w, bias,
                                                                      (const bf16*)res, (bf16*)out, g, pg);
  else
    conv3x3_patch_kernel<S, false><<<grid, 64 * kPatchNW, pp.lds, s>>>((const bf16*)src, (const bf16*)w, bias,
                                                                       (const bf16*)res, (bf16*)out, g, pg);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

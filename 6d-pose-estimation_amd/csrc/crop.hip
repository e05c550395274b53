// GPU crop / pad / resize / normalise of LineMOD frames -- the per-sample body of
// LineMODDatasetRGBD.__getitem__ (data/dataset_rgbd.py:104-206) and
// LineMODDatasetRGB.__getitem__ (data/dataset_rgb.py:95-145) after the file reads,
// batched: one launch turns B full frames (640x480 RGB u8 + u16 depth in mm) into
// the model inputs the DataLoader would have produced.
//
// One thread per output pixel (all three colour channels + depth): square crop
// geometry recomputed per thread from the sample's jittered bbox (a few scalar
// double ops, exactly the reference's Python arithmetic), zero padding folded into
// the gather (pixels outside the frame read as 0 = cv2.copyMakeBorder constant 0),
// cv2.resize INTER_LINEAR restated (8U: 11-bit fixed-point weights, vertical pass
// as OpenCV's SIMD body rounds; 16U: float weights, round-half-even; exact 2x:
// INTER_AREA), then ToTensor/Normalize and the depth normalisation.  Outputs are
// NCHW fp32 (rgb), (B,1,S,S) / (B,S,S) fp32 (depth), written coalesced along x.
// Built with -ffp-contract=off: every fp32 op rounds like numpy / torch-CPU.
// HBM-bound gather; algorithmic bytes per crop: <= 5 * crop^2 read (clipped to
// the frame) + S^2 * (12 + 4 + 4) written.
#include <math.h>

#include "common.h"

namespace {

constexpr int kThreads = 256;
constexpr int kCoefBits = 11;
constexpr int kCoefScale = 1 << kCoefBits;

struct CropGeom {
  int x1, y1;      // crop origin in ORIGINAL image coordinates (may be negative)
  int n;           // crop side int(size)
  int pad_l, pad_t;
  int x1p, y1p;    // origin in padded coordinates (dataset_rgbd.py:138-139)
};

// dataset_rgbd.py:120-139 (Python float = double, int() truncates toward zero)
__device__ __forceinline__ CropGeom crop_geom(const int32_t* bb, int H, int W) {
  const int x = bb[0], y = bb[1], w = bb[2], h = bb[3];
  const double c_x = (double)x + (double)w / 2.0, c_y = (double)y + (double)h / 2.0;
  const double size = (double)(w > h ? w : h) * 1.2;
  CropGeom g;
  g.x1 = (int)(c_x - size / 2.0);
  g.y1 = (int)(c_y - size / 2.0);
  g.n = (int)size;
  if (g.n < 1) g.n = 1;   // the reference raises on an empty crop (cv2.resize)
  g.pad_l = g.x1 < 0 ? -g.x1 : 0;
  g.pad_t = g.y1 < 0 ? -g.y1 : 0;
  const int pad_r = g.x1 + g.n - W > 0 ? g.x1 + g.n - W : 0;
  const int pad_b = g.y1 + g.n - H > 0 ? g.y1 + g.n - H : 0;
  const bool padded = g.pad_l > 0 || g.pad_t > 0 || pad_r > 0 || pad_b > 0;
  g.x1p = padded ? g.x1 + g.pad_l : g.x1;
  g.y1p = padded ? g.y1 + g.pad_t : g.y1;
  return g;
}

// cv::resizeGeneric_ tables for one output index: fx = (float)((d + 0.5) * scale - 0.5),
// sx = floor(fx), fx -= sx; x only: reset to (0, 0) / (n-1, 0) at the edges
__device__ __forceinline__ void lin_coef(int d, int n, int S, bool clamp_edges, int& s, float& f) {
  const double scale = 1.0 / ((double)S / (double)n);
  f = (float)(((double)d + 0.5) * scale - 0.5);
  s = (int)floorf(f);
  f = f - (float)s;
  if (clamp_edges) {
    if (s < 0) { f = 0.f; s = 0; }
    if (s >= n - 1) { f = 0.f; s = n - 1; }
  }
}

__device__ __forceinline__ int fix_coef(float c) { return (int)rintf(c * (float)kCoefScale); }   // cvRound

__global__ __launch_bounds__(kThreads) void crop_rgbd_kernel(
    const uint8_t* __restrict__ rgb, int bgr, const uint16_t* __restrict__ depth, int H, int W,
    const int32_t* __restrict__ bbox_orig, const int32_t* __restrict__ bbox_aug, const float* __restrict__ K, int S,
    const float* __restrict__ mean_std, float* __restrict__ rgb_out, float* __restrict__ depth_out,
    float* __restrict__ depth_raw_out, float* __restrict__ center_out, float* __restrict__ K_out,
    uint8_t* __restrict__ u8_out) {
  const int b = blockIdx.y;
  const int pix = blockIdx.x * kThreads + threadIdx.x;
  const CropGeom g = crop_geom(bbox_aug + 4 * b, H, W);
  const float scale32 = (float)((double)S / (double)g.n);   // np.float32(img_size / crop_size)

  if (pix == 0) {
    if (center_out) {
      // dataset_rgbd.py:105,148-156 (float32 arithmetic, NEP 50 weak Python scalars)
      const int32_t* bo = bbox_orig + 4 * b;
      const float cgx = (float)((double)bo[0] + (double)bo[2] / 2.0);
      const float cgy = (float)((double)bo[1] + (double)bo[3] / 2.0);
      float ccx = (cgx + (float)g.pad_l) - (float)g.x1p;
      float ccy = (cgy + (float)g.pad_t) - (float)g.y1p;
      ccx = fminf(fmaxf(ccx * scale32, 0.f), (float)(S - 1));
      ccy = fminf(fmaxf(ccy * scale32, 0.f), (float)(S - 1));
      center_out[2 * b] = ccx;
      center_out[2 * b + 1] = ccy;
    }
    if (K_out) {
      // dataset_rgbd.py:159-169
      const float* k = K + 9 * b;
      float* ko = K_out + 9 * b;
      ko[0] = k[0] * scale32; ko[1] = 0.f; ko[2] = ((k[2] + (float)g.pad_l) - (float)g.x1p) * scale32;
      ko[3] = 0.f; ko[4] = k[4] * scale32; ko[5] = ((k[5] + (float)g.pad_t) - (float)g.y1p) * scale32;
      ko[6] = 0.f; ko[7] = 0.f; ko[8] = 1.f;
    }
  }
  if (pix >= S * S) return;
  const int oy = pix / S, ox = pix - oy * S;
  const int n = g.n;
  const int64_t HW = (int64_t)H * W;
  const uint8_t* img = rgb + (int64_t)b * HW * 3;
  const uint16_t* dimg = depth ? depth + (int64_t)b * HW : nullptr;

  // crop pixel (r, c) -> frame pixel (y1 + r, x1 + c); zero outside the frame
  auto in_frame = [&](int r, int c, int64_t& off) {
    const int yy = g.y1 + r, xx = g.x1 + c;
    off = (int64_t)yy * W + xx;
    return (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
  };
  auto px3 = [&](int r, int c, int (&v)[3]) {
    int64_t off;
    if (in_frame(r, c, off)) {
      const uint8_t* p = img + off * 3;
      v[0] = p[bgr ? 2 : 0]; v[1] = p[1]; v[2] = p[bgr ? 0 : 2];
    } else {
      v[0] = v[1] = v[2] = 0;
    }
  };
  auto pxd = [&](int r, int c) -> int {
    int64_t off;
    return (dimg && in_frame(r, c, off)) ? (int)dimg[off] : 0;
  };

  int outc[3];
  int dval;
  if (n == 2 * S) {
    // exact 2x downscale: cv::resize switches INTER_LINEAR to INTER_AREA (2x2 mean)
    const int r = 2 * oy, c = 2 * ox;
    int a[3], bq[3], cq[3], dq[3];
    px3(r, c, a); px3(r, c + 1, bq); px3(r + 1, c, cq); px3(r + 1, c + 1, dq);
#pragma unroll
    for (int k = 0; k < 3; ++k) outc[k] = (a[k] + bq[k] + cq[k] + dq[k] + 2) >> 2;
    dval = (pxd(r, c) + pxd(r, c + 1) + pxd(r + 1, c) + pxd(r + 1, c + 1) + 2) >> 2;
  } else {
    int sx, sy;
    float fx, fy;
    lin_coef(ox, n, S, true, sx, fx);
    lin_coef(oy, n, S, false, sy, fy);
    const bool edge = sx >= n - 1;   // dx >= xmax: S[sx] * ONE
    const int c0 = sx, c1 = edge ? sx : sx + 1;
    const int r0 = sy < 0 ? 0 : (sy > n - 1 ? n - 1 : sy);
    const int r1 = sy + 1 < 0 ? 0 : (sy + 1 > n - 1 ? n - 1 : sy + 1);
    // 8U: HResizeLinear (int) + VResizeLinearVec_32s8u
    const int a0 = fix_coef(1.f - fx), a1 = fix_coef(fx);
    const int b0 = fix_coef(1.f - fy), b1 = fix_coef(fy);
    int p00[3], p01[3], p10[3], p11[3];
    px3(r0, c0, p00); px3(r0, c1, p01); px3(r1, c0, p10); px3(r1, c1, p11);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int h0 = p00[k] * a0 + (edge ? 0 : p01[k] * a1);
      const int h1 = p10[k] * a0 + (edge ? 0 : p11[k] * a1);
      const int t = (((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16);
      const int v = (t + 2) >> 2;
      outc[k] = v < 0 ? 0 : (v > 255 ? 255 : v);
    }
    // 16U: float weights, mul + add, round half to even, saturate
    if (dimg) {
      const float fa0 = 1.f - fx, fb0 = 1.f - fy;
      const float d00 = (float)pxd(r0, c0), d10 = (float)pxd(r1, c0);
      const float h0 = edge ? d00 * 1.f : d00 * fa0 + (float)pxd(r0, c1) * fx;
      const float h1 = edge ? d10 * 1.f : d10 * fa0 + (float)pxd(r1, c1) * fx;
      const float v = rintf(h0 * fb0 + h1 * fy);
      dval = v < 0.f ? 0 : (v > 65535.f ? 65535 : (int)v);
    } else {
      dval = 0;
    }
  }

  // ToTensor (u8 / 255) + Normalize ((x - mean) / std), NCHW
  const int64_t plane = (int64_t)S * S;
  if (u8_out) {   // the resized uint8 crop, HWC (the PIL image ColorJitter receives)
    uint8_t* o = u8_out + ((int64_t)b * plane + pix) * 3;
    o[0] = (uint8_t)outc[0]; o[1] = (uint8_t)outc[1]; o[2] = (uint8_t)outc[2];
  }
  if (rgb_out) {
    float* o = rgb_out + (int64_t)b * 3 * plane + pix;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float v = (float)outc[k] / 255.f;
      if (mean_std) v = (v - mean_std[k]) / mean_std[3 + k];
      o[k * plane] = v;
    }
  }
  // dataset_rgbd.py:176-186
  const float raw = (float)dval / 1000.f;
  if (depth_raw_out) depth_raw_out[(int64_t)b * plane + pix] = raw;
  if (depth_out) {
    float dn = (raw - 0.1f) / 1.5f;
    dn = fminf(fmaxf(dn, 0.f), 1.f);
    if (raw < 0.01f) dn = 0.f;
    depth_out[(int64_t)b * plane + pix] = dn;
  }
}

}  // namespace

extern "C" int pose6d_crop_rgbd(const uint8_t* rgb, int32_t bgr, const uint16_t* depth, int32_t B, int32_t H,
                                int32_t W, const int32_t* bbox_orig, const int32_t* bbox_aug, const float* K,
                                int32_t S, const float* mean_std, float* rgb_out, float* depth_out,
                                float* depth_raw_out, float* center_out, float* K_out, void* stream) {
  P6_CHECK_ARG(rgb != nullptr && bbox_aug != nullptr, "pose6d_crop_rgbd: rgb and bbox_aug are required");
  P6_CHECK_ARG(B >= 0 && H > 0 && W > 0 && S > 0 && (int64_t)S * S < (1ll << 31), "pose6d_crop_rgbd: bad shape");
  P6_CHECK_ARG(center_out == nullptr || bbox_orig != nullptr, "pose6d_crop_rgbd: center_out needs bbox_orig");
  P6_CHECK_ARG(K_out == nullptr || K != nullptr, "pose6d_crop_rgbd: K_out needs K");
  if (B == 0) return POSE6D_OK;
  const dim3 grid(p6::ceil_div((int64_t)S * S, kThreads), B);
  crop_rgbd_kernel<<<grid, kThreads, 0, p6::stream_of(stream)>>>(rgb, bgr, depth, H, W, bbox_orig, bbox_aug, K, S,
                                                                 mean_std, rgb_out, depth_out, depth_raw_out,
                                                                 center_out, K_out, nullptr);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

// ---------------------------------------------------------------- train transform
// The reference's train_transform (train_rgbd_geometric.py:41-47) on the resized
// uint8 crop: ColorJitter(brightness, contrast, saturation, hue) in a random op order
// -> ToTensor -> Normalize -> RandomErasing(p, scale, ratio, value 0).  ColorJitter's
// arithmetic is Pillow's (torchvision applies it to a PIL image): ImageEnhance =
// Image.blend against a degenerate image (black / the constant int(mean L + 0.5) /
// the L image), float alpha, truncating; hue through Pillow's HSV conversion with
// torchvision's uint8 hue-band shift -- restated in oracle/augment.py and pinned there
// against Pillow itself.  One 1024-thread workgroup per crop holds the crop in LDS
// (S * S * 3 bytes: 147 KiB at 224) while the four ops run in place, the contrast
// mean being a workgroup reduction of the current image.
// Random parameters: counter-based draws (splitmix64 of seed, crop, draw index) with
// torchvision's distributions (get_params of ColorJitter / RandomErasing); every
// crop's parameters are written to params_out so a checker can replay them.
namespace {

constexpr int kAugThreads = 1024;
constexpr int kAugParams = 16;   // perm[4], factor[4] (NaN: op off), erase i, j, h, w (-1: none), 4 spare

struct AugCfg {
  float lo[4], hi[4];   // brightness, contrast, saturation, hue ranges (lo == hi == NaN: off)
  float p, scale_lo, scale_hi, log_r_lo, log_r_hi;
};

__device__ __forceinline__ uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// draw k of crop b: a uniform double in [0, 1)
__device__ __forceinline__ double u01(uint64_t seed, int b, int k) {
  const uint64_t x = splitmix(seed ^ splitmix(((uint64_t)(uint32_t)b << 32) | (uint32_t)k));
  return (double)(x >> 11) * 0x1.0p-53;
}

// a float32 tensor's uniform_(lo, hi) value
__device__ __forceinline__ float uf(uint64_t seed, int b, int k, float lo, float hi) {
  return (float)((double)lo + ((double)hi - (double)lo) * u01(seed, b, k));
}

// Pillow ImagingBlend on one uint8 band value
__device__ __forceinline__ int blend_u8(int d, int v, float a) {
  if (a == 0.f) return d;
  if (a == 1.f) return v;
  const float t = (float)d + a * (float)(v - d);
  if (a >= 0.f && a <= 1.f) return (int)(uint8_t)t;
  return t <= 0.f ? 0 : (t >= 255.f ? 255 : (int)(uint8_t)t);
}

__device__ __forceinline__ int lum_u8(int r, int g, int b) { return (r * 19595 + g * 38470 + b * 7471 + 0x8000) >> 16; }

__device__ __forceinline__ int clip8(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

// Pillow rgb2hsv_row / hsv2rgb (oracle/augment.py spells out the rounding of each step)
__device__ __forceinline__ void rgb2hsv(int r, int g, int b, int& h8, int& s8, int& v8) {
  const int maxc = max(r, max(g, b)), minc = min(r, min(g, b));
  v8 = maxc;
  if (maxc == minc) { h8 = 0; s8 = 0; return; }
  const float cr = (float)(maxc - minc);
  const float s = cr / (float)maxc;
  const float rc = (float)(maxc - r) / cr, gc = (float)(maxc - g) / cr, bc = (float)(maxc - b) / cr;
  float h;
  if (r == maxc) h = bc - gc;
  else if (g == maxc) h = (float)(2.0 + (double)rc - (double)bc);
  else h = (float)(4.0 + (double)gc - (double)rc);
  h = (float)fmod((double)h / 6.0 + 1.0, 1.0);
  h8 = clip8((int)((double)h * 255.0));
  s8 = clip8((int)((double)s * 255.0));
}

__device__ __forceinline__ void hsv2rgb(int h8, int s8, int v8, int& r, int& g, int& b) {
  if (s8 == 0) { r = g = b = v8; return; }
  const double hf = (double)(float)h8;
  const double i = floor(hf * 6.0 / 255.0);
  const double f = (double)(float)(hf * 6.0 / 255.0 - i);
  const double fs = (double)(float)((double)(float)s8 / 255.0);
  const double vf = (double)(float)v8;
  const int p = clip8((int)round(vf * (1.0 - fs)));
  const int q = clip8((int)round(vf * (1.0 - fs * f)));
  const int t = clip8((int)round(vf * (1.0 - fs * (1.0 - f))));
  switch ((int)i % 6) {
    case 0: r = v8; g = t; b = p; break;
    case 1: r = q; g = v8; b = p; break;
    case 2: r = p; g = v8; b = t; break;
    case 3: r = p; g = q; b = v8; break;
    case 4: r = t; g = p; b = v8; break;
    default: r = v8; g = p; b = q; break;
  }
}

__global__ __launch_bounds__(kAugThreads) void augment_kernel(const uint8_t* __restrict__ src, int S,
                                                              const float* __restrict__ mean_std, AugCfg cfg,
                                                              uint64_t seed, float* __restrict__ rgb_out,
                                                              float* __restrict__ params_out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t img[];   // [S][S][3]
  __shared__ int red[kAugThreads / 64];
  __shared__ float prm[kAugParams];
  const int b = blockIdx.x, tid = threadIdx.x;
  const int npx = S * S, nbytes = npx * 3;
  const uint8_t* in = src + (int64_t)b * nbytes;
  for (int i = tid * 16; i < nbytes; i += kAugThreads * 16) {
    if (i + 16 <= nbytes) {
      *reinterpret_cast<uint4*>(img + i) = *reinterpret_cast<const uint4*>(in + i);
    } else {
      for (int k = i; k < nbytes; ++k) img[k] = in[k];
    }
  }
  if (tid == 0) {
    // ColorJitter.get_params: fn_idx = randperm(4), then each enabled factor
    int perm[4] = {0, 1, 2, 3};
    for (int i = 3; i > 0; --i) {   // Fisher-Yates
      const int j = (int)(u01(seed, b, 3 - i) * (double)(i + 1));
      const int t = perm[i]; perm[i] = perm[j]; perm[j] = t;
    }
    for (int k = 0; k < 4; ++k) {
      prm[k] = (float)perm[k];
      prm[4 + k] = isnan(cfg.lo[k]) ? cfg.lo[k] : uf(seed, b, 3 + k, cfg.lo[k], cfg.hi[k]);
    }
    // RandomErasing.forward / get_params (value 0): p, then up to 10 attempts
    float box[4] = {-1.f, -1.f, -1.f, -1.f};
    if (u01(seed, b, 7) < (double)cfg.p) {
      const double area = (double)S * (double)S;
      for (int att = 0; att < 10; ++att) {
        const int k0 = 8 + 4 * att;
        const double ea = area * (double)uf(seed, b, k0, cfg.scale_lo, cfg.scale_hi);
        const double ar = (double)expf(uf(seed, b, k0 + 1, cfg.log_r_lo, cfg.log_r_hi));
        const int h = (int)rint(sqrt(ea * ar)), w = (int)rint(sqrt(ea / ar));   // round(): half to even
        if (!(h < S && w < S)) continue;
        box[0] = (float)(int)(u01(seed, b, k0 + 2) * (double)(S - h + 1));
        box[1] = (float)(int)(u01(seed, b, k0 + 3) * (double)(S - w + 1));
        box[2] = (float)h;
        box[3] = (float)w;
        break;
      }
    }
    for (int k = 0; k < 4; ++k) prm[8 + k] = box[k];
    for (int k = 12; k < kAugParams; ++k) prm[k] = 0.f;
    if (params_out)
      for (int k = 0; k < kAugParams; ++k) params_out[b * kAugParams + k] = prm[k];
  }
  __syncthreads();
  for (int step = 0; step < 4; ++step) {
    const int op = (int)prm[step];
    const float f = prm[4 + op];
    if (isnan(f)) continue;   // op disabled (block-uniform)
    int mean = 0;
    if (op == 1) {            // contrast: int(mean(L) + 0.5) of the current image
      int sum = 0;
      for (int p = tid; p < npx; p += kAugThreads) sum += lum_u8(img[3 * p], img[3 * p + 1], img[3 * p + 2]);
      sum = p6::wave_sum(sum);
      if ((tid & 63) == 0) red[tid >> 6] = sum;
      __syncthreads();
      int tot = 0;
#pragma unroll
      for (int w = 0; w < kAugThreads / 64; ++w) tot += red[w];
      mean = (int)((double)tot / (double)npx + 0.5);
    }
    const int shift = op == 3 ? ((int)(int8_t)(int)((double)f * 255.0) & 255) : 0;
    for (int p = tid; p < npx; p += kAugThreads) {
      int r = img[3 * p], g = img[3 * p + 1], bl = img[3 * p + 2];
      if (op == 0) {
        r = blend_u8(0, r, f); g = blend_u8(0, g, f); bl = blend_u8(0, bl, f);
      } else if (op == 1) {
        r = blend_u8(mean, r, f); g = blend_u8(mean, g, f); bl = blend_u8(mean, bl, f);
      } else if (op == 2) {
        const int l = lum_u8(r, g, bl);
        r = blend_u8(l, r, f); g = blend_u8(l, g, f); bl = blend_u8(l, bl, f);
      } else {
        int h8, s8, v8;
        rgb2hsv(r, g, bl, h8, s8, v8);
        hsv2rgb((h8 + shift) & 255, s8, v8, r, g, bl);
      }
      img[3 * p] = (uint8_t)r; img[3 * p + 1] = (uint8_t)g; img[3 * p + 2] = (uint8_t)bl;
    }
    __syncthreads();
  }
  // ToTensor + Normalize + RandomErasing (value 0), NCHW fp32, coalesced along x
  const int bi = (int)prm[8], bj = (int)prm[9], bh = (int)prm[10], bw = (int)prm[11];
  float* o = rgb_out + (int64_t)b * 3 * npx;
  for (int p = tid; p < npx; p += kAugThreads) {
    const int y = p / S, x = p - y * S;
    const bool erased = bh > 0 && y >= bi && y < bi + bh && x >= bj && x < bj + bw;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      float v = (float)img[3 * p + k] / 255.f;
      if (mean_std) v = (v - mean_std[k]) / mean_std[3 + k];
      o[(int64_t)k * npx + p] = erased ? 0.f : v;
    }
  }
}

}  // namespace

extern "C" int64_t pose6d_crop_train_workspace(int32_t B, int32_t S) { return (int64_t)B * S * S * 3; }

extern "C" int pose6d_crop_rgbd_train(const uint8_t* rgb, int32_t bgr, const uint16_t* depth, int32_t B, int32_t H,
                                      int32_t W, const int32_t* bbox_orig, const int32_t* bbox_aug, const float* K,
                                      int32_t S, const float* mean_std, float brightness, float contrast,
                                      float saturation, float hue, float erase_p, float erase_scale_lo,
                                      float erase_scale_hi, float erase_ratio_lo, float erase_ratio_hi,
                                      uint64_t seed, uint8_t* workspace, float* rgb_out, float* depth_out,
                                      float* depth_raw_out, float* center_out, float* K_out, float* params_out,
                                      void* stream) {
  P6_CHECK_ARG(rgb != nullptr && bbox_aug != nullptr && workspace != nullptr && rgb_out != nullptr,
               "pose6d_crop_rgbd_train: rgb, bbox_aug, workspace and rgb_out are required");
  P6_CHECK_ARG(B >= 0 && H > 0 && W > 0 && S > 0 && S <= 232, "pose6d_crop_rgbd_train: bad shape (S <= 232: the "
               "crop must fit one workgroup's LDS)");
  P6_CHECK_ARG(center_out == nullptr || bbox_orig != nullptr, "pose6d_crop_rgbd_train: center_out needs bbox_orig");
  P6_CHECK_ARG(K_out == nullptr || K != nullptr, "pose6d_crop_rgbd_train: K_out needs K");
  P6_CHECK_ARG(brightness >= 0.f && contrast >= 0.f && saturation >= 0.f && hue >= 0.f && hue <= 0.5f,
               "pose6d_crop_rgbd_train: ColorJitter factors must be >= 0 (hue <= 0.5)");
  P6_CHECK_ARG(erase_p >= 0.f && erase_p <= 1.f && erase_scale_lo <= erase_scale_hi && erase_ratio_lo > 0.f &&
                   erase_ratio_lo <= erase_ratio_hi,
               "pose6d_crop_rgbd_train: bad RandomErasing arguments");
  if (B == 0) return POSE6D_OK;
  hipStream_t s = p6::stream_of(stream);
  const dim3 grid(p6::ceil_div((int64_t)S * S, kThreads), B);
  crop_rgbd_kernel<<<grid, kThreads, 0, s>>>(rgb, bgr, depth, H, W, bbox_orig, bbox_aug, K, S, nullptr, nullptr,
                                             depth_out, depth_raw_out, center_out, K_out, workspace);
  P6_LAUNCH_CHECK();
  // ColorJitter._check_input: value v -> [max(0, 1 - v), 1 + v] (hue: [-v, v]); 0 -> the op is off
  AugCfg cfg;
  const float v[4] = {brightness, contrast, saturation, hue};
  for (int k = 0; k < 4; ++k) {
    if (v[k] == 0.f) {
      cfg.lo[k] = cfg.hi[k] = __builtin_nanf("");
    } else if (k == 3) {
      cfg.lo[k] = -v[k]; cfg.hi[k] = v[k];
    } else {
      cfg.lo[k] = 1.f - v[k] > 0.f ? 1.f - v[k] : 0.f; cfg.hi[k] = 1.f + v[k];
    }
  }
  cfg.p = erase_p;
  cfg.scale_lo = erase_scale_lo;
  cfg.scale_hi = erase_scale_hi;
  cfg.log_r_lo = logf(erase_ratio_lo);   // torch.log(torch.tensor(ratio)): float32
  cfg.log_r_hi = logf(erase_ratio_hi);
  const int lds = S * S * 3;
  augment_kernel<<<B, kAugThreads, lds, s>>>(workspace, S, mean_std, cfg, seed, rgb_out, params_out);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

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
    float* __restrict__ depth_raw_out, float* __restrict__ center_out, float* __restrict__ K_out) {
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
                                                                 center_out, K_out);
  P6_LAUNCH_CHECK();
  return POSE6D_OK;
}

"""ORACLE (test infrastructure only -- never imported by the product path).

CPU restatement of the reference's per-sample crop pipeline, used to check the
HIP crop kernel (pose6d_crop_rgbd) bit for bit:

  * geometry: data/dataset_rgbd.py:104-169 (square crop x1.2 around the jittered
    bbox, zero padding, crop-adjusted centre and intrinsics) and
    data/dataset_rgb.py:95-130 (same crop; original centre and K);
  * bbox jitter draw order: dataset_rgbd.py:110-118 (0.05 / 0.1),
    dataset_rgb.py:101-110 (0.15 / 0.2) -- np.random.uniform x4, int() truncation;
  * cv2.resize(crop, (224, 224)) INTER_LINEAR (dataset_rgbd.py:172-173,
    dataset_rgb.py:131), restated from OpenCV 4.12's resize.cpp (opencv-python
    4.12, requirements.txt): 8U via 11-bit fixed-point coefficients with the
    vertical pass as the SIMD body computes it (VResizeLinearVec_32s8u:
    ((S0>>4)*b0 >> 16) + ((S1>>4)*b1 >> 16) + 2 >> 2, saturated) -- the 224*3
    row is a whole number of vectors, so no scalar tail; 16U via float
    coefficients, mul+add, round-half-even; the exact 2x case switches to
    INTER_AREA (2x2 mean, (sum + 2) >> 2);
  * depth_raw = f32(depth) / 1000, normalised (d - 0.1) / 1.5 clipped to [0, 1],
    zero where depth_raw < 0.01 (dataset_rgbd.py:176-186);
  * torchvision ToTensor + Normalize of the val transform
    (train_rgbd_geometric.py:49-53): (u8 / 255 - mean) / std in fp32.

PARITY UNPINNED for the resize: cv2 is not installed in this image (SURVEY.md
§8c) and no stand-in is written for it, so the restatement is checked against
hand-computed cases (tests/test_crop.py), not against cv2's own output.  The
geometry and normalisation follow the reference lines cited above.
Train-mode photometric augmentation (ColorJitter, RandomErasing on PIL) is not
restated (out of scope: DESIGN.md).
"""
import math

import numpy as np

COEF_BITS = 11
COEF_SCALE = 1 << COEF_BITS
IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def jitter_bbox(bbox, rgbd=True, rng=np.random):
    """dataset_rgbd.py:110-118 / dataset_rgb.py:101-110 (same draw order)."""
    x, y, w, h = (int(v) for v in bbox)
    a, b = (0.05, 0.1) if rgbd else (0.15, 0.2)
    jx = int(rng.uniform(-a, a) * w)
    jy = int(rng.uniform(-a, a) * h)
    sw = int(rng.uniform(-b, b) * w)
    sh = int(rng.uniform(-b, b) * h)
    return x + jx, y + jy, w + sw, h + sh


def crop_geometry(bbox_aug, h_img, w_img):
    """dataset_rgbd.py:120-145: (x1, y1) in ORIGINAL image coordinates, crop size,
    pad_l, pad_t, x1/y1 in padded coordinates."""
    x, y, w, h = (int(v) for v in bbox_aug)
    c_x, c_y = x + w / 2, y + h / 2
    size = max(w, h) * 1.2
    x1 = int(c_x - size / 2)
    y1 = int(c_y - size / 2)
    pad_l = max(0, -x1)
    pad_t = max(0, -y1)
    pad_r = max(0, (x1 + int(size)) - w_img)
    pad_b = max(0, (y1 + int(size)) - h_img)
    x1p, y1p = x1, y1
    if pad_l > 0 or pad_t > 0 or pad_r > 0 or pad_b > 0:
        x1p, y1p = x1 + pad_l, y1 + pad_t
    return x1, y1, int(size), pad_l, pad_t, x1p, y1p


def crop_pixels(img, x1, y1, n):
    """img[y1:y1+n, x1:x1+n] of the zero-padded image (original coords, zeros outside)."""
    H, W = img.shape[:2]
    out = np.zeros((n, n) + img.shape[2:], img.dtype)
    ys, xs = max(0, y1), max(0, x1)
    ye, xe = min(H, y1 + n), min(W, x1 + n)
    if ye > ys and xe > xs:
        out[ys - y1:ye - y1, xs - x1:xe - x1] = img[ys:ye, xs:xe]
    return out


def _coeffs(dsize, ssize, clamp_edges):
    """cv::resizeGeneric_ tables: source index and fractional weight per output
    index (fx computed in double, stored as float; edge resets for x only)."""
    scale = 1.0 / (dsize / ssize)
    idx = np.zeros(dsize, np.int64)
    frac = np.zeros(dsize, np.float32)
    for d in range(dsize):
        f = np.float32((d + 0.5) * scale - 0.5)
        s = math.floor(f)
        f = np.float32(f - np.float32(s))
        if clamp_edges:
            if s < 0:
                f, s = np.float32(0.0), 0
            if s >= ssize - 1:
                f, s = np.float32(0.0), ssize - 1
        idx[d], frac[d] = s, f
    return idx, frac


def _round_half_even(x):
    return np.rint(x).astype(np.int64)


def resize_linear_u8(src, dsize=224):
    """cv2.resize(src (n, n, C) uint8, (dsize, dsize)) INTER_LINEAR."""
    n = src.shape[0]
    if n == 2 * dsize:
        return _area2(src)
    C = src.shape[2]
    sx, fx = _coeffs(dsize, n, True)
    sy, fy = _coeffs(dsize, n, False)
    ax0 = _round_half_even((np.float32(1.0) - fx) * np.float32(COEF_SCALE))
    ax1 = _round_half_even(fx * np.float32(COEF_SCALE))
    by0 = _round_half_even((np.float32(1.0) - fy) * np.float32(COEF_SCALE))
    by1 = _round_half_even(fy * np.float32(COEF_SCALE))
    S = src.astype(np.int64)
    sx1 = np.minimum(sx + 1, n - 1)
    edge = sx >= n - 1                     # dx >= xmax: S[sx] * ONE only
    hrow = S[:, sx, :] * ax0[None, :, None] + np.where(edge[None, :, None], 0, S[:, sx1, :] * ax1[None, :, None])
    r0 = np.clip(sy, 0, n - 1)
    r1 = np.clip(sy + 1, 0, n - 1)
    t0 = ((hrow[r0] >> 4) * by0[:, None, None]) >> 16
    t1 = ((hrow[r1] >> 4) * by1[:, None, None]) >> 16
    return np.clip((t0 + t1 + 2) >> 2, 0, 255).astype(np.uint8).reshape(dsize, dsize, C)


def resize_linear_u16(src, dsize=224):
    """cv2.resize(src (n, n) uint16, (dsize, dsize)) INTER_LINEAR (float weights)."""
    n = src.shape[0]
    if n == 2 * dsize:
        return _area2(src)
    sx, fx = _coeffs(dsize, n, True)
    sy, fy = _coeffs(dsize, n, False)
    ax0, ax1 = np.float32(1.0) - fx, fx
    by0, by1 = np.float32(1.0) - fy, fy
    S = src.astype(np.float32)
    sx1 = np.minimum(sx + 1, n - 1)
    edge = sx >= n - 1
    hrow = np.where(edge[None, :], S[:, sx] * np.float32(1.0),
                    (S[:, sx] * ax0[None, :]).astype(np.float32) + (S[:, sx1] * ax1[None, :]).astype(np.float32))
    hrow = hrow.astype(np.float32)
    r0 = np.clip(sy, 0, n - 1)
    r1 = np.clip(sy + 1, 0, n - 1)
    v = (hrow[r0] * by0[:, None]).astype(np.float32) + (hrow[r1] * by1[:, None]).astype(np.float32)
    return np.clip(np.rint(v.astype(np.float32)), 0, 65535).astype(np.uint16)


def _area2(src):
    """INTER_AREA fast path for an exact 2x downscale: (2x2 sum + 2) >> 2."""
    S = src.astype(np.int64)
    s = S[0::2, 0::2] + S[0::2, 1::2] + S[1::2, 0::2] + S[1::2, 1::2]
    return ((s + 2) >> 2).astype(src.dtype)


def resized_crop_u8(rgb, bbox_aug, img_size=224):
    """The uint8 (S, S, 3) crop after cv2.resize: the PIL image the train transform's
    ColorJitter receives (dataset_rgbd.py:172, 196-197)."""
    x1, y1, crop, _, _, _, _ = crop_geometry(bbox_aug, rgb.shape[0], rgb.shape[1])
    return resize_linear_u8(crop_pixels(rgb, x1, y1, crop), img_size)


def crop_sample(rgb, depth, bbox_orig, bbox_aug, K, img_size=224, mean=IMAGENET_MEAN, std=IMAGENET_STD):
    """One sample of LineMODDatasetRGBD.__getitem__ after the file reads
    (dataset_rgbd.py:104-206, val transform).  rgb (H, W, 3) uint8 RGB, depth
    (H, W) uint16 or None, K (3, 3).  Returns rgb (3, S, S), depth (1, S, S),
    depth_raw (S, S), centre (2,), K_crop (3, 3), all float32."""
    h_img, w_img = rgb.shape[:2]
    if depth is None:
        depth = np.zeros((h_img, w_img), np.uint16)
    cam_K = np.asarray(K, np.float32).reshape(3, 3)
    xo, yo, wo, ho = (int(v) for v in bbox_orig)
    center_gt = np.array([xo + wo / 2, yo + ho / 2], dtype=np.float32)
    x1, y1, crop, pad_l, pad_t, x1p, y1p = crop_geometry(bbox_aug, h_img, w_img)
    rgb_crop = crop_pixels(rgb, x1, y1, crop)
    depth_crop = crop_pixels(depth, x1, y1, crop)
    center_in_crop = np.array([center_gt[0] + pad_l - x1p, center_gt[1] + pad_t - y1p], dtype=np.float32)
    scale = img_size / crop
    center = np.clip(center_in_crop * np.float32(scale), 0, img_size - 1).astype(np.float32)
    fx, fy, cx, cy = cam_K[0, 0], cam_K[1, 1], cam_K[0, 2], cam_K[1, 2]
    s32 = np.float32(scale)
    K_crop = np.array([[fx * s32, 0, (cx + np.float32(pad_l) - np.float32(x1p)) * s32],
                       [0, fy * s32, (cy + np.float32(pad_t) - np.float32(y1p)) * s32],
                       [0, 0, 1]], dtype=np.float32)
    rgb_r = resize_linear_u8(rgb_crop, img_size)
    d_r = resize_linear_u16(depth_crop, img_size).astype(np.float32)
    depth_raw = (d_r / np.float32(1000.0)).astype(np.float32)
    dn = ((depth_raw - np.float32(0.1)) / np.float32(1.5)).astype(np.float32)
    dn = np.clip(dn, np.float32(0), np.float32(1))
    dn[depth_raw < np.float32(0.01)] = 0
    x = rgb_r.astype(np.float32).transpose(2, 0, 1) / np.float32(255.0)
    m = np.array(mean, np.float32)[:, None, None]
    s = np.array(std, np.float32)[:, None, None]
    x = ((x - m) / s).astype(np.float32)
    return x, dn[None].astype(np.float32), depth_raw, center, K_crop

"""ORACLE (test infrastructure only -- never imported by the product path).

CPU restatement of the reference's train-time photometric augmentation
(scripts/training/train_rgbd_geometric.py:41-47):

    ToPILImage -> ColorJitter(0.3, 0.3, 0.3, 0.05) -> ToTensor
               -> Normalize(ImageNet mean / std) -> RandomErasing(p=0.2, scale=(0.02, 0.1))

applied by data/dataset_rgbd.py:196-197 to the 224x224 uint8 RGB crop (after the
cv2 resize).  torchvision==0.24.1 is absent from this image, so its two classes are
restated from its published source (transforms.ColorJitter.get_params / forward,
functional_pil.adjust_{brightness,contrast,saturation,hue}, RandomErasing.get_params
/ forward); ColorJitter's PIL arithmetic (ImageEnhance.Brightness / Contrast / Color
= Image.blend against a degenerate image; convert("L"); convert("HSV") and back;
ImageStat mean) is restated from Pillow's C code and PINNED against the Pillow that
IS importable here (tests/test_augment.py: every RGB triple through the HSV round
trip and the L conversion, blends at the jitter's factor range, whole-image ops).

The random draws are NOT torch's generator stream: the GPU kernel draws its
parameters from a counter-based RNG (seed, crop, draw) with torchvision's
distributions, reports them, and this oracle replays the SAME parameters:
  perm   -- a permutation of the four ops (torch.randperm(4) in torchvision)
  b, c, s -- factors U[0.7, 1.3]; h -- U[-0.05, 0.05]
  erase  -- (i, j, h, w) of the erased box, or none (probability 1 - p).
The parameter distributions are property-tested instead (tests/test_augment.py).
"""
import numpy as np

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def to_l(img):
    """Pillow rgb2l: L = (R*19595 + G*38470 + B*7471 + 0x8000) >> 16 (Convert.c)."""
    i = img.astype(np.uint32)
    return ((i[..., 0] * 19595 + i[..., 1] * 38470 + i[..., 2] * 7471 + 0x8000) >> 16).astype(np.uint8)


def blend(deg, img, alpha):
    """Pillow ImagingBlend (Blend.c) on uint8 bands: float alpha (the C parameter is a
    float), temp = (float) in1 + alpha * (float)(in2 - in1) in single precision;
    interpolation (0 <= alpha <= 1) truncates, extrapolation clips then truncates."""
    a = np.float32(alpha)
    if a == np.float32(0.0):
        return np.broadcast_to(deg, img.shape).astype(np.uint8).copy()
    if a == np.float32(1.0):
        return img.copy()
    d = np.broadcast_to(deg, img.shape).astype(np.int32)
    temp = d.astype(np.float32) + a * (img.astype(np.int32) - d).astype(np.float32)
    if np.float32(0.0) <= a <= np.float32(1.0):
        return temp.astype(np.uint8)
    out = np.where(temp <= 0, 0, np.where(temp >= 255, 255, temp))
    return out.astype(np.float32).astype(np.uint8)


def adjust_brightness(img, f):
    """ImageEnhance.Brightness: blend(black, img, f)."""
    return blend(np.zeros_like(img), img, f)


def adjust_contrast(img, f):
    """ImageEnhance.Contrast: degenerate = the constant int(mean(L) + 0.5)
    (ImageStat mean: histogram sum / count in double)."""
    lum = to_l(img)
    mean = int(float(lum.astype(np.int64).sum()) / lum.size + 0.5)
    return blend(np.full_like(img, mean), img, f)


def adjust_saturation(img, f):
    """ImageEnhance.Color: degenerate = img.convert("L").convert("RGB")."""
    lum = to_l(img)
    return blend(np.repeat(lum[..., None], 3, axis=-1), img, f)


def rgb_to_hsv(img):
    """Pillow rgb2hsv_row (Convert.c, following colorsys): float math, h via fmod in
    double, bands truncated to uint8."""
    r, g, b = (img[..., k].astype(np.int32) for k in range(3))
    maxc = np.maximum(r, np.maximum(g, b))
    minc = np.minimum(r, np.minimum(g, b))
    v = maxc
    eq = maxc == minc
    cr = (maxc - minc).astype(np.float32)
    crs = np.where(eq, np.float32(1.0), cr)
    s = cr / np.where(maxc == 0, np.float32(1.0), maxc.astype(np.float32))
    rc = (maxc - r).astype(np.float32) / crs
    gc = (maxc - g).astype(np.float32) / crs
    bc = (maxc - b).astype(np.float32) / crs
    # `h = 2.0 + rc - bc`: the double literals make the sums double, stored into float h
    d = np.float64
    h = np.where(r == maxc, bc - gc,
                 np.where(g == maxc, (2.0 + rc.astype(d) - bc.astype(d)).astype(np.float32),
                          (4.0 + gc.astype(d) - rc.astype(d)).astype(np.float32))).astype(np.float32)
    # float h promoted to double for /6.0 + 1.0 and fmod; stored back into the float h
    h = np.fmod(h.astype(np.float64) / 6.0 + 1.0, 1.0).astype(np.float32)
    uh = np.clip((h.astype(np.float64) * 255.0).astype(np.int64), 0, 255)
    us = np.clip((s.astype(np.float64) * 255.0).astype(np.int64), 0, 255)
    uh = np.where(eq, 0, uh)
    us = np.where(eq, 0, us)
    return np.stack([uh, us, v], -1).astype(np.uint8)


def hsv_to_rgb(hsv):
    """Pillow hsv2rgb (Convert.c): sector i = floor(h*6/255) in double; p, q, t
    rounded (C round: half away from zero) in double."""
    hf = hsv[..., 0].astype(np.float32).astype(np.float64)
    i = np.floor(hf * 6.0 / 255.0)
    f = (hf * 6.0 / 255.0 - i).astype(np.float32).astype(np.float64)
    fs = (hsv[..., 1].astype(np.float32).astype(np.float64) / 255.0).astype(np.float32).astype(np.float64)
    vf = hsv[..., 2].astype(np.float32).astype(np.float64)

    def rnd(x):   # C round(): half away from zero
        return np.sign(x) * np.floor(np.abs(x) + 0.5)
    p = np.clip(rnd(vf * (1.0 - fs)), 0, 255).astype(np.uint8)
    q = np.clip(rnd(vf * (1.0 - fs * f)), 0, 255).astype(np.uint8)
    t = np.clip(rnd(vf * (1.0 - fs * (1.0 - f))), 0, 255).astype(np.uint8)
    vv = hsv[..., 2]
    i = i.astype(np.int64) % 6
    sel = [(vv, t, p), (q, vv, p), (p, vv, t), (p, q, vv), (t, p, vv), (vv, p, q)]
    out = np.zeros(hsv.shape, np.uint8)
    for k, (a, b_, c) in enumerate(sel):
        m = i == k
        out[..., 0] = np.where(m, a, out[..., 0])
        out[..., 1] = np.where(m, b_, out[..., 1])
        out[..., 2] = np.where(m, c, out[..., 2])
    grey = hsv[..., 1] == 0
    for k in range(3):
        out[..., k] = np.where(grey, vv, out[..., k])
    return out


def hue_shift(hue_factor):
    """torchvision functional_pil.adjust_hue: np_h += np.int8(hue_factor * 255).astype(np.uint8)
    (truncation toward zero, two's-complement wrap of the hue band)."""
    return int(np.int8(np.float64(hue_factor) * 255)) & 0xFF


def adjust_hue(img, hue_factor):
    hsv = rgb_to_hsv(img)
    hsv[..., 0] = (hsv[..., 0].astype(np.int32) + hue_shift(hue_factor)) & 0xFF
    return hsv_to_rgb(hsv)


def color_jitter(img, perm, b, c, s, h):
    """transforms.ColorJitter.forward: the four adjustments in the drawn order."""
    for fn in perm:
        if fn == 0:
            img = adjust_brightness(img, b)
        elif fn == 1:
            img = adjust_contrast(img, c)
        elif fn == 2:
            img = adjust_saturation(img, s)
        else:
            img = adjust_hue(img, h)
    return img


def to_tensor_normalize(img):
    """ToTensor (u8 / 255 in fp32) + Normalize ((x - mean) / std, fp32) -> (3, H, W)."""
    x = img.astype(np.float32) / np.float32(255.0)
    m = np.array(IMAGENET_MEAN, np.float32)
    sd = np.array(IMAGENET_STD, np.float32)
    return ((x - m) / sd).transpose(2, 0, 1).copy()


def random_erase(x, box):
    """RandomErasing(value=0): zero the (i, j, h, w) box of the normalised tensor."""
    if box is not None:
        i, j, hh, ww = box
        x = x.copy()
        x[:, i:i + hh, j:j + ww] = 0.0
    return x


def train_transform(img, perm, b, c, s, h, box):
    """The whole train transform of one 224x224 uint8 RGB crop."""
    return random_erase(to_tensor_normalize(color_jitter(img, perm, b, c, s, h)), box)

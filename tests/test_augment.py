"""Train-time photometric augmentation (train_rgbd_geometric.py:41-47:
ColorJitter(0.3, 0.3, 0.3, 0.05) + ToTensor + Normalize + RandomErasing(p=0.2,
scale=(0.02, 0.1))).

CPU: the oracle's restatement of Pillow's arithmetic (oracle/augment.py) against the
Pillow importable in this image -- every RGB triple through convert("L"), the HSV
conversion both ways, and ImageEnhance.Brightness / Contrast / Color at factors
across the jitter range on random images.  torchvision (absent) is restated: its
parameter draw and op order are checked as properties on the GPU kernel's draws.
GPU: pose6d_crop_rgbd_train against the oracle replaying the kernel's own drawn
parameters, bit for bit; parameter distributions; identity / wrap / erase cases."""
import numpy as np
import pytest

from oracle import augment as A


def _all_rgb():
    c = np.arange(1 << 24, dtype=np.uint32)
    return np.stack([(c >> 16) & 255, (c >> 8) & 255, c & 255], -1).astype(np.uint8).reshape(4096, 4096, 3)


def test_oracle_color_conversions_match_pillow():
    Image = pytest.importorskip("PIL.Image")
    rgb = _all_rgb()
    assert np.array_equal(np.array(Image.fromarray(rgb, "RGB").convert("L")), A.to_l(rgb))
    assert np.array_equal(np.array(Image.fromarray(rgb, "RGB").convert("HSV")), A.rgb_to_hsv(rgb))
    # the same bytes read as HSV triples: every (h, s, v) back to RGB
    assert np.array_equal(np.array(Image.fromarray(rgb, "HSV").convert("RGB")), A.hsv_to_rgb(rgb))


@pytest.mark.parametrize("seed", range(6))
def test_oracle_enhance_ops_match_pillow(seed):
    Image = pytest.importorskip("PIL.Image")
    ImageEnhance = pytest.importorskip("PIL.ImageEnhance")
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, (64, 80, 3), dtype=np.uint8)
    if seed % 2:   # smooth image with saturated areas (clipping paths)
        img = np.clip(img.astype(np.int32) // 2 + 150, 0, 255).astype(np.uint8)
    pil = Image.fromarray(img, "RGB")
    factors = [0.7, 1.3, 1.0, 0.0] + list(rng.uniform(0.7, 1.3, 6))
    for f in factors:
        assert np.array_equal(np.array(ImageEnhance.Brightness(pil).enhance(f)), A.adjust_brightness(img, f)), f
        assert np.array_equal(np.array(ImageEnhance.Contrast(pil).enhance(f)), A.adjust_contrast(img, f)), f
        assert np.array_equal(np.array(ImageEnhance.Color(pil).enhance(f)), A.adjust_saturation(img, f)), f
    for hf in [-0.05, 0.05, 0.0, -0.031, 0.0449] + list(rng.uniform(-0.05, 0.05, 4)):
        h, s, v = pil.convert("HSV").split()
        nh = np.array(h, dtype=np.uint8)
        nh += np.int8(hf * 255).astype(np.uint8)   # torchvision functional_pil.adjust_hue
        ref = Image.merge("HSV", (Image.fromarray(nh, "L"), s, v)).convert("RGB")
        assert np.array_equal(np.array(ref), A.adjust_hue(img, hf)), hf


def test_oracle_transform_identity_and_erase():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (224, 224, 3), dtype=np.uint8)
    # factors 1 / hue 0: ColorJitter is the identity except the HSV round trip (hue op)
    same = A.color_jitter(img, [0, 1, 2], 1.0, 1.0, 1.0, 0.0)
    assert np.array_equal(same, img)
    x = A.train_transform(img, [0, 1, 2], 1.0, 1.0, 1.0, 0.0, (10, 20, 30, 40))
    ref = A.to_tensor_normalize(img)
    assert np.all(x[:, 10:40, 20:60] == 0)
    ref[:, 10:40, 20:60] = 0
    assert np.array_equal(x, ref)


# ----------------------------------------------------------------- GPU: the kernel
H, W = 480, 640
BBOXES = [(200, 150, 120, 90), (-20, -30, 100, 140), (600, 430, 90, 70), (310, 220, 9, 12), (100, 100, 187, 150),
          (150, 60, 374, 300), (33, 417, 57, 61), (400, 100, 200, 180)]


def _run(aug, B=32, seed=0):
    import torch
    from pose6d.data import CropRGBD
    rng = np.random.default_rng(seed)
    rgb = rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)
    if seed % 2:   # smooth, saturated content (contrast / clipping / grey-pixel paths)
        rgb = np.clip(rgb.astype(np.int32) // 3 + 170, 0, 255).astype(np.uint8)
        rgb[:, ::7] = 128
    depth = rng.integers(300, 1600, (B, H, W), dtype=np.uint16)
    bb = np.array([BBOXES[i % len(BBOXES)] for i in range(B)], np.int32)
    K = np.tile(np.array([[572.4114, 0, 325.2611], [0, 573.57043, 242.04899], [0, 0, 1]], np.float32), (B, 1, 1))
    d = lambda a: torch.from_numpy(a).cuda()
    crop = CropRGBD(224, augment=aug)
    out = crop(d(rgb), d(depth), d(bb), d(bb), d(K))
    torch.cuda.synchronize()
    params = crop.last_params.cpu().numpy() if crop.last_params is not None else None
    return rgb, bb, [o.cpu().numpy() for o in out], params


def _replay(rgb, bb, params, i):
    from oracle import crop as OC
    img = OC.resized_crop_u8(rgb[i], bb[i])
    p = params[i]
    box = None if p[10] < 0 else tuple(int(v) for v in p[8:12])
    return A.train_transform(img, [int(v) for v in p[:4]], *[float(v) for v in p[4:8]], box)


def _replay_nan_aware(rgb, bb, params, i):
    # factors reported NaN = op off: the oracle skips it (torchvision's None)
    from oracle import crop as OC
    img = OC.resized_crop_u8(rgb[i], bb[i])
    p = params[i]
    perm = [int(v) for v in p[:4] if not np.isnan(p[4 + int(v)])]
    f = [1.0 if np.isnan(v) else float(v) for v in p[4:8]]
    box = None if p[10] < 0 else tuple(int(v) for v in p[8:12])
    return A.random_erase(A.to_tensor_normalize(A.color_jitter(img, perm, *f)), box)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [0, 1, 2])
def test_train_transform_matches_oracle_bit_for_bit(seed):
    from pose6d.data import TrainAugment
    rgb, bb, out, params = _run(TrainAugment(seed=seed), seed=seed)
    for i in range(len(bb)):
        assert np.array_equal(out[0][i], _replay(rgb, bb, params, i)), f"crop {i}, params {params[i]}"


@pytest.mark.gpu
def test_train_transform_disabled_ops_and_wide_hue():
    """Ops switched off (factor 0 -> torchvision's None: no HSV round trip), and a
    hue range of +-0.5 (every shift of the uint8 hue band, wrapping both ways)."""
    from pose6d.data import TrainAugment
    rgb, bb, out, params = _run(TrainAugment(brightness=0, contrast=0.5, saturation=0, hue=0.5, erase_p=0.5), seed=5)
    assert np.isnan(params[:, 4]).all() and np.isnan(params[:, 6]).all()
    assert (params[:, 7] < -0.25).any() and (params[:, 7] > 0.25).any()
    for i in range(len(bb)):
        assert np.array_equal(out[0][i], _replay_nan_aware(rgb, bb, params, i)), f"crop {i}"


@pytest.mark.gpu
def test_train_transform_identity_equals_val_transform():
    """All jitter off and p = 0: the train path reproduces the val crop exactly; with
    p = 1 every crop has exactly its reported box zeroed and nothing else changed."""
    import torch
    from pose6d.data import TrainAugment
    rgb, bb, out_id, params = _run(TrainAugment(0, 0, 0, 0, erase_p=0.0), seed=3)
    _, _, out_val, _ = _run(None, seed=3)
    assert (params[:, 8:12] == -1).all()
    for a, b in zip(out_id, out_val):
        assert np.array_equal(a, b)
    _, _, out_er, params = _run(TrainAugment(0, 0, 0, 0, erase_p=1.0, seed=9), seed=3)
    assert (params[:, 10] > 0).all()
    for i in range(len(bb)):
        r, c, h, w = (int(v) for v in params[i, 8:12])
        assert 0 <= r and r + h <= 224 and 0 <= c and c + w <= 224
        ref = out_val[0][i].copy()
        ref[:, r:r + h, c:c + w] = 0
        assert np.array_equal(out_er[0][i], ref)
    for a, b in zip(out_er[1:], out_val[1:]):   # depth / centre / K untouched by the transform
        assert np.array_equal(a, b)
    del torch


@pytest.mark.gpu
def test_train_transform_parameter_distributions():
    """torchvision's distributions: a uniform random op order (randperm(4)), factors
    U[0.7, 1.3] / hue U[-0.05, 0.05], erasing with probability 0.2 and an area of
    0.02-0.1 of the crop at aspect 0.3-3.3 (up to the integer rounding of h, w)."""
    from pose6d.data import TrainAugment
    aug = TrainAugment(seed=123)
    ps = np.concatenate([_run(aug, B=32, seed=s)[3] for s in range(24)])   # 768 crops, fresh draws per call
    n = len(ps)
    perms = {tuple(int(v) for v in p[:4]) for p in ps}
    assert len(perms) == 24
    assert all(sorted(p) == [0, 1, 2, 3] for p in perms)
    first = np.bincount(ps[:, 0].astype(int), minlength=4) / n
    assert np.all(np.abs(first - 0.25) < 0.06), first
    for k in range(3):
        f = ps[:, 4 + k]
        assert f.min() >= 0.7 and f.max() <= 1.3 and abs(f.mean() - 1.0) < 0.03
    assert ps[:, 7].min() >= -0.05 and ps[:, 7].max() <= 0.05 and abs(ps[:, 7].mean()) < 0.005
    er = ps[ps[:, 10] > 0]
    assert abs(len(er) / n - 0.2) < 4 * (0.2 * 0.8 / n) ** 0.5, len(er) / n
    h, w = er[:, 10], er[:, 11]
    area = h * w / 224.0 ** 2
    assert area.min() > 0.015 and area.max() < 0.11
    assert (h / w).min() > 0.25 and (h / w).max() < 3.6
    assert (er[:, 8] + h <= 224).all() and (er[:, 9] + w <= 224).all() and (er[:, 8:10] >= 0).all()


def test_train_augment_seed_depends_on_rank():
    """Data-parallel ranks with one user seed draw different parameters (the rank is
    mixed into every kernel seed); rank 0 keeps the single-process sequence."""
    from pose6d.data import TrainAugment
    r0, r1, r0b = TrainAugment(seed=7, rank=0), TrainAugment(seed=7, rank=1), TrainAugment(seed=7)
    s0 = [r0.next_seed() for _ in range(4)]
    s1 = [r1.next_seed() for _ in range(4)]
    assert s0 == [r0b.next_seed() for _ in range(4)]   # no process group: rank 0
    assert len(set(s0) | set(s1)) == 8
    assert s0[0] == (7 * 0x9E3779B97F4A7C15 + 1) & 0xFFFFFFFFFFFFFFFF

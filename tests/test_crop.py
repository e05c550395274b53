"""GPU crop/resize/normalise of full frames (pose6d_crop_rgbd, pose6d/data.py)
against the oracle's restatement of data/dataset_rgbd.py:104-206 (oracle/crop.py).

The resize half of the oracle is PARITY UNPINNED (cv2 is absent from the image):
its CPU tests below pin it with hand-computed cases (identity at 224, constant
images, the exact-2x area path, zero padding); the GPU tests demand the kernel
reproduce the oracle bit for bit on every output."""
import numpy as np
import pytest
import torch

from oracle import crop as OC

H, W = 480, 640


def _frames(B, seed):
    rng = np.random.default_rng(seed)
    rgb = rng.integers(0, 256, (B, H, W, 3), dtype=np.uint8)
    depth = rng.integers(300, 1600, (B, H, W), dtype=np.uint16)
    depth[rng.random((B, H, W)) < 0.05] = 0
    K = np.tile(np.array([[572.4114, 0, 325.2611], [0, 573.57043, 242.04899], [0, 0, 1]], np.float32), (B, 1, 1))
    return rgb, depth, K


# (x, y, w, h): interior, padded left/top, padded right/bottom, tiny (upscale),
# crop side exactly 224 (187 * 1.2), exactly 448 (374 * 1.2 -> INTER_AREA), larger
# than the frame, odd sizes
BBOXES = [(200, 150, 120, 90), (-20, -30, 100, 140), (600, 430, 90, 70), (310, 220, 9, 12), (100, 100, 187, 150),
          (150, 60, 374, 300), (-100, -50, 900, 700), (33, 417, 57, 61)]


# ----------------------------------------------------------------- CPU: oracle pins
def test_oracle_geometry_hand_computed():
    # c = (140, 80), size = 96.0 -> x1 = 92, y1 = 32, no padding
    x1, y1, n, pl, pt, x1p, y1p = OC.crop_geometry((100, 50, 80, 60), H, W)
    assert (x1, y1, n, pl, pt, x1p, y1p) == (92, 32, 96, 0, 0, 92, 32)
    # c = (30, 40), size = 120 -> x1 = -30, y1 = -20: padded, origin (0, 0) in padded coords
    x1, y1, n, pl, pt, x1p, y1p = OC.crop_geometry((-20, -10, 100, 100), H, W)
    assert (x1, y1, n, pl, pt, x1p, y1p) == (-30, -20, 120, 30, 20, 0, 0)
    rgb, depth, K = _frames(1, 0)
    x, d, raw, c, Kc = OC.crop_sample(rgb[0], depth[0], (100, 50, 80, 60), (100, 50, 80, 60), K[0])
    s = np.float32(224 / 96)
    assert np.array_equal(c, np.array([(np.float32(140.0) - 92) * s, (np.float32(80.0) - 32) * s], np.float32))
    assert Kc[0, 0] == np.float32(572.4114) * s and Kc[0, 2] == (np.float32(325.2611) - np.float32(92)) * s


def test_oracle_resize_identity_and_constant():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, (224, 224, 3), dtype=np.uint8)
    assert np.array_equal(OC.resize_linear_u8(img), img)
    d = rng.integers(0, 65536, (224, 224)).astype(np.uint16)
    assert np.array_equal(OC.resize_linear_u16(d), d)
    for n in (37, 150, 301, 447, 449):
        for v in (0, 1, 127, 254, 255):
            c = np.full((n, n, 3), v, np.uint8)
            assert np.all(OC.resize_linear_u8(c) == v), (n, v)
        c = np.full((n, n), 1234, np.uint16)
        assert np.all(OC.resize_linear_u16(c) == 1234)


def test_oracle_resize_area_2x_and_padding():
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (448, 448, 3), dtype=np.uint8)
    s = img.astype(np.int64)
    ref = (s[0::2, 0::2] + s[0::2, 1::2] + s[1::2, 0::2] + s[1::2, 1::2] + 2) >> 2
    assert np.array_equal(OC.resize_linear_u8(img), ref.astype(np.uint8))
    frame = rng.integers(1, 256, (H, W, 3), dtype=np.uint8)
    crop = OC.crop_pixels(frame, -30, -20, 120)
    assert np.all(crop[:20] == 0) and np.all(crop[:, :30] == 0) and np.array_equal(crop[20:, 30:], frame[:100, :90])


def test_oracle_linear_weights_2to1_column():
    # upscaling a 2-pixel image: interior outputs are convex combinations (monotone)
    img = np.zeros((2, 2, 3), np.uint8)
    img[:, 1] = 200
    out = OC.resize_linear_u8(img)[0, :, 0].astype(int)
    assert out[0] == 0 and out[-1] == 200 and np.all(np.diff(out) >= 0)


def test_jitter_draw_order():
    from pose6d.data import jitter_bboxes
    bb = np.array([(200, 150, 120, 90), (10, 20, 30, 40), (5, 5, 7, 300)])
    for rgbd in (True, False):
        got = jitter_bboxes(bb, rgbd, np.random.RandomState(9))
        r = np.random.RandomState(9)
        assert [tuple(g) for g in got] == [OC.jitter_bbox(b, rgbd, r) for b in bb]


# ----------------------------------------------------------------- GPU: kernel == oracle
def _run_gpu(rgb, depth, bo, ba, K, bgr=False, normalize=True):
    from pose6d.data import CropRGBD
    dev = "cuda"
    crop = CropRGBD(224, normalize=normalize, bgr=bgr)
    d = torch.from_numpy(depth).to(dev) if depth is not None else None
    out = crop(torch.from_numpy(rgb).to(dev), d, torch.from_numpy(bo).to(dev), torch.from_numpy(ba).to(dev),
               torch.from_numpy(K).to(dev))
    torch.cuda.synchronize()
    return [t.cpu().numpy() for t in out]


def _check(got, rgb, depth, bo, ba, K, normalize=True):
    for i in range(len(bo)):
        kw = {} if normalize else {"mean": (0.0, 0.0, 0.0), "std": (1.0, 1.0, 1.0)}
        ref = OC.crop_sample(rgb[i], None if depth is None else depth[i], bo[i], ba[i], K[i], **kw)
        names = ("rgb", "depth", "depth_raw", "center", "K")
        for name, g, r in zip(names, got, ref):
            assert np.array_equal(g[i], r), f"sample {i} bbox {tuple(ba[i])}: {name} differs " \
                                            f"(max |d| {np.abs(g[i].astype(np.float64) - r).max():.3g})"


@pytest.mark.gpu
def test_crop_kernel_bit_exact():
    B = len(BBOXES)
    rgb, depth, K = _frames(B, 1)
    bo = np.array(BBOXES, np.int32)
    ba = np.array([OC.jitter_bbox(b, True, np.random.RandomState(i)) for i, b in enumerate(bo)], np.int32)
    ba[4], ba[5], ba[6] = bo[4], bo[5], bo[6]     # keep the exact-224 / exact-448 / oversize cases
    got = _run_gpu(rgb, depth, bo, ba, K)
    _check(got, rgb, depth, bo, ba, K)


@pytest.mark.gpu
def test_crop_kernel_no_depth_bgr_and_plain_totensor():
    B = 4
    rgb, _, K = _frames(B, 2)
    bo = np.array(BBOXES[:B], np.int32)
    got = _run_gpu(rgb, None, bo, bo, K, normalize=False)
    _check(got, rgb, None, bo, bo, K, normalize=False)
    assert np.all(got[1] == 0) and np.all(got[2] == 0)
    bgr = np.ascontiguousarray(rgb[..., ::-1])
    got_bgr = _run_gpu(bgr, None, bo, bo, K, bgr=True, normalize=False)
    assert np.array_equal(got_bgr[0], got[0])


@pytest.mark.gpu
def test_crop_random_bboxes_batch32():
    """The bench workload shape: 32 frames of 640x480, bbox w, h ~ U[40, 200]
    inside the frame, jittered like the training set."""
    B = 32
    rng = np.random.default_rng(7)
    rgb, depth, K = _frames(B, 3)
    w = rng.integers(40, 201, B)
    h = rng.integers(40, 201, B)
    bo = np.stack([rng.integers(0, W - w), rng.integers(0, H - h), w, h], 1).astype(np.int32)
    ba = np.array([OC.jitter_bbox(b, True, np.random.RandomState(100 + i)) for i, b in enumerate(bo)], np.int32)
    got = _run_gpu(rgb, depth, bo, ba, K)
    _check(got, rgb, depth, bo, ba, K)

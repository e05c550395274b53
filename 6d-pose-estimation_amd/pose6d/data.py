"""Device-side input crops for the pose models: the per-sample body of the
reference's LineMODDatasetRGBD / LineMODDatasetRGB.__getitem__
(data/dataset_rgbd.py:85-206, data/dataset_rgb.py:83-147) after the file reads,
batched into one pose6d_crop_rgbd launch.

The host keeps what is cheap and must stay bit-identical: the bbox jitter is
drawn with the reference's np.random calls in the reference's order
(`jitter_bboxes`), the rotation-matrix -> quaternion conversion and labels stay
with the caller.  Decoding the PNGs (cv2.imread) is I/O and stays on the host;
the full frames are uploaded once per batch and everything after the read --
padding, crop, resize, ToTensor/Normalize, depth normalisation, crop-adjusted
centre and intrinsics -- runs on the GPU.

The reference's TRAIN transform (train_rgbd_geometric.py:41-47: ColorJitter(0.3,
0.3, 0.3, 0.05) on the PIL crop, ToTensor, Normalize, RandomErasing(p=0.2,
scale=(0.02, 0.1))) runs on the GPU too: `CropRGBD(..., augment=TrainAugment())`
(pose6d_crop_rgbd_train -- torchvision's op order and parameter distributions,
Pillow's uint8 arithmetic, counter-based random draws keyed by (seed, batch counter,
crop); each crop's drawn parameters are returned for inspection / replay).
"""
import numpy as np
import torch

from ._lib import Pose6dError, call, query, require_device, stream

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


def jitter_bboxes(bboxes, rgbd=True, rng=np.random):
    """dataset_rgbd.py:110-118 (rgbd=True: +-5 % shift, +-10 % size) or
    dataset_rgb.py:101-110 (+-15 %, +-20 %): four rng.uniform draws per sample in
    the reference's order, int() truncation.  bboxes: (B, 4) ints -> (B, 4) int32."""
    a, b = (0.05, 0.1) if rgbd else (0.15, 0.2)
    out = np.zeros((len(bboxes), 4), np.int32)
    for i, (x, y, w, h) in enumerate(np.asarray(bboxes).astype(np.int64).tolist()):
        jx = int(rng.uniform(-a, a) * w)
        jy = int(rng.uniform(-a, a) * h)
        sw = int(rng.uniform(-b, b) * w)
        sh = int(rng.uniform(-b, b) * h)
        out[i] = (x + jx, y + jy, w + sw, h + sh)
    return out


class TrainAugment:
    """transforms.ColorJitter(brightness, contrast, saturation, hue) +
    transforms.RandomErasing(p, scale, ratio, value=0) of the reference's
    train_transform (train_rgbd_geometric.py:41-47), as pose6d_crop_rgbd_train runs
    them.  Each call of the owning CropRGBD draws fresh parameters: the kernel seed is
    (seed, rank, calls so far) -- deterministic for a given seed, rank and call sequence.

    `rank` (default: the torch.distributed rank when a process group is initialised,
    else 0) is mixed into every kernel seed, so that data-parallel ranks sharing one
    `seed` draw different jitter / erase parameters for their crop b (the reference's
    DataLoader workers draw from independent torch RNG streams).  Rank 0 keeps the
    single-process sequence.  The seed reaches the kernel as a by-value argument:
    do not capture a CropRGBD(augment=...) call into a hipGraph -- a replay would
    repeat the captured call's parameters."""

    def __init__(self, brightness=0.3, contrast=0.3, saturation=0.3, hue=0.05, erase_p=0.2, erase_scale=(0.02, 0.1),
                 erase_ratio=(0.3, 3.3), seed=0, rank=None):
        self.jitter = (float(brightness), float(contrast), float(saturation), float(hue))
        self.erase = (float(erase_p), float(erase_scale[0]), float(erase_scale[1]), float(erase_ratio[0]),
                      float(erase_ratio[1]))
        self.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        if rank is None:
            import torch.distributed as dist
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        self.rank = int(rank)
        self.calls = 0

    def next_seed(self):
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise Pose6dError("TrainAugment: the augmented crop must not be graph-captured (its seed is a "
                              "by-value kernel argument: every replay would repeat the same parameters)")
        s = (self.seed * 0x9E3779B97F4A7C15 + self.calls * 0xD1B54A32D192ED03 + 1
             + self.rank * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
        self.calls += 1
        return s


class CropRGBD:
    """Batched crop of full frames into the model inputs of the RGB-D datasets.

    __call__(rgb, depth, bbox_orig, bbox_aug=None, K) with device tensors
      rgb (B, H, W, 3) uint8 (RGB, or BGR with bgr=True), depth (B, H, W) uint16 mm
      or int16/int32 holding mm values < 65536 (converted), or None;
      bbox_orig / bbox_aug (B, 4) int (x, y, w, h); K (B, 3, 3) float
    returns (rgb (B,3,S,S), depth (B,1,S,S), depth_raw (B,S,S), bbox_center (B,2),
    camera_matrix (B,3,3)) -- the tensors dataset_rgbd.py:206 returns, batched.
    """

    def __init__(self, img_size=224, normalize=True, bgr=False, mean=IMAGENET_MEAN, std=IMAGENET_STD, augment=None):
        self.img_size = img_size
        self.augment = augment   # TrainAugment: the train transform (else the val transform)
        self.last_params = None  # (B, 16) per-crop parameters of the last augmented call
        self._ws = None
        self.normalize = normalize
        self.bgr = bgr
        self._ms = torch.tensor(list(mean) + list(std), dtype=torch.float32)
        self._ms_dev = {}

    def _mean_std(self, dev):
        if not self.normalize:
            return None
        t = self._ms_dev.get(dev)
        if t is None:
            t = self._ms_dev[dev] = self._ms.to(dev)
        return t

    def __call__(self, rgb, depth, bbox_orig, bbox_aug, K, out=None):
        require_device(rgb, depth, bbox_orig, bbox_aug, K)
        if rgb.dtype != torch.uint8 or rgb.dim() != 4 or rgb.shape[-1] != 3:
            raise Pose6dError(f"CropRGBD: rgb must be (B, H, W, 3) uint8, got {tuple(rgb.shape)} {rgb.dtype}")
        B, H, W, _ = rgb.shape
        dev = rgb.device
        if depth is not None:
            if tuple(depth.shape) != (B, H, W):
                raise Pose6dError(f"CropRGBD: depth must be (B, H, W) = {(B, H, W)}, got {tuple(depth.shape)}")
            if depth.dtype != torch.uint16:
                depth = depth.to(torch.int32).clamp_(0, 65535).to(torch.uint16)
            depth = depth.contiguous()
        if bbox_aug is None:
            bbox_aug = bbox_orig
        bo = bbox_orig.to(torch.int32).contiguous()
        ba = bbox_aug.to(torch.int32).contiguous()
        Kc = K.to(torch.float32).reshape(B, 3, 3).contiguous()
        S = self.img_size
        if out is None:
            out = (torch.empty(B, 3, S, S, device=dev), torch.empty(B, 1, S, S, device=dev),
                   torch.empty(B, S, S, device=dev), torch.empty(B, 2, device=dev), torch.empty(B, 3, 3, device=dev))
        if self.augment is None:
            call("crop_rgbd", rgb.contiguous(), int(self.bgr), depth, B, H, W, bo, ba, Kc, S, self._mean_std(dev),
                 *out, stream())
            return out
        nws = query("crop_train_workspace", B, S)
        if self._ws is None or self._ws.numel() < nws or self._ws.device != dev:
            self._ws = torch.empty(nws, device=dev, dtype=torch.uint8)
        self.last_params = torch.empty(B, 16, device=dev)
        a = self.augment
        call("crop_rgbd_train", rgb.contiguous(), int(self.bgr), depth, B, H, W, bo, ba, Kc, S, self._mean_std(dev),
             *a.jitter, *a.erase, a.next_seed(), self._ws, *out, self.last_params, stream())
        return out

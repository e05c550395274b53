"""LineMOD evaluation on the device path.

What sits around the hot path when the reference scores a model on LineMOD:

* the sample index of LineMODDatasetRGB / LineMODDatasetRGBD._load_data
  (data/dataset_rgb.py:31-78, data/dataset_rgbd.py:31-82): numeric object
  folders in sorted order; folders without gt.yml / info.yml (RGB-D: or without
  depth/) are skipped; PNG frames in sorted name order; the interleaved split
  on the frame's position i (i % 10 == 8 -> 'val', 9 -> 'test', else 'train');
  one sample per annotation of a frame present in both YAMLs whose obj_id
  matches the folder; obj_id = int(folder) - 1;
* the labels of __getitem__ (dataset_rgbd.py:97-102,182-185): quaternion =
  scipy Rotation.from_matrix(cam_R_m2c).as_quat() [x, y, z, w] as fp32,
  translation = fp32(cam_t_m2c) / 1000; the RGB dataset's bbox centre and K
  are the original-image ones (dataset_rgb.py:96,139-141), the RGB-D dataset's
  the crop-adjusted ones CropRGBD computes;
* evaluate_model of scripts/visualization/compare_all_models.py:65-104:
  batches in index order (DataLoader batch_size 16, shuffle=False), one
  ADDLoss.eval_metrics per batch, the mean of the per-batch values;
plus the per-object filter the reference lacks (`objects=("06",)` = cat).

Frames are decoded on the host with PIL.  PNG is lossless, so the RGB bytes
equal cv2.imread + COLOR_BGR2RGB, and 16-bit depth reads unchanged (the
IMREAD_UNCHANGED of dataset_rgbd.py:92); a missing depth file gives zeros like
dataset_rgbd.py:93-94.  Everything after the read -- pad, crop, resize,
ToTensor/Normalize, depth normalisation, crop intrinsics -- is one CropRGBD
launch per batch on the GPU.  Train-mode photometric augmentation (ColorJitter,
RandomErasing) is not part of this path (pose6d/data.py).
"""
import os

import numpy as np
import torch

from ._lib import Pose6dError
from .data import CropRGBD, jitter_bboxes

CAT_FOLDER = "06"   # LineMOD cat: folder 06 -> obj_id 5


def _split(i):
    """dataset_rgbd.py:58-65."""
    c = i % 10
    return "val" if c == 8 else "test" if c == 9 else "train"


def _safe_yaml(path):
    import yaml
    with open(path, "r") as f:
        return yaml.safe_load(f)


def load_rgb(path):
    """(H, W, 3) uint8 RGB of a PNG frame."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im.convert("RGB"), dtype=np.uint8)


def load_depth(path, shape):
    """(H, W) uint16 depth in mm; zeros when the file is missing or unreadable
    (dataset_rgbd.py:92-94)."""
    from PIL import Image
    try:
        with Image.open(path) as im:
            a = np.asarray(im)
    except (OSError, ValueError):
        return np.zeros(shape, np.uint16)
    if a.ndim == 3:      # IMREAD_UNCHANGED keeps every channel; the dataset only ever reads 1-channel depth
        raise Pose6dError(f"{path}: depth must be single-channel, got shape {a.shape}")
    return a.astype(np.uint16)


class LineMODSet:
    """The sample index of LineMODDatasetRGB(D)(root_dir, mode) plus batched,
    device-side sample preparation.

    objects: optional iterable of folder names ("06") or zero-based obj_ids (5)
    to keep -- the per-object filter of §8f #3; None keeps every object.
    """

    def __init__(self, root_dir, mode="train", rgbd=True, img_size=224, augment_bbox=True, objects=None):
        if not os.path.exists(root_dir):
            raise FileNotFoundError(f"Root dir not found: {root_dir}")
        self.root_dir, self.mode, self.rgbd, self.img_size = root_dir, mode, rgbd, img_size
        self.augment_bbox = augment_bbox and mode == "train"
        keep = None
        if objects is not None:
            keep = {str(int(o) + 1).zfill(2) if isinstance(o, (int, np.integer)) else str(o).zfill(2)
                    for o in objects}
        self.all_data = []
        for obj_folder in [f for f in sorted(os.listdir(root_dir)) if f.isdigit()]:
            if keep is not None and obj_folder not in keep:
                continue
            self._load_folder(obj_folder)
        self._crop = CropRGBD(img_size)

    def _load_folder(self, obj_folder):
        """dataset_rgbd.py:36-82 / dataset_rgb.py:35-78 for one object folder."""
        base = os.path.join(self.root_dir, obj_folder)
        gt_path, info_path = os.path.join(base, "gt.yml"), os.path.join(base, "info.yml")
        rgb_path, depth_path = os.path.join(base, "rgb"), os.path.join(base, "depth")
        if not os.path.exists(gt_path) or not os.path.exists(info_path):
            return
        if self.rgbd and not os.path.exists(depth_path):
            return
        gts, infos = _safe_yaml(gt_path), _safe_yaml(info_path)
        images = sorted(img for img in os.listdir(rgb_path) if img.endswith(".png"))
        for i, img_name in enumerate(images):
            frame_id = int(img_name.split(".")[0])
            if _split(i) != self.mode or frame_id not in gts or frame_id not in infos:
                continue
            for anno in gts[frame_id]:
                if str(int(anno["obj_id"])).zfill(2) == obj_folder:
                    item = {"img_path": os.path.join(rgb_path, img_name), "obj_id": int(obj_folder) - 1,
                            "bbox": anno["obj_bb"], "cam_R_m2c": anno["cam_R_m2c"], "cam_t_m2c": anno["cam_t_m2c"],
                            "cam_K": infos[frame_id]["cam_K"]}
                    if self.rgbd:
                        item["depth_path"] = os.path.join(depth_path, img_name)
                    self.all_data.append(item)

    def __len__(self):
        return len(self.all_data)

    @staticmethod
    def labels(items):
        """(quaternion (B,4), translation (B,3), obj_id (B,) int64) on the host,
        each built the way dataset_rgbd.py:182-185 builds it per sample."""
        from scipy.spatial.transform import Rotation
        q = torch.stack([torch.tensor(Rotation.from_matrix(np.array(it["cam_R_m2c"]).reshape(3, 3)).as_quat(),
                                      dtype=torch.float32) for it in items])
        t = torch.stack([torch.tensor(np.array(it["cam_t_m2c"]), dtype=torch.float32) / 1000.0 for it in items])
        ids = torch.tensor([it["obj_id"] for it in items], dtype=torch.long)
        return q, t, ids

    def batch(self, indices, device, rng=np.random):
        """The collated DataLoader batch for samples `indices`, on `device`:
        RGB-D (rgb, depth, depth_raw, quaternion, translation, obj_id, bbox_center,
        camera_matrix) as dataset_rgbd.py:206; RGB (rgb, quaternion, translation,
        obj_id, bbox_center, camera_matrix) as dataset_rgb.py:147."""
        items = [self.all_data[i] for i in indices]
        if not items:
            raise Pose6dError("LineMODSet.batch: empty index list")
        rgbs = [load_rgb(it["img_path"]) for it in items]
        shape = rgbs[0].shape
        if any(r.shape != shape for r in rgbs):
            raise Pose6dError(f"LineMODSet.batch: frames of one batch must share a size, got "
                              f"{sorted({r.shape for r in rgbs})}")
        rgb = torch.from_numpy(np.stack(rgbs)).to(device, non_blocking=True)
        depth = None
        if self.rgbd:
            depth = torch.from_numpy(np.stack([load_depth(it["depth_path"], shape[:2]) for it in items]))
            depth = depth.to(device, non_blocking=True)
        bo = np.array([it["bbox"] for it in items], np.int64)
        ba = jitter_bboxes(bo, self.rgbd, rng) if self.augment_bbox else bo.astype(np.int32)
        K = torch.from_numpy(np.stack([np.array(it["cam_K"]).reshape(3, 3).astype(np.float32) for it in items]))
        out = self._crop(rgb, depth, torch.from_numpy(bo.astype(np.int32)).to(device),
                         torch.from_numpy(ba).to(device), K.to(device))
        q, t, ids = (x.to(device) for x in self.labels(items))
        if self.rgbd:
            crop_rgb, crop_depth, depth_raw, center, Kc = out
            return crop_rgb, crop_depth, depth_raw, q, t, ids, center, Kc
        # dataset_rgb.py:96,139-141: original-image centre (Python float -> fp32) and K
        center = torch.tensor([[x + w / 2, y + h / 2] for x, y, w, h in bo.tolist()], dtype=torch.float32)
        return out[0], q, t, ids, center.to(device), K.to(device)

    def batches(self, batch_size=16, device="cuda", rng=np.random):
        """Index-order batches (DataLoader(shuffle=False, drop_last=False))."""
        for s in range(0, len(self), batch_size):
            yield self.batch(range(s, min(s + batch_size, len(self))), device, rng)


def evaluate_model(model, model_name, loader, criterion, is_rgbd=False, needs_geometry=False):
    """compare_all_models.py:65-104: per-batch eval_metrics, mean of the batch
    means.  `loader` yields the batches LineMODSet.batches makes (or any
    iterable of the reference's collated tuples already on the device)."""
    if model is None:
        return None
    model.eval()
    add, adds, acc = [], [], []
    with torch.no_grad():
        for batch in loader:
            if is_rgbd:
                rgb, depth, depth_raw, gt_rot, gt_trans, obj_ids, bbox_center, cam_matrix = batch
                if "Geometric" in model_name:
                    pred_rot, pred_trans = model(rgb, depth, depth_raw, bbox_center, cam_matrix)
                else:
                    pred_rot, pred_trans = model(rgb, depth)
            else:
                rgb, gt_rot, gt_trans, obj_ids, bbox_center, cam_matrix = batch
                if needs_geometry:
                    pred_rot, pred_trans = model(rgb, bbox_center, cam_matrix)
                else:
                    pred_rot, pred_trans = model(rgb)
            m = criterion.eval_metrics(pred_rot, pred_trans, gt_rot, gt_trans, obj_ids)
            add.append(m["add_mean"])
            adds.append(m["add_s_mean"])
            acc.append(m["add_01d_acc"])
    return {"ADD (mm)": np.mean(add), "ADD-S (mm)": np.mean(adds), "ADD-0.1d (%)": np.mean(acc)}

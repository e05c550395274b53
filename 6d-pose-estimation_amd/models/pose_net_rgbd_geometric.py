"""Drop-in for the reference's models/pose_net_rgbd_geometric.py.

PoseNetRGBDGeometric (pose_net_rgbd_geometric.py:13-85): ResNet50 on RGB -> BN-MLP
rotation head -> quaternion normalise; translation from one depth pixel through
the pinhole model (no learned part, no gradient).  Same constructor, forward
signature, parameter names and state_dict as the reference; the trunk, head,
normalise and pinhole run on pose6d's HIP kernels.
"""
import torch
import torch.nn as nn

from pose6d import ops
from pose6d.model_base import EngineModel
from pose6d.resnet import load_pretrained, resnet50_trunk


class PoseNetRGBDGeometric(EngineModel):
    """RGB backbone for rotation; translation directly from the depth sensor."""

    def __init__(self, pretrained=True):
        super().__init__()
        self.backbone = resnet50_trunk(3)
        if pretrained:
            load_pretrained(self.backbone)
        self.rot_head = nn.Sequential(
            nn.Linear(2048, 1024), nn.BatchNorm1d(1024), nn.ReLU(), nn.Dropout(0.3),
            nn.Linear(1024, 512), nn.BatchNorm1d(512), nn.ReLU(), nn.Dropout(0.2),
            nn.Linear(512, 4))
        self._p6_init()

    def forward(self, rgb, depth=None, depth_raw=None, bbox_center=None, camera_matrix=None):
        """RGB -> rotation; depth sensor -> translation (pose_net_rgbd_geometric.py:40-54)."""
        features = self._run_trunk("backbone", self.backbone, rgb, 3)
        rotation = ops.normalize(self._run_head("rot_head", self.rot_head, features, salt=1, copy=False))
        self._advance_seed()
        if depth_raw is not None and bbox_center is not None and camera_matrix is not None:
            translation = self._compute_pinhole_translation(depth_raw, bbox_center, camera_matrix)
        else:
            translation = torch.zeros(rgb.size(0), 3, device=rgb.device)
            translation[:, 2] = 0.5
        return rotation, translation

    def _compute_pinhole_translation(self, depth_raw, bbox_center, camera_matrix):
        """pose_net_rgbd_geometric.py:56-85 (HIP kernel pose6d_pinhole_depth)."""
        return ops.pinhole_depth(depth_raw, bbox_center, camera_matrix)

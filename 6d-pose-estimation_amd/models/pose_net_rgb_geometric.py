"""Drop-in for the reference's models/pose_net_rgb_geometric.py
(PoseNetRGBGeometric, pose_net_rgb_geometric.py:8-109).

ResNet50 -> rotation head (normalised with ||q|| + 1e-8); lightweight z-CNN +
z-MLP -> depth z; x, y from the pinhole model (differentiable in z).
"""
import torch
import torch.nn as nn

from pose6d import ops
from pose6d.model_base import EngineModel
from pose6d.resnet import load_pretrained, resnet50_trunk


class PoseNetRGBGeometric(EngineModel):
    """Learns rotation and Z-depth; computes X, Y with the pinhole camera model."""

    def __init__(self, pretrained=True):
        super().__init__()
        self.rgb_backbone = resnet50_trunk(3)
        if pretrained:
            load_pretrained(self.rgb_backbone)
        self.rot_head = nn.Sequential(
            nn.Linear(2048, 1024), nn.BatchNorm1d(1024), nn.ReLU(), nn.Dropout(0.3),
            nn.Linear(1024, 512), nn.BatchNorm1d(512), nn.ReLU(), nn.Dropout(0.2),
            nn.Linear(512, 4))
        self.z_backbone = nn.Sequential(
            nn.Conv2d(3, 32, kernel_size=7, stride=2, padding=3), nn.BatchNorm2d(32), nn.ReLU(), nn.MaxPool2d(2),
            nn.Conv2d(32, 64, kernel_size=5, stride=1, padding=2), nn.BatchNorm2d(64), nn.ReLU(), nn.MaxPool2d(2),
            nn.Conv2d(64, 128, kernel_size=3, stride=1, padding=1), nn.BatchNorm2d(128), nn.ReLU(), nn.MaxPool2d(2),
            nn.Conv2d(128, 256, kernel_size=3, stride=1, padding=1), nn.BatchNorm2d(256), nn.ReLU(),
            nn.MaxPool2d(2),
            nn.AdaptiveAvgPool2d(1), nn.Flatten())
        self.z_predictor = nn.Sequential(
            nn.Linear(256, 128), nn.ReLU(), nn.Dropout(0.2),
            nn.Linear(128, 64), nn.ReLU(),
            nn.Linear(64, 1))
        self.z_predictor[-1].bias.data.fill_(0.5)   # pose_net_rgb_geometric.py:68
        self._p6_init()

    def forward(self, rgb, bbox_center=None, camera_matrix=None):
        """pose_net_rgb_geometric.py:70-91."""
        rgb_features = self._run_trunk("rgb_backbone", self.rgb_backbone, rgb, 3)
        rotation = ops.normalize_eps(self._run_head("rot_head", self.rot_head, rgb_features, salt=1, copy=False))
        z_features = self._run_trunk("z_backbone", self.z_backbone, rgb, 3, kind="zcnn")
        z_pred = self._run_head("z_predictor", self.z_predictor, z_features, salt=2)
        self._advance_seed()
        if bbox_center is not None and camera_matrix is not None:
            translation = self._compute_pinhole_translation(z_pred, bbox_center, camera_matrix)
        else:
            translation = torch.cat([torch.zeros_like(z_pred), torch.zeros_like(z_pred), z_pred], dim=1)
        return rotation, translation

    def _compute_pinhole_translation(self, z_pred, bbox_center, camera_matrix):
        """pose_net_rgb_geometric.py:93-109 (HIP kernels pose6d_pinhole_z_fwd/_bwd)."""
        return ops.pinhole_z(z_pred, bbox_center, camera_matrix)

"""Drop-in for the reference's models/pose_net_rgb.py (PoseNetRGB, pose_net_rgb.py:8-65).

ResNet50 trunk + two BN-MLP heads (rotation -> normalised quaternion, translation
with z-bias 0.5), on pose6d's HIP kernels; reference parameter names/state_dict.
"""
import torch.nn as nn

from pose6d import ops
from pose6d.model_base import EngineModel
from pose6d.resnet import load_pretrained, resnet50_trunk


def _bn_mlp(out_dim):
    return nn.Sequential(
        nn.Linear(2048, 2048), nn.BatchNorm1d(2048), nn.ReLU(), nn.Dropout(0.3),
        nn.Linear(2048, 1024), nn.BatchNorm1d(1024), nn.ReLU(), nn.Dropout(0.2),
        nn.Linear(1024, 512), nn.ReLU(),
        nn.Linear(512, out_dim))


class PoseNetRGB(EngineModel):
    """Predicts rotation (quaternion) and translation (x, y, z) from RGB."""

    def __init__(self, pretrained=True):
        super().__init__()
        self.backbone = resnet50_trunk(3)
        if pretrained:
            load_pretrained(self.backbone)
        self.rot_head = _bn_mlp(4)
        self.trans_head = _bn_mlp(3)
        # translation bias -> typical depth (pose_net_rgb.py:53-54)
        self.trans_head[-1].bias.data.fill_(0)
        self.trans_head[-1].bias.data[2] = 0.5
        self._p6_init()

    def forward(self, x):
        """RGB image -> (rotation, translation) (pose_net_rgb.py:56-65)."""
        features = self._run_trunk("backbone", self.backbone, x, 3)
        rotation = ops.normalize(self._run_head("rot_head", self.rot_head, features, salt=1, copy=False))
        translation = self._run_head("trans_head", self.trans_head, features, salt=2)
        self._advance_seed()
        return rotation, translation

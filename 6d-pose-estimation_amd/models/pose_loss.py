"""Drop-in for the reference's models/pose_loss.py (PoseLoss, pose_loss.py:7-65).

Same constructor, same forward signature; the loss and its gradient run in
pose6d's HIP kernels (pose6d_pose_loss_fwd / _bwd) -- one launch each.
"""
import torch
import torch.nn as nn

from pose6d import ops


class PoseLoss(nn.Module):
    """Rotation loss (geodesic or quaternion-L1) + L1 translation loss."""

    def __init__(self, rot_weight=1.0, trans_weight=1.0, rotation_loss='geodesic'):
        super().__init__()
        self.rot_weight = rot_weight
        self.trans_weight = trans_weight
        self.rotation_loss_type = rotation_loss

    def forward(self, pred_rot, pred_trans, gt_rot, gt_trans, obj_ids=None):
        mode = 0 if self.rotation_loss_type == 'geodesic' else 1
        return ops.pose_loss(pred_rot, pred_trans, gt_rot, gt_trans, float(self.rot_weight),
                             float(self.trans_weight), mode)

    def train_loss(self, pred_rot, pred_trans, gt_rot, gt_trans, obj_ids=None):
        """Alias for forward() (pose_loss.py:63-65)."""
        return self.forward(pred_rot, pred_trans, gt_rot, gt_trans, obj_ids)

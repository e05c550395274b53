"""Drop-in for the reference's models/pose_net_rgbd.py (CrossModalAttention,
PoseNetRGBD; pose_net_rgbd.py:8-142).

Two ResNet50 trunks (RGB, and depth with a 1-channel stem) -> LayerNorm each ->
cross-modal attention (8 heads of 256) with a residual onto the RGB feature ->
concat (B, 4096) -> fusion MLP (Linear / LayerNorm / GELU / Dropout) -> rotation
(normalised) and translation heads.  Same parameter names, shapes and
state_dict keys as the reference (672 entries); all math runs on pose6d's HIP
kernels (trunks: TrunkEngine; norms + attention: FusionEngine; MLPs: HeadEngine).
"""
import torch
import torch.nn as nn

from pose6d import fusion, ops
from pose6d.model_base import EngineModel
from pose6d.resnet import load_pretrained, resnet50_trunk


class CrossModalAttention(nn.Module):
    """Cross-modal attention for RGB-Depth feature fusion (pose_net_rgbd.py:8-35)."""

    def __init__(self, dim, num_heads=8, dropout=0.1):
        super().__init__()
        self.num_heads = num_heads
        self.head_dim = dim // num_heads
        self.scale = self.head_dim ** -0.5
        self.q_proj = nn.Linear(dim, dim)
        self.k_proj = nn.Linear(dim, dim)
        self.v_proj = nn.Linear(dim, dim)
        self.out_proj = nn.Linear(dim, dim)
        self.dropout = nn.Dropout(dropout)
        self._p6_engine = None
        self.register_buffer("_p6_seed", torch.tensor([torch.initial_seed() & 0x7FFFFFFFFFFF], dtype=torch.int64),
                             persistent=False)

    def forward(self, rgb_feat, depth_feat):
        """out_proj(dropout(softmax(q k^T * scale)) v) (pose_net_rgbd.py:23-35)."""
        if self._p6_engine is None:
            self._p6_engine = fusion.FusionEngine(self)
        out = fusion.run(self._p6_engine, rgb_feat, depth_feat, self.training, seed_dev=self._p6_seed, salt=11)
        if self.training:
            with torch.no_grad():
                self._p6_seed.add_(1)
        return out


class PoseNetRGBD(EngineModel):
    """RGB-D pose estimation with cross-modal attention fusion (pose_net_rgbd.py:38-142)."""

    def __init__(self, pretrained=True):
        super().__init__()
        self.rgb_backbone = resnet50_trunk(3)
        self.depth_backbone = resnet50_trunk(3)
        if pretrained:
            load_pretrained(self.rgb_backbone)
            load_pretrained(self.depth_backbone)
        # depth stem: a fresh 1-channel conv (default nn.Conv2d init, pose_net_rgbd.py:55);
        # with pretrained weights it is the RGB stem summed over its input channels (:57-59)
        rgb_conv1 = self.depth_backbone[0]
        self.depth_backbone[0] = nn.Conv2d(1, 64, kernel_size=7, stride=2, padding=3, bias=False)
        if pretrained:
            with torch.no_grad():
                self.depth_backbone[0].weight.copy_(rgb_conv1.weight.sum(dim=1, keepdim=True))
        feat_dim, fused_dim = 2048, 1024
        self.rgb_norm = nn.LayerNorm(feat_dim)
        self.depth_norm = nn.LayerNorm(feat_dim)
        self.cross_attention = CrossModalAttention(feat_dim, num_heads=8, dropout=0.1)
        self.fusion = nn.Sequential(
            nn.Linear(feat_dim * 2, fused_dim), nn.LayerNorm(fused_dim), nn.GELU(), nn.Dropout(0.2),
            nn.Linear(fused_dim, fused_dim), nn.LayerNorm(fused_dim), nn.GELU())
        self.rot_head = nn.Sequential(
            nn.Linear(fused_dim, 512), nn.LayerNorm(512), nn.GELU(), nn.Dropout(0.1),
            nn.Linear(512, 256), nn.GELU(), nn.Linear(256, 4))
        self.trans_head = nn.Sequential(
            nn.Linear(fused_dim, 512), nn.LayerNorm(512), nn.GELU(), nn.Dropout(0.1),
            nn.Linear(512, 256), nn.GELU(), nn.Linear(256, 3))
        self._init_weights()
        self._p6_init()

    def _init_weights(self):
        """xavier-uniform Linear weights, zero biases, translation z-bias 0.5 (pose_net_rgbd.py:107-116)."""
        for m in [self.fusion, self.rot_head, self.trans_head]:
            for layer in m:
                if isinstance(layer, nn.Linear):
                    nn.init.xavier_uniform_(layer.weight)
                    if layer.bias is not None:
                        nn.init.zeros_(layer.bias)
        self.trans_head[-1].bias.data[2] = 0.5

    def forward(self, rgb, depth, depth_raw=None, bbox_center=None, camera_matrix=None):
        """RGB + depth -> (rotation, translation) (pose_net_rgbd.py:118-142); the
        geometric arguments are accepted and unused, as in the reference."""
        rgb_feat = self._run_trunk("rgb_backbone", self.rgb_backbone, rgb, 3)
        depth_feat = self._run_trunk("depth_backbone", self.depth_backbone, depth, 1)
        eng = self._engine("fusion_core", lambda: fusion.FusionEngine(self.cross_attention, self.rgb_norm,
                                                                      self.depth_norm))
        combined = fusion.run(eng, rgb_feat, depth_feat, self.training, seed_dev=self._p6_seed, salt=3)
        fused = self._run_head("fusion", self.fusion, combined, salt=4)
        rotation = ops.normalize(self._run_head("rot_head", self.rot_head, fused, salt=5, copy=False))
        translation = self._run_head("trans_head", self.trans_head, fused, salt=6)
        self._advance_seed()
        return rotation, translation

    def count_parameters(self):
        """Count trainable parameters (pose_net_rgbd.py:144-146)."""
        return sum(p.numel() for p in self.parameters() if p.requires_grad)

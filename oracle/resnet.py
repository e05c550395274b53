"""ORACLE — test infrastructure only.  torch-CPU fp32 functional restatement of
the four PoseNet models of SFR-Vision/6d-pose-estimation.

The trunk is torchvision==0.24.1's ResNet50 (requirements.txt:6; third-party and
absent from this image), restated from its published definition: stem conv7x7/s2
+ BN + ReLU + maxpool3/s2, Bottleneck v1.5 stages [3, 4, 6, 3] (stride on the
3x3), AdaptiveAvgPool(1); wrapped as nn.Sequential(*children[:-1]) by every
model (pose_net_rgb.py:18-20), hence the state_dict prefixes `<trunk>.0` (conv1),
`.1` (bn1), `.4`-`.7` (layer1-4).

Every function takes `P`, a dict of parameters AND buffers keyed by the
reference's state_dict names.  In training mode BatchNorm uses batch statistics
and updates P's running buffers in place (torch semantics: biased variance for
normalisation, unbiased for running_var, momentum 0.1).  Dropout is the identity
here (parity runs use Dropout in eval).
"""
import torch
import torch.nn.functional as F

LAYERS = [3, 4, 6, 3]
PLANES = [64, 128, 256, 512]
STRIDES = [1, 2, 2, 2]


def _bn(x, P, name, training):
    return F.batch_norm(x, P[name + ".running_mean"], P[name + ".running_var"], P[name + ".weight"],
                        P[name + ".bias"], training=training, momentum=0.1, eps=1e-5)


def _bn_count(P, name, training):
    if training:
        P[name + ".num_batches_tracked"] += 1


def bn(x, P, name, training):
    _bn_count(P, name, training)
    return _bn(x, P, name, training)


def trunk(x, P, pre, training):
    """ResNet50 without fc: (B, Cin, H, W) -> (B, 2048)."""
    x = F.conv2d(x, P[f"{pre}.0.weight"], stride=2, padding=3)
    x = F.relu(bn(x, P, f"{pre}.1", training))
    x = F.max_pool2d(x, 3, 2, 1)
    inplanes = 64
    for li, (n, planes, stride) in enumerate(zip(LAYERS, PLANES, STRIDES)):
        for bi in range(n):
            s = stride if bi == 0 else 1
            b = f"{pre}.{4 + li}.{bi}"
            idn = x
            y = F.relu(bn(F.conv2d(x, P[b + ".conv1.weight"]), P, b + ".bn1", training))
            y = F.relu(bn(F.conv2d(y, P[b + ".conv2.weight"], stride=s, padding=1), P, b + ".bn2", training))
            y = bn(F.conv2d(y, P[b + ".conv3.weight"]), P, b + ".bn3", training)
            if bi == 0:
                idn = bn(F.conv2d(x, P[b + ".downsample.0.weight"], stride=s), P, b + ".downsample.1", training)
            x = F.relu(y + idn)
            inplanes = planes * 4
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


def _trunk_or(features, x, P, pre, training):
    """The trunk's (B, 2048) features, or -- when `features` maps this trunk's
    prefix to a tensor -- that tensor (the trunk hook the model fixture of
    tests/golden/models.npz is checked through: it pins everything around the trunk)."""
    if features is not None and pre in features:
        return features[pre]
    return trunk(x, P, pre, training)


def _lin(x, P, name):
    return F.linear(x, P[name + ".weight"], P[name + ".bias"])


def bn_mlp(x, P, pre, dims, training):
    """Linear/BN1d/ReLU/Dropout blocks then ReLU?/Linear, as in pose_net_rgb.py:23-35
    (dims = [in, h1, h2, (h3,) out]; `h3` present -> a plain Linear+ReLU before out)."""
    idx = 0
    x = F.relu(bn(_lin(x, P, f"{pre}.{idx}"), P, f"{pre}.{idx + 1}", training)); idx += 4
    x = F.relu(bn(_lin(x, P, f"{pre}.{idx}"), P, f"{pre}.{idx + 1}", training)); idx += 4
    if len(dims) == 5:
        x = F.relu(_lin(x, P, f"{pre}.{idx}")); idx += 2
    return _lin(x, P, f"{pre}.{idx}")


def normalize(q):
    return F.normalize(q, p=2, dim=1)


def pinhole_rgbd_geometric(depth_raw, bbox_center, K):
    """pose_net_rgbd_geometric.py:56-85."""
    B = depth_raw.shape[0]
    if K.dim() == 2:
        K = K.unsqueeze(0).expand(B, -1, -1)
    fx, fy, cx, cy = K[:, 0, 0], K[:, 1, 1], K[:, 0, 2], K[:, 1, 2]
    u = bbox_center[:, 0].clamp(0, 223)
    v = bbox_center[:, 1].clamp(0, 223)
    ui = u.long().clamp(0, 223)
    vi = v.long().clamp(0, 223)
    z = depth_raw[torch.arange(B), vi, ui]
    z = torch.where(z > 0.01, z, torch.tensor(0.5))
    z = torch.clamp(z, min=0.1, max=2.0)
    return torch.stack([(u - cx) * z / fx, (v - cy) * z / fy, z], dim=1)


def pinhole_rgb_geometric(z, bbox_center, K):
    """pose_net_rgb_geometric.py:93-109 (no clamps)."""
    if K.dim() == 2:
        K = K.unsqueeze(0).expand(z.size(0), -1, -1)
    fx, fy = K[:, 0, 0].unsqueeze(1), K[:, 1, 1].unsqueeze(1)
    cx, cy = K[:, 0, 2].unsqueeze(1), K[:, 1, 2].unsqueeze(1)
    u, v = bbox_center[:, 0].unsqueeze(1), bbox_center[:, 1].unsqueeze(1)
    return torch.cat([(u - cx) * z / fx, (v - cy) * z / fy, z], dim=1)


def forward_rgb(P, x, training, features=None):
    """pose_net_rgb.py:56-65."""
    f = _trunk_or(features, x, P, "backbone", training)
    rot = normalize(bn_mlp(f, P, "rot_head", [2048, 2048, 1024, 512, 4], training))
    trans = bn_mlp(f, P, "trans_head", [2048, 2048, 1024, 512, 3], training)
    return rot, trans


def forward_rgbd_geometric(P, rgb, depth=None, depth_raw=None, bbox_center=None, K=None, training=False,
                           features=None):
    """pose_net_rgbd_geometric.py:40-54."""
    f = _trunk_or(features, rgb, P, "backbone", training)
    rot = normalize(bn_mlp(f, P, "rot_head", [2048, 1024, 512, 4], training))
    if depth_raw is not None and bbox_center is not None and K is not None:
        trans = pinhole_rgbd_geometric(depth_raw, bbox_center, K)
    else:
        trans = torch.zeros(rgb.size(0), 3)
        trans[:, 2] = 0.5
    return rot, trans


def z_backbone(x, P, training):
    """pose_net_rgb_geometric.py:36-55."""
    for i in (0, 4, 8, 12):
        x = F.conv2d(x, P[f"z_backbone.{i}.weight"], P[f"z_backbone.{i}.bias"], stride=2 if i == 0 else 1,
                     padding={0: 3, 4: 2, 8: 1, 12: 1}[i])
        x = F.max_pool2d(F.relu(bn(x, P, f"z_backbone.{i + 1}", training)), 2)
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)


def forward_rgb_geometric(P, rgb, bbox_center=None, K=None, training=False, features=None):
    """pose_net_rgb_geometric.py:70-91."""
    f = _trunk_or(features, rgb, P, "rgb_backbone", training)
    r = bn_mlp(f, P, "rot_head", [2048, 1024, 512, 4], training)
    rot = r / (torch.norm(r, dim=1, keepdim=True) + 1e-8)
    z = z_backbone(rgb, P, training)
    z = F.relu(_lin(z, P, "z_predictor.0"))
    z = F.relu(_lin(z, P, "z_predictor.3"))
    z = _lin(z, P, "z_predictor.5")
    if bbox_center is not None and K is not None:
        trans = pinhole_rgb_geometric(z, bbox_center, K)
    else:
        trans = torch.cat([torch.zeros_like(z), torch.zeros_like(z), z], dim=1)
    return rot, trans


def _ln(x, P, name):
    return F.layer_norm(x, (x.shape[-1],), P[name + ".weight"], P[name + ".bias"], eps=1e-5)


def cross_attention(r, d, P, pre="cross_attention", heads=8):
    """pose_net_rgbd.py:23-35 (dropout = identity)."""
    B, D = r.shape
    hd = D // heads
    q = _lin(r, P, pre + ".q_proj").view(B, heads, hd)
    k = _lin(d, P, pre + ".k_proj").view(B, heads, hd)
    v = _lin(d, P, pre + ".v_proj").view(B, heads, hd)
    a = ((q @ k.transpose(-2, -1)) * hd ** -0.5).softmax(dim=-1)
    return _lin((a @ v).reshape(B, -1), P, pre + ".out_proj")


def _gelu_head(x, P, pre):
    x = F.gelu(_ln(_lin(x, P, pre + ".0"), P, pre + ".1"))
    x = F.gelu(_lin(x, P, pre + ".4"))
    return _lin(x, P, pre + ".6")


def forward_rgbd(P, rgb, depth, depth_raw=None, bbox_center=None, K=None, training=False, features=None):
    """pose_net_rgbd.py:118-142."""
    B = rgb.size(0)
    r = _ln(_trunk_or(features, rgb, P, "rgb_backbone", training), P, "rgb_norm")
    d = _ln(_trunk_or(features, depth, P, "depth_backbone", training), P, "depth_norm")
    r_enh = r + cross_attention(r, d, P)
    x = torch.cat([r_enh, d], dim=1)
    x = F.gelu(_ln(_lin(x, P, "fusion.0"), P, "fusion.1"))
    x = F.gelu(_ln(_lin(x, P, "fusion.4"), P, "fusion.5"))
    rot = normalize(_gelu_head(x, P, "rot_head"))
    trans = _gelu_head(x, P, "trans_head")
    assert rot.shape == (B, 4)
    return rot, trans

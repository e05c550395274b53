"""ResNet50 module tree with torchvision's parameter names (the trunk every
reference model wraps as nn.Sequential(*list(resnet50().children())[:-1]),
pose_net_rgb.py:18-20).  Parameters only: the computation runs in
pose6d.trunk.TrunkEngine on the HIP kernels.

torchvision==0.24.1 (requirements.txt:6) is absent from this image; this restates
its public ResNet50 definition (Bottleneck v1.5, layers [3, 4, 6, 3]) and init
(kaiming_normal_(fan_out, relu) for convs, BN weight 1 / bias 0), so state_dicts
interchange with the reference's (same keys, shapes, OIHW layout).
"""
import os
import warnings

import torch
import torch.nn as nn

LAYERS = [3, 4, 6, 3]
PLANES = [64, 128, 256, 512]
STRIDES = [1, 2, 2, 2]
EXPANSION = 4


class Bottleneck(nn.Module):
    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * EXPANSION, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * EXPANSION)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride


def _layer(inplanes, planes, blocks, stride):
    ds = None
    if stride != 1 or inplanes != planes * EXPANSION:
        ds = nn.Sequential(nn.Conv2d(inplanes, planes * EXPANSION, 1, stride=stride, bias=False),
                           nn.BatchNorm2d(planes * EXPANSION))
    mods = [Bottleneck(inplanes, planes, stride, ds)]
    for _ in range(1, blocks):
        mods.append(Bottleneck(planes * EXPANSION, planes))
    return nn.Sequential(*mods)


def resnet50_trunk(in_channels=3):
    """nn.Sequential(conv1, bn1, relu, maxpool, layer1..4, avgpool) == children()[:-1]."""
    mods = [nn.Conv2d(in_channels, 64, 7, stride=2, padding=3, bias=False), nn.BatchNorm2d(64), nn.ReLU(inplace=True),
            nn.MaxPool2d(3, 2, 1)]
    inplanes = 64
    for n, planes, stride in zip(LAYERS, PLANES, STRIDES):
        mods.append(_layer(inplanes, planes, n, stride))
        inplanes = planes * EXPANSION
    mods.append(nn.AdaptiveAvgPool2d((1, 1)))
    seq = nn.Sequential(*mods)
    for m in seq.modules():
        if isinstance(m, nn.Conv2d):
            nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
        elif isinstance(m, nn.BatchNorm2d):
            nn.init.constant_(m.weight, 1)
            nn.init.constant_(m.bias, 0)
    return seq


class PretrainedWeightsUnavailable(RuntimeError):
    """pretrained=True without local ImageNet weights (the reference's
    resnet50(weights=ResNet50_Weights.DEFAULT) raises when the download fails)."""


def load_pretrained(seq):
    """ImageNet weights (torchvision ResNet50_Weights.DEFAULT, pose_net_rgbd_geometric.py:23-25)
    cannot be downloaded here; POSE6D_RESNET50_WEIGHTS must name a local torchvision
    resnet50 state_dict (loaded weights_only).  Without one this raises, as the
    reference does when its download is impossible, so that an unchanged training
    script cannot silently train from random init; POSE6D_ALLOW_RANDOM_INIT=1 opts
    into the random init explicitly (a warning is still emitted)."""
    path = os.environ.get("POSE6D_RESNET50_WEIGHTS")
    if not path or not os.path.exists(path):
        msg = ("pretrained=True: no local ResNet50 ImageNet weights (set POSE6D_RESNET50_WEIGHTS to a torchvision "
               "resnet50 state_dict, or POSE6D_ALLOW_RANDOM_INIT=1 to train from random init)")
        if os.environ.get("POSE6D_ALLOW_RANDOM_INIT", "") not in ("1", "true", "yes"):
            raise PretrainedWeightsUnavailable(msg + (f"; {path!r} does not exist" if path else ""))
        warnings.warn(msg + ": using random init", RuntimeWarning, stacklevel=3)
        return False
    sd = torch.load(path, map_location="cpu", weights_only=True)
    names = {"conv1": "0", "bn1": "1", "layer1": "4", "layer2": "5", "layer3": "6", "layer4": "7"}
    mapped = {}
    for k, v in sd.items():
        head = k.split(".")[0]
        if head in names:
            mapped[names[head] + k[len(head):]] = v
    seq.load_state_dict(mapped, strict=True)
    return True

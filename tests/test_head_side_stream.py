"""The one-GPU step with the head's Linear weight gradients on a side stream
(pose6d.train.step_body(branch=True), the captured graph's parallel branch) equals the
one-chain step (POSE6D_HEAD_WGRAD_SIDE off) bit for bit: the same launches on the same
operands, only their overlap differs."""
import copy
import warnings

import pytest
import torch


def _trainers(dtype, B=4):
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    warnings.simplefilter("ignore")
    torch.manual_seed(0)
    m0 = PoseNetRGBDGeometric(pretrained=False)
    return [RGBDGeometricTrainer(copy.deepcopy(m0).cuda(), B, dtype=dtype) for _ in range(2)]


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_head_wgrad_side_stream_bit_identical(dtype, monkeypatch):
    from bench import synth_batch
    from pose6d import train
    side, chain = _trainers(dtype)
    data = synth_batch(4, torch.device("cuda"), seed=21)
    monkeypatch.setattr(train, "POSE6D_HEAD_WGRAD_SIDE", True)
    side.capture(data, warmup=1)
    monkeypatch.setattr(train, "POSE6D_HEAD_WGRAD_SIDE", False)
    chain.capture(data, warmup=1)
    assert hasattr(side, "_side") and not hasattr(chain, "_side")
    for step in range(3):
        side.step()
        chain.step()
        torch.cuda.synchronize()
        assert torch.equal(side.arena.grad, chain.arena.grad), f"step {step}: gradients differ"
        assert torch.equal(side.arena.flat, chain.arena.flat), f"step {step}: parameters differ"
        assert torch.equal(side.m, chain.m) and torch.equal(side.v, chain.v), f"step {step}: moments differ"
        assert torch.equal(side.loss, chain.loss)

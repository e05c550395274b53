"""Checkpoint interop: the reference's checkpoint dict
(train_rgbd_geometric.py:151-157 -- epoch, model_state_dict, optimizer_state_dict,
best_acc, curr_acc) written and resumed by the fused trainer, and by the drop-in
module driven the reference's way (torch AdamW), loadable with the safe loader."""
import io
import warnings

import pytest
import torch


def _roundtrip(obj):
    buf = io.BytesIO()
    torch.save(obj, buf)
    buf.seek(0)
    return torch.load(buf, weights_only=True)


def test_reference_style_checkpoint_cpu():
    """Drop-in module + torch AdamW exactly as train_rgbd_geometric.py:64-65 builds
    them: the saved dict reloads (weights_only=True) into fresh instances with
    the reference's key names (334 entries) and identical tensors."""
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    warnings.simplefilter("ignore")
    torch.manual_seed(0)
    m = PoseNetRGBDGeometric(pretrained=False)
    opt = torch.optim.AdamW(m.parameters(), lr=1e-4, weight_decay=1e-4)
    for p in m.parameters():
        p.grad = torch.randn_like(p) * 1e-3
    opt.step()
    ck = _roundtrip({"epoch": 3, "model_state_dict": m.state_dict(), "optimizer_state_dict": opt.state_dict(),
                     "best_acc": 12.5, "curr_acc": 10.0})
    m2 = PoseNetRGBDGeometric(pretrained=False)
    m2.load_state_dict(ck["model_state_dict"])
    opt2 = torch.optim.AdamW(m2.parameters(), lr=1e-4, weight_decay=1e-4)
    opt2.load_state_dict(ck["optimizer_state_dict"])
    assert len(ck["model_state_dict"]) == 334
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a, b), k
    assert ck["epoch"] + 1 == 4


@pytest.mark.gpu
def test_trainer_checkpoint_interop():
    """Fused trainer -> reference checkpoint -> torch AdamW resumes with the same
    moments; and torch AdamW's next update equals the trainer's AdamW kernel on
    the same gradient (no clipping)."""
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    from bench import synth_batch
    warnings.simplefilter("ignore")
    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = PoseNetRGBDGeometric(pretrained=False).to(dev)
    tr = RGBDGeometricTrainer(model, 4, dtype=torch.bfloat16)
    data = synth_batch(4, dev, seed=5)
    for _ in range(2):
        tr.step(data)
    torch.cuda.synchronize()
    ck = _roundtrip(tr.checkpoint(epoch=1, best_acc=3.0, curr_acc=2.0))
    assert set(ck) == {"epoch", "model_state_dict", "optimizer_state_dict", "best_acc", "curr_acc"}

    # the reference's resume path on a fresh module
    m2 = PoseNetRGBDGeometric(pretrained=False).to(dev)
    m2.load_state_dict(ck["model_state_dict"])
    opt = torch.optim.AdamW(m2.parameters(), lr=1e-4, weight_decay=1e-4)
    opt.load_state_dict(ck["optimizer_state_dict"])
    params2 = list(m2.parameters())
    for p, q in zip(model.parameters(), params2):
        st = opt.state[q]
        o = tr.arena.offsets[tr.arena._index_of(p)]
        assert torch.equal(st["exp_avg"].reshape(-1), tr.m[o:o + p.numel()])
        assert torch.equal(st["exp_avg_sq"].reshape(-1), tr.v[o:o + p.numel()])
        assert float(st["step"]) == 2.0

    # one more update on an identical synthetic gradient, no clipping
    g = torch.randn(tr.arena.numel, device=dev, generator=torch.Generator(device=dev).manual_seed(1)) * 1e-3
    for p, q in zip(model.parameters(), params2):
        o = tr.arena.offsets[tr.arena._index_of(p)]
        q.grad = g[o:o + p.numel()].view_as(q).clone()
    opt.step()
    tr.arena.grad.copy_(g)
    tr.hp[7] = 0.0
    tr._optimizer()
    torch.cuda.synchronize()
    for (k, p), q in zip(model.named_parameters(), params2):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-6, atol=1e-7, msg=k)

    # and back: a torch AdamW state_dict resumes the trainer (moments, step, lr)
    m3 = PoseNetRGBDGeometric(pretrained=False).to(dev)
    tr3 = RGBDGeometricTrainer(m3, 4, dtype=torch.bfloat16)
    nxt = tr3.load_checkpoint({"epoch": 7, "model_state_dict": m2.state_dict(),
                               "optimizer_state_dict": opt.state_dict()})
    assert nxt == 8 and float(tr3.hp[5]) == 3.0
    for p, q in zip(m3.parameters(), params2):
        o = tr3.arena.offsets[tr3.arena._index_of(p)]
        assert torch.equal(p.detach(), q.detach())
        assert torch.equal(tr3.m[o:o + p.numel()], opt.state[q]["exp_avg"].reshape(-1))


@pytest.mark.gpu
def test_trainer_clip_and_adamw_match_torch():
    """The trainer's clip-norm + AdamW launches (pose6d_sumsq_partial_step +
    pose6d_adamw_step) against torch.nn.utils.clip_grad_norm_(params, 1.0) +
    torch.optim.AdamW (train_rgbd_geometric.py:111-112) on a gradient whose norm
    is well above 1, so the clip is active."""
    from models.pose_net_rgbd_geometric import PoseNetRGBDGeometric
    from pose6d.train import RGBDGeometricTrainer
    warnings.simplefilter("ignore")
    torch.manual_seed(0)
    dev = torch.device("cuda")
    model = PoseNetRGBDGeometric(pretrained=False).to(dev)
    tr = RGBDGeometricTrainer(model, 4, dtype=torch.bfloat16)
    m2 = PoseNetRGBDGeometric(pretrained=False).to(dev)
    m2.load_state_dict(model.state_dict())
    params2 = list(m2.parameters())
    opt = torch.optim.AdamW(params2, lr=1e-4, weight_decay=1e-4)
    gen = torch.Generator(device=dev).manual_seed(3)
    for _ in range(3):
        g = torch.randn(tr.arena.numel, device=dev, generator=gen) * 0.05   # total norm ~ 250
        for p, q in zip(model.parameters(), params2):
            o = tr.arena.offsets[tr.arena._index_of(p)]
            q.grad = g[o:o + p.numel()].view_as(q).clone()
        norm_ref = torch.nn.utils.clip_grad_norm_(params2, 1.0)
        opt.step()
        tr.arena.grad.copy_(g)
        tr._optimizer()
        torch.cuda.synchronize()
        torch.testing.assert_close(tr.norm[0], norm_ref.float(), rtol=1e-5, atol=0)
    for (k, p), q in zip(model.named_parameters(), params2):
        torch.testing.assert_close(p.detach(), q.detach(), rtol=1e-6, atol=1e-7, msg=k)

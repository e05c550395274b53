"""Single-image inference (the reference's inference_*.py call the
model on one crop at a time): B=1 eval forward of every model against the oracle,
and the same forward captured into a hipGraph and replayed (the latency path
bench.py's `inference_b1` times) giving the eager result bit for bit."""
import pytest
import torch

from tests.test_models import EXPECTED, _close, _inputs, _model_forward, _oracle_run, _models

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", list(EXPECTED))
def test_b1_eval_forward_and_graph_replay(name):
    torch.manual_seed(0)
    m = _models()[name](pretrained=False)
    P0 = {k: v.clone() for k, v in m.state_dict().items()}
    m = m.cuda().eval()
    g = torch.Generator().manual_seed(3)
    inp = _inputs(1, 224, g)
    cin = {k: v.cuda() for k, v in inp.items()}
    with torch.no_grad():
        rot, trans = _model_forward(name, m, cin)
        rr, tr, _, _ = _oracle_run(name, P0, inp, False, torch.float32)
        _close(rot, rr, 1e-4, "rotation")
        _close(trans, tr, 1e-4, "translation")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            _model_forward(name, m, cin)
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            grot, gtrans = _model_forward(name, m, cin)
        cin["rgb"].copy_(torch.randn(1, 3, 224, 224, generator=g).cuda())   # new crop, same buffers
        graph.replay()
        rot2, trans2 = _model_forward(name, m, cin)
        torch.cuda.synchronize()
    assert torch.equal(grot, rot2) and torch.equal(gtrans, trans2)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("name", list(EXPECTED))
def test_eval_bn_folded_into_conv_is_bit_identical(name, dtype):
    """Eval forward with BN + residual + ReLU applied in the conv epilogue
    (pose6d_conv2d_fwd_act) equals the separate conv / bn_act launches bit for bit."""
    torch.manual_seed(0)
    m = _models()[name](pretrained=False).cuda().eval().set_compute_dtype(dtype)
    g = torch.Generator().manual_seed(5)
    cin = {k: v.cuda() for k, v in _inputs(2, 224, g).items()}
    outs = []
    for fold in (False, True):
        with torch.no_grad():
            _model_forward(name, m, cin)   # creates the engines
            for eng in m.engines().values():
                if hasattr(eng, "eval_fuse"):
                    eng.eval_fuse = fold
            rot, trans = _model_forward(name, m, cin)
        torch.cuda.synchronize()
        outs.append((rot.clone(), trans.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_eval_downsample_in_block_launch_is_bit_identical(dtype):
    """Eval trunk with each downsampling Bottleneck's conv3 + downsample conv + both
    BatchNorms + add + ReLU in ONE launch (pose6d_conv2d_fwd_act_dual) equals the
    separate downsample launch + fused conv3 epilogue bit for bit (all four stages:
    stride 1 at layer1, stride 2 at layers 2-4), with non-trivial running statistics."""
    from pose6d.resnet import resnet50_trunk
    from pose6d.trunk import TrunkEngine
    torch.manual_seed(0)
    seq = resnet50_trunk(3)
    g = torch.Generator().manual_seed(11)
    for mod in seq.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            C = mod.num_features
            mod.running_mean.copy_(torch.randn(C, generator=g) * 0.1)
            mod.running_var.copy_(torch.rand(C, generator=g) + 0.5)
            mod.weight.data.copy_(torch.rand(C, generator=g) + 0.5)
            mod.bias.data.copy_(torch.randn(C, generator=g) * 0.1)
    seq = seq.cuda().eval()
    eng = TrunkEngine(seq, 3)
    eng.set_dtype(dtype)
    x = torch.randn(4, 3, 224, 224, generator=g).cuda()
    eng.eval_dual_rows = 0   # every stage (batch 4 grids are small: the default tile is 64x64 too)
    feats = []
    for dual in (False, True):
        eng.eval_dual = dual
        with torch.no_grad():
            feats.append(eng.forward(x, False).clone())
        torch.cuda.synchronize()
    # 4 blocks x (conv3, downsample); fp32 layer4's downsample (K = 1024 on a
    # 128-tile grid) splits K in its own launch, so that pair stays separate
    assert len(eng._dual_pairs()) == (6 if dtype == torch.float32 else 8)
    assert torch.equal(feats[0], feats[1])


@pytest.mark.parametrize("name", list(EXPECTED))
def test_eval_head_linear_bn1d_fused_is_bit_identical(name):
    """Eval heads: each Linear -> BatchNorm1d (+ ReLU) pair as one GEMM with the BN in
    its store (pose6d_gemm_f32_bn_eval) equals the separate launches bit for bit,
    with non-trivial running statistics."""
    torch.manual_seed(0)
    m = _models()[name](pretrained=False)
    g = torch.Generator().manual_seed(13)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm1d):
            C = mod.num_features
            mod.running_mean.copy_(torch.randn(C, generator=g) * 0.1)
            mod.running_var.copy_(torch.rand(C, generator=g) + 0.5)
            mod.weight.data.copy_(torch.rand(C, generator=g) + 0.5)
    m = m.cuda().eval()
    cin = {k: v.cuda() for k, v in _inputs(8, 224, g).items()}
    from pose6d.head import HeadEngine
    outs = []
    for fuse in (False, True):
        with torch.no_grad():
            _model_forward(name, m, cin)   # creates the engines
            heads = [e for e in m.engines().values() if isinstance(e, HeadEngine)]
            assert heads
            for e in heads:
                e.fuse_eval_bn = fuse
            rot, trans = _model_forward(name, m, cin)
        torch.cuda.synchronize()
        outs.append((rot.clone(), trans.clone()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])

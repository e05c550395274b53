"""Algorithmic flops / bytes the bench's roofline object prices each conv launch at
(pose6d.steptime.conv_flops / conv_bytes), on hand-counted cases.  CPU only."""
from pose6d import steptime as ST

BF16, F32 = 1, 0


def _bwd_args(name, dt, dres, mask, dx, N, H, W, Cin, Cout, KH, stride, Ho):
    head = (dt, "x", "dy", "wt", dres) + ((mask,) if name != "conv2d_backward_chain" else ()) + (dx, "dw", 0, "ws", 0)
    return head + (N, H, W, Cin, Cin, Cout, KH, KH, stride, KH // 2, Ho, Ho, None, None, "st")


def test_fused_1x1_backward_bytes_and_flops():
    # layer1 conv3 backward (64 -> 256, 56x56, batch 32), residual gradient + ReLU bits
    a = _bwd_args("conv2d_backward_chain_bn", BF16, "dres", "mask", "dx", 32, 56, 56, 64, 256, 1, 1, 56)
    M = 32 * 56 * 56
    sym = "conv_bwd_kernel<0, 2, 3>"
    assert ST.conv_flops("conv2d_backward_chain_bn", a, sym) == 2 * 2.0 * M * 256 * 64
    x, dy, w, dw = M * 64 * 2, M * 256 * 2, 256 * 64 * 2, 256 * 64 * 4
    dgrad = x + dy + w + x + M * 64 // 8        # + dres read + ReLU bits
    wgrad = x + dy + dw
    assert ST.conv_bytes("conv2d_backward_chain_bn", a, sym) == dgrad + wgrad - dy
    assert ST.conv_geom("conv2d_backward_chain_bn", a) == "32 56x56 64->256 k1s1"


def test_separate_backward_launches_and_reduce():
    a = _bwd_args("conv2d_backward_chain", F32, None, None, "dx", 4, 14, 14, 256, 256, 3, 1, 14)
    M = 4 * 14 * 14
    x, dy, w = M * 256 * 4, M * 256 * 4, 256 * 9 * 256 * 4
    assert ST.conv_bytes("conv2d_backward_chain", a, "conv_lds_kernel<float, 64, 64, 3, 4, false, 4>") == x + dy + w
    assert ST.conv_bytes("conv2d_backward_chain", a, "conv_wgrad_kernel<float, 128, 128>") == x + dy + 256 * 9 * 256 * 4
    assert ST.conv_bytes("conv2d_backward_chain", a, "wgrad_reduce_kernel<16>") == 0.0
    assert ST.conv_flops("conv2d_backward_chain", a, "wgrad_reduce_kernel<16>") == 0.0


def test_forward_bytes():
    # conv2d_fwd(dtype, x, wp, bias, y, stats, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, stream)
    a = (BF16, "x", "w", None, "y", "st", 32, 56, 56, 64, 64, 3, 3, 1, 1, 56, 56, "s")
    M = 32 * 56 * 56
    assert ST.conv_bytes("conv2d_fwd", a, "conv_lds_kernel") == 2 * (M * 64 + 64 * 9 * 64 + M * 64)
    assert ST.conv_flops("conv2d_fwd", a, "conv_lds_kernel") == 2.0 * M * 64 * 9 * 64
    # conv2d_fwd_act(dtype, x, w, bias, out, N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo, scale, shift, res, ...)
    r = (BF16, "x", "w", None, "o", 32, 56, 56, 64, 256, 1, 1, 1, 0, 56, 56, "sc", "sh", "res", None, None, 1, "s")
    assert ST.conv_bytes("conv2d_fwd_act", r, "conv_lds_kernel") == 2 * (M * 64 + 256 * 64 + 2 * M * 256)
    assert ST.conv_bytes("bn_act", r, "bn_act_kernel") is None


def test_bn_reduce_epilogue_bytes():
    """pose6d_conv2d_backward_chain_bn's epilogue also reads the BN's y (+ a second BN's
    y2) and its ReLU bits: priced from the pose6d_bn_reduce_t the call passes."""
    import ctypes

    from pose6d.trunk import _BnReduce
    sym = "conv_bwd_kernel<0, 2, 3>"
    M = 32 * 56 * 56
    x = M * 256 * 2
    base = _bwd_args("conv2d_backward_chain_bn", BF16, "dres", "mask", "dx", 32, 56, 56, 256, 64, 1, 1, 56)
    plain = ST.conv_bytes("conv2d_backward_chain_bn", base, sym)
    one = _BnReduce(y=1, relu_mask=None, y2=None)
    two = _BnReduce(y=1, relu_mask=1, y2=1)
    a1 = base[:-2] + (ctypes.addressof(one), "st")
    a2 = base[:-2] + (ctypes.addressof(two), "st")
    assert ST.conv_bytes("conv2d_backward_chain_bn", a1, sym) == plain + x
    assert ST.conv_bytes("conv2d_backward_chain_bn", a2, sym) == plain + 2 * x + M * 256 // 8

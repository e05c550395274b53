"""Convolutional trunk engine: runs a ResNet50 trunk (or the RGB-Geometric z-CNN)
forward and backward on the pose6d HIP kernels.

Replaces what torchvision/cuDNN do behind `self.backbone(x)` in every reference
model (e.g. pose_net_rgbd_geometric.py:43) and the autograd backward of it.

Design (MI355X-first):
  * activations NHWC in `dtype` (bf16 for training throughput, fp32 for parity);
  * every conv = one implicit-GEMM MFMA launch whose epilogue also emits the
    BatchNorm batch-statistics partials; BN+ReLU(+residual) = one vectorised pass;
  * conv weights: fp32 OIHW masters (the nn.Parameters, so state_dicts interchange
    with the reference) packed to the kernel layouts by ONE launch per step;
  * all buffers preallocated per (batch, H, W, dtype) -> the whole step is
    graph-capturable (no allocation, no host sync inside forward/backward).
Only one forward's activations are kept: backward() must follow the forward it
differentiates (checked with a generation counter).
"""
import ctypes

import numpy as np
import torch
import torch.nn as nn

from ._lib import DT_BF16, DT_F32, Pose6dError, call, query, require_device, stream

DTYPES = {torch.float32: DT_F32, torch.bfloat16: DT_BF16}


class _WgradReduce(ctypes.Structure):
    """pose6d_wgrad_reduce_t (include/pose6d.h)."""
    _fields_ = [("ws", ctypes.c_void_p), ("dw", ctypes.c_void_p)] + [
        (n, ctypes.c_int32) for n in ("dtype", "N", "H", "W", "Cin", "Cin_real", "Cout", "KH", "KW", "stride", "pad",
                                      "Ho", "Wo", "accumulate")]


class _BnReduce(ctypes.Structure):
    """pose6d_bn_reduce_t (include/pose6d.h): the BN whose backward sums a data
    gradient's epilogue accumulates."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("y", "mean", "invstd", "relu_scale", "relu_shift", "relu_mask",
                                                "partial", "y2", "mean2", "invstd2", "partial2")] + [
        ("rows", ctypes.c_int32)]


class _BnStats(ctypes.Structure):
    """pose6d_bn_stats_t (include/pose6d.h): one BN of pose6d_bn_finalize_dual."""
    _fields_ = [(n, ctypes.c_void_p) for n in ("partial", "gamma", "beta", "running_mean", "running_var",
                                                "num_batches", "scale", "shift", "save_mean", "save_invstd")] + [
        ("momentum", ctypes.c_float), ("eps", ctypes.c_float), ("C", ctypes.c_int32)]


def _bn_stats(op):
    bn = op.bn
    p = [op.stats, bn.weight, bn.bias, bn.running_mean, bn.running_var, bn.num_batches_tracked, op.scale, op.shift,
         op.mean, op.inv]
    return _BnStats(*[t.data_ptr() if t is not None else None for t in p],
                    float(bn.momentum if bn.momentum is not None else 0.1), float(bn.eps), op.cout)


# pose6d_bn_fold_t (include/pose6d.h): eval-mode BN fold table entry
_FOLD = np.dtype([("gamma", "<u8"), ("beta", "<u8"), ("rmean", "<u8"), ("rvar", "<u8"), ("scale", "<u8"),
                  ("shift", "<u8"), ("smean", "<u8"), ("sinv", "<u8"), ("eps", "<f4"), ("C", "<i4")])
_DESC = np.dtype([("w", "<u8"), ("wp", "<u8"), ("wt", "<u8"), ("O", "<i4"), ("I", "<i4"), ("Ip", "<i4"),
                  ("KH", "<i4"), ("KW", "<i4"), ("Kpad", "<i4"), ("KWp", "<i4"), ("reserved", "<i4"),
                  ("start", "<i8")])


def pack_geom(dtype, cin_pad, k, stride, pad):
    """(taps per packed kernel row, Kpad) of a forward filter (pose6d_conv_pack_geom)."""
    kwp, kpad = ctypes.c_int32(), ctypes.c_int32()
    call("conv_pack_geom", DTYPES[dtype], cin_pad, k, k, stride, pad, ctypes.byref(kwp),
         ctypes.byref(kpad))
    return kwp.value, kpad.value


def pack_single(w, cin_pad, dtype, with_t=True, stride=1, pad=None):
    """Pack one OIHW fp32 device weight -> (wp [O][Kpad], wt [Ipad][KH][KW][O] or None).
    stride / pad (default: 'same' padding) select the forward layout (pose6d_conv_pack_geom:
    the 4-channel 7x7 / stride-2 stems use the row-tap layout)."""
    O, I, KH, KW = w.shape
    kwp, Kpad = pack_geom(dtype, cin_pad, KH, stride, KH // 2 if pad is None else pad)
    wp = torch.empty(O, Kpad, device=w.device, dtype=dtype)
    wt = torch.empty(cin_pad, KH, KW, O, device=w.device, dtype=dtype) if with_t else None
    w = w.detach().float().contiguous()
    rec = np.zeros(1, _DESC)
    rec[0] = (w.data_ptr(), wp.data_ptr(), wt.data_ptr() if wt is not None else 0, O, I, cin_pad, KH, KW, Kpad, kwp,
              0, 0)
    d = torch.from_numpy(rec.view(np.uint8).copy()).to(w.device)
    call("pack_conv_weights", DTYPES[dtype], d, 1, O * Kpad, stream())
    torch.cuda.current_stream().synchronize()   # `d` / `w` are temporaries
    return wp, wt


class _Act:
    """An NHWC activation tensor of the trunk graph."""

    def __init__(self, C, H, W, name):
        self.C, self.H, self.W, self.name = C, H, W, name
        self.t = None      # forward value
        self.g = None      # gradient buffer
        self.pending = None  # gradient contribution waiting for the producer's dgrad (residual)


class _ConvOp:
    def __init__(self, conv, bn, src, name):
        self.conv, self.bn, self.src, self.name = conv, bn, src, name
        self.cin = conv.in_channels
        self.cin_pad = 4 if self.cin < 8 else self.cin
        self.cout = conv.out_channels
        self.k = conv.kernel_size[0]
        self.stride = conv.stride[0]
        self.pad = conv.padding[0]
        self.H, self.W = src.H, src.W
        self.Ho = (self.H + 2 * self.pad - self.k) // self.stride + 1
        self.Wo = (self.W + 2 * self.pad - self.k) // self.stride + 1
        self.out = _Act(self.cout, self.Ho, self.Wo, name + ".y")
        self.act_op = None   # the _ActOp applying this conv's BN (set by _ActOp)
        self.needs_dgrad = True


class _ActOp:
    """out = relu?(bn(y) [+ res_act | + bn_res(y_res)])"""

    def __init__(self, cop, relu, res_act=None, res_conv=None, name=""):
        self.cop, self.relu, self.res_act, self.res_conv = cop, relu, res_act, res_conv
        cop.act_op = self   # the BN+act applied to this conv's output
        self.out = _Act(cop.cout, cop.Ho, cop.Wo, name)
        self.pooled = False   # applied inside the following max pool (its output is never stored)


class _PoolOp:
    def __init__(self, src, k, s, p, name):
        self.src, self.k, self.s, self.p = src, k, s, p
        self.act = None   # the plain BN+ReLU this pool applies on the fly (pose6d_bn_relu_maxpool_fwd)
        Ho = (src.H + 2 * p - k) // s + 1
        Wo = (src.W + 2 * p - k) // s + 1
        self.out = _Act(src.C, Ho, Wo, name)


class TrunkEngine:
    """Executes an nn.Sequential trunk (ResNet50 children[:-1] or the z-CNN)."""

    def __init__(self, seq, in_channels, kind="resnet50"):
        self.seq = seq
        self.kind = kind
        self.in_channels = in_channels
        self._shape = None
        self.generation = 0
        self._saved_gen = -1
        self._pack_key = None
        self._build(224, 224)   # op graph (geometry is re-derived in prepare())

    # ------------------------------------------------------------ graph build
    def _build(self, H, W):
        self.ops = []
        self.convs = []
        x = _Act(4 if self.in_channels < 8 else self.in_channels, H, W, "input")
        self.input = x

        def conv_bn(conv, bn, src, name):
            op = _ConvOp(conv, bn, src, name)
            self.ops.append(op)
            self.convs.append(op)
            return op

        if self.kind == "resnet50":
            s = self.seq
            c = conv_bn(s[0], s[1], x, "stem")
            c.needs_dgrad = False
            a = _ActOp(c, True, name="stem.act")
            self.ops.append(a)
            p = _PoolOp(a.out, 3, 2, 1, "stem.pool")
            self.ops.append(p)
            cur = p.out
            for li in range(4):
                for bi, blk in enumerate(s[4 + li]):
                    nm = f"layer{li + 1}.{bi}"
                    # the downsample conv runs first in forward, so in backward it comes
                    # after conv1 and adds its data gradient into conv1's in place: a
                    # stride-2 1x1 then touches only the even pixels it reaches
                    # (pose6d_conv2d_backward with dres == dx skips the empty classes)
                    cd = None
                    if blk.downsample is not None:
                        cd = conv_bn(blk.downsample[0], blk.downsample[1], cur, nm + ".down")
                    c1 = conv_bn(blk.conv1, blk.bn1, cur, nm + ".conv1")
                    a1 = _ActOp(c1, True, name=nm + ".a1"); self.ops.append(a1)
                    c2 = conv_bn(blk.conv2, blk.bn2, a1.out, nm + ".conv2")
                    a2 = _ActOp(c2, True, name=nm + ".a2"); self.ops.append(a2)
                    c3 = conv_bn(blk.conv3, blk.bn3, a2.out, nm + ".conv3")
                    if cd is not None:
                        o = _ActOp(c3, True, res_conv=cd, name=nm + ".out")
                    else:
                        o = _ActOp(c3, True, res_act=cur, name=nm + ".out")
                    self.ops.append(o)
                    cur = o.out
            self.final = cur
        elif self.kind == "zcnn":
            s = self.seq
            cur = x
            for i in (0, 4, 8, 12):
                c = conv_bn(s[i], s[i + 1], cur, f"z{i}")
                if i == 0:
                    c.needs_dgrad = False
                a = _ActOp(c, True, name=f"z{i}.act"); self.ops.append(a)
                mp = s[i + 3]
                p = _PoolOp(a.out, mp.kernel_size, mp.stride, mp.padding, f"z{i}.pool"); self.ops.append(p)
                cur = p.out
            self.final = cur
        else:
            raise ValueError(self.kind)
        # act -> pool pairs whose activation feeds only the pool (stem, z-CNN): one pass
        for i, op in enumerate(self.ops[:-1]):
            nxt = self.ops[i + 1]
            if (isinstance(op, _ActOp) and isinstance(nxt, _PoolOp) and nxt.src is op.out and op.relu
                    and op.res_act is None and op.res_conv is None
                    and not any(o is not nxt and (getattr(o, "src", None) is op.out
                                                  or getattr(o, "res_act", None) is op.out) for o in self.ops)):
                op.pooled, nxt.act = True, op
        self.feat_dim = self.final.C

    # ------------------------------------------------------------ allocation
    def prepare(self, B, H, W, dtype, device):
        key = (B, H, W, dtype, device)
        if self._shape == key:
            return
        if dtype not in DTYPES:
            raise Pose6dError(f"unsupported trunk dtype {dtype}")
        self._build(H, W)
        self._shape = key
        self.B, self.dtype, self.dt, self.device = B, dtype, DTYPES[dtype], device
        e = lambda *s, dt=dtype: torch.empty(*s, device=device, dtype=dt)
        f32 = lambda *s: torch.empty(*s, device=device, dtype=torch.float32)
        self.input.t = e(B, H, W, self.input.C)
        ws_w, ws_bn, ws_sk = 0, 0, 0
        for op in self.ops:
            o = op.out
            o.t = e(B, o.H, o.W, o.C)
            o.g = e(B, o.H, o.W, o.C)
            if isinstance(op, _ConvOp):
                M = B * op.Ho * op.Wo
                op.KWp, op.Kpad = pack_geom(dtype, op.cin_pad, op.k, op.stride, op.pad)
                op.wp = e(op.cout, op.Kpad)
                op.wt = e(op.cin_pad, op.k, op.k, op.cout) if op.needs_dgrad else None
                rows = query("conv_stats_rows", B, op.Ho, op.Wo, op.cout)
                op.stats_rows = rows
                op.stats = f32(2, op.cout, rows)   # channel-major BN partials
                op.scale, op.shift, op.mean, op.inv = (f32(op.cout) for _ in range(4))
                ws_w = max(ws_w, query("conv2d_wgrad_workspace", self.dt, B, op.Ho, op.Wo, op.cin_pad, op.cout, op.k,
                                       op.k))
                ws_sk = max(ws_sk, query("conv_splitk_workspace", self.dt, 0, B, op.H, op.W, op.cin_pad, op.cout, op.k,
                                         op.k, op.stride, op.pad, op.Ho, op.Wo))
                ws_bn = max(ws_bn, (query("bn_bwd_workspace_rows", M) * 2 + 3) * op.cout)
            elif isinstance(op, _ActOp):
                residual = op.res_act is not None or op.res_conv is not None
                # residual BN + ReLU: one mask bit per element replaces re-reading `out` in
                # backward, and the identity branch's gradient dz = dout * mask is never
                # written out: its consumers (the next block's conv1 data gradient, the
                # downsample BN's backward) apply the bits to dout themselves
                vec = 8 if dtype == torch.bfloat16 else 4
                op.mbits = (torch.empty(B * o.H * o.W * o.C // vec, device=device, dtype=torch.uint8)
                            if (op.relu and residual) else None)
                op.dz = e(B, o.H, o.W, o.C) if (residual and op.mbits is None) else None
                if op.res_conv is not None and op.mbits is not None:   # both BNs' partials at once
                    ws_bn = max(ws_bn, 2 * (query("bn_bwd_workspace_rows", B * o.H * o.W) * 2 + 3) * o.C)
            elif isinstance(op, _PoolOp):
                op.argmax = torch.empty(B, o.H, o.W, o.C, device=device, dtype=torch.uint8)
        # training BN finalize + apply as one launch (pose6d_bn_finalize_act) where the form
        # allows it: ready flags per BN (zeroed once) and one epoch counter per engine
        self.bn_epoch = torch.zeros(1, device=device, dtype=torch.int64)
        for op in self.ops:
            if isinstance(op, _ActOp):
                op.fin_flags = None
                if self._fin_act_ok(op):
                    n = query("bn_finalize_act_flags", op.cop.stats_rows, op.cop.cout)
                    op.fin_flags = torch.zeros(max(n, 1), device=device, dtype=torch.int32)
        self._plan_bn_reduce(B, f32)
        ws_bn = max(ws_bn, 6 * max(op.cout for op in self.convs))   # pose6d_bn_bwd_partials' coefficients
        self.ws_wgrad = f32(max(ws_w // 4, 1))
        self.ws_wgrad2 = f32(max(ws_w // 4, 1))   # ping-pong: a deferred slab reduce reads the other one
        self.ws_bn = f32(max(ws_bn, 1))
        self.ws_fin = None   # pose6d_bn_finalize needs no workspace (one launch)
        # this engine's split-K workspace (arrival counters zeroed once, re-armed by every
        # launch; partial tiles): engines on different streams never share one
        self.ws_sk = torch.zeros(max(ws_sk, 1), device=device, dtype=torch.uint8) if ws_sk else None
        self.ws_sk_bytes = ws_sk
        self.feat = f32(B, self.feat_dim)
        self.feat_grad_in = None
        self._fold_dev, self._fold_key = None, None
        # weight packing descriptors (one launch for all convs)
        self._desc_dev = None
        self._pack_key = None
        self._build_pack_table()

    @staticmethod
    def _fin_act_ok(op):
        """pose6d_bn_finalize_act's forms: a BN + (ReLU) + identity / no residual that is
        stored (not applied inside a max pool), channels a multiple of 64."""
        return not op.pooled and op.res_conv is None and op.cop.cout % 64 == 0

    def _plan_bn_reduce(self, B, f32):
        """A conv whose input is a BN + ReLU output that no other conv reads (each
        bottleneck's conv2 / conv3, and conv1 of a block fed by an identity block) writes
        that activation's whole gradient in one data-gradient launch: its epilogue also
        sums the BN's backward partials (pose6d_conv2d_backward_chain_bn), so the BN
        backward is finalize + apply (pose6d_bn_bwd_partials), without re-reading dout.
        A downsampling block's input (read by conv1 and the downsample conv, the latter
        adding into the former's gradient in place) keeps the three-pass backward."""
        producer = {id(op.out): op for op in self.ops if isinstance(op, _ActOp)}
        readers = {}
        for op in self.convs:
            readers.setdefault(id(op.src), []).append(op)
        for op in self.ops:
            if isinstance(op, _ActOp):
                op.bnr = None
            elif isinstance(op, _ConvOp):
                op.bnr_desc = None
        for op in self.convs:
            p = producer.get(id(op.src))
            if (p is None or p.pooled or not p.relu or not op.needs_dgrad or len(readers[id(op.src)]) != 1
                    or p.res_act is not None and p.mbits is None or p.res_conv is not None and p.mbits is None):
                continue
            rows = query("conv2d_backward_bn_rows", self.dt, B, op.H, op.W, op.cin_pad, op.cout, op.k, op.k,
                         op.stride, op.pad, op.Ho, op.Wo)
            if rows <= 0:
                continue
            c, r = p.cop, p.res_conv
            part = f32(2, c.cout, rows)
            part2 = f32(2, r.cout, rows) if r is not None else None
            ptr = lambda t: t.data_ptr() if t is not None else None
            plain = p.mbits is None
            op.bnr_desc = _BnReduce(ptr(c.out.t), ptr(c.mean), ptr(c.inv), ptr(c.scale) if plain else None,
                                    ptr(c.shift) if plain else None, ptr(p.mbits), ptr(part),
                                    ptr(r.out.t) if r else None, ptr(r.mean) if r else None,
                                    ptr(r.inv) if r else None, ptr(part2), rows)
            p.bnr = (part, part2, rows)

    def _eval_fold(self, st):
        """Eval scale/shift (+ saved mean / invstd) of every BN from its running
        statistics: ONE launch (pose6d_bn_eval_fold) instead of one per BN."""
        key = tuple((op.bn.weight.data_ptr(), op.bn.bias.data_ptr(), op.bn.running_mean.data_ptr(),
                     op.bn.running_var.data_ptr(), float(op.bn.eps)) for op in self.convs)
        if key != self._fold_key:
            assert query("bn_fold_desc_size") == _FOLD.itemsize
            rec = np.zeros(len(self.convs), dtype=_FOLD)
            for i, op in enumerate(self.convs):
                bn = op.bn
                rec[i] = (bn.weight.data_ptr(), bn.bias.data_ptr(), bn.running_mean.data_ptr(),
                          bn.running_var.data_ptr(), op.scale.data_ptr(), op.shift.data_ptr(), op.mean.data_ptr(),
                          op.inv.data_ptr(), float(bn.eps), op.cout)
            self._fold_dev = torch.from_numpy(rec.view(np.uint8).copy()).to(self.device)
            self._fold_key = key
        call("bn_eval_fold", self._fold_dev, len(self.convs), max(op.cout for op in self.convs), st)

    def _build_pack_table(self):
        n = len(self.convs)
        sz = query("pack_desc_size")
        assert sz == 64, sz
        rec = np.zeros(n, dtype=_DESC)
        start = 0
        for i, op in enumerate(self.convs):
            w = op.conv.weight
            rec[i] = (w.data_ptr(), op.wp.data_ptr(), op.wt.data_ptr() if op.wt is not None else 0, op.cout, op.cin,
                      op.cin_pad, op.k, op.k, op.Kpad, op.KWp, 0, start)
            start += op.cout * op.Kpad
        self._pack_total = start
        self._desc_host = rec   # (host copy: pose6d_adamw_packed_jobs reads it)
        self._desc_dev = torch.from_numpy(rec.view(np.uint8).copy()).to(self.device)
        self._desc_ptrs = tuple(op.conv.weight.data_ptr() for op in self.convs)

    def pack_weights(self, force=False):
        """Re-pack the conv weights if the fp32 masters changed (optimizer step,
        load_state_dict, .to()).  One kernel launch for all convs."""
        ptrs = tuple(op.conv.weight.data_ptr() for op in self.convs)
        if ptrs != self._desc_ptrs:
            self._build_pack_table()
        key = (ptrs, tuple(op.conv.weight._version for op in self.convs))
        if force or key != self._pack_key:
            call("pack_conv_weights", self.dt, self._desc_dev, len(self.convs), self._pack_total, stream())
            self._pack_key = key

    # ------------------------------------------------------------ forward
    def forward(self, x, training, pack=True, inference=False):
        """x: (B, C, H, W) fp32 on device -> features (B, feat_dim) fp32 (engine buffer).
        Eval mode folds each BatchNorm into its conv's epilogue: such a forward keeps no
        backward state, so backward() after it raises (`inference` is accepted for the
        autograd bridge; the trunk's eval forward is the same either way)."""
        require_device(x)
        B, C, H, W = x.shape
        if C != self.in_channels:
            raise Pose6dError(f"trunk expects {self.in_channels} input channels, got {C}")
        padw = self._stem_pad_cols(W, self.dtype_req)
        self.prepare(B, H, W + padw, self.dtype_req, x.device)
        if pack:
            self.pack_weights()
        st = stream()
        dt = self.dt
        xf = x.detach()
        if xf.dtype != torch.float32:
            xf = xf.float()
        if padw:
            # odd-width bf16 input to a row-tap stem: one zero column on the right (exact:
            # see _stem_pad_cols); torch does the copy, the trunk runs on the even width
            xf = torch.nn.functional.pad(xf, (0, padw))
        xf = xf.contiguous()
        call("nchw_to_nhwc", dt, xf, self.input.t, B, C, H, W + padw, self.input.C, st)
        # eval: the BN (running statistics) is known before the conv runs, so the conv's
        # epilogue applies BN (+ residual) + ReLU and stores the activation directly
        fold = not training and self.eval_fuse
        dual = {}
        if fold:
            self._eval_fold(st)
            dual = self._dual_pairs()
        # training: a downsampling block's two BN finalizes (bn3, downsample BN: same
        # output grid) as one launch after conv3 (pose6d_bn_finalize_dual)
        fused_fin = training and not fold and self.bn_fused_finalize_act
        if fused_fin:
            self.bn_epoch.add_(1)   # a fresh epoch for this forward's finalize -> apply hand-offs
        fin2 = {}
        if training and not fold and self.bn_dual_finalize:
            pos = {id(o): i for i, o in enumerate(self.ops)}
            for op in self.ops:
                if isinstance(op, _ActOp) and op.res_conv is not None:
                    c3, r = op.cop, op.res_conv
                    if (pos[id(r)] < pos[id(c3)] and c3.stats_rows == r.stats_rows
                            and (c3.Ho, c3.Wo) == (r.Ho, r.Wo)):
                        fin2[c3] = r
                        fin2[r] = None
        for op in self.ops:
            if isinstance(op, _ConvOp):
                if op in dual:
                    if dual[op] is None:
                        continue   # a downsample conv: computed inside its block's last conv launch
                    a = op.act_op
                    r = a.res_conv
                    call("conv2d_fwd_act_dual", dt, op.src.t, op.wp, r.src.t, r.wp, a.out.t, B, op.Ho, op.Wo,
                         op.cin_pad, op.cout, r.H, r.W, r.cin_pad, r.stride, op.scale, op.shift, r.scale, r.shift,
                         int(a.relu), st)
                    continue
                bias = op.conv.bias
                bias = bias.detach() if bias is not None else None
                bn = op.bn
                fin = ("bn_finalize", op.stats, op.stats_rows, op.cout, B * op.Ho * op.Wo, bn.weight.detach(),
                       bn.bias.detach(), bn.running_mean, bn.running_var, bn.num_batches_tracked,
                       float(bn.momentum if bn.momentum is not None else 0.1), float(bn.eps), int(training),
                       op.scale, op.shift, op.mean, op.inv, self.ws_fin, st)
                a = getattr(op, "act_op", None)
                if fold and a is not None and not a.pooled:
                    res, rs, rb = None, None, None
                    if a.res_conv is not None:
                        res, rs, rb = a.res_conv.out.t, a.res_conv.scale, a.res_conv.shift
                    elif a.res_act is not None:
                        res = a.res_act.t
                    call("conv2d_fwd_act", dt, op.src.t, op.wp, bias, a.out.t, B, op.H, op.W, op.cin_pad, op.cout,
                         op.k, op.k, op.stride, op.pad, op.Ho, op.Wo, op.scale, op.shift, res, rs, rb, int(a.relu),
                         self.ws_sk, self.ws_sk_bytes, st)
                    continue
                call("conv2d_fwd", dt, op.src.t, op.wp, bias, op.out.t, op.stats if training else None, B, op.H,
                     op.W, op.cin_pad, op.cout, op.k, op.k, op.stride, op.pad, op.Ho, op.Wo, self.ws_sk,
                     self.ws_sk_bytes, st)
                if fold:
                    pass
                elif fused_fin and a is not None and getattr(a, "fin_flags", None) is not None:
                    pass   # finalized inside its BN's apply launch (pose6d_bn_finalize_act)
                elif op in fin2:
                    r = fin2[op]
                    if r is not None:   # conv3: both BNs now; the downsample BN's finalize waited for it
                        a, b = _bn_stats(op), _bn_stats(r)
                        call("bn_finalize_dual", ctypes.addressof(a), ctypes.addressof(b), op.stats_rows,
                             B * op.Ho * op.Wo, st)
                else:
                    call(*fin)
            elif isinstance(op, _ActOp):
                if op.pooled or fold:
                    continue   # applied by the following pool / by its conv's epilogue
                c = op.cop
                M = B * c.Ho * c.Wo
                mb = op.mbits if training else None
                if fused_fin and op.fin_flags is not None:
                    st_ = _bn_stats(c)
                    call("bn_finalize_act", dt, ctypes.addressof(st_), c.stats_rows, M, c.out.t,
                         op.res_act.t if op.res_act else None, int(op.relu), op.out.t, mb, op.fin_flags,
                         self.bn_epoch, st)
                    continue
                if op.res_conv is not None:
                    r = op.res_conv
                    call("bn_act_fwd_mask", dt, c.out.t, c.scale, c.shift, r.out.t, r.scale, r.shift, int(op.relu),
                         op.out.t, mb, M, c.cout, st)
                else:
                    call("bn_act_fwd_mask", dt, c.out.t, c.scale, c.shift, op.res_act.t if op.res_act else None, None,
                         None, int(op.relu), op.out.t, mb, M, c.cout, st)
            elif op.act is not None:
                s, c = op.src, op.act.cop
                call("bn_relu_maxpool_fwd", dt, c.out.t, c.scale, c.shift, op.out.t, op.argmax, B, s.H, s.W, s.C,
                     op.k, op.s, op.p, op.out.H, op.out.W, st)
            else:
                s = op.src
                call("maxpool_fwd", dt, s.t, op.out.t, op.argmax, B, s.H, s.W, s.C, op.k, op.s, op.p, op.out.H,
                     op.out.W, st)
        f = self.final
        call("avgpool_fwd", dt, f.t, self.feat, B, f.H * f.W, f.C, st)
        self.generation += 1
        self._saved_gen = self.generation if training else -1
        self._eval_gen = -1 if training else self.generation
        return self.feat

    def _stem_pad_cols(self, W, dtype):
        """1 if the first conv is a bf16 row-tap stem (4-channel 7x7 / stride 2,
        pose6d_conv_pack_geom) and W is odd, else 0.  The bf16 row-tap kernels read two
        pixels per 16-byte chunk from even pixel offsets, so they need an even row pitch
        (pose6d_conv2d_fwd refuses odd W); a zero column appended on the right gives the
        same output width -- floor((W + 1 + 2p - k) / s) == floor((W + 2p - k) / s) for
        the stride-2 stems at odd W -- and every window that reaches it reads zero
        padding there already, so the result is the odd-width conv's exactly (the stem
        has no data gradient; its weight gradient sees a zero column)."""
        if dtype != torch.bfloat16 or W % 2 == 0:
            return 0
        c = self.seq[0]
        k, s, p = c.kernel_size[1], c.stride[1], c.padding[1]
        cin_pad = 4 if self.in_channels < 8 else self.in_channels
        if pack_geom(dtype, cin_pad, k, s, p)[0] == k:
            return 0   # not a row-tap stem: any width works
        assert (W + 1 + 2 * p - k) // s == (W + 2 * p - k) // s, "row-tap stem: padding would change Wo"
        return 1

    def _dual_pairs(self):
        """Eval: each Bottleneck with a downsample branch gets its output from ONE launch
        (pose6d_conv2d_fwd_act_dual: conv3 and the downsample conv as two GEMMs of one
        workgroup, both BatchNorms + add + ReLU in the epilogue; bit-identical to the
        separate launches) -- the downsample output never makes an HBM round trip.
        Only for the big-grid stages (layer1/layer2 at batch 32: >= 16384 output rows):
        the pair runs on the 64x64 tile with both accumulator sets, which lost to the
        separate launches (128x128 tiles) on layer3/layer4 (eval trace).
        Returns {conv3: its downsample conv, downsample conv: None}; `eval_dual` /
        `eval_dual_rows` (engine attributes: the tests compare both paths) switch it off /
        set the row threshold."""
        if not self.eval_dual:
            return {}
        ks = 64 if self.dtype == torch.bfloat16 else 32
        min_rows = self.eval_dual_rows
        pairs = {}
        for op in self.ops:
            if not isinstance(op, _ActOp) or op.res_conv is None or op.pooled:
                continue
            c3, r = op.cop, op.res_conv
            ok = (c3.k == 1 and c3.stride == 1 and c3.pad == 0 and r.k == 1 and r.pad == 0
                  and c3.conv.bias is None and r.conv.bias is None
                  and c3.cin_pad % ks == 0 and r.cin_pad % ks == 0 and c3.cout == r.cout
                  and (r.Ho, r.Wo) == (c3.Ho, c3.Wo) and self.B * c3.Ho * c3.Wo >= min_rows)
            # the dual kernel has no split-K: a pair whose separate launches split K
            # (small grids, long K) stays separate, so both paths agree bit for bit
            ok = ok and all(query("conv_variant", self.dt, 0, self.B, c.H, c.W, c.cin_pad, c.cout, 1, 1, c.stride, 0,
                                  c.Ho, c.Wo) >> 16 == 1 for c in (c3, r))
            if ok:
                pairs[c3] = r
                pairs[r] = None
        return pairs

    # ------------------------------------------------------------ backward
    def backward(self, dfeat, grad_of, accumulate=False, on_conv_done=None):
        """dfeat: (B, feat_dim) fp32.  grad_of(param) -> fp32 tensor receiving that
        parameter's gradient (written, or added if accumulate).  Input gets no grad."""
        if self._saved_gen != self.generation:
            if getattr(self, "_eval_gen", -1) == self.generation:
                raise Pose6dError("TrunkEngine.backward after an eval-mode forward: the trunk's eval BatchNorm is "
                                  "folded into the conv epilogues and keeps no backward state; train() the module "
                                  "(the reference's training scripts do) to differentiate through it")
            raise Pose6dError("TrunkEngine.backward: activations of the matching training forward were overwritten")
        st = stream()
        dt = self.dt
        B = self.B
        acc = int(accumulate)
        f = self.final
        dfeat = dfeat.detach().float().contiguous()
        call("avgpool_bwd", dt, dfeat, f.g, B, f.H * f.W, f.C, st)
        for op in self.ops:
            op.out.pending = None
        self.input.pending = None
        # weight-gradient slab reduces ride on the next conv's fused launch
        # (pose6d_conv2d_backward_chain): `pending` = the conv whose dW still waits
        ws_pp = (self.ws_wgrad, self.ws_wgrad2)
        slot = 0
        pending, pending_op = None, None
        deferred = ctypes.c_int32(0)

        def conv_done(o):
            if on_conv_done is not None:
                on_conv_done(o)

        for op in reversed(self.ops):
            if isinstance(op, _ActOp):
                c = op.cop
                M = B * c.Ho * c.Wo
                bn = c.bn
                # ReLU mask: recomputed from the raw conv output when there is no residual
                # (saves reading the forward output), read from it otherwise
                plain = op.relu and op.res_act is None and op.res_conv is None
                out = op.out.t if (op.relu and not plain) else None
                rs, rb = (c.scale, c.shift) if plain else (None, None)
                r = op.res_conv
                if op.bnr is not None and self.bwd_conv_bn_reduce:
                    # the consumer's data gradient already summed this BN's partials
                    part, part2, rows = op.bnr
                    call("bn_bwd_partials", dt, part, rows, op.out.g, op.mbits, rs, rb, c.out.t, c.mean, c.inv,
                         bn.weight.detach(), grad_of(bn.weight), grad_of(bn.bias), c.out.g, part2,
                         r.out.t if r else None, r.mean if r else None, r.inv if r else None,
                         r.bn.weight.detach() if r else None, grad_of(r.bn.weight) if r else None,
                         grad_of(r.bn.bias) if r else None, r.out.g if r else None, acc, self.ws_bn, M, c.cout, st)
                    if op.res_act is not None:
                        op.res_act.pending = (op.out.g, op.mbits)
                    continue
                if r is not None and op.mbits is not None and self.bwd_dual_bn:
                    # downsampling block: its last BN and the branch BN share dout * mask --
                    # both backwards in one reduce / finalize / apply
                    call("bn_bwd_mask_dual", dt, op.out.g, op.mbits, c.out.t, c.mean, c.inv, bn.weight.detach(),
                         grad_of(bn.weight), grad_of(bn.bias), c.out.g, r.out.t, r.mean, r.inv,
                         r.bn.weight.detach(), grad_of(r.bn.weight), grad_of(r.bn.bias), r.out.g, acc, self.ws_bn,
                         M, c.cout, st)
                    continue
                if op.mbits is not None:
                    call("bn_bwd_mask", dt, op.out.g, op.mbits, c.out.t, c.mean, c.inv, bn.weight.detach(),
                         grad_of(bn.weight), grad_of(bn.bias), acc, c.out.g, op.dz, self.ws_bn, M, c.cout, st)
                else:
                    call("bn_bwd", dt, op.out.g, out, rs, rb, c.out.t, c.mean, c.inv, bn.weight.detach(),
                         grad_of(bn.weight), grad_of(bn.bias), acc, c.out.g, op.dz, self.ws_bn, M, c.cout, st)
                if op.res_conv is not None:
                    r = op.res_conv
                    # identity branch = bn_r(y_r) (no ReLU of its own): its dz is the masked dout
                    if op.mbits is not None:
                        call("bn_bwd_mask", dt, op.out.g, op.mbits, r.out.t, r.mean, r.inv, r.bn.weight.detach(),
                             grad_of(r.bn.weight), grad_of(r.bn.bias), acc, r.out.g, None, self.ws_bn, M, r.cout,
                             st)
                    else:
                        call("bn_bwd", dt, op.dz, None, None, None, r.out.t, r.mean, r.inv, r.bn.weight.detach(),
                             grad_of(r.bn.weight), grad_of(r.bn.bias), acc, r.out.g, None, self.ws_bn, M, r.cout, st)
                elif op.res_act is not None:
                    # the identity gradient: dz itself, or (dout, mask bits) applied by the consumer
                    op.res_act.pending = op.dz if op.mbits is None else (op.out.g, op.mbits)
            elif isinstance(op, _ConvOp):
                dy = op.out.g
                M = B * op.Ho * op.Wo
                dres, dx, dmask = None, None, None
                if op.needs_dgrad:
                    src = op.src
                    if src.pending is not None and src.g is not None:
                        # a contribution is waiting: fuse it into this dgrad's epilogue (in
                        # place when it already sits in src.g: dres == dx; as dout * mask
                        # bits when it is a residual BN's masked output gradient)
                        dres, dx = src.pending, src.g
                        if isinstance(dres, tuple):
                            dres, dmask = dres
                        src.pending = None
                    elif src.pending is None and self._has_later_consumer(op):
                        # first of two contributions (conv1; the downsample conv adds to it)
                        dx = src.g
                        src.pending = src.g
                    else:
                        dx = src.g
                if op.conv.bias is not None:   # before conv_done(op) can mark the bucket ready
                    call("channel_sum", dt, dy, M, op.cout, grad_of(op.conv.bias), acc, st)
                # data + weight gradient: one fused launch on the bf16 fast path
                ws = ws_pp[slot]
                dw = grad_of(op.conv.weight)
                args = (dt, op.src.t, dy, op.wt, dres, dx, dw, acc, ws, ws.numel() * 4, B, op.H, op.W, op.cin_pad,
                        op.cin, op.cout, op.k, op.k, op.stride, op.pad, op.Ho, op.Wo)
                job = _WgradReduce(ws.data_ptr(), dw.data_ptr(), dt, B, op.H, op.W, op.cin_pad, op.cin, op.cout,
                                   op.k, op.k, op.stride, op.pad, op.Ho, op.Wo, acc)
                prev = ctypes.addressof(pending) if pending is not None else None
                if op.bnr_desc is not None and self.bwd_conv_bn_reduce:
                    call("conv2d_backward_chain_bn", dt, op.src.t, dy, op.wt, dres, dmask, *args[5:], prev,
                         ctypes.addressof(deferred), ctypes.addressof(op.bnr_desc), st)
                elif dmask is not None:
                    call("conv2d_backward_chain_masked", dt, op.src.t, dy, op.wt, dres, dmask, *args[5:], prev,
                         ctypes.addressof(deferred), st)
                else:
                    call("conv2d_backward_chain", *args, prev, ctypes.addressof(deferred), st)
                if pending_op is not None:
                    conv_done(pending_op)          # its reduce ran in this launch (or just before it)
                if deferred.value:
                    pending, pending_op = job, op
                    slot ^= 1
                else:
                    pending, pending_op = None, None
                    conv_done(op)

            else:
                s = op.src
                call("maxpool_bwd", dt, op.out.g, op.argmax, s.g, B, s.H, s.W, s.C, op.k, op.s, op.p, op.out.H,
                     op.out.W, st)
        if pending is not None:
            call("wgrad_reduce", ctypes.addressof(pending), st)
            conv_done(pending_op)

    def _has_later_consumer(self, op):
        """True if op.src is also consumed by a conv processed later in backward
        (i.e. earlier in forward): the downsample conv of a block shares its input
        with the block's conv1."""
        idx = self.ops.index(op)
        for prev in self.ops[:idx]:
            if isinstance(prev, _ConvOp) and prev.src is op.src and prev.needs_dgrad:
                return True
        return False

    dtype_req = torch.float32
    # eval-forward fusions (bit-identical to the separate launches; attributes, not
    # environment, so the tests can compare both paths): BN + residual + ReLU in the conv
    # epilogue, and a downsampling block's two convs in one launch for >= eval_dual_rows
    # output rows
    eval_fuse = True
    eval_dual = True
    eval_dual_rows = 16384
    # training backward: a downsampling block's two BatchNorm backwards in one set of
    # launches (bit-identical to two pose6d_bn_bwd_mask calls; attribute for the tests)
    bwd_dual_bn = True
    # training forward: a downsampling block's two BN finalizes in one launch
    # (bit-identical to two pose6d_bn_finalize calls; attribute for the tests)
    bn_dual_finalize = True
    # training forward: each other BN's finalize + apply in one launch (pose6d_bn_finalize_act;
    # bit-identical to the two launches).  Off: measured slower -- the apply workgroups'
    # flag poll + write-through parameter reads cost more than the launch boundary they
    # remove (bf16 step 4.57 -> 4.70 ms, fp32 11.76 -> 11.89; profiles/r06_bn_finalize_act.txt)
    bn_fused_finalize_act = False
    # training backward: a BN + ReLU whose output gradient one data-gradient launch
    # completes gets its reduce pass from that launch's epilogue (attribute for the tests)
    bwd_conv_bn_reduce = True

    def set_dtype(self, dtype):
        self.dtype_req = dtype

    def params_in_grad_order(self):
        """Parameters in the order backward() finishes their gradients."""
        out = []
        for op in reversed(self.ops):
            if isinstance(op, _ActOp):
                out += [op.cop.bn.weight, op.cop.bn.bias]
                if op.res_conv is not None:
                    out += [op.res_conv.bn.weight, op.res_conv.bn.bias]
            elif isinstance(op, _ConvOp):
                out.append(op.conv.weight)
                if op.conv.bias is not None:
                    out.append(op.conv.bias)
        return out

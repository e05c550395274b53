"""Fully-connected head engine: executes an nn.Sequential of Linear / BatchNorm1d /
LayerNorm / ReLU / GELU / Dropout forward and backward on the pose6d HIP kernels
(fp32).

Replaces the rot/trans/z heads of the reference (pose_net_rgb.py:23-50,
pose_net_rgb_geometric.py:23-33,58-65, pose_net_rgbd_geometric.py:28-38) and the
fusion MLP / heads of PoseNetRGBD (pose_net_rgbd.py:80-105).
Linear -> BatchNorm1d -> ReLU -> Dropout runs as 2 launches (GEMM + fused
BN/ReLU/dropout column kernel), Linear -> LayerNorm -> GELU -> Dropout as 2
(GEMM + fused row kernel); buffers are preallocated per batch size.
"""
import ctypes

import torch
import torch.nn as nn

from ._lib import Pose6dError, call, require_device, stream


class _Stage:
    pass


class HeadEngine:
    def __init__(self, seq):
        self.seq = seq
        self.stages = self._parse(list(seq))
        self._B = None
        self.generation = 0
        self._saved_gen = -1
        self.fuse_eval_bn = True   # False: the two separate launches (tests compare the two)

    @staticmethod
    def _parse(mods):
        stages, i = [], 0
        while i < len(mods):
            m = mods[i]
            st = _Stage()
            if isinstance(m, nn.Linear):
                st.kind, st.mod = "linear", m
                i += 1
            elif isinstance(m, nn.BatchNorm1d):
                st.kind, st.mod, st.act, st.drop = "bn1d", m, 0, None
                i += 1
                if i < len(mods) and isinstance(mods[i], nn.ReLU):
                    st.act = 1
                    i += 1
                if i < len(mods) and isinstance(mods[i], nn.Dropout):
                    st.drop = mods[i]
                    i += 1
            elif isinstance(m, nn.LayerNorm):
                if len(m.normalized_shape) != 1 or not m.elementwise_affine or m.bias is None:
                    raise Pose6dError("HeadEngine: LayerNorm must be affine over the last dimension")
                st.kind, st.mod, st.act, st.drop = "ln", m, 0, None
                i += 1
                if i < len(mods) and isinstance(mods[i], (nn.ReLU, nn.GELU)):
                    if isinstance(mods[i], nn.GELU) and getattr(mods[i], "approximate", "none") != "none":
                        raise Pose6dError("only exact (erf) GELU is implemented")
                    st.act = 1 if isinstance(mods[i], nn.ReLU) else 2
                    i += 1
                if i < len(mods) and isinstance(mods[i], nn.Dropout):
                    st.drop = mods[i]
                    i += 1
            elif isinstance(m, (nn.ReLU, nn.GELU, nn.Dropout)):
                st.kind, st.act, st.drop = "act", 0, None
                if isinstance(m, nn.ReLU):
                    st.act = 1
                    i += 1
                elif isinstance(m, nn.GELU):
                    if getattr(m, "approximate", "none") != "none":
                        raise Pose6dError("only exact (erf) GELU is implemented")
                    st.act = 2
                    i += 1
                if i < len(mods) and isinstance(mods[i], nn.Dropout):
                    st.drop = mods[i]
                    i += 1
            elif isinstance(m, nn.Flatten):
                i += 1
                continue
            else:
                raise Pose6dError(f"HeadEngine: unsupported layer {type(m).__name__}")
            stages.append(st)
        return stages

    def _prepare(self, B, in_dim, device):
        if self._B == (B, in_dim, device):
            return
        self._B = (B, in_dim, device)
        d = in_dim
        for st in self.stages:
            if st.kind == "linear":
                if st.mod.in_features != d:
                    raise Pose6dError("HeadEngine: shape mismatch")
                d = st.mod.out_features
            st.dim = d
            st.y = torch.empty(B, d, device=device, dtype=torch.float32)
            st.dx = torch.empty(B, (st.mod.in_features if st.kind == "linear" else d), device=device,
                                dtype=torch.float32)
            if st.kind in ("bn1d", "act", "ln"):
                st.mask = torch.empty(B, d, device=device, dtype=torch.uint8)
            if st.kind == "ln":
                if st.mod.normalized_shape[0] != d:
                    raise Pose6dError("HeadEngine: LayerNorm width mismatch")
                st.smean = torch.empty(B, device=device, dtype=torch.float32)
                st.srstd = torch.empty(B, device=device, dtype=torch.float32)
            if st.kind == "bn1d":
                st.smean = torch.empty(d, device=device, dtype=torch.float32)
                st.sinv = torch.empty(d, device=device, dtype=torch.float32)
        self.out_dim = d
        widest = max([in_dim] + [st.dim for st in self.stages])
        self.ws = torch.empty(16 * B * widest, device=device, dtype=torch.float32)   # split-K partials

    def forward(self, x, training, seed_dev=None, salt=0, inference=False):
        """x: (B, in) fp32 device tensor -> (B, out) (engine buffer).  inference=True:
        no backward will follow this forward (autograd.run's no-autograd branch), so
        eval Linear + BatchNorm1d pairs may skip the buffers only backward reads."""
        require_device(x)
        x = x.detach().float().contiguous()
        B = x.shape[0]
        self._prepare(B, x.shape[1], x.device)
        st_ = stream()
        cur = x
        self.x = x
        # eval without autograd: a Linear followed by an eval BatchNorm1d (no dropout)
        # stores the normalised output directly (pose6d_gemm_f32_bn_eval, bit-identical
        # to the two launches); nothing reads the Linear's raw output then.  Decided by
        # the caller (`inference`), not by torch.is_grad_enabled(): grad mode is off
        # inside autograd.Function.forward too, where a backward does follow
        fuse_bn = inference and not training and B <= 32 and self.fuse_eval_bn
        skip = -1
        for i, st in enumerate(self.stages):
            st.x = cur
            if i == skip:
                cur = st.y
                continue
            nxt = self.stages[i + 1] if i + 1 < len(self.stages) else None
            if (fuse_bn and st.kind == "linear" and nxt is not None and nxt.kind == "bn1d" and not nxt.mod.training
                    and not (nxt.drop is not None and nxt.drop.training and nxt.drop.p > 0)):
                m, bn = st.mod, nxt.mod
                K, N = m.in_features, m.out_features
                nxt.x, nxt.p, nxt.bn_train = st.y, 0.0, False
                call("gemm_f32_bn_eval", cur, K, m.weight.detach(), nxt.y, N,
                     m.bias.detach() if m.bias is not None else None, B, N, K, bn.weight.detach(), bn.bias.detach(),
                     bn.running_mean, bn.running_var, float(bn.eps), nxt.act, self.ws, self.ws.numel(), st_)
                skip = i + 1
                cur = st.y
                continue
            if st.kind == "linear":
                m = st.mod
                K, N = m.in_features, m.out_features
                call("gemm_f32", cur, K, 1, m.weight.detach(), 1, K, st.y, N,
                     m.bias.detach() if m.bias is not None else None, B, N, K, 1.0, 0.0, self.ws, self.ws.numel(),
                     st_)
            else:
                # per-module flags, as nn.Dropout / nn.BatchNorm1d themselves behave
                p = float(st.drop.p) if (st.drop is not None and st.drop.training and st.drop.p > 0) else 0.0
                if p > 0 and seed_dev is None:
                    raise Pose6dError("dropout in training needs a device seed")
                if st.kind == "bn1d":
                    bn = st.mod
                    st.bn_train = bn.training
                    call("bn1d_fwd", cur, st.y, B, st.dim, bn.weight.detach(), bn.bias.detach(), bn.running_mean,
                         bn.running_var, bn.num_batches_tracked, float(bn.momentum if bn.momentum is not None else 0.1),
                         float(bn.eps), int(bn.training), st.act, p, seed_dev, (salt * 131 + i) & 0xFFFFFFFFFFFF,
                         st.mask, st.smean, st.sinv, st_)
                elif st.kind == "ln":
                    ln = st.mod
                    call("layernorm_fwd", cur, st.dim, st.y, st.dim, None, B, st.dim, ln.weight.detach(),
                         ln.bias.detach(), float(ln.eps), st.act, p, seed_dev, (salt * 131 + i) & 0xFFFFFFFFFFFF,
                         st.mask, st.smean, st.srstd, st_)
                else:
                    call("act_fwd", cur, st.y, B * st.dim, st.act, p, seed_dev, (salt * 131 + i) & 0xFFFFFFFFFFFF,
                         st.mask, st_)
                st.p = p
            cur = st.y
        self.training = training
        self.generation += 1
        self._saved_gen = -1 if skip >= 0 else self.generation   # fused: no backward state
        return cur

    def backward(self, dy, grad_of, accumulate=False, need_dx=True, wgrad_stream=None):
        """wgrad_stream (a torch.cuda.Stream, optional): the Linear weight gradients,
        which nothing downstream of the head's data gradient reads, run there -- each
        after the current stream's work up to its launch -- so they overlap the trunk
        backward; the caller joins it (current_stream().wait_stream) before anything
        reads those gradients.  Their operands (the saved inputs, the stage gradients)
        are persistent buffers, next written by the following step's forward."""
        if self._saved_gen != self.generation:
            raise Pose6dError("HeadEngine.backward without matching forward")
        st_ = stream()
        B = dy.shape[0]
        g = dy.detach().float().contiguous()
        acc = int(accumulate)
        for idx in range(len(self.stages) - 1, -1, -1):
            st = self.stages[idx]
            last = idx == 0
            if st.kind == "linear":
                m = st.mod
                K, N = m.in_features, m.out_features
                # dW[N][K] = dy^T x and db = colsum(dy), one launch
                ws_ = st_
                if wgrad_stream is not None:
                    wgrad_stream.wait_stream(torch.cuda.current_stream())
                    ws_ = ctypes.c_void_p(wgrad_stream.cuda_stream)
                call("linear_wgrad", g, N, st.x, K, grad_of(m.weight),
                     grad_of(m.bias) if m.bias is not None else None, N, K, B, acc, ws_)
                if last and not need_dx:
                    return None
                call("gemm_f32", g, N, 1, m.weight.detach(), K, 1, st.dx, K, None, B, K, N, 1.0, 0.0, self.ws,
                     self.ws.numel(), st_)
            elif st.kind == "bn1d":
                bn = st.mod
                call("bn1d_bwd", g, st.x, st.y, B, st.dim, bn.weight.detach(), st.smean, st.sinv,
                     int(st.bn_train), st.act, st.p, st.mask, st.dx, grad_of(bn.weight), grad_of(bn.bias), acc,
                     st_)
            elif st.kind == "ln":
                ln = st.mod
                call("layernorm_bwd", g, st.dim, None, 0, st.x, st.dim, B, st.dim, ln.weight.detach(),
                     ln.bias.detach(), st.smean, st.srstd, st.act, st.p, st.mask, st.dx, st.dim, 0,
                     grad_of(ln.weight), grad_of(ln.bias), acc, st_)
            else:
                call("act_bwd", g, st.x, st.dx, B * st.dim, st.act, st.p, st.mask, st_)
            g = st.dx
        return g

    def params_in_grad_order(self):
        out = []
        for st in reversed(self.stages):
            if st.kind == "linear":
                out += [st.mod.weight] + ([st.mod.bias] if st.mod.bias is not None else [])
            elif st.kind in ("bn1d", "ln"):
                out += [st.mod.weight, st.mod.bias]
        return out

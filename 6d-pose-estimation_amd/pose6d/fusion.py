"""Cross-modal fusion engine of PoseNetRGBD (pose_net_rgbd.py:8-35,127-134) on the
pose6d HIP kernels (fp32):

    r   = rgb_norm(rgb_feat)                    LayerNorm(2048)       (:127)
    d   = depth_norm(depth_feat)                LayerNorm(2048)       (:128)
    q, k, v = q_proj(r), k_proj(d), v_proj(d)                         (:26-28)
    o   = dropout(softmax(q k^T * hd^-0.5)) v   per sample, 8 heads   (:30-34)
    out = [r + out_proj(o), d]                  residual + cat        (:131-134)

Launch plan (7 launches forward, 14 backward at batch 32): the two LayerNorms
write straight into the two halves of the (B, 4096) concatenation, out_proj
accumulates onto the rgb half in the GEMM epilogue (beta = 1), and the backward
LayerNorms take the residual / concatenation gradient as their second input —
no elementwise add or cat kernels exist on this path.

With norms=False the engine is CrossModalAttention.forward alone
(out = out_proj(o), no residual / cat).
"""
import torch

from ._lib import Pose6dError, call, require_device, stream


class FusionEngine:
    def __init__(self, attn, rgb_norm=None, depth_norm=None):
        self.attn = attn
        self.rgb_norm, self.depth_norm = rgb_norm, depth_norm
        self.norms = rgb_norm is not None
        if self.norms != (depth_norm is not None):
            raise Pose6dError("FusionEngine: give both LayerNorms or neither")
        self.D = attn.q_proj.in_features
        self.H, self.hd = attn.num_heads, attn.head_dim
        if self.H * self.hd != self.D:
            raise Pose6dError("FusionEngine: dim must equal num_heads * head_dim")
        self._key = None
        self.generation = 0
        self._saved_gen = -1

    def _prepare(self, B, device):
        if self._key == (B, device):
            return
        self._key = (B, device)
        D, H = self.D, self.H
        f = dict(device=device, dtype=torch.float32)
        self.out = torch.empty(B, 2 * D if self.norms else D, **f)
        self.R = torch.empty(B, D, **f)            # normalised rgb (q_proj input)
        self.Q, self.K, self.V, self.O = (torch.empty(B, D, **f) for _ in range(4))
        self.dQ, self.dK, self.dV, self.dO = (torch.empty(B, D, **f) for _ in range(4))
        self.dR, self.dDn = torch.empty(B, D, **f), torch.empty(B, D, **f)
        self.probs = torch.empty(B, H, H, **f)
        self.mask = torch.empty(B, H, H, device=device, dtype=torch.uint8)
        self.stats = torch.empty(4, B, **f)        # mean / rstd of the two LayerNorms
        self.ws = torch.empty(16 * B * D, **f)     # split-K GEMM partials

    def _linear(self, x, ldx, lin, y, ldy, beta, st):
        call("gemm_f32", x, ldx, 1, lin.weight.detach(), 1, lin.in_features, y, ldy, lin.bias.detach(), x.shape[0],
             lin.out_features, lin.in_features, 1.0, beta, self.ws, self.ws.numel(), st)

    def forward(self, rgb_feat, depth_feat, training, seed_dev=None, salt=0):
        require_device(rgb_feat, depth_feat)
        rgb_feat = rgb_feat.detach().float().contiguous()
        depth_feat = depth_feat.detach().float().contiguous()
        B, D = rgb_feat.shape[0], self.D
        if rgb_feat.shape != (B, D) or depth_feat.shape != (B, D):
            raise Pose6dError(f"FusionEngine: expected two (B, {D}) features")
        self._prepare(B, rgb_feat.device)
        st = stream()
        a = self.attn
        p = float(a.dropout.p) if (a.dropout.training and a.dropout.p > 0) else 0.0
        if p > 0 and seed_dev is None:
            raise Pose6dError("dropout in training needs a device seed")
        self.p = p
        self.rgb_in, self.depth_in = rgb_feat, depth_feat
        if self.norms:
            out_r, out_d = self.out[:, :D], self.out[:, D:]
            for ln, x, y, y2, k in ((self.rgb_norm, rgb_feat, out_r, self.R, 0), (self.depth_norm, depth_feat, out_d,
                                                                                    None, 2)):
                call("layernorm_fwd", x, D, y, 2 * D, y2, B, D, ln.weight.detach(), ln.bias.detach(), float(ln.eps),
                     0, 0.0, None, 0, None, self.stats[k], self.stats[k + 1], st)
            self.Rv, self.ldR = self.R, D
            self.Dv, self.ldD = out_d, 2 * D
            tgt, ldt, beta = out_r, 2 * D, 1.0
        else:
            self.Rv, self.ldR = rgb_feat, D
            self.Dv, self.ldD = depth_feat, D
            tgt, ldt, beta = self.out, D, 0.0
        self._linear(self.Rv, self.ldR, a.q_proj, self.Q, D, 0.0, st)
        self._linear(self.Dv, self.ldD, a.k_proj, self.K, D, 0.0, st)
        self._linear(self.Dv, self.ldD, a.v_proj, self.V, D, 0.0, st)
        call("xattn_fwd", self.Q, self.K, self.V, self.O, B, self.H, self.hd, float(a.scale), p, seed_dev,
             (salt * 131 + 7) & 0xFFFFFFFFFFFF, self.probs, self.mask, st)
        self._linear(self.O, D, a.out_proj, tgt, ldt, beta, st)
        self.generation += 1
        self._saved_gen = self.generation
        return self.out

    def _linear_bwd(self, dy, lddy, x, ldx, lin, dx, dx_beta, grad_of, acc, st):
        """dW (+)= dy^T x, db (+)= colsum(dy), dx = dy W (+ dx_beta * dx)."""
        B = dy.shape[0]
        N, K = lin.out_features, lin.in_features
        call("linear_wgrad", dy, lddy, x, ldx, grad_of(lin.weight), grad_of(lin.bias), N, K, B, acc, st)
        if dx is not None:
            call("gemm_f32", dy, lddy, 1, lin.weight.detach(), K, 1, dx, K, None, B, K, N, 1.0, dx_beta, self.ws,
                 self.ws.numel(), st)

    def backward(self, dout, grad_of, accumulate=False):
        """dout: gradient of the engine output -> (d rgb_feat, d depth_feat)."""
        if self._saved_gen != self.generation:
            raise Pose6dError("FusionEngine.backward without matching forward")
        st = stream()
        a = self.attn
        D = self.D
        g = dout.detach().float().contiguous()
        B = g.shape[0]
        acc = int(accumulate)
        ldg = 2 * D if self.norms else D
        g_r = g[:, :D]
        self._linear_bwd(g_r, ldg, self.O, D, a.out_proj, self.dO, 0.0, grad_of, acc, st)
        call("xattn_bwd", self.dO, self.Q, self.K, self.V, self.probs, self.mask, B, self.H, self.hd,
             float(a.scale), self.p, self.dQ, self.dK, self.dV, st)
        self._linear_bwd(self.dQ, D, self.Rv, self.ldR, a.q_proj, self.dR, 0.0, grad_of, acc, st)
        self._linear_bwd(self.dK, D, self.Dv, self.ldD, a.k_proj, self.dDn, 0.0, grad_of, acc, st)
        self._linear_bwd(self.dV, D, self.Dv, self.ldD, a.v_proj, self.dDn, 1.0, grad_of, acc, st)
        if not self.norms:
            return self.dR, self.dDn
        d_rgb = torch.empty(B, D, device=g.device, dtype=torch.float32)
        d_depth = torch.empty(B, D, device=g.device, dtype=torch.float32)
        # rgb: q-projection gradient + the residual branch; depth: k/v gradient + the cat branch
        for ln, x, dy, dy2, dx, k in ((self.rgb_norm, self.rgb_in, self.dR, g_r, d_rgb, 0),
                                      (self.depth_norm, self.depth_in, self.dDn, g[:, D:], d_depth, 2)):
            call("layernorm_bwd", dy, D, dy2, ldg, x, D, B, D, ln.weight.detach(), ln.bias.detach(), self.stats[k],
                 self.stats[k + 1], 0, 0.0, None, dx, D, 0, grad_of(ln.weight), grad_of(ln.bias), acc, st)
        return d_rgb, d_depth

    def params(self):
        a = self.attn
        out = []
        if self.norms:
            out += [self.rgb_norm.weight, self.rgb_norm.bias, self.depth_norm.weight, self.depth_norm.bias]
        for lin in (a.q_proj, a.k_proj, a.v_proj, a.out_proj):
            out += [lin.weight, lin.bias]
        return out


class _FusionFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, rgb_feat, depth_feat, eng, training, extra, *params):
        out = eng.forward(rgb_feat, depth_feat, training, **extra)
        ctx.eng, ctx.gen, ctx.params = eng, eng.generation, params
        return out.clone()

    @staticmethod
    def backward(ctx, dout):
        eng = ctx.eng
        if eng.generation != ctx.gen:
            raise Pose6dError("backward through the fusion engine after another forward of the same module")
        grads = {id(p): torch.empty_like(p) for p in ctx.params}
        d_rgb, d_depth = eng.backward(dout, lambda p: grads[id(p)])
        d_rgb = d_rgb.clone() if ctx.needs_input_grad[0] else None
        d_depth = d_depth.clone() if ctx.needs_input_grad[1] else None
        return (d_rgb, d_depth, None, None, None) + tuple(grads[id(p)] for p in ctx.params)


def run(eng, rgb_feat, depth_feat, training, **extra):
    params = eng.params()
    if torch.is_grad_enabled() and (rgb_feat.requires_grad or depth_feat.requires_grad or
                                    any(p.requires_grad for p in params)):
        return _FusionFn.apply(rgb_feat, depth_feat, eng, training, extra, *params)
    return eng.forward(rgb_feat, depth_feat, training, **extra).clone()

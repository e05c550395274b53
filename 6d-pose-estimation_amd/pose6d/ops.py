"""torch.autograd.Functions over the pose6d C ABI (small head / loss ops).

Every op checks that its tensors live on the ROCm device and calls exactly one
HIP entry point per direction.  No CPU fallback exists.
"""
import torch

from ._lib import call, require_device, stream


def _f32(t):
    return t.detach().to(torch.float32).contiguous()


class _PoseLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pr, pt, gr, gt, wr, wt, mode):
        require_device(pr, pt, gr, gt)
        pr_, pt_, gr_, gt_ = _f32(pr), _f32(pt), _f32(gr), _f32(gt)
        B = pr_.shape[0]
        loss = torch.empty((), device=pr.device, dtype=torch.float32)
        call("pose_loss_fwd", pr_, pt_, gr_, gt_, B, wr, wt, mode, loss, stream())
        ctx.save_for_backward(pr_, pt_, gr_, gt_)
        ctx.cfg = (wr, wt, mode)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        pr, pt, gr, gt = ctx.saved_tensors
        wr, wt, mode = ctx.cfg
        grot = torch.empty_like(pr)
        gtr = torch.empty_like(pt)
        call("pose_loss_bwd", pr, pt, gr, gt, pr.shape[0], wr, wt, mode, _f32(dloss), grot, gtr, stream())
        return grot, gtr, None, None, None, None, None


def pose_loss(pred_rot, pred_trans, gt_rot, gt_trans, rot_weight=1.0, trans_weight=1.0, mode=0):
    """PoseLoss.forward (pose_loss.py:19-28); mode 0 geodesic, 1 quaternion-L1."""
    return _PoseLoss.apply(pred_rot, pred_trans, gt_rot, gt_trans, rot_weight, trans_weight, mode)


class _RowNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, mode):
        require_device(x)
        x_ = _f32(x)
        y = torch.empty_like(x_)
        call("rownorm_fwd", x_, y, x_.shape[0], x_.shape[1], mode, stream())
        ctx.save_for_backward(x_)
        ctx.mode = mode
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dx = torch.empty_like(x)
        call("rownorm_bwd", x, _f32(dy), dx, x.shape[0], x.shape[1], ctx.mode, stream())
        return dx, None


def normalize(x):
    """F.normalize(x, p=2, dim=1) (pose_net_rgb.py:61)."""
    return _RowNorm.apply(x, 0)


def normalize_eps(x):
    """x / (||x|| + 1e-8) (pose_net_rgb_geometric.py:75)."""
    return _RowNorm.apply(x, 1)


def _kmat(K, B):
    K_ = _f32(K)
    if K_.dim() == 2:
        return K_, 0
    assert K_.shape[0] == B, "camera_matrix batch mismatch"
    return K_, 1


def pinhole_depth(depth_raw, bbox_center, K):
    """PoseNetRGBDGeometric._compute_pinhole_translation (pose_net_rgbd_geometric.py:56-85).
    No gradient flows (the reference's translation is a function of inputs only)."""
    require_device(depth_raw, bbox_center, K)
    d = _f32(depth_raw)
    B, H, W = d.shape
    K_, kb = _kmat(K, B)
    t = torch.empty(B, 3, device=d.device, dtype=torch.float32)
    call("pinhole_depth", d, H, W, _f32(bbox_center), K_, kb, B, t, stream())
    return t


class _PinholeZ(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, bbox, K):
        require_device(z, bbox, K)
        z_ = _f32(z).reshape(-1)
        B = z_.shape[0]
        K_, kb = _kmat(K, B)
        bb = _f32(bbox)
        t = torch.empty(B, 3, device=z.device, dtype=torch.float32)
        call("pinhole_z_fwd", z_, bb, K_, kb, B, t, stream())
        ctx.save_for_backward(bb, K_)
        ctx.kb = kb
        ctx.zshape = z.shape
        return t

    @staticmethod
    def backward(ctx, dt):
        bb, K_ = ctx.saved_tensors
        B = bb.shape[0]
        dz = torch.empty(B, device=dt.device, dtype=torch.float32)
        call("pinhole_z_bwd", _f32(dt), bb, K_, ctx.kb, B, dz, stream())
        return dz.reshape(ctx.zshape), None, None


def pinhole_z(z, bbox_center, K):
    """PoseNetRGBGeometric._compute_pinhole_translation (pose_net_rgb_geometric.py:93-109)."""
    return _PinholeZ.apply(z, bbox_center, K)

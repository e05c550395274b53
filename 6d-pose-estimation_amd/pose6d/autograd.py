"""torch.autograd bridges for the trunk and head engines, so the drop-in models
work under the reference scripts' `loss.backward()` + torch optimizers unchanged.

One Function per engine call (not per layer): forward runs the engine, backward
runs the engine's backward and hands autograd one fresh gradient per parameter.
"""
import torch

from ._lib import Pose6dError


class _EngineFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, eng, training, extra, *params):
        out = eng.forward(x, training, **extra)
        ctx.eng = eng
        ctx.gen = eng.generation
        ctx.params = params
        ctx.x_needs_grad = ctx.needs_input_grad[0]
        return out.clone()

    @staticmethod
    def backward(ctx, dout):
        eng = ctx.eng
        if eng.generation != ctx.gen:
            raise Pose6dError("backward through a pose6d engine after another forward of the same module "
                              "(its saved activations were overwritten)")
        grads = {id(p): torch.empty_like(p, memory_format=torch.contiguous_format) for p in ctx.params}
        dx = eng.backward(dout, lambda p: grads[id(p)])
        dx = dx.clone() if (dx is not None and ctx.x_needs_grad) else None
        return (dx, None, None, None) + tuple(grads[id(p)] for p in ctx.params)


def run(eng, x, training, params, copy=True, **extra):
    """Apply an engine with autograd when gradients are needed.  Without autograd the
    engine's output buffer is returned as is when copy=False (the caller consumes it
    before the engine runs again: trunk features feeding the heads)."""
    params = [p for p in params]
    if torch.is_grad_enabled() and (x.requires_grad or any(p.requires_grad for p in params)):
        return _EngineFn.apply(x, eng, training, extra, *params)
    out = eng.forward(x, training, inference=True, **extra)
    return out.clone() if copy else out

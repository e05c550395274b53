"""Per-kernel timing of a TrunkEngine's convolutions with HIP events (on the stream
the kernels are launched on), grouped by kernel symbol so the averages line up
with rocprofv3 --kernel-trace --stats rows."""
import collections

import torch

from ._lib import call, query, stream

# pose6d_conv_variant tile codes -> (BM, BN, waves per workgroup)
TILES = {0: (128, 128, 4), 1: (128, 64, 4), 2: (64, 128, 4), 3: (64, 64, 4), 4: (128, 128, 8), 5: (128, 64, 8)}


def _tname(dtype):
    return "__bf16" if dtype == torch.bfloat16 else "float"


def _sym(v, T):
    bm, bn, nw = TILES[v & 15]
    mode = (v >> 4) & 15
    if (v >> 8) & 1:
        return f"conv_lds_kernel<{T}, {bm}, {bn}, {mode}, {(v >> 12) & 15}, false, {nw}>"
    return f"conv_igemm_kernel<{T}, {bm}, {bn}, {mode}, false>"


def conv_launches(eng, fused=True):
    """(symbol, flops, launch-callable, name) for every conv pass of one training
    step, issued the way the step issues them (fused=True: one conv_bwd_kernel
    launch for the data + weight gradient where pose6d_conv2d_backward fuses them;
    False: the separate dgrad and wgrad(+reduce) passes)."""
    B, dt, T = eng.B, eng.dt, _tname(eng.dtype)
    st = stream()
    out = []
    for op in eng.convs:
        M = B * op.Ho * op.Wo
        K = op.k * op.k * op.cin
        flops = 2.0 * M * op.cout * K
        sym = _sym(query("conv_variant", dt, 0, B, op.H, op.W, op.cin_pad, op.cout, op.k, op.k, op.stride, op.pad,
                         op.Ho, op.Wo), T)

        def fwd(op=op):
            call("conv2d_fwd", dt, op.src.t, op.wp, op.conv.bias, op.out.t, op.stats, B, op.H, op.W, op.cin_pad,
                 op.cout, op.k, op.k, op.stride, op.pad, op.Ho, op.Wo, eng.ws_sk, eng.ws_sk_bytes, st)
        out.append((sym, flops, fwd, op.name + ".fwd"))
        bv = query("bwd_variant", dt, B, op.H, op.W, op.cin_pad, op.cout, op.k, op.k, op.stride, op.pad, op.Ho,
                   op.Wo) if (op.needs_dgrad and fused) else 0
        if bv:
            # the step's fused data + weight gradient launch (conv2d_backward phase 1;
            # the slab reduce is its own kernel and row in rocprof)
            # conv_bwd_kernel<DMODE, DS, WS[, float]>: WS = POSE6D_WGRAD_STAGES (3, bf16) or
            # POSE6D_WGRAD_STAGES_F32 (2, fp32; csrc/wgrad_body.h)
            if eng.dtype == torch.float32:
                sym = f"conv_bwd_kernel<{(bv >> 4) & 15}, {bv & 15}, 2, float>"
            else:
                sym = f"conv_bwd_kernel<{(bv >> 4) & 15}, {bv & 15}, 3>"
            dw = torch.empty_like(op.conv.weight)

            def bwd(op=op, dw=dw):
                call("conv2d_backward_ex", dt, op.src.t, op.out.g, op.wt, None, op.src.g, dw, 0, eng.ws_wgrad,
                     eng.ws_wgrad.numel() * 4, B, op.H, op.W, op.cin_pad, op.cin, op.cout, op.k, op.k, op.stride,
                     op.pad, op.Ho, op.Wo, 1, st)
            out.append((sym, 2 * flops, bwd, op.name + ".bwd"))
            continue
        if op.needs_dgrad:
            sym = _sym(query("conv_variant", dt, 1, B, op.H, op.W, op.cin_pad, op.cout, op.k, op.k, op.stride,
                             op.pad, op.Ho, op.Wo), T)

            def dgrad(op=op):
                call("conv2d_dgrad", dt, op.out.g, op.wt, None, op.src.g, B, op.H, op.W, op.cin_pad, op.cout, op.k,
                     op.k, op.stride, op.pad, op.Ho, op.Wo, st)
            out.append((sym, flops, dgrad, op.name + ".dgrad"))
        v = query("wgrad_variant", dt, M, op.cout, op.k * op.k * op.cin_pad, op.cin_pad)
        if (v >> 8) & 1 and eng.dtype == torch.float32:
            pw = str(op.k == 1 and op.stride == 1 and op.pad == 0).lower()
            sym = f"conv_wgrad_lds_f32_kernel<{v >> 12}, {pw}, {128 if v & 2 else 64}>"
        elif (v >> 8) & 1:
            sym = f"conv_wgrad_lds_kernel<64, 64, {v >> 12}>"
        else:
            sym = f"conv_wgrad_kernel<{T}, {128 if v & 2 else 64}, {128 if v & 1 else 64}>"
        dw = torch.empty_like(op.conv.weight)

        def wgrad(op=op, dw=dw):
            call("conv2d_wgrad", dt, op.src.t, op.out.g, dw, 0, eng.ws_wgrad, eng.ws_wgrad.numel() * 4, B, op.H,
                 op.W, op.cin_pad, op.cin, op.cout, op.k, op.k, op.stride, op.pad, op.Ho, op.Wo, st)
        out.append((sym + "+reduce", flops, wgrad, op.name + ".wgrad"))
    return out


def time_launches(launches, reps=10):
    """Average duration of each launch (events bracket `reps` back-to-back launches)."""
    res = []
    s = torch.cuda.current_stream()
    for sym, flops, fn, name in launches:
        fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            fn()
        e1.record(s)
        e1.synchronize()
        res.append((sym, flops, e0.elapsed_time(e1) / reps * 1e-3, name))
    return res


def by_symbol(timed):
    agg = collections.OrderedDict()
    for sym, flops, t, name in timed:
        a = agg.setdefault(sym, {"launches": 0, "time_s": 0.0, "flops": 0.0})
        a["launches"] += 1
        a["time_s"] += t
        a["flops"] += flops
    return agg

"""Per-layer conv timing sweep (GPU box): every distinct ResNet50 conv shape at
batch 32 bf16, fwd / dgrad / wgrad, each implementation x tile, TFLOP/s.
usage: python tools/conv_bench.py [--passes fwd,dgrad] [--impls base,fast] [--tiles 0,1,2,3]
Plans are chosen through pose6d_tuning_t (the *_tuned entry points); --env / --wgrad-env
sweep tuning fields, e.g. --env "conv_tile=4,conv_stages=2;conv_s2=0"."""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "6d-pose-estimation_amd")]

import pose6d._lib as _plib  # noqa: E402
from pose6d._lib import Tuning, call, query, stream  # noqa: E402
from pose6d.trunk import DTYPES, pack_single  # noqa: E402

# (H, W, Cin, Cout, k, s, p) per distinct ResNet50 conv (input geometry)
SHAPES = [
    (224, 224, 4, 64, 7, 2, 3),
    (56, 56, 64, 64, 1, 1, 0), (56, 56, 64, 64, 3, 1, 1), (56, 56, 64, 256, 1, 1, 0), (56, 56, 256, 64, 1, 1, 0),
    (56, 56, 256, 128, 1, 1, 0), (56, 56, 128, 128, 3, 2, 1), (28, 28, 128, 512, 1, 1, 0), (56, 56, 256, 512, 1, 2, 0),
    (28, 28, 512, 128, 1, 1, 0), (28, 28, 128, 128, 3, 1, 1), (28, 28, 512, 256, 1, 1, 0),
    (28, 28, 256, 256, 3, 2, 1), (14, 14, 256, 1024, 1, 1, 0), (28, 28, 512, 1024, 1, 2, 0),
    (14, 14, 1024, 256, 1, 1, 0), (14, 14, 256, 256, 3, 1, 1), (14, 14, 1024, 512, 1, 1, 0),
    (14, 14, 512, 512, 3, 2, 1), (7, 7, 512, 2048, 1, 1, 0), (14, 14, 1024, 2048, 1, 2, 0),
    (7, 7, 2048, 512, 1, 1, 0), (7, 7, 512, 512, 3, 1, 1),
]


GRAPH = False
TUNE = Tuning()   # the plan override the timed calls pass (mutated by the sweeps)


def _set_tune(**kw):
    for f, _ in Tuning._fields_:
        setattr(TUNE, f, -1)
    for k, v in kw.items():
        setattr(TUNE, k, int(v))


def timeit(fn, reps=20):
    fn()
    if GRAPH:   # the calls replayed from one hipGraph: no host-issue floor (~6 us per ctypes call)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(reps):
                fn()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            g.replay()
        e1.record()
        e1.synchronize()
        return e0.elapsed_time(e1) / (5 * reps) * 1e-3
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        fn()
    e1.record(s)
    e1.synchronize()
    return e0.elapsed_time(e1) / reps * 1e-3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--passes", default="fwd,dgrad,wgrad")
    ap.add_argument("--impls", default="base,fast")
    ap.add_argument("--tiles", default="auto,0,1,3")
    ap.add_argument("--stages", default="auto", help="fast-path LDS ring depths to sweep, e.g. auto,2,3,4,6")
    ap.add_argument("--wgrad-env", default="", help="';'-separated field=V[,field=V] pose6d_tuning_t settings to "
                                                     "sweep for wgrad")
    ap.add_argument("--env", default="", help="';'-separated field=V[,field=V] pose6d_tuning_t settings to sweep "
                                           "for fwd / dgrad")
    ap.add_argument("--B", type=int, default=32)
    ap.add_argument("--only", default="", help="comma-separated indices into SHAPES")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--lib", default="", help="load this libpose6d build instead (tools/conv_exp.sh variants)")
    ap.add_argument("--graph", action="store_true", help="time replays of a captured graph (GPU time, no host floor)")
    a = ap.parse_args()
    global GRAPH
    GRAPH = a.graph
    if a.lib:
        _plib.LIB_PATH = os.path.abspath(a.lib)
    dtype = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    B, dt, dev = a.B, DTYPES[dtype], "cuda"
    st = stream()
    tot = {}
    flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev) if "fwdcold" in a.passes else None
    for (H, W, Cin, Cout, k, s, p) in (SHAPES if not a.only else [SHAPES[int(i)] for i in a.only.split(",")]):
        Ho, Wo = (H + 2 * p - k) // s + 1, (W + 2 * p - k) // s + 1
        x = torch.randn(B, H, W, Cin, device=dev).to(dtype)
        w = torch.randn(Cout, Cin, k, k, device=dev) * 0.05
        wp, wt = pack_single(w, Cin, dtype, stride=s, pad=p)
        y = torch.empty(B, Ho, Wo, Cout, device=dev, dtype=dtype)
        dy = torch.randn(B, Ho, Wo, Cout, device=dev).to(dtype)
        dx = torch.empty(B, H, W, Cin, device=dev, dtype=dtype)
        stats = torch.empty(query("conv_stats_rows", B, Ho, Wo, Cout), 2, Cout, device=dev)
        # room for any split plan the --wgrad-env sweep selects (the call checks the size)
        ws = torch.empty(max(query("conv2d_wgrad_workspace_tuned", dt, B, Ho, Wo, Cin, Cout, k, k,
                                   Tuning(wgrad_base=1).ref), 256 << 20) // 4,
                         device=dev)
        dw = torch.empty(Cout, Cin, k, k, device=dev)
        skw = torch.zeros(64 << 20, device=dev, dtype=torch.uint8)   # split-K workspace (caller-provided)
        flops = 2.0 * B * Ho * Wo * Cout * Cin * k * k
        sc, sh = torch.rand(Cout, device=dev) + 0.5, torch.randn(Cout, device=dev) * 0.1
        res = torch.randn(B, Ho, Wo, Cout, device=dev).to(dtype) if "fwdactres" in a.passes else None
        # the residual junction's gradient added in the data-gradient epilogue (bwdres*)
        dres = torch.randn(B, H, W, Cin, device=dev).to(dtype) if "bwdres" in a.passes else None
        if "bwdrescold" in a.passes and flush is None:
            flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
        fns = {
            "fwd": lambda: call("conv2d_fwd_tuned", dt, x, wp, None, y, stats, B, H, W, Cin, Cout, k, k, s, p, Ho,
                                Wo, TUNE.ref, skw, skw.numel(), stream()),
            # tuned, no BN statistics (stats-free plans: the 3x3 patch kernel)
            "fwdnst": lambda: call("conv2d_fwd_tuned", dt, x, wp, None, y, None, B, H, W, Cin, Cout, k, k, s, p, Ho,
                                   Wo, TUNE.ref, skw, skw.numel(), stream()),
            # no BN statistics (as in eval without the fold)
            "fwdns": lambda: call("conv2d_fwd", dt, x, wp, None, y, None, B, H, W, Cin, Cout, k, k, s, p, Ho, Wo,
                                  skw, skw.numel(), stream()),
            # each call behind a 512 MB write (caches hold none of the conv's operands), minus that write's time
            "fwdcold": lambda: (flush.zero_(), call("conv2d_fwd", dt, x, wp, None, y, stats, B, H, W, Cin, Cout, k,
                                                    k, s, p, Ho, Wo, skw, skw.numel(), stream())),
            "flush": lambda: flush.zero_(),
            # eval epilogue: BN (+ residual) + ReLU applied before the store (pose6d_conv2d_fwd_act)
            "fwdact": lambda: call("conv2d_fwd_act", dt, x, wp, None, y, B, H, W, Cin, Cout, k, k, s, p, Ho, Wo, sc,
                                   sh, None, None, None, 1, skw, skw.numel(), stream()),
            "fwdactres": lambda: call("conv2d_fwd_act", dt, x, wp, None, y, B, H, W, Cin, Cout, k, k, s, p, Ho, Wo,
                                      sc, sh, res, None, None, 1, skw, skw.numel(), stream()),
            "dgrad": lambda: call("conv2d_dgrad_tuned", dt, dy, wt, None, dx, B, H, W, Cin, Cout, k, k, s, p, Ho, Wo,
                                  TUNE.ref, skw, skw.numel(), stream()),
            "dgradip": lambda: call("conv2d_dgrad", dt, dy, wt, dx, dx, B, H, W, Cin, Cout, k, k, s, p, Ho, Wo, stream()),
            "bwdip": lambda: call("conv2d_backward", dt, x, dy, wt, dx, dx, dw, 0, ws, ws.numel() * 4, B, H, W, Cin,
                                  Cin, Cout, k, k, s, p, Ho, Wo, stream()),
            "bwd": lambda: call("conv2d_backward_tuned", dt, x, dy, wt, None, dx, dw, 0, ws, ws.numel() * 4, B, H, W,
                                Cin, Cin, Cout, k, k, s, p, Ho, Wo, TUNE.ref, stream()),
            "bwdres": lambda: call("conv2d_backward_tuned", dt, x, dy, wt, dres, dx, dw, 0, ws, ws.numel() * 4, B, H,
                                   W, Cin, Cin, Cout, k, k, s, p, Ho, Wo, TUNE.ref, stream()),
            # behind a 512 MB write (operands from HBM, as in the step), minus that write's time (--passes flush)
            "bwdrescold": lambda: (flush.zero_(), call("conv2d_backward_tuned", dt, x, dy, wt, dres, dx, dw, 0, ws,
                                                       ws.numel() * 4, B, H, W, Cin, Cin, Cout, k, k, s, p, Ho, Wo,
                                                       TUNE.ref, stream())),
            "wgrad": lambda: call("conv2d_wgrad_tuned", dt, x, dy, dw, 0, ws, ws.numel() * 4, B, H, W, Cin, Cin, Cout,
                                  k, k, s, p, Ho, Wo, TUNE.ref, stream()),
        }
        line = f"{H:3d}x{W:<3d} {Cin:4d}->{Cout:<4d} k{k}s{s} |"
        if "fwdcold" in a.passes.split(",") or "bwdrescold" in a.passes.split(","):
            line += f" flush:{timeit(fns['flush']) * 1e6:6.1f}us"
        for ps in a.passes.split(","):
            if ps in ("dgrad", "bwd", "dgradip", "bwdip", "bwdres", "bwdrescold") and Cin % 8:
                continue   # the stem has no data gradient
            sweep = a.wgrad_env if ps == "wgrad" else a.env
            if sweep:
                for spec in ["auto"] + sweep.split(";"):
                    kv = [] if spec == "auto" else [e.split("=") for e in spec.split(",")]
                    _set_tune(**{k_: v_ for k_, v_ in kv})
                    sec = timeit(fns[ps])
                    _set_tune()
                    line += f" {ps[0]}[{spec}]:{sec * 1e6:6.1f}us/{flops / sec / 1e12:5.0f}T"
                continue
            impls = {"wgrad": ["base"], "bwd": ["fast"], "bwdip": ["fast"], "bwdres": ["fast"],
                     "bwdrescold": ["fast"]}.get(ps, a.impls.split(","))
            tiles = a.tiles.split(",") if ps not in ("wgrad", "bwd", "bwdip", "bwdres", "bwdrescold") else ["auto"]
            for impl in impls:
                stages = a.stages.split(",") if impl == "fast" else ["auto"]
                for t in tiles:
                    for nst in stages:
                        kw = {"conv_base": int(impl == "base"), "wgrad_base": int(impl == "base")}
                        if t != "auto":
                            kw["conv_tile"] = t
                        if nst != "auto":
                            kw["conv_stages"] = nst
                        _set_tune(**kw)
                        try:
                            sec = timeit(fns[ps])
                        except Exception as e:  # noqa: BLE001
                            line += f" {ps}:{impl}/{t}/{nst}=ERR({str(e)[:120]})"
                            continue
                        tf = flops / sec / 1e12
                        tag = f"{ps}/{impl[0]}{t}" + (f"s{nst}" if impl == "fast" else "")
                        line += f" {tag}:{sec * 1e6:6.1f}us/{tf:5.0f}T"
                        if t == "auto" and nst == "auto":
                            tot[(ps, impl)] = tot.get((ps, impl), 0.0) + sec
        _set_tune()
        print(line, flush=True)
    print("totals (auto tile, one instance per distinct shape):",
          {f"{k[0]}/{k[1]}": round(v * 1e3, 3) for k, v in tot.items()})


if __name__ == "__main__":
    main()

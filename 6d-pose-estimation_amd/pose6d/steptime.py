"""Per-kernel durations measured INSIDE a captured step (hipGraph), with HIP events.

The graph of a step is captured exactly as the trainer captures it; then, before it
is instantiated, one event-record node is spliced in front of every node and one
after the last (hipGraphAddEventRecordNode, graph surgery through the HIP runtime
torch already loaded).  Replaying it gives, for every kernel of the step, the time
between the event before it and the event after it: the kernel as the step issues
it (same arguments, same predecessor, same cache state), not an isolated replay.

While the step is captured, every pose6d entry point called (pose6d._lib.call) is
logged with the graph's node count after it, so each kernel node maps back to the
call (and conv geometry) that launched it: that gives algorithmic flops per node.

Each event node adds a nearly constant cost to the interval it closes (the marker
packet between two dispatches: ~3 us on MI355X).  run(plain_ms=...) calibrates it
against the uninstrumented replay of the same step: overhead per node = (instrumented
step - plain step) / nodes, subtracted from every node.  With it the in-step averages
agree with rocprofv3 --kernel-trace of the plain replay within ~1 % (profiles/r03*).

Used by bench.py for the `roofline` object and the per-symbol breakdown.
"""
import collections
import ctypes

import torch

from . import _lib

_hip = None


def hip():
    global _hip
    if _hip is None:
        h = ctypes.CDLL("libamdhip64.so.7")   # soname: the runtime torch already loaded
        vp, sz = ctypes.c_void_p, ctypes.c_size_t
        P = ctypes.POINTER
        sig = {
            "hipGraphGetNodes": [vp, P(vp), P(sz)],
            "hipGraphNodeGetType": [vp, P(ctypes.c_int)],
            "hipGraphNodeGetDependencies": [vp, P(vp), P(sz)],
            "hipGraphRemoveDependencies": [vp, P(vp), P(vp), sz],
            "hipGraphAddDependencies": [vp, P(vp), P(vp), sz],
            "hipGraphAddEventRecordNode": [P(vp), vp, P(vp), sz, vp],
            "hipGraphKernelNodeGetParams": [vp, ctypes.c_void_p],
            "hipEventCreate": [P(vp)],
            "hipEventDestroy": [vp],
            "hipEventElapsedTime": [P(ctypes.c_float), vp, vp],
            "hipStreamGetCaptureInfo_v2": [vp, P(ctypes.c_int), P(ctypes.c_ulonglong), P(vp), P(vp), P(sz)],
        }
        for n, a in sig.items():
            f = getattr(h, n)
            f.argtypes = a
            f.restype = ctypes.c_int
        h.hipKernelNameRefByPtr.argtypes = [vp, vp]
        h.hipKernelNameRefByPtr.restype = ctypes.c_char_p
        _hip = h
    return _hip


def _ok(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed (hipError {rc})")


class _KernelNodeParams(ctypes.Structure):
    _fields_ = [("block", ctypes.c_uint * 3), ("extra", ctypes.c_void_p), ("func", ctypes.c_void_p),
                ("grid", ctypes.c_uint * 3), ("kernelParams", ctypes.c_void_p), ("sharedMemBytes", ctypes.c_uint)]


_demangle = None


def short_name(mangled):
    """Demangled kernel name without namespace, return type and argument list:
    'conv_bwd_kernel<0, 2, 3, false>' (the prefix of rocprofv3's kernel names)."""
    global _demangle
    if _demangle is None:
        cxx = ctypes.CDLL("libstdc++.so.6")
        _demangle = cxx.__cxa_demangle
        _demangle.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        _demangle.restype = ctypes.c_void_p
    st = ctypes.c_int(0)
    p = _demangle(mangled, None, None, ctypes.byref(st))
    if (st.value != 0 or not p) and b"DF16b" in mangled:
        # libstdc++ 11 does not know the __bf16 mangling (DF16b): spell it as the
        # vendor type u6__bf16, which demangles to "__bf16" with the same substitutions
        p = _demangle(mangled.replace(b"DF16b", b"u6__bf16"), None, None, ctypes.byref(st))
    if st.value != 0 or not p:
        return mangled.decode()
    s = ctypes.string_at(p).decode()
    ctypes.CDLL(None).free(ctypes.c_void_p(p))
    s = s.replace("(anonymous namespace)::", "")
    if s.startswith("void "):
        s = s[5:]
    depth, cut = 0, len(s)
    for i, ch in enumerate(s):   # drop the argument list: the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    return s[:cut]


def _graph_nodes(graph):
    h = hip()
    n = ctypes.c_size_t(0)
    _ok(h.hipGraphGetNodes(graph, None, ctypes.byref(n)), "hipGraphGetNodes")
    arr = (ctypes.c_void_p * max(n.value, 1))()
    _ok(h.hipGraphGetNodes(graph, arr, ctypes.byref(n)), "hipGraphGetNodes")
    return [arr[i] for i in range(n.value)]


def _deps(node):
    h = hip()
    n = ctypes.c_size_t(0)
    _ok(h.hipGraphNodeGetDependencies(node, None, ctypes.byref(n)), "hipGraphNodeGetDependencies")
    arr = (ctypes.c_void_p * max(n.value, 1))()
    _ok(h.hipGraphNodeGetDependencies(node, arr, ctypes.byref(n)), "hipGraphNodeGetDependencies")
    return [arr[i] for i in range(n.value)]


class _CallLog:
    """_lib.call observer during capture: (name, args, graph node count after it)."""

    def __init__(self, stream_ptr):
        self.stream = stream_ptr
        self.entries = []

    def node_count(self):
        h = hip()
        status, cid = ctypes.c_int(0), ctypes.c_ulonglong(0)
        g, deps, nd = ctypes.c_void_p(0), ctypes.c_void_p(0), ctypes.c_size_t(0)
        _ok(h.hipStreamGetCaptureInfo_v2(ctypes.c_void_p(self.stream), ctypes.byref(status), ctypes.byref(cid),
                                         ctypes.byref(g), ctypes.byref(deps), ctypes.byref(nd)),
            "hipStreamGetCaptureInfo_v2")
        if status.value != 1 or not g.value:   # 1 = hipStreamCaptureStatusActive
            return None
        n = ctypes.c_size_t(0)
        _ok(hip().hipGraphGetNodes(g, None, ctypes.byref(n)), "hipGraphGetNodes")
        return n.value

    def __call__(self, name, args):
        self.entries.append((name, args, self.node_count()))


def conv_flops(name, args, sym):
    """Algorithmic flops (2 per multiply-add, real input channels) of the kernel `sym`
    launched by pose6d_<name>(*args); None for a non-conv call, 0 for the weight-
    gradient slab reduce."""
    if "reduce" in sym and "wgrad" in sym:
        return 0.0
    if name in ("conv2d_fwd", "conv2d_fwd_act"):
        N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo = args[6:17] if name == "conv2d_fwd" else args[5:16]
        cin = 3 if Cin == 4 else Cin   # the padded stem input (RGB padded to 4 channels)
        return 2.0 * N * Ho * Wo * Cout * KH * KW * cin
    if name in _BWD_N_INDEX:
        i0 = _BWD_N_INDEX[name]
        N, H, W, Cin, Cin_real, Cout, KH, KW, stride, pad, Ho, Wo = args[i0:i0 + 12]
        one = 2.0 * N * Ho * Wo * Cout * KH * KW * Cin_real
        if sym.startswith("conv_bwd_kernel"):
            return 2 * one          # data + weight gradient in one launch
        if args[i0 - 5] is None:    # dx == NULL: weight gradient only (the stem)
            return one if "wgrad" in sym else 0.0
        return one                  # a separate data-gradient or weight-gradient launch
    if name == "conv2d_fwd_act_dual":
        N, Ho, Wo, Cin, Cout, Hd, Wd, Cind = args[6:14]
        return 2.0 * N * Ho * Wo * Cout * (Cin + Cind)
    return None


def conv_bytes(name, args, sym):
    """Algorithmic HBM bytes of the kernel `sym` launched by pose6d_<name>(*args): every
    operand read once and every result written once (activations in the call's dtype,
    weights as packed, fp32 dW, the residual gradient and its ReLU bits where the call
    carries them); None where conv_flops is None, 0 for the slab reduce (its bytes ride
    in the fused launch that carries it)."""
    if "reduce" in sym and "wgrad" in sym:
        return 0.0
    if name in ("conv2d_fwd", "conv2d_fwd_act"):
        dt = args[0]
        N, H, W, Cin, Cout, KH, KW, stride, pad, Ho, Wo = args[6:17] if name == "conv2d_fwd" else args[5:16]
        e = 4 if dt == 0 else 2
        b = e * (N * H * W * Cin + Cout * KH * KW * Cin + N * Ho * Wo * Cout)
        if name == "conv2d_fwd_act" and args[18] is not None:   # residual added in the epilogue
            b += e * N * Ho * Wo * Cout
        return float(b)
    if name in _BWD_N_INDEX:
        i0 = _BWD_N_INDEX[name]
        dt = args[0]
        e = 4 if dt == 0 else 2
        N, H, W, Cin, Cin_real, Cout, KH, KW, stride, pad, Ho, Wo = args[i0:i0 + 12]
        x = N * H * W * Cin * e
        dy = N * Ho * Wo * Cout * e
        w = Cout * KH * KW * Cin * e
        dw = Cout * KH * KW * Cin_real * 4
        dres = args[4] is not None   # in place (dres == dx) it is still read
        dgrad = (x + dy + w + (x if dres else 0) + (N * H * W * Cin // 8 if name != "conv2d_backward_chain" and
                                                     args[5] is not None else 0))
        wgrad = x + dy + dw
        bn = args[-2] if name == "conv2d_backward_chain_bn" else None
        if bn:
            # the BN-reduce epilogue reads the BN's input y (and a second BN's y2) and
            # its ReLU bits: pose6d_bn_reduce_t {y, mean, invstd, rs, rb, relu_mask,
            # partial, y2, ...}, 8-byte pointers
            ptr = ctypes.c_void_p.from_address
            dgrad += x
            if ptr(bn + 5 * 8).value:
                dgrad += N * H * W * Cin // 8
            if ptr(bn + 7 * 8).value:
                dgrad += x
        if sym.startswith("conv_bwd_kernel"):
            return float(dgrad + wgrad - dy)   # dY read once by the fused launch
        if args[i0 - 5] is None:
            return float(wgrad) if "wgrad" in sym else 0.0
        return float(wgrad if "wgrad" in sym else dgrad)
    if name == "conv2d_fwd_act_dual":
        dt = args[0]
        e = 4 if dt == 0 else 2
        N, Ho, Wo, Cin, Cout, Hd, Wd, Cind = args[6:14]
        return float(e * (N * Ho * Wo * (Cin + Cout + Cind) + Cout * (Cin + Cind)))   # xd read at the sampled pixels
    return None


# index of N in the argument list of the backward entry points
_BWD_N_INDEX = {"conv2d_backward_chain": 10, "conv2d_backward_chain_masked": 11, "conv2d_backward_chain_bn": 11}


def conv_geom(name, args):
    """'N HxW Cin->Cout kKsS' of a conv call (None otherwise), for per-launch listings."""
    idx = {"conv2d_fwd": 6, "conv2d_fwd_act": 5, **_BWD_N_INDEX}
    if name not in idx:
        return None
    i = idx[name]
    if name.startswith("conv2d_backward"):
        N, H, W, Cin, _, Cout, KH, _, stride = args[i:i + 9]
    else:
        N, H, W, Cin, Cout, KH, _, stride = args[i:i + 8]
    return f"{N} {H}x{W} {Cin}->{Cout} k{KH}s{stride}"


class StepTimer:
    """Capture `step()` into a graph with an event before every node; `run(reps)`
    replays it and returns one record per kernel node with its mean duration."""

    def __init__(self, step, device, warm=True):
        h = hip()
        s = torch.cuda.Stream(device=device)
        s.wait_stream(torch.cuda.current_stream())
        if warm:
            with torch.cuda.stream(s):
                step()
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph(keep_graph=True)
        # thread-local capture: under a live RCCL group the watchdog thread queries the
        # events of in-flight collectives meanwhile, which a global-mode capture forbids
        with torch.cuda.graph(self.graph, stream=s, capture_error_mode="thread_local"):
            log = _CallLog(torch.cuda.current_stream().cuda_stream)
            _lib.observers.append(log)
            try:
                step()
            finally:
                _lib.observers.remove(log)
        raw = ctypes.c_void_p(self.graph.raw_cuda_graph())
        nodes = _graph_nodes(raw)
        # the capture of one stream is a chain: node i depends on node i - 1 only
        for i, nd in enumerate(nodes):
            d = _deps(nd)
            if d != ([] if i == 0 else [nodes[i - 1]]):
                raise RuntimeError("StepTimer: captured graph is not a single chain")
        # node index -> the pose6d call that created it
        owner = [None] * len(nodes)
        prev = 0
        for name, args, cnt in log.entries:
            if cnt is None:
                continue
            for j in range(prev, min(cnt, len(nodes))):
                owner[j] = (name, args)
            prev = max(prev, cnt)
        self.events = []
        for i in range(len(nodes) + 1):
            e = ctypes.c_void_p()
            _ok(h.hipEventCreate(ctypes.byref(e)), "hipEventCreate")
            self.events.append(e)
        self.records = []
        for i, nd in enumerate(nodes):
            t = ctypes.c_int(-1)
            _ok(h.hipGraphNodeGetType(nd, ctypes.byref(t)), "hipGraphNodeGetType")
            sym = None
            if t.value == 0:   # kernel node
                p = _KernelNodeParams()
                _ok(h.hipGraphKernelNodeGetParams(nd, ctypes.byref(p)), "hipGraphKernelNodeGetParams")
                nm = h.hipKernelNameRefByPtr(p.func, None)
                sym = short_name(nm) if nm else "?"
            name, args = owner[i] if owner[i] else (None, None)
            fl = conv_flops(name, args, sym) if (sym and name) else None
            nb = conv_bytes(name, args, sym) if (sym and name) else None
            self.records.append({"node": i, "type": t.value, "kernel": sym, "call": name, "flops": fl, "bytes": nb,
                                 "geom": conv_geom(name, args) if name else None})
            # splice: deps(node) -> event_i -> node
            ev = ctypes.c_void_p()
            if i == 0:
                _ok(h.hipGraphAddEventRecordNode(ctypes.byref(ev), raw, None, 0, self.events[0]), "addEventRecord")
            else:
                a = (ctypes.c_void_p * 1)(nodes[i - 1])
                b = (ctypes.c_void_p * 1)(nd)
                _ok(h.hipGraphRemoveDependencies(raw, a, b, 1), "hipGraphRemoveDependencies")
                _ok(h.hipGraphAddEventRecordNode(ctypes.byref(ev), raw, a, 1, self.events[i]), "addEventRecord")
            a = (ctypes.c_void_p * 1)(ev)
            b = (ctypes.c_void_p * 1)(nd)
            _ok(h.hipGraphAddDependencies(raw, a, b, 1), "hipGraphAddDependencies")
        ev = ctypes.c_void_p()
        a = (ctypes.c_void_p * 1)(nodes[-1])
        _ok(h.hipGraphAddEventRecordNode(ctypes.byref(ev), raw, a, 1, self.events[-1]), "addEventRecord")
        self.graph.instantiate()
        self.stream = s

    def run(self, reps=10, plain_ms=None):
        """Replay `reps` times; each kernel record gets 'us' = mean in-step duration
        (minus the calibrated per-node event overhead when `plain_ms`, the step's
        uninstrumented replay time, is given) and 'us_raw' = the raw event interval."""
        h = hip()
        n = len(self.records)
        acc = [0.0] * n
        total = 0.0
        ms = ctypes.c_float(0.0)
        for _ in range(reps + 1):
            self.graph.replay()
            torch.cuda.synchronize()
            if _ == 0:
                continue   # first replay warms the instantiated graph
            for i in range(n):
                _ok(h.hipEventElapsedTime(ctypes.byref(ms), self.events[i], self.events[i + 1]), "elapsed")
                acc[i] += ms.value
            _ok(h.hipEventElapsedTime(ctypes.byref(ms), self.events[0], self.events[n]), "elapsed")
            total += ms.value
        self.total_ms = total / reps
        self.overhead_us = 0.0
        if plain_ms is not None and plain_ms < self.total_ms:
            self.overhead_us = (self.total_ms - plain_ms) * 1e3 / n
        for r, a in zip(self.records, acc):
            r["us_raw"] = a / reps * 1e3
            r["us"] = max(r["us_raw"] - self.overhead_us, 0.0)
        return [r for r in self.records if r["type"] == 0]

    def close(self):
        h = hip()
        for e in self.events:
            h.hipEventDestroy(e)
        self.events = []


def by_symbol(records):
    """{kernel symbol: {launches, time_us, flops}} over kernel records, by total time."""
    agg = collections.OrderedDict()
    for r in records:
        a = agg.setdefault(r["kernel"], {"launches": 0, "time_us": 0.0, "time_raw_us": 0.0, "flops": 0.0,
                                         "flops_known": True, "bytes": 0.0})
        a["launches"] += 1
        a["time_us"] += r["us"]
        a["time_raw_us"] += r.get("us_raw", r["us"])
        if r["flops"] is None:
            a["flops_known"] = False
        else:
            a["flops"] += r["flops"]
            a["bytes"] += r.get("bytes") or 0.0
    return collections.OrderedDict(sorted(agg.items(), key=lambda kv: -kv[1]["time_us"]))

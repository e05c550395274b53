"""ctypes binding of libpose6d.so (the C ABI declared in include/pose6d.h).

The library is the product: there is no CPU or eager-PyTorch fallback.  Loading
fails loudly if the .so is missing, and every op raises if handed a tensor that
is not on a ROCm device.
"""
import ctypes
import os
import re

import torch  # noqa: F401  (loads torch's HIP runtime first; libpose6d binds to the same libamdhip64.so.7)

HERE = os.path.dirname(os.path.abspath(__file__))
# POSE6D_LIB: another build of the same library (A/B timing of two builds on one box)
LIB_PATH = os.environ.get("POSE6D_LIB") or os.path.join(HERE, "lib", "libpose6d.so")
HEADER = os.path.join(os.path.dirname(os.path.dirname(HERE)), "include", "pose6d.h")

DT_F32 = 0
DT_BF16 = 1

_lib = None


class Pose6dError(RuntimeError):
    pass


_CT = {
    "int": ctypes.c_int, "int32_t": ctypes.c_int32, "int64_t": ctypes.c_int64, "float": ctypes.c_float,
    "double": ctypes.c_double, "void": None, "char": ctypes.c_char, "uint64_t": ctypes.c_uint64,
    "uint8_t": ctypes.c_uint8,
}


def _parse_header(path):
    """Parse `int pose6d_xxx(args);` prototypes -> {name: [ctypes argtypes]}."""
    src = open(path).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    protos = {}
    for m in re.finditer(r"\b(int64_t|int|const char\s*\*)\s*(pose6d_\w+)\s*\(([^)]*)\)\s*;", src):
        name, args = m.group(2), m.group(3).strip()
        types = []
        if args and args != "void":
            for a in args.split(","):
                a = a.strip()
                if "*" in a:
                    types.append(ctypes.c_void_p)
                else:
                    base = a.replace("const", "").split()[0]
                    types.append(_CT[base])
        protos[name] = (types, m.group(1))
    return protos


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise Pose6dError(f"libpose6d.so not built ({LIB_PATH}); run `python -c 'import __graft_entry__ as g; g.build()'`"
                          " or `make -C 6d-pose-estimation_amd/csrc`")
    lib = ctypes.CDLL(LIB_PATH)
    protos = _parse_header(HEADER) if os.path.exists(HEADER) else {}
    missing = []
    for name, (argtypes, ret) in protos.items():
        if not hasattr(lib, name):   # a header newer than the build: fails when called
            missing.append(name)
            continue
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = {"int": ctypes.c_int, "int64_t": ctypes.c_int64}.get(ret, ctypes.c_char_p)
    lib._protos = protos
    lib._missing = missing
    _lib = lib
    return lib


class Tuning(ctypes.Structure):
    """pose6d_tuning_t (include/pose6d.h): explicit plan overrides for the conv
    entry points' *_tuned forms (tests / tuning tools only; -1 = default)."""
    _fields_ = [(n, ctypes.c_int32) for n in ("conv_tile", "conv_stages", "conv_s2", "conv_base", "wgrad_stages",
                                               "wgrad_base", "bwd_separate", "conv_splitk", "wgrad_splits",
                                               "bwd_order", "conv_patch")]

    def __init__(self, **kw):
        super().__init__(*([-1] * len(self._fields_)))
        for k, v in kw.items():
            setattr(self, k, int(v))

    @property
    def ref(self):
        # byref, not addressof: the argument object keeps the struct alive for the call,
        # so `Tuning(...).ref` passed inline does not hand the library freed memory
        return ctypes.byref(self)


def symbols():
    load()
    return sorted(_lib._protos)


def query(name, *args):
    """Call a size-query entry point (returns its value, no error code)."""
    return getattr(load(), "pose6d_" + name)(*args)


def call(name, *args):
    """Call pose6d_<name>; tensors are passed as data pointers; raise on error."""
    lib = load()
    if "pose6d_" + name in lib._missing:
        raise Pose6dError(f"pose6d_{name} is declared in include/pose6d.h but missing from {LIB_PATH} "
                          "(stale build: rebuild the library)")
    fn = getattr(lib, "pose6d_" + name)
    conv = []
    for a in args:
        if isinstance(a, torch.Tensor):
            conv.append(ctypes.c_void_p(a.data_ptr()))
        elif a is None:
            conv.append(None)
        else:
            conv.append(a)
    rc = fn(*conv)
    if rc != 0:
        raise Pose6dError(f"pose6d_{name} failed ({rc}): {lib.pose6d_last_error().decode()}")
    for ob in observers:   # profiling only (pose6d.steptime maps graph nodes back to calls)
        ob(name, args)


observers = []


def stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def require_device(*tensors):
    for t in tensors:
        if t is not None and isinstance(t, torch.Tensor) and not t.is_cuda:
            raise Pose6dError("pose6d ops run only on a ROCm device (MI355X); got a CPU tensor. "
                              "There is no CPU fallback by design.")

"""CPU oracle for the *_to_all reductions -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker (never as the thing measured or shipped).

Wraps oracle/liboracle.so (our C restatement, reduce_oracle.c) and, when it
was built, oracle/_ref/libref_ops.so (the reference's own operator functions
from src/reduce/reduce-op.c:79-158). See reduce_oracle.c for what is pinned.
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

OPS = ["sum", "prod", "and", "or", "xor", "min", "max"]
DTYPES = ["short", "int", "long", "longlong", "float", "double", "longdouble", "complexf", "complexd"]
NP = {
    "short": np.int16, "int": np.int32, "long": np.int64, "longlong": np.int64,
    "float": np.float32, "double": np.float64, "longdouble": np.longdouble,
    "complexf": np.complex64, "complexd": np.complex128,
}
# reference src/reduce/reduce-op.c:405-448
MATRIX = {
    "sum": DTYPES, "prod": DTYPES,
    "and": ["short", "int", "long", "longlong"],
    "or": ["short", "int", "long", "longlong"],
    "xor": ["short", "int", "long", "longlong"],
    "max": ["short", "int", "long", "longlong", "float", "double", "longdouble"],
    "min": ["short", "int", "long", "longlong", "float", "double", "longdouble"],
}
PAIRS = [(op, t) for op in ["sum", "prod", "and", "or", "xor", "max", "min"] for t in MATRIX[op]]
assert len(PAIRS) == 44

_lib = None
_ref = None


def _load():
    global _lib
    if _lib is None:
        path = os.path.join(HERE, "liboracle.so")
        if not os.path.exists(path):
            raise RuntimeError(f"{path} missing: run `make -C oracle`")
        lib = ctypes.CDLL(path)
        lib.oracle_fold.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
        lib.oracle_fold.restype = ctypes.c_int
        lib.oracle_reduce_pe.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_size_t]
        lib.oracle_reduce_pe.restype = ctypes.c_int
        lib.oracle_cpu_baseline_double_sum.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        lib.oracle_cpu_baseline_double_sum.restype = ctypes.c_double
        lib.oracle_cpu_baseline.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_size_t, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        lib.oracle_cpu_baseline.restype = ctypes.c_double
        _lib = lib
    return _lib


def ref_available():
    return os.path.exists(os.path.join(HERE, "_ref", "libref_ops.so"))


def _load_ref():
    global _ref
    if _ref is None:
        _ref = ctypes.CDLL(os.path.join(HERE, "_ref", "libref_ops.so"))
    return _ref


def reduce_pe(op, dtype, srcs, me):
    """Result the reference computes on active-set member `me` (srcs in active-set order)."""
    lib = _load()
    n = len(srcs[0])
    srcs = [np.ascontiguousarray(s, dtype=NP[dtype]) for s in srcs]
    out = np.empty(n, dtype=NP[dtype])
    arr = (ctypes.c_void_p * len(srcs))(*[s.ctypes.data for s in srcs])
    rc = lib.oracle_reduce_pe(OPS.index(op), DTYPES.index(dtype), len(srcs), me, arr, out.ctypes.data, n)
    if rc != 0:
        raise ValueError(f"oracle: undefined reduction {op}/{dtype}")
    return out


def reduce_all(op, dtype, srcs):
    return [reduce_pe(op, dtype, srcs, me) for me in range(len(srcs))]


def ref_reduce_pe(op, dtype, srcs, me):
    """Same as reduce_pe but every element operation is the REFERENCE's compiled
    operator function (oracle/_ref); the fold order is restated from
    reduce-op.c:226-264 (own source first, then ascending, skipping self)."""
    ref = _load_ref()
    fn = getattr(ref, f"ref_{op}_{dtype}")
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long]
    fn.restype = None
    srcs = [np.ascontiguousarray(s, dtype=NP[dtype]) for s in srcs]
    acc = srcs[me].copy()
    for i, s in enumerate(srcs):
        if i != me:
            fn(acc.ctypes.data, s.ctypes.data, len(acc))
    return acc


def cpu_baseline_double_sum(npes, n, warm=1, reps=3):
    """Median seconds per call of the reference algorithm (restated) on npes
    host processes with a shared-memory transport, max over PEs."""
    return _load().oracle_cpu_baseline_double_sum(npes, n, warm, reps)


def cpu_baseline(op, dtype, npes, n, warm=1, reps=3, pin=True):
    """The reference algorithm (reduce-op.c:226-266, restated in C) as npes
    forked host processes, each pinned to a CPU of its own from this process's
    affinity mask (skipping its first two CPUs when there are spare ones):
    (median seconds per call, max over PEs; CPUs used).
    op/dtype: sum on int (config 1) or double."""
    cpus = (ctypes.c_int * npes)()
    t = _load().oracle_cpu_baseline(OPS.index(op), DTYPES.index(dtype), npes, n, warm, reps, 1 if pin else 0, cpus)
    if t < 0:
        raise RuntimeError("oracle_cpu_baseline failed")
    return t, list(cpus)


def value_bytes(dtype):
    """Bytes of an element that carry its value (x87 long double: 10 of 16)."""
    return 10 if dtype == "longdouble" else np.dtype(NP[dtype]).itemsize


def as_value_bytes(a, dtype):
    """uint8 view [n, value_bytes] for bit comparisons (drops long double padding)."""
    a = np.ascontiguousarray(a, dtype=NP[dtype])
    b = a.view(np.uint8).reshape(len(a), a.itemsize)
    return b[:, :value_bytes(dtype)]


# ---------------------------------------------------------------------------
# data-movement collectives: restated semantics
# ---------------------------------------------------------------------------
def broadcast(srcs, root, targets_before):
    """reference src/broadcast/broadcast-linear.c:61-82: every member but the
    root gets the root's source; the root's target keeps its old contents."""
    return [t.copy() if i == root else srcs[root].copy() for i, t in enumerate(targets_before)]


def fcollect(srcs):
    """reference src/fcollect/fcollect-linear.c:60-93: member i's block lands
    at offset i * nelems, in active-set order, on every member."""
    out = np.concatenate(srcs) if srcs else np.zeros(0)
    return [out.copy() for _ in srcs]


def collect(srcs):
    """reference src/collect/collect-linear.c:60-156: like fcollect with
    per-member lengths; offsets are the running sum in active-set order."""
    return fcollect(srcs)

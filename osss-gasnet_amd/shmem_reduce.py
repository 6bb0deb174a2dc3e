"""ctypes binding of libshmem_reduce.so for tests and bench.py.

The product is the C library (include/shmem.h, shmemx.h, mi355_reduce.h);
this module only loads it and marshals numpy arrays and pointers, the way an
OpenSHMEM test program in C would call it. It never computes a reduction
itself: if the library is missing, loading fails loudly.
"""
import ctypes
import hashlib
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SHMEM_REDUCE_LIBDIR: a variant build of the same library (e.g. lib/probe,
# csrc/Makefile `probe`) for measurement tools; default: the in-tree lib/
LIB_DIR = os.environ.get("SHMEM_REDUCE_LIBDIR") or os.path.join(HERE, "lib")
LIB_PATH = os.path.join(LIB_DIR, "libshmem_reduce.so")

OPS = ["sum", "prod", "and", "or", "xor", "min", "max"]           # enum mi355_op
DTYPES = ["short", "int", "long", "longlong", "float", "double",   # enum mi355_dtype
          "longdouble", "complexf", "complexd"]
NP = {
    "short": np.int16, "int": np.int32, "long": np.int64, "longlong": np.int64,
    "float": np.float32, "double": np.float64, "longdouble": np.longdouble,
    "complexf": np.complex64, "complexd": np.complex128,
}
# torch dtype name -> the shmem type whose C type has its layout (LP64: long = long long = int64)
TORCH_DTYPES = {"int16": "short", "int32": "int", "int64": "long", "float32": "float", "float64": "double",
                "complex64": "complexf", "complex128": "complexd"}
ALGORITHMS = {"auto": 0, "p2p": 1, "exact": 2, "rccl": 3}          # enum shmemx_reduce_algorithm
ORDERS = {"reference": 0, "pe_start": 1}                            # enum shmemx_reduce_order
SHMEM_REDUCE_SYNC_SIZE = 128
SHMEM_REDUCE_MIN_WRKDATA_SIZE = 64
SHMEM_SYNC_VALUE = -1

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_i = ctypes.c_int


class CallInfo(ctypes.Structure):
    """shmemx_call_info (include/shmemx.h): what the last *_to_all call ran"""
    _fields_ = [("schedule", ctypes.c_char * 64), ("kernel", ctypes.c_char * 256), ("ordered", _i),
                ("sources", _i), ("outputs", _i), ("peer_sources", _i), ("launches", _i),
                ("bytes_per_buffer", ctypes.c_ulonglong), ("alg_bytes", ctypes.c_ulonglong),
                ("peer_bytes", ctypes.c_ulonglong)]


def load(path=LIB_PATH):
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    sig = {
        "shmem_init": ([], None), "shmem_finalize": ([], None),
        "shmem_my_pe": ([], _i), "shmem_n_pes": ([], _i),
        "shmem_malloc": ([_sz], _vp), "shmem_free": ([_vp], None),
        "shmem_barrier_all": ([], None),
        "shmem_barrier": ([_i, _i, _i, _vp], None),
        "shmem_global_exit": ([_i], None),
        "shmemx_barrier_on_stream": ([_i, _i, _i, _vp], None),
        "shmemx_malloc_device": ([_sz], _vp), "shmemx_free_device": ([_vp], None),
        "shmemx_is_device_symmetric": ([_vp], _i), "shmemx_peer_device_ptr": ([_vp, _i], _vp),
        "shmemx_set_reduce_algorithm": ([_i], _i), "shmemx_get_reduce_algorithm": ([], _i),
        "shmemx_set_reduce_order": ([_i], _i), "shmemx_get_reduce_order": ([], _i),
        "shmemx_set_persistent": ([_i], _i),
        "shmemx_persistent_stats": ([ctypes.POINTER(ctypes.c_long)] * 2, None),
        "shmemx_external_map_stats": ([ctypes.POINTER(ctypes.c_long)] * 3, None),
        "shmemx_external_map_flush": ([], None),
        "shmemx_device_id": ([], _i), "shmemx_device_synchronize": ([], None),
        "shmemx_threshold_calibration": ([ctypes.POINTER(ctypes.c_double), _i], _i),
        "shmemx_peer_link": ([_i, ctypes.POINTER(_i), ctypes.POINTER(_i)], _i),
        "shmemx_memcpy": ([_vp, _vp, _sz], None), "shmemx_wtime": ([], ctypes.c_double),
        "shmemx_kernel_timing": ([_i], None),
        "shmemx_rccl_init": ([ctypes.c_double], _i),
        "shmemx_last_call_info": ([ctypes.POINTER(CallInfo)], _i),
        "shmemx_coherence_selftest": ([ctypes.POINTER(_i)] * 3, None),
        "shmemx_coherence_sysload": ([ctypes.POINTER(_i)] * 2, None),
        "shmemx_kernel_timing_stats": ([ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_double)], None),
        "shmemx_kernel_timing_phase_stats": ([_i, ctypes.POINTER(ctypes.c_long), ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_double)], None),
        "mi355_dtype_size": ([_i], _sz), "mi355_op_supported": ([_i, _i], _i),
        "mi355_combine": ([_i, _i, _vp, ctypes.POINTER(_vp), _i, _sz, _vp], _i),
        "mi355_combine_orders": ([_i, _i, ctypes.POINTER(_vp), ctypes.POINTER(_vp), _i, _sz, _vp], _i),
        "mi355_copy_segments": ([ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_sz), _i, _vp], _i),
        "mi355_shard_bounds": ([_sz, _sz, _i, _i, ctypes.POINTER(_sz), ctypes.POINTER(_sz)], None),
    }
    for name, (args, res) in sig.items():
        f = getattr(lib, name)
        f.argtypes = args
        f.restype = res
    return lib


class Shmem:
    """One PE's view of the library (call init() once per process)."""

    def __init__(self, path=LIB_PATH):
        self.lib = load(path)
        self._psync = np.full(SHMEM_REDUCE_SYNC_SIZE, SHMEM_SYNC_VALUE, dtype=np.int64)
        self._psync_ptr = self._psync.ctypes.data
        self._fns = {}

    def _reduction(self, op, dtype):
        f = self._fns.get((op, dtype))
        if f is None:
            f = getattr(self.lib, f"shmem_{dtype}_{op}_to_all")
            f.restype = None
            f.argtypes = [_vp, _vp, _i, _i, _i, _i, _vp, _vp]
            self._fns[(op, dtype)] = f
        return f

    # ---- runtime
    def init(self):
        self.lib.shmem_init()

    def finalize(self):
        self.lib.shmem_finalize()

    def my_pe(self):
        return self.lib.shmem_my_pe()

    def n_pes(self):
        return self.lib.shmem_n_pes()

    def barrier_all(self):
        self.lib.shmem_barrier_all()

    def malloc_device(self, nbytes):
        return self.lib.shmemx_malloc_device(nbytes)

    def free_device(self, ptr):
        self.lib.shmemx_free_device(ptr)

    def threshold_calibration(self):
        """None, or the init-time threshold calibration (shmemx_threshold_calibration):
        {"fused": [(bytes, fused_us, multi_launch_us)...], "oneshot": [(bytes, oneshot_us, twoshot_us)...]}"""
        us = (ctypes.c_double * 22)()
        if not self.lib.shmemx_threshold_calibration(us, 22):
            return None
        fs = [64 << 10, 256 << 10, 512 << 10, 1 << 20, 2 << 20, 4 << 20]
        os_ = [16 << 10, 32 << 10, 64 << 10, 128 << 10, 256 << 10]
        return {"fused": [(b, us[i], us[6 + i]) for i, b in enumerate(fs)],
                "oneshot": [(b, us[12 + i], us[17 + i]) for i, b in enumerate(os_)]}

    def peer_device_ptr(self, ptr, pe):
        """PE pe's copy of a device-heap object, addressable by kernels on
        this PE's GPU (shmemx_peer_device_ptr); None if not mapped."""
        return self.lib.shmemx_peer_device_ptr(ptr, pe)

    def malloc(self, nbytes):
        return self.lib.shmem_malloc(nbytes)

    def free(self, ptr):
        self.lib.shmem_free(ptr)

    def set_algorithm(self, name):
        return self.lib.shmemx_set_reduce_algorithm(ALGORITHMS[name])

    def set_order(self, name):
        """"reference": every PE gets the reference's result for itself; "pe_start": PE_start's everywhere"""
        return self.lib.shmemx_set_reduce_order(ORDERS[name])

    def set_fused_max(self, nbytes):
        """fused-kernel threshold in bytes per PE (collective setting, shmemx.h); returns the previous"""
        f = self.lib.shmemx_set_fused_max_bytes
        f.argtypes, f.restype = [ctypes.c_size_t], ctypes.c_size_t
        return int(f(nbytes))

    def thresholds(self):
        """(fused_max, oneshot_max) in bytes per PE (shmemx.h)"""
        for name in ("shmemx_get_fused_max_bytes", "shmemx_get_oneshot_max_bytes"):
            getattr(self.lib, name).restype = ctypes.c_size_t
        return int(self.lib.shmemx_get_fused_max_bytes()), int(self.lib.shmemx_get_oneshot_max_bytes())

    def set_oneshot_max(self, nbytes):
        """one-shot threshold in bytes per PE (collective setting, shmemx.h); returns the previous"""
        f = self.lib.shmemx_set_oneshot_max_bytes
        f.argtypes, f.restype = [ctypes.c_size_t], ctypes.c_size_t
        return int(f(nbytes))

    def set_persistent(self, enable):
        """opt-in persistent fused server (shmemx.h); returns the previous setting"""
        return bool(self.lib.shmemx_set_persistent(1 if enable else 0))

    def persistent_stats(self):
        """(calls served by a resident server, servers launched) since init"""
        a, b = ctypes.c_long(), ctypes.c_long()
        self.lib.shmemx_persistent_stats(ctypes.byref(a), ctypes.byref(b))
        return a.value, b.value

    def external_map_fallbacks(self):
        """calls staged because a member could not open a peer's buffer (shmemx.h)"""
        self.lib.shmemx_external_map_fallbacks.restype = ctypes.c_long
        return int(self.lib.shmemx_external_map_fallbacks())

    def external_map_stats(self):
        """(peers' allocations mapped now, opened, closed since init): device
        buffers outside the heap that calls mapped (shmemx.h)"""
        a, b, c = ctypes.c_long(), ctypes.c_long(), ctypes.c_long()
        self.lib.shmemx_external_map_stats(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return a.value, b.value, c.value

    def sync(self):
        self.lib.shmemx_device_synchronize()

    # ---- data movement (hipMemcpy, blocking)
    def put(self, dptr, arr):
        arr = np.ascontiguousarray(arr)
        self.lib.shmemx_memcpy(dptr, arr.ctypes.data, arr.nbytes)

    def get(self, dptr, n, dtype):
        out = np.empty(n, dtype=NP[dtype] if isinstance(dtype, str) else dtype)
        self.lib.shmemx_memcpy(out.ctypes.data, dptr, out.nbytes)
        return out

    # ---- the reduction entry points (include/shmem.h)
    def to_all(self, op, dtype, target, source, nreduce, PE_start=0, logPE_stride=0, PE_size=None,
               pWrk=None, pSync=None):
        if PE_size is None:
            PE_size = self.n_pes()
        if pSync is None:
            pSync = self._psync_ptr
        self._reduction(op, dtype)(target, source, nreduce, PE_start, logPE_stride, PE_size, pWrk, pSync)

    def to_all_tensors(self, op, target, source, PE_start=0, logPE_stride=0, PE_size=None):
        """shmem_<T>_<op>_to_all on two contiguous device tensors of one dtype
        (T from the tensor's dtype; long double has no torch dtype). They need
        not come from the symmetric heap: at PE_size > 1 the members map each
        other's allocations for the call (shmemx.h, extmap.c). Blocking, like
        the C call: on return `target` holds this PE's result."""
        if target.dtype != source.dtype or target.numel() != source.numel():
            raise ValueError("target and source must have the same dtype and number of elements")
        if not (target.is_contiguous() and source.is_contiguous()) or target.device.type != "cuda" \
                or source.device.type != "cuda":
            raise ValueError("target and source must be contiguous GPU tensors")
        dtype = TORCH_DTYPES.get(str(source.dtype).replace("torch.", ""))
        if dtype is None:
            raise TypeError(f"no shmem_*_to_all for {source.dtype}")
        self.to_all(op, dtype, target.data_ptr(), source.data_ptr(), source.numel(), PE_start, logPE_stride, PE_size)

    def heap_tensor(self, n, dtype):
        """A 1-D torch tensor of n elements of torch dtype `dtype` in the
        device symmetric heap (collective, like shmemx_malloc_device): the
        buffer the stream-ordered, graph-capturable reductions take. The tensor
        does not own the memory: free it with free_device(t.data_ptr()) once
        no tensor or queued work uses it."""
        import torch
        name = TORCH_DTYPES.get(str(dtype).replace("torch.", ""))
        if name is None:
            raise TypeError(f"no shmem_*_to_all for {dtype}")
        np_dt = np.dtype(NP[name])
        ptr = self.malloc_device(max(1, n) * np_dt.itemsize)
        if not ptr:
            raise MemoryError("device symmetric heap exhausted")

        class _HeapBuffer:
            __cuda_array_interface__ = {"shape": (n,), "typestr": np_dt.str, "data": (ptr, False), "version": 3,
                                        "strides": None}

        t = torch.as_tensor(_HeapBuffer(), device=f"cuda:{self.lib.shmemx_device_id()}")
        if t.data_ptr() != ptr:
            raise RuntimeError("torch copied the heap buffer instead of wrapping it")
        return t

    def _stream_reduction(self, op, dtype):
        key = ("stream", op, dtype)
        f = self._fns.get(key)
        if f is None:
            f = getattr(self.lib, f"shmemx_{dtype}_{op}_to_all_on_stream")
            f.restype = None
            f.argtypes = [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp]
            self._fns[key] = f
        return f

    # ---- stream-ordered variants (include/shmemx.h)
    def to_all_on_stream(self, op, dtype, target, source, nreduce, PE_start, logPE_stride, PE_size, stream):
        self._stream_reduction(op, dtype)(target, source, nreduce, PE_start, logPE_stride, PE_size, None,
                                          self._psync_ptr, stream)

    def barrier_on_stream(self, PE_start, logPE_stride, PE_size, stream):
        self.lib.shmemx_barrier_on_stream(PE_start, logPE_stride, PE_size, stream)

    # ---- HIP streams and graphs, for callers of the stream-ordered API
    #      (resolved through the library's own libamdhip64 dependency)
    def _hip(self, name, *args):
        rc = getattr(self.lib, name)(*args)
        if rc != 0:
            raise RuntimeError(f"{name} failed: {rc}")

    def stream_create(self):
        s = _vp()
        self._hip("hipStreamCreate", ctypes.byref(s))
        return s.value

    def stream_sync(self, stream):
        self._hip("hipStreamSynchronize", _vp(stream))

    def stream_destroy(self, stream):
        self._hip("hipStreamDestroy", _vp(stream))

    def capture_begin(self, stream, mode=2):  # hipStreamCaptureModeRelaxed
        self._hip("hipStreamBeginCapture", _vp(stream), _i(mode))

    def capture_end(self, stream):
        g, e = _vp(), _vp()
        self._hip("hipStreamEndCapture", _vp(stream), ctypes.byref(g))
        self._hip("hipGraphInstantiate", ctypes.byref(e), g, None, None, _sz(0))
        return g.value, e.value

    def graph_launch(self, exe, stream):
        self._hip("hipGraphLaunch", _vp(exe), _vp(stream))

    def graph_destroy(self, graph, exe):
        self._hip("hipGraphExecDestroy", _vp(exe))
        self._hip("hipGraphDestroy", _vp(graph))

    # ---- the combine layer (include/mi355_reduce.h)
    def combine(self, op, dtype, dst, srcs, n, stream=None):
        arr = (_vp * len(srcs))(*srcs)
        return self.lib.mi355_combine(OPS.index(op), DTYPES.index(dtype), dst, arr, len(srcs), n, stream)

    def combine_orders(self, op, dtype, dsts, srcs, n, stream=None):
        """dsts[q] (or None) <- the fold in member q's reference order (mi355_combine_orders)"""
        d = (_vp * len(dsts))(*[x if x else None for x in dsts])
        s = (_vp * len(srcs))(*srcs)
        return self.lib.mi355_combine_orders(OPS.index(op), DTYPES.index(dtype), d, s, len(srcs), n, stream)

    def last_call_info(self):
        """dict of shmemx_last_call_info, or None before the first call"""
        ci = CallInfo()
        if self.lib.shmemx_last_call_info(ctypes.byref(ci)) != 0:
            return None
        d = {f: getattr(ci, f) for f, _ in CallInfo._fields_}
        d["schedule"] = ci.schedule.decode()
        d["kernel"] = ci.kernel.decode()
        return d

    def coherence_selftest(self):
        """(ran, passed, stale_without_acquire) of the init-time peer-read coherence test"""
        a, b, c = _i(), _i(), _i()
        self.lib.shmemx_coherence_selftest(ctypes.byref(a), ctypes.byref(b), ctypes.byref(c))
        return bool(a.value), bool(b.value), bool(c.value)

    def coherence_sysload(self):
        """(sysload_fresh, acquires_skipped): the coherence test's check of the
        fused kernel's system-coherent loads, and whether its acquires are off"""
        a, b = _i(), _i()
        self.lib.shmemx_coherence_sysload(ctypes.byref(a), ctypes.byref(b))
        return bool(a.value), bool(b.value)

    PRODUCER_FIELDS = ("fused_plain_no_acquire", "fused_sysload", "fused_after_acquire",
                       "host_plain_no_acquire", "host_sysload", "host_after_acquire")

    def coherence_producer(self):
        """(ran, {field: fresh}) of the init test of a caller's producer path
        (plain stores in a null-stream kernel, then the fused kernel's or the
        multi-launch schedules' ordering; shmemx.h shmemx_coherence_producer)"""
        ran, fresh = _i(), (ctypes.c_int * 6)()
        self.lib.shmemx_coherence_producer(ctypes.byref(ran), fresh)
        return bool(ran.value), {k: bool(fresh[i]) for i, k in enumerate(self.PRODUCER_FIELDS)}

    def device_wait_report(self):
        """(slow, us): the init timing of device barriers over the job (shmemx.h
        shmemx_device_wait_report); slow = host barriers and no fused kernel"""
        slow, us = _i(), ctypes.c_double()
        self.lib.shmemx_device_wait_report(ctypes.byref(slow), ctypes.byref(us))
        return bool(slow.value), us.value

    def kernel_timing(self, enable):
        self.lib.shmemx_kernel_timing(1 if enable else 0)

    def kernel_timing_stats(self):
        n, tot, avg = ctypes.c_long(), ctypes.c_double(), ctypes.c_double()
        self.lib.shmemx_kernel_timing_stats(ctypes.byref(n), ctypes.byref(tot), ctypes.byref(avg))
        return n.value, tot.value, avg.value

    def kernel_timing_phase_stats(self, phase):
        """phase 0: each call's dominant kernel; 1: the P2P all-gather copy"""
        n, tot, avg = ctypes.c_long(), ctypes.c_double(), ctypes.c_double()
        self.lib.shmemx_kernel_timing_phase_stats(phase, ctypes.byref(n), ctypes.byref(tot), ctypes.byref(avg))
        return n.value, tot.value, avg.value


BENCH_LIB_PATH = os.path.join(LIB_DIR, "libshmem_bench.so")


def bench_loop(path=BENCH_LIB_PATH, name="double_sum"):
    """bench.py's timed loop in C (csrc/bench_loop.c): K back-to-back
    shmem_<name>_to_all calls (double_sum, float_max, longlong_and). Load
    after the main library."""
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    f = getattr(ctypes.CDLL(path), f"shmemb_{name}_loop")
    f.argtypes = [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i]
    f.restype = None
    return f


def bench_rotating(path=BENCH_LIB_PATH):
    """csrc/bench_loop.c shmemb_double_sum_rotating: K calls over npairs
    disjoint (target, source) pairs taken in turn; returns
    f(targets, sources, nreduce, pe_start, log_stride, pe_size, psync, k)."""
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    f = ctypes.CDLL(path).shmemb_double_sum_rotating
    f.argtypes = [_vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _i]
    f.restype = None

    def run(targets, sources, nreduce, pe_start, log_stride, pe_size, psync, k):
        t = (_vp * len(targets))(*targets)
        s = (_vp * len(sources))(*sources)
        f(t, s, len(targets), nreduce, pe_start, log_stride, pe_size, None, psync, k)
    return run


def bench_call_times(path=BENCH_LIB_PATH):
    """csrc/bench_loop.c shmemb_double_sum_times: K shmem_double_sum_to_all
    calls, each timed alone; returns f(target, source, nreduce, PE_start,
    logPE_stride, PE_size, k) -> numpy array of k durations in us"""
    import numpy as np
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
    f = ctypes.CDLL(path).shmemb_double_sum_times
    f.argtypes = [_vp, _vp, _i, _i, _i, _i, _vp, _vp, _i, _vp]
    f.restype = None

    def run(target, source, nreduce, pe_start, log_stride, pe_size, psync, k):
        out = np.zeros(k)
        f(target, source, nreduce, pe_start, log_stride, pe_size, None, psync, k, out.ctypes.data)
        return out
    return run


def kernel_code_hash(path=LIB_PATH):
    """sha256 (16 hex digits) of the gfx950 code objects the library carries
    (its .hip_fatbin ELF section): the machine code PMC counter profiles
    describe. Host-only changes leave it unchanged; any change to a kernel,
    a kernel header or the device compile flags changes it (the build is
    deterministic: rebuilding the same sources gives the same bytes).
    profiles/pmc_traffic.json records it per entry and bench.py reports an
    entry's HBM traffic only for a library with the same hash."""
    import struct
    with open(path, "rb") as f:
        b = f.read()
    shoff = struct.unpack_from("<Q", b, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    secs = [struct.unpack_from("<IIQQQQ", b, shoff + i * shentsize) for i in range(shnum)]
    stroff = secs[shstrndx][4]
    for name, _typ, _flags, _addr, off, size in secs:
        if b[stroff + name:b.index(b"\0", stroff + name)] == b".hip_fatbin":
            return hashlib.sha256(b[off:off + size]).hexdigest()[:16]
    raise RuntimeError(f"{path} has no .hip_fatbin section")


def shard_bounds(lib, n, elem_size, nshards, i):
    lo, hi = _sz(), _sz()
    lib.mi355_shard_bounds(n, elem_size, nshards, i, ctypes.byref(lo), ctypes.byref(hi))
    return lo.value, hi.value

"""GPU: the public shmem_<T>_<op>_to_all entry points on a 1-PE active set,
in-process (this pytest process is PE 0 of 1).

With one PE the reference computes target = source (reduce-op.c:226-229, with
the temporary target of :197-215 when they overlap); these tests cover every
buffer kind the entry point classifies: host (shmem_malloc), device symmetric,
device non-symmetric (plain hipMalloc), overlapping and unaligned.
"""
import ctypes

import numpy as np
import pytest

import gen_golden
import oracle
import shmem_reduce

pytestmark = pytest.mark.gpu


def same_bits(a, b, dtype):
    return (oracle.as_value_bytes(a, dtype) == oracle.as_value_bytes(b, dtype)).all()


@pytest.mark.parametrize("op,dtype", oracle.PAIRS)
def test_identity_host_and_device(shm, op, dtype):
    n = 1000
    es = np.dtype(oracle.NP[dtype]).itemsize
    x = gen_golden.values(np.random.default_rng(1), op, dtype, n)
    # host symmetric buffers (shmem_malloc): staged through the GPU
    hs, ht = shm.malloc(n * es), shm.malloc(n * es)
    ctypes.memmove(hs, x.ctypes.data, n * es)
    shm.to_all(op, dtype, ht, hs, n, 0, 0, 1)
    got = np.empty(n, dtype=oracle.NP[dtype])
    ctypes.memmove(got.ctypes.data, ht, n * es)
    assert same_bits(got, x, dtype)
    shm.free(ht)
    shm.free(hs)
    # device symmetric buffers
    ds, dt = shm.malloc_device(n * es), shm.malloc_device(n * es)
    shm.put(ds, x)
    shm.to_all(op, dtype, dt, ds, n, 0, 0, 1)
    assert same_bits(shm.get(dt, n, dtype), x, dtype)
    shm.free_device(dt)
    shm.free_device(ds)


@pytest.mark.parametrize("delta", [0, 3, -3, 200, -200])
def test_overlapping_target_is_memmove(shm, delta):
    """target = source + delta elements; the result must be the ORIGINAL source
    (the reference copies through a temporary when the ranges overlap)."""
    n = 5000
    x = np.arange(n, dtype=np.float64) * 1.5
    base = shm.malloc_device((n + 512) * 8)
    src = base + 256 * 8
    tgt = src + delta * 8
    shm.put(src, x)
    shm.to_all("sum", "double", tgt, src, n, 0, 0, 1)
    assert (shm.get(tgt, n, "double") == x).all()
    shm.free_device(base)


def test_overlap_larger_than_scratch(shm):
    """Overlap handling is chunked through scratch (3 MiB here) in memmove order."""
    n = 3 << 20  # 24 MiB of doubles
    x = np.arange(n, dtype=np.float64)
    base = shm.malloc_device((n + 2048) * 8)
    for delta in (777, -777):
        src = base + 1024 * 8
        shm.put(src, x)
        tgt = src + delta * 8
        shm.to_all("sum", "double", tgt, src, n, 0, 0, 1)
        assert (shm.get(tgt, n, "double") == x).all(), delta
    shm.free_device(base)


def test_non_symmetric_device_memory(shm):
    hip = ctypes.CDLL("libamdhip64.so")
    n = 12345
    x = np.random.default_rng(3).integers(-1000, 1000, n).astype(np.int32)
    ps, pt = ctypes.c_void_p(), ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(ps), ctypes.c_size_t(n * 4)) == 0
    assert hip.hipMalloc(ctypes.byref(pt), ctypes.c_size_t(n * 4)) == 0
    shm.put(ps.value, x)
    assert not shm.lib.shmemx_is_device_symmetric(ps.value)
    shm.to_all("xor", "int", pt.value, ps.value, n, 0, 0, 1)
    assert (shm.get(pt.value, n, "int") == x).all()
    hip.hipFree(ps)
    hip.hipFree(pt)


def test_zero_elements_is_a_no_op(shm):
    d = shm.malloc_device(64)
    shm.put(d, np.full(8, 7.0))
    shm.to_all("sum", "double", d + 0, d + 0, 0, 0, 0, 1)
    assert (shm.get(d, 8, "double") == 7.0).all()
    shm.free_device(d)


def test_static_host_array_source(shm):
    """Sources need not come from shmem_malloc (the reference allows global arrays)."""
    x = np.linspace(-1, 1, 777)
    t = np.zeros_like(x)
    shm.to_all("max", "double", t.ctypes.data, x.ctypes.data, len(x), 0, 0, 1)
    assert (t == x).all()


def test_kernel_timing_counts_launches(shm):
    n = 1 << 20
    a, b = shm.malloc_device(8 * n), shm.malloc_device(8 * n)
    shm.kernel_timing(True)
    for _ in range(3):
        shm.to_all("sum", "double", b, a, n, 0, 0, 1)
    k, tot, avg = shm.kernel_timing_stats()
    k1, _, _ = shm.kernel_timing_phase_stats(1)   # no all-gather leg on one PE
    shm.kernel_timing(False)
    assert k == 3 and tot > 0 and avg > 0 and k1 == 0
    shm.free_device(b)
    shm.free_device(a)


def test_peer_link_has_no_self_link(shm):
    t, h = ctypes.c_int(-7), ctypes.c_int(-7)
    assert shm.lib.shmemx_peer_link(0, ctypes.byref(t), ctypes.byref(h)) == -1   # PE 0 is this PE
    assert shm.lib.shmemx_peer_link(5, ctypes.byref(t), ctypes.byref(h)) == -1   # no such PE
    assert (t.value, h.value) == (-7, -7)


def test_psync_is_left_at_sync_value(shm):
    psync = np.full(shmem_reduce.SHMEM_REDUCE_SYNC_SIZE, -1, dtype=np.int64)
    x = np.ones(100)
    t = np.zeros(100)
    shm.to_all("sum", "double", t.ctypes.data, x.ctypes.data, 100, 0, 0, 1, pSync=psync.ctypes.data)
    assert (psync == -1).all()


@pytest.mark.parametrize("op,dtype", [("sum", "double"), ("max", "float"), ("min", "int"), ("prod", "long"),
                                      ("sum", "complexd"), ("sum", "complexf"),
                                      ("sum", "short"), ("prod", "short"), ("min", "short")])
def test_rccl_glue_one_rank(shm, op, dtype):
    """The RCCL schedule's glue (csrc/rccl.c: non-blocking communicator
    bring-up with a deadline, type/op mapping, complex sum as 2n reals, short
    widened to int32 and truncated back) on a
    1-rank communicator, where ncclAllReduce is the identity. Multi-rank RCCL
    needs one GPU per rank (RCCL refuses two ranks on one device), so this is
    what the one-GPU box can run."""
    assert shm.lib.shmemx_rccl_init(30.0) == 0
    f = shm.lib.shmemi_rccl_allreduce
    f.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]
    f.restype = ctypes.c_int
    assert shm.lib.shmemi_rccl_supported(shmem_reduce.OPS.index(op), shmem_reduce.DTYPES.index(dtype))
    n = 4099
    es = np.dtype(oracle.NP[dtype]).itemsize
    x = gen_golden.values(np.random.default_rng(9), op, dtype, n)
    ds, dt = shm.malloc_device(n * es), shm.malloc_device(n * es)
    shm.put(ds, x)
    assert f(shmem_reduce.OPS.index(op), shmem_reduce.DTYPES.index(dtype), ds, dt, n) == 0
    assert same_bits(shm.get(dt, n, dtype), x, dtype)
    shm.free_device(dt)
    shm.free_device(ds)


def test_peer_device_ptr(shm):
    """shmemx_peer_device_ptr (round 6): this PE's own copy of a device-heap
    object is its own address; anything outside the device heap, or a PE
    outside the job, gives NULL (the peers' mappings are exercised by
    bench.py's xGMI legs, tests/test_gpu_bench.py)."""
    d = shm.malloc_device(4096)
    try:
        assert shm.peer_device_ptr(d, 0) == d
        assert shm.peer_device_ptr(d + 100, 0) == d + 100
        assert shm.peer_device_ptr(d, 1) is None and shm.peer_device_ptr(d, -1) is None
        h = np.zeros(16)
        assert shm.peer_device_ptr(h.ctypes.data, 0) is None
        hs = shm.malloc(4096)
        assert shm.peer_device_ptr(hs, 0) is None   # the host heap is not the device heap
        shm.free(hs)
    finally:
        shm.free_device(d)

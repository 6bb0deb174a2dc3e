"""CPU: shmem_malloc's symmetric host heap (csrc/hostheap.c) on several PE
processes without a GPU (SHMEM_BOOTSTRAP_ONLY=1).

The reference's heap is one host segment per PE carved by one allocator per
PE (comms-inline.h:766-845, memalloc.c:71-154): the same sequence of
collective shmem_malloc calls gives every block the same offset everywhere,
and a peer's copy of an object is that peer's segment base + the offset. So
shmem_getmem / shmem_putmem (putget.c:249-256) and the broadcast / fcollect
/ collect collectives (broadcast-linear.c:61-82, fcollect-linear.c:60-93,
collect-linear.c:60-156) work on shmem_malloc'd objects. Checked here with
host-memory local sides (plain memory copies; the device-side variants are
tests/test_gpu_coll.py's), against the oracle's restated semantics.
"""
import os
import sys

import textwrap

import numpy as np
import pytest

import test_bootstrap

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PRE = f"""
import numpy as np
sys.path.insert(0, {os.path.join(ROOT, 'oracle')!r})
import oracle
L = shm.lib
vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
for name in ("shmem_putmem", "shmem_getmem"):
    getattr(L, name).argtypes = [vp, vp, sz, i]
for b in (32, 64):
    getattr(L, f"shmem_broadcast{{b}}").argtypes = [vp, vp, sz, i, i, i, i, vp]
    for k in ("fcollect", "collect"):
        getattr(L, f"shmem_{{k}}{{b}}").argtypes = [vp, vp, sz, i, i, i, vp]
def arr(p, n, dt):
    return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(np.ctypeslib.as_ctypes_type(dt))), shape=(n,))
def src(pe, n, dt=np.int64, seed=0):
    return np.random.default_rng(seed * 1009 + pe).integers(-2**31, 2**31, n).astype(dt)
"""


def spawn(npes, body, tmp_path, **kw):
    return test_bootstrap.spawn(npes, PRE + textwrap.dedent(body), tmp_path, **kw)


def test_symmetric_offsets_first_fit(tmp_path):
    """Same call sequence, same offsets on every PE; a freed gap is reused
    first-fit; blocks page-aligned; offsets identical across PEs (checked
    through a remote put at each block's start)."""
    body = """
    base = shm.malloc(4096)
    sizes = [1000 + 17 * k for k in range(10)]
    ptrs = [shm.malloc(s) for s in sizes]
    offs = [p - base for p in ptrs]
    assert all(p % 4096 == 0 for p in ptrs) and offs == sorted(offs) and len(set(offs)) == len(offs), offs
    shm.free(ptrs[3]); shm.free(ptrs[4])
    q = shm.malloc(5000)              # fits the two freed 4 KiB pages: first fit
    assert q == ptrs[3], (q - base, offs[3])
    r = shm.malloc(9000)              # does not fit any gap: after the last block
    assert r - base > offs[-1], (r - base, offs[-1])
    # every PE writes its rank at the start of PE (me+1)'s copy of each block
    shm.barrier_all()
    nxt = (me + 1) % npes
    for p in ptrs[:3] + [q, r] + ptrs[5:]:
        x = np.array([1000 + me], dtype=np.int64)
        L.shmem_putmem(p, x.ctypes.data, 8, nxt)
    shm.barrier_all()
    prv = (me - 1) % npes
    for p in ptrs[:3] + [q, r] + ptrs[5:]:
        assert arr(p, 1, np.int64)[0] == 1000 + prv
    print('OFFS', *offs)
    shm.finalize()
    """
    res = spawn(3, body, tmp_path)
    for rc, out in res:
        assert rc == 0, out
    offs = [ln for rc, out in res for ln in out.splitlines() if ln.startswith("OFFS")]
    assert len(set(offs)) == 1, offs


def test_putmem_getmem_between_pes(tmp_path):
    """Each PE gets every other PE's block and puts its own into every other
    PE's slot array; unaligned sizes and offsets; page-locked or plain local
    buffers."""
    body = """
    n = 12345
    s = shm.malloc(n * 8); t = shm.malloc(npes * n * 8)
    arr(s, n, np.int64)[:] = src(me, n)
    arr(t, npes * n, np.int64)[:] = -1
    shm.barrier_all()
    for q in range(npes):
        mine = src(me, n)                                   # plain numpy memory as the local side
        L.shmem_putmem(t + me * n * 8 + 8, mine.ctypes.data + 8, (n - 3) * 8, q)
    shm.barrier_all()
    got = arr(t, npes * n, np.int64).reshape(npes, n)
    for q in range(npes):
        assert (got[q, 1:n - 2] == src(q, n)[1:n - 2]).all() and got[q, 0] == -1 and (got[q, n - 2:] == -1).all()
    for q in range(npes):
        out = np.zeros(n, dtype=np.int64)
        L.shmem_getmem(out.ctypes.data, s, n * 8, q)
        assert (out == src(q, n)).all(), q
    shm.barrier_all()
    print('ok')
    shm.finalize()
    """
    for rc, out in spawn(4, body, tmp_path):
        assert rc == 0, out


@pytest.mark.parametrize("bits", [32, 64])
def test_collectives_on_host_heap(tmp_path, bits):
    """broadcast (every root, a strided active set), fcollect and collect
    with shmem_malloc'd sources, into host-heap and plain targets, against
    oracle.broadcast / fcollect / collect."""
    body = f"""
    bits = {bits}
    dt = np.int32 if bits == 32 else np.int64
    es = bits // 8
    cap = 4096
    s = shm.malloc(cap * es); t = shm.malloc(8 * cap * es)
    psync = (ctypes.c_long * 128)(*([-1] * 128))
    members = list(range(0, npes, 2))              # PE_start 0, logPE_stride 1
    size = len(members)
    n = 777
    mine = members.index(me) if me in members else None
    # broadcast from every root, target in the host heap
    for root in range(size):
        arr(s, n, dt)[:] = src(me, n, dt, root)
        arr(t, n, dt)[:] = -7
        if mine is not None:
            getattr(L, f"shmem_broadcast{{bits}}")(t, s, n, root, 0, 1, size, psync)
            want = oracle.broadcast([src(q, n, dt, root) for q in members], root, [np.full(n, -7, dt)] * size)
            assert (arr(t, n, dt) == want[mine]).all(), root
        shm.barrier_all()
    # fcollect over every PE, target plain host memory
    arr(s, n, dt)[:] = src(me, n, dt, 50)
    out = np.zeros(npes * n, dtype=dt)
    getattr(L, f"shmem_fcollect{{bits}}")(out.ctypes.data, s, n, 0, 0, npes, psync)
    assert (out == oracle.fcollect([src(q, n, dt, 50) for q in range(npes)])[me]).all()
    shm.barrier_all()
    # collect: per-PE lengths
    k = (me * 37 + 5) % 100
    arr(s, k, dt)[:] = src(me, k, dt, 60)
    getattr(L, f"shmem_collect{{bits}}")(t, s, k, 0, 0, npes, psync)
    want = oracle.collect([src(q, (q * 37 + 5) % 100, dt, 60) for q in range(npes)])[me]
    assert (arr(t, len(want), dt) == want).all()
    shm.barrier_all()
    print('ok')
    shm.finalize()
    """
    for rc, out in spawn(5, body, tmp_path):
        assert rc == 0, out


def test_non_symmetric_remote_address_is_fatal(tmp_path):
    body = """
    x = np.zeros(4, dtype=np.int64)
    if me == 0:
        L.shmem_getmem(x.ctypes.data, x.ctypes.data, 32, 1)
    shm.barrier_all()
    print('UNREACHABLE')
    """
    res = spawn(2, body, tmp_path)
    assert any("is not symmetric" in out for _, out in res), res
    for rc, out in res:
        assert rc != 0 and "UNREACHABLE" not in out


def test_heap_exhaustion_returns_null(tmp_path):
    """No room left: shmem_malloc returns NULL on every PE after its barrier,
    with a NOTICE trace, as the reference's shmalloc (symmem.c:150-153); the
    job goes on, and the space is usable again once freed."""
    body = """
    p = shm.malloc(8 << 20)
    q = shm.malloc(9 << 20)    # more than the 16 MiB segment has left
    assert not q, q
    shm.free(p)
    r = shm.malloc(9 << 20)    # fits now: first fit from the start
    assert r and r == p, (r, p)
    arr(r, 4, np.int64)[:] = me
    shm.barrier_all()
    out = np.zeros(4, dtype=np.int64)
    L.shmem_getmem(out.ctypes.data, r, 32, (me + 1) % npes)
    assert (out == (me + 1) % npes).all(), out
    shm.barrier_all()
    print('ok')
    shm.finalize()
    """
    res = spawn(2, body, tmp_path, extra={"SHMEM_SYMMETRIC_HEAP_SIZE": "16M", "SHMEM_LOG_LEVELS": "NOTICE"})
    for rc, out in res:
        assert rc == 0 and "ok" in out, out
    assert any("NOTICE" in out and "no room left" in out for _, out in res), res

"""CPU: the multi-PE runtime without a GPU (SHMEM_BOOTSTRAP_ONLY=1).

Several processes bring up the bootstrap segment, run many active-set
barriers under random delays and check ordering through a shared file;
a reduction call without a GPU must abort loudly (there is no CPU path).
"""
import os
import subprocess
import sys
import textwrap
import uuid

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "osss-gasnet_amd")


def spawn(npes, body, tmp_path, timeout=120, extra=None):
    code = textwrap.dedent(f"""
        import os, sys, random, time, ctypes
        sys.path.insert(0, {PKG!r})
        import shmem_reduce
        shm = shmem_reduce.Shmem(); shm.init()
        me, npes = shm.my_pe(), shm.n_pes()
    """) + textwrap.dedent(body)
    env = dict(os.environ, SHMEM_BOOTSTRAP_ONLY="1", SHMEM_NPES=str(npes), SHMEM_JOB_ID=uuid.uuid4().hex[:12],
               SHMEM_BARRIER_TIMEOUT="60", TMPDIR=str(tmp_path))
    env.update(extra or {})
    procs = [subprocess.Popen([sys.executable, "-c", code], env=dict(env, SHMEM_PE=str(pe)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for pe in range(npes)]
    res = []
    for p in procs:
        out, _ = p.communicate(timeout=timeout)
        res.append((p.returncode, out))
    return res


@pytest.mark.parametrize("npes", [2, 3, 5])
def test_barrier_orders_phases(tmp_path, npes):
    """In each round every PE appends its mark after a random delay, then
    barriers; after the barrier every PE must see all marks of that round."""
    body = f"""
    log = os.path.join({str(tmp_path)!r}, 'log')
    for r in range(40):
        time.sleep(random.random() * 0.003)
        with open(log, 'a') as f:
            f.write(f'{{r}} {{me}}\\n')
        shm.barrier_all()
        seen = [l.split() for l in open(log).read().split('\\n') if l]
        got = sum(1 for a, b in seen if int(a) == r)
        assert got == npes, (r, got)
        shm.barrier_all()
    shm.finalize()
    print('ok', me)
    """
    for rc, out in spawn(npes, body, tmp_path):
        assert rc == 0, out


def test_strided_active_set_barriers_run_concurrently(tmp_path):
    """Barriers on {0,2} and {1,3} (logPE_stride 1) interleave without crosstalk."""
    body = """
    import numpy as np
    psync = np.full(128, -1, dtype=np.int64)
    start = me % 2
    for r in range(200):
        shm.lib.shmem_barrier(start, 1, 2, psync.ctypes.data)
    assert (psync == -1).all()
    shm.barrier_all()
    shm.finalize()
    """
    for rc, out in spawn(4, body, tmp_path):
        assert rc == 0, out


def test_reduction_without_gpu_fails_loudly(tmp_path):
    body = """
    import numpy as np
    x = np.ones(10); t = np.zeros(10)
    shm.to_all('sum', 'double', t.ctypes.data, x.ctypes.data, 10, 0, 0, npes)
    print('UNREACHABLE')
    """
    for rc, out in spawn(2, body, tmp_path):
        assert rc != 0
        assert "UNREACHABLE" not in out
        assert "no GPU" in out or "aborting" in out


def test_global_exit_stops_every_pe(tmp_path):
    body = """
    if me == 1:
        shm.lib.shmem_global_exit(7)
    shm.barrier_all()
    print('UNREACHABLE')
    """
    res = spawn(3, body, tmp_path)
    assert res[1][0] == 7
    for rc, out in res:
        assert rc != 0 and "UNREACHABLE" not in out


def test_host_malloc_is_collective_and_aligned(tmp_path):
    body = """
    ptrs = [shm.malloc(1000 + 17 * i) for i in range(10)]
    assert all(p % 4096 == 0 for p in ptrs)
    for p in ptrs: shm.free(p)
    assert shm.malloc(0) is None
    shm.finalize()
    """
    for rc, out in spawn(2, body, tmp_path):
        assert rc == 0, out


def test_identity_from_torchrun_env(tmp_path):
    """RANK/WORLD_SIZE (torch.distributed.run) give the PE identity."""
    body = """
    assert (me, npes) == (int(os.environ['RANK']), 2)
    shm.barrier_all(); shm.finalize()
    """
    code_env = {"SHMEM_NPES": "", "SHMEM_PE": ""}
    env = dict(os.environ, SHMEM_BOOTSTRAP_ONLY="1", SHMEM_JOB_ID=uuid.uuid4().hex[:12], WORLD_SIZE="2")
    env.update(code_env)
    code = textwrap.dedent(f"""
        import os, sys
        sys.path.insert(0, {PKG!r})
        import shmem_reduce
        shm = shmem_reduce.Shmem(); shm.init()
        me, npes = shm.my_pe(), shm.n_pes()
    """) + textwrap.dedent(body)
    procs = [subprocess.Popen([sys.executable, "-c", code], env=dict(env, RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.STDOUT, text=True) for r in range(2)]
    for p in procs:
        out, _ = p.communicate(timeout=60)
        assert p.returncode == 0, out


def test_get_put_with_null_buffer_name_it(tmp_path):
    """shmem_getmem / shmem_putmem with a NULL local buffer (e.g. an unchecked
    failed shmemx_malloc_device) abort with the call and the argument named,
    before any GPU work."""
    body = """
    f = shm.lib.shmem_getmem if me == 0 else shm.lib.shmem_putmem
    f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    x = (ctypes.c_char * 64)()
    if me == 0:
        f(None, ctypes.addressof(x), 64, 1)
    else:
        f(ctypes.addressof(x), None, 64, 0)
    print('UNREACHABLE')
    """
    res = spawn(2, body, tmp_path)
    for rc, out in res:
        assert rc != 0 and "UNREACHABLE" not in out, out
    assert any("shmem_getmem: NULL dest" in out for _, out in res), res
    assert any("shmem_putmem: NULL source" in out or "aborting" in out for _, out in res), res


def test_job_above_32_pes(tmp_path):
    """A job of more PEs than a device barrier holds (MI355_FUSED_MAX_MEMBERS
    = 32): the bootstrap, host barriers, the symmetric host heap and an
    fcollect over all 40 PEs. On a GPU such a job skips the init's timed
    device barrier (runtime.c device_wait_test) and its collectives take the
    host-barrier schedules (reduce.c device_flags_ok)."""
    body = """
    import numpy as np
    L = shm.lib
    vp, sz, i = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
    L.shmem_fcollect64.argtypes = [vp, vp, sz, i, i, i, vp]
    L.shmem_getmem.argtypes = [vp, vp, sz, i]
    psync = (ctypes.c_long * 128)(*([-1] * 128))
    s = shm.malloc(64); t = shm.malloc(npes * 64)
    np.ctypeslib.as_array(ctypes.cast(s, ctypes.POINTER(ctypes.c_int64)), shape=(8,))[:] = me * 100 + np.arange(8)
    shm.barrier_all()
    L.shmem_fcollect64(t, s, 8, 0, 0, npes, psync)
    got = np.ctypeslib.as_array(ctypes.cast(t, ctypes.POINTER(ctypes.c_int64)), shape=(npes * 8,)).reshape(npes, 8)
    assert (got == np.arange(npes)[:, None] * 100 + np.arange(8)).all()
    out = np.zeros(8, dtype=np.int64)
    L.shmem_getmem(out.ctypes.data, s, 64, (me + 17) % npes)
    assert (out == ((me + 17) % npes) * 100 + np.arange(8)).all()
    shm.barrier_all()
    print('ok', me)
    shm.finalize()
    """
    res = spawn(40, body, tmp_path, timeout=240)
    for rc, out in res:
        assert rc == 0 and "ok" in out, out

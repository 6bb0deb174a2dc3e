"""CPU: SHMEM_DEBUG=1's collective argument check and the init-time settings
check, on PE processes without a GPU (SHMEM_BOOTSTRAP_ONLY=1).

nreduce == 0 calls are pure synchronization (the reference still runs both
barriers, reduce-op.c:230,266) and need no GPU, so the exchange runs here
for real: matching calls over changing and disjoint active sets must pass,
and a member passing a different operator, type, nreduce or active set must
end the job with a message naming the field (reference debug checks:
reduce-op.c:395-398, utils.h:74-129). The GPU-side counterpart with real
buffers is tests/test_gpu_checks.py."""
import time

from test_bootstrap import spawn

DBG = {"SHMEM_DEBUG": "1"}


def test_matching_calls_pass(tmp_path):
    body = """
    rng = random.Random(17)              # the same sequence on every PE
    jitter = random.Random(me)           # per PE (must not consume rng)
    t = (ctypes.c_double * 4)()
    for k in range(300):
        op, dt = rng.choice([('sum', 'double'), ('max', 'int'), ('xor', 'long'), ('prod', 'complexf')])
        kind = rng.randrange(4)
        if kind == 0:                     # the whole job
            sets = [(0, 0, npes)]
        elif kind == 1:                   # two disjoint halves at once
            sets = [(0, 0, 2), (2, 0, npes - 2)]
        elif kind == 2:                   # strided: even / odd PEs
            sets = [(0, 1, (npes + 1) // 2), (1, 1, npes // 2)]
        else:                             # a sub-range
            sets = [(1, 0, npes - 1)]
        for s in sets:
            if me in [s[0] + i * (1 << s[1]) for i in range(s[2])]:
                time.sleep(jitter.random() * 0.0005)
                shm.to_all(op, dt, ctypes.addressof(t), ctypes.addressof(t), 0, *s)
    shm.barrier_all()
    shm.finalize()
    print('ok', me)
    """
    for rc, out in spawn(4, body, tmp_path, extra=DBG):
        assert rc == 0 and "ok" in out, out


def mismatch(tmp_path, npes, call, expect, may_return=()):
    body = """
    t = (ctypes.c_double * 4)()
    p = ctypes.addressof(t)
    shm.to_all('sum', 'double', p, p, 0, 0, 0, npes)          # a matching call first
    print('T0 %.6f' % time.time(), flush=True)
    """ + call + """
    print('RETURNED', flush=True)
    """
    t_start = time.time()
    res = spawn(npes, body, tmp_path, extra=dict(DBG, SHMEM_BARRIER_TIMEOUT="600"))
    dt = time.time() - t_start
    outs = [o for _, o in res]
    assert all(rc != 0 for pe, (rc, _) in enumerate(res) if pe not in may_return), outs
    assert not any("RETURNED" in o for pe, o in enumerate(outs) if pe not in may_return), outs
    assert any(e in o for o in outs for e in expect), outs
    t0 = min(float(ln.split()[1]) for o in outs for ln in o.splitlines() if ln.startswith("T0 "))
    assert time.time() - t0 < 5.0 and dt < 60, (dt, outs)
    return outs


def test_different_operator(tmp_path):
    mismatch(tmp_path, 2, "shm.to_all('sum' if me == 0 else 'max', 'double', p, p, 0, 0, 0, npes)",
             ["reduction operator (enum mi355_op) is 0 on PE 0 but 6 on PE 1",
              "reduction operator (enum mi355_op) is 6 on PE 1 but 0 on PE 0"])


def test_different_type(tmp_path):
    mismatch(tmp_path, 2, "shm.to_all('max', 'int' if me == 0 else 'long', p, p, 0, 0, 0, npes)",
             ["element type (enum mi355_dtype) is"])


def test_different_nreduce(tmp_path):
    # PE 1's nreduce > 0 would need a GPU after the check: the check comes first
    mismatch(tmp_path, 2, "shm.to_all('sum', 'double', p, p, 0 if me == 0 else 3, 0, 0, npes)",
             ["nreduce is 0 on PE 0 but 3 on PE 1", "nreduce is 3 on PE 1 but 0 on PE 0"])


def test_different_active_set(tmp_path):
    # PE 0 and PE 1 disagree on PE_size; PE 2 (in PE 1's set only) waits in a barrier
    call = ("if me == 2:\n        shm.barrier_all()\n"
            "    else:\n        shm.to_all('sum', 'double', p, p, 0, 0, 0, 2 if me == 0 else 3)")
    mismatch(tmp_path, 3, call, ["PE_size is 2 on PE 0 but 3 on PE 1", "PE_size is 3 on PE 1 but 2 on PE 0"])


def test_different_fused_threshold(tmp_path):
    """shmemx_set_fused_max_bytes is a collective setting: a PE that set another
    threshold would take another schedule than its peers (round 4)."""
    call = ("shm.set_fused_max(1 << 20 if me == 0 else 2 << 20)\n"
            "    shm.to_all('sum', 'double', p, p, 0, 0, 0, npes)")
    mismatch(tmp_path, 2, call, ["fused-kernel threshold in bytes (SHMEM_FUSED_MAX_BYTES / shmemx_set_fused_max_bytes) "
                                 "is 1048576 on PE 0 but 2097152 on PE 1",
                                 "is 2097152 on PE 1 but 1048576 on PE 0"])


def test_different_stride(tmp_path):
    call = "shm.to_all('sum', 'double', p, p, 0, 0, 0 if me != 2 else 1, 2)\n    shm.barrier_all()"
    # PEs 0, 1 call over (0, 0, 2), a correct collective of theirs; PE 2 over
    # (0, 1, 2) = {0, 2}: it learns of the mismatch at PE 0's next
    # synchronization (here shmem_barrier_all) and aborts the job; PEs 0 and
    # 1 may already be through (PE 2's arrivals satisfied their barriers)
    mismatch(tmp_path, 3, call, ["passed this call's synchronization from another call"], may_return=(0, 1))


def test_settings_must_agree(tmp_path):
    body = """
    print('INIT-RETURNED', flush=True)
    shm.finalize()
    """
    # the spawn helper passes one environment to every PE: PE 1 picks its own order from SHMEM_PE
    import os
    res = spawn(2, body, tmp_path, extra={"SHMEM_REDUCE_ORDER": "reference"})
    assert all(rc == 0 for rc, _ in res), res
    env_hook = os.path.join(str(tmp_path), "sitecustomize.py")
    with open(env_hook, "w") as f:
        f.write("import os\nif os.environ.get('SHMEM_PE') == '1': os.environ['SHMEM_REDUCE_ORDER'] = 'pe_start'\n")
    res = spawn(2, body, tmp_path, extra={"PYTHONPATH": str(tmp_path)})
    outs = [o for _, o in res]
    assert all(rc != 0 for rc, _ in res) and not any("INIT-RETURNED" in o for o in outs), outs
    assert any("SHMEM_REDUCE_ORDER differs between PEs" in o for o in outs), outs


def test_external_map_setting_must_agree(tmp_path):
    """SHMEM_EXTERNAL_MAP decides whether a member joins the per-call record
    exchange for device buffers outside the heap (csrc/extmap.c): PEs that
    differ would wait on each other for ever, so init aborts naming it."""
    import os
    body = """
    print('INIT-RETURNED', flush=True)
    shm.finalize()
    """
    with open(os.path.join(str(tmp_path), "sitecustomize.py"), "w") as f:
        f.write("import os\nif os.environ.get('SHMEM_PE') == '1': os.environ['SHMEM_EXTERNAL_MAP'] = '0'\n")
    res = spawn(2, body, tmp_path, extra={"PYTHONPATH": str(tmp_path)})
    outs = [o for _, o in res]
    assert all(rc != 0 for rc, _ in res) and not any("INIT-RETURNED" in o for o in outs), outs
    assert any("SHMEM_EXTERNAL_MAP differs between PEs" in o for o in outs), outs

"""GPU: the job-level checks added in round 3, on PE processes sharing the
one test GPU.

* the init-time coherence test of peer-heap reads (runtime.c
  coherence_test): it runs and passes on the real layout; a simulated stale
  re-read after the acquire (SHMEM_TEST_IPC_FAIL=stale on PE 1) makes every
  PE fall back to the RCCL schedule cleanly (reference contract: a blocking
  get returns the peer's current data, comms-inline.h:2224-2238);
* SHMEM_DEBUG=1's collective argument check (reference debug checks
  reduce-op.c:395-398, utils.h:74-129): a member passing a different
  nreduce / PE_size / operator ends the job within seconds, with a message
  naming the field, instead of reading wrong offsets or waiting out the
  barrier timeout; matching calls (also disjoint sets at once, and
  stream-ordered ones) pass;
* settings that must agree across PEs (SHMEM_REDUCE_ORDER, ...) abort init.
"""
import os
import subprocess
import sys
import time
import uuid

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
pytestmark = [pytest.mark.gpu, pytest.mark.multipe]

PRELUDE = ("import sys, os, time\nsys.path[:0] = [%r, %r, %r]\n" % (HERE, os.path.join(ROOT, "osss-gasnet_amd"),
                                                                     os.path.join(ROOT, "oracle")) +
           "import numpy as np, shmem_reduce\nshm = shmem_reduce.Shmem(); shm.init()\n"
           "me, npes = shm.my_pe(), shm.n_pes()\n")


def spawn(npes, code, extra=None, per_pe=None, timeout=120):
    env = dict(os.environ, SHMEM_NPES=str(npes), SHMEM_JOB_ID=uuid.uuid4().hex[:12], SHMEM_DEVICE="0",
               SHMEM_DEVICE_HEAP_SIZE="32M", SHMEM_DEVICE_SCRATCH_SIZE="3M", SHMEM_BARRIER_TIMEOUT="120")
    env.update(extra or {})
    procs = []
    for pe in range(npes):
        e = dict(env, SHMEM_PE=str(pe))
        e.update((per_pe or {}).get(pe, {}))
        procs.append(subprocess.Popen([sys.executable, "-c", PRELUDE + code], env=e, stdout=subprocess.PIPE,
                                      stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            outs.append(p.communicate(timeout=timeout)[0])
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    return [p.returncode for p in procs], outs, time.time()


# ---------------------------------------------------------------------------
# coherence self-test
# ---------------------------------------------------------------------------
COH = ("ran, passed, stale = shm.coherence_selftest()\n"
       "print('COH', int(ran), int(passed), int(stale), 'ALG', shm.lib.shmemx_get_reduce_algorithm(), flush=True)\n"
       "x = np.random.default_rng(5 + me).random(4099) - 0.5\n"
       "d = shm.malloc_device(4099 * 8); shm.put(d, x)\n"
       "shm.to_all('sum', 'double', d, d, 4099, 0, 0, npes)\n"
       "want = np.random.default_rng(5).random(4099) - 0.5 + (np.random.default_rng(6).random(4099) - 0.5)\n"
       "print('EXACT', bool((shm.get(d, 4099, 'double') == want).all()), flush=True)\n"
       "info = shm.last_call_info(); print('SCHED', info['schedule'], flush=True)\n"
       "shm.finalize()\n")


def parse(out, key):
    return [ln.split()[1:] for ln in out.splitlines() if ln.startswith(key + " ")]


def test_coherence_selftest_runs_and_passes():
    rcs, outs, _ = spawn(2, COH)
    for rc, out in zip(rcs, outs):
        assert rc == 0, out[-2000:]
        coh = parse(out, "COH")[0]
        assert coh[:2] == ["1", "1"] and coh[4] == "0", out  # ran, passed; P2P (auto) kept
        assert parse(out, "EXACT")[0] == ["True"] and parse(out, "SCHED")[0] == ["fused-twoshot"], out


@pytest.mark.parametrize("mode", ["stale", "producer"])
def test_stale_reread_falls_back_to_rccl(mode):
    """PE 1 reports its re-read after the acquire stale -- of the library's own
    write-through marker (stale), or of a caller's plain-store words after the
    multi-launch ordering (producer, round 4's producer-path test): every PE
    learns it at init and runs the RCCL schedule (RCCL joins the two ranks on
    the one GPU through its socket transport, NCCL_HOSTID per PE, as in
    test_gpu_multipe.test_rccl_schedule_multi_rank); a 2-PE double sum is
    a + b either way, so the result stays exact."""
    per_pe = {pe: {"NCCL_HOSTID": f"shmem-stale-test-pe{pe}"} for pe in range(2)}
    rcs, outs, _ = spawn(2, COH, extra={"SHMEM_TEST_IPC_FAIL": mode, "NCCL_SOCKET_IFNAME": "lo",
                                        "NCCL_IB_DISABLE": "1"}, per_pe=per_pe)
    for rc, out in zip(rcs, outs):
        assert rc == 0, out[-2000:]
        coh = parse(out, "COH")[0]
        # ran, failed, (stale marker), algorithm RCCL
        assert coh[:2] == ["1", "0"] and coh[4] == "3", out
        assert coh[2] == ("1" if mode == "stale" else "0"), out
        assert parse(out, "EXACT")[0] == ["True"] and parse(out, "SCHED")[0] == ["rccl"], out
    assert "init coherence test" in outs[0]


SYSLOAD = ("import oracle\n"
           "fresh, skipped = shm.coherence_sysload()\n"
           "print('SYS', int(fresh), int(skipped), flush=True)\n"
           "d = shm.malloc_device(40000 * 8); t = shm.malloc_device(40000 * 8)\n"
           "bad = 0\n"
           "for k in range(24):\n"
           "    n = 40000 if k % 2 else 3000\n"          # fused two-shot (ordered) / one-shot
           "    xs = [np.random.default_rng(1000 * k + p).random(n) - 0.5 for p in range(npes)]\n"
           "    shm.put(d, xs[me])\n"                     # the same buffers rewritten every call
           "    shm.to_all('sum', 'double', t, d, n, 0, 0, npes)\n"
           "    got = shm.get(t, n, 'double')\n"
           "    bad += int((got.view(np.uint64) != oracle.reduce_pe('sum', 'double', xs, me).view(np.uint64)).sum())\n"
           "print('BAD', bad, 'SCHED', shm.last_call_info()['schedule'], flush=True)\n"
           "shm.finalize()\n")


@pytest.mark.parametrize("env,want", [({}, ["1", "1"]), ({"SHMEM_TEST_IPC_FAIL": "sysload"}, ["0", "0"]),
                                      ({"SHMEM_FUSED_ACQUIRE": "1"}, ["1", "0"])],
                         ids=["acquires-skipped", "sysload-stale-keeps-acquires", "forced-acquires"])
def test_fused_acquires_follow_the_sysload_check(env, want):
    """The fused kernel reads the members' buffers with system-coherent loads
    and skips its per-block acquires only when the init coherence test saw
    those loads fresh on every PE: here (one GPU) they are; a simulated stale
    result on PE 1, or SHMEM_FUSED_ACQUIRE=1, keeps the acquires. Every way,
    24 calls on rewritten buffers (ordered two-shot and one-shot, 3 PEs) are
    bit-exact on every PE."""
    rcs, outs, _ = spawn(3, SYSLOAD, extra=env)
    for rc, out in zip(rcs, outs):
        assert rc == 0, out[-2000:]
        assert parse(out, "SYS")[0] == want, out
        assert parse(out, "BAD")[0] == ["0", "SCHED", "fused-twoshot"], out


FUSED_OFF = ("import oracle\n"
             "print('THR', *shm.thresholds(), flush=True)\n"
             "shm.set_fused_max(1 << 20)\n"
             "print('THR2', *shm.thresholds(), flush=True)\n"
             "d = shm.malloc_device(40000 * 8); t = shm.malloc_device(40000 * 8)\n"
             "bad, scheds = 0, set()\n"
             "for k in range(6):\n"
             "    n = 40000 if k % 2 else 3000\n"
             "    xs = [np.random.default_rng(1000 * k + p).random(n) - 0.5 for p in range(npes)]\n"
             "    shm.put(d, xs[me])\n"
             "    shm.to_all('sum', 'double', t, d, n, 0, 0, npes)\n"
             "    scheds.add(shm.last_call_info()['schedule'])\n"
             "    got = shm.get(t, n, 'double')\n"
             "    bad += int((got.view(np.uint64) != oracle.reduce_pe('sum', 'double', xs, me).view(np.uint64)).sum())\n"
             "print('BAD', bad, 'SCHED', *sorted(scheds), flush=True)\n"
             "shm.finalize()\n")


def test_stale_fused_ordering_turns_the_fused_kernel_off():
    """PE 1 reports a caller's plain stores stale through the
    fused kernel's flag ordering, with system-coherent loads AND after an
    acquire (SHMEM_TEST_IPC_FAIL=producer_fused): every PE turns the fused
    kernel off at init (fused_max 0, the warning on PE 0), the setter cannot
    turn it back on, and the calls run the multi-launch schedule, bit-exact."""
    rcs, outs, _ = spawn(3, FUSED_OFF, extra={"SHMEM_TEST_IPC_FAIL": "producer_fused"})
    for rc, out in zip(rcs, outs):
        assert rc == 0, out[-2000:]
        assert parse(out, "THR")[0][0] == "0" and parse(out, "THR2")[0][0] == "0", out
        assert parse(out, "BAD")[0] == ["0", "SCHED", "p2p"], out
    assert "the fused kernel is disabled" in outs[0], outs[0]


def test_timesliced_device_waits_use_host_barriers():
    """PE 1 votes its device-side waits slow (SHMEM_TEST_IPC_FAIL=slowwait, as
    when more PEs share a GPU than it schedules together): every PE records
    the slow waits, turns the fused kernel off (the setter cannot re-enable
    it) and runs host barriers; the results stay bit-exact. Without the fault
    the init timing is recorded and nothing is turned off."""
    code = FUSED_OFF.replace("shm.finalize()\n", "print('DW', *shm.device_wait_report(), flush=True)\nshm.finalize()\n")
    rcs, outs, _ = spawn(3, code, extra={"SHMEM_TEST_IPC_FAIL": "slowwait"})
    for rc, out in zip(rcs, outs):
        assert rc == 0, out[-2000:]
        assert parse(out, "THR")[0][0] == "0" and parse(out, "THR2")[0][0] == "0", out
        bad = parse(out, "BAD")[0]
        assert bad[0] == "0" and not any("fused" in x for x in bad[2:]), out
        slow, us = parse(out, "DW")[0]
        assert slow == "True" and float(us) > 0.0, out
    assert "host barriers, no fused kernel" in outs[0], outs[0]
    # without the fault: the timing is recorded, nothing turned off
    rcs, outs, _ = spawn(3, code)
    for rc, out in zip(rcs, outs):
        assert rc == 0, out[-2000:]
        slow, us = parse(out, "DW")[0]
        assert slow == "False" and 0.0 < float(us) < 1000.0, out
        assert parse(out, "BAD")[0][0] == "0", out


CALIB = ("import oracle\n"
         "cal = shm.threshold_calibration()\n"
         "fm, om = shm.thresholds()\n"
         "print('CAL', int(cal is not None), fm, om, flush=True)\n"
         "if cal is not None:\n"
         "    for b, f, m in cal['fused']: print('F', b, f, m, flush=True)\n"
         "    for b, o, t in cal['oneshot']: print('O', b, o, t, flush=True)\n"
         "d = shm.malloc_device(8 << 20); t = shm.malloc_device(8 << 20)\n"
         "bad, scheds = 0, []\n"
         "for k, nb in enumerate([16 << 10, 64 << 10, 256 << 10, 1 << 20, 2 << 20, 4 << 20, 8 << 20]):\n"
         "    n = nb // 8\n"
         "    xs = [np.random.default_rng(300 * k + p).random(n) - 0.5 for p in range(npes)]\n"
         "    shm.put(d, xs[me])\n"
         "    shm.to_all('sum', 'double', t, d, n, 0, 0, npes)\n"
         "    scheds.append('%d:%s' % (nb, shm.last_call_info()['schedule']))\n"
         "    got = shm.get(t, n, 'double')\n"
         "    bad += int((got.view(np.uint64) != oracle.reduce_pe('sum', 'double', xs, me).view(np.uint64)).sum())\n"
         "print('BAD', bad, flush=True)\n"
         "print('SCHED', *scheds, flush=True)\n"
         "shm.finalize()\n")


def test_thresholds_calibrated_at_init():
    """the fused / one-shot thresholds from measurement on the
    job's own layout (reduce.c shmemi_calibrate_thresholds): every PE gets the
    same thresholds, each the largest size of the prefix of measured sizes
    where the fused (one-shot) call was no slower; calls below and above them
    take the schedules they select, bit-exact on every PE."""
    rcs, outs, _ = spawn(3, CALIB, extra={"SHMEM_THRESHOLD_CALIBRATE": "1", "SHMEM_DEVICE_SCRATCH_SIZE": "24M"})
    cals = []
    for rc, out in zip(rcs, outs):
        assert rc == 0, out[-2000:]
        cal = parse(out, "CAL")[0]
        assert cal[0] == "1", out
        fm, om = int(cal[1]), int(cal[2])
        cals.append((fm, om))
        fs = [(int(b), float(f), float(m)) for b, f, m in parse(out, "F")]
        os_ = [(int(b), float(o), float(t)) for b, o, t in parse(out, "O")]
        assert len(fs) == 6 and len(os_) == 5 and all(f > 0 and m > 0 for _, f, m in fs), out
        # the rule: the largest size of the winning prefix
        want_f = 0
        for b, f, m in fs:
            if f > m:
                break
            want_f = b
        want_o = 0
        for b, o, t in os_:
            if o > t:
                break
            want_o = b
        assert (fm, om) == (want_f, want_o), (fm, om, fs, os_)
        assert parse(out, "BAD")[0] == ["0"], out
        for x in parse(out, "SCHED")[0]:
            nb, sched = x.split(":")
            if int(nb) <= fm:
                assert sched.startswith("fused-" + ("oneshot" if int(nb) <= om else "twoshot")), (x, fm, om)
            else:
                assert sched == "p2p", (x, fm)
    assert len(set(cals)) == 1, cals   # one decision for the job


def test_calibration_settings_must_agree():
    """A threshold given on one PE only would make that PE skip the
    calibration its peers run: init aborts naming the setting instead."""
    rcs, outs, _ = spawn(2, "print('UP', flush=True)\nshm.finalize()\n", extra={"SHMEM_THRESHOLD_CALIBRATE": "1"},
                         per_pe={1: {"SHMEM_FUSED_MAX_BYTES": "2M"}}, timeout=60)
    assert any(rc != 0 for rc in rcs) and any("SHMEM_THRESHOLD_CALIBRATE" in o for o in outs), outs


# ---------------------------------------------------------------------------
# SHMEM_DEBUG=1 collective argument check
# ---------------------------------------------------------------------------
def run_mismatch(npes, body):
    code = ("d = shm.malloc_device(1 << 16)\n"
            "shm.to_all('sum', 'double', d, d, 100, 0, 0, npes)\n"   # a matching call first
            "print('T0 %.6f' % time.time(), flush=True)\n" + body)
    rcs, outs, t_end = spawn(npes, code, extra={"SHMEM_DEBUG": "1", "SHMEM_BARRIER_TIMEOUT": "600"})
    t0 = min(float(parse(o, "T0")[0][0]) for o in outs if parse(o, "T0"))
    return rcs, outs, t_end - t0


def test_debug_check_names_a_different_nreduce():
    rcs, outs, dt = run_mismatch(2, "shm.to_all('sum', 'double', d, d, 100 if me == 0 else 99, 0, 0, npes)\n"
                                    "print('RETURNED', flush=True)\n")
    assert all(rc != 0 for rc in rcs) and not any("RETURNED" in o for o in outs), outs
    assert any("nreduce is 100 on PE 0 but 99 on PE 1" in o or "nreduce is 99 on PE 1 but 100 on PE 0" in o
               for o in outs), outs
    assert dt < 5.0, dt


def test_debug_check_names_a_different_active_set():
    # PE 0 and PE 1 disagree on PE_size; PE 2 waits in shmem_barrier_all
    body = ("if me == 2:\n    shm.barrier_all()\n"
            "else:\n    shm.to_all('max', 'int', d, d, 64, 0, 0, 2 if me == 0 else 3)\n"
            "print('RETURNED', flush=True)\n")
    rcs, outs, dt = run_mismatch(3, body)
    assert all(rc != 0 for rc in rcs) and not any("RETURNED" in o for o in outs), outs
    assert any("PE_size is" in o for o in outs), outs
    assert dt < 5.0, dt


def test_debug_check_names_a_different_operator():
    body = ("f = 'sum' if me == 0 else 'max'\nshm.to_all(f, 'double', d, d, 64, 0, 0, npes)\n"
            "print('RETURNED', flush=True)\n")
    rcs, outs, dt = run_mismatch(2, body)
    assert all(rc != 0 for rc in rcs) and not any("RETURNED" in o for o in outs), outs
    assert any("reduction operator" in o for o in outs), outs
    assert dt < 5.0, dt


def test_debug_check_passes_matching_calls():
    """Matching calls under SHMEM_DEBUG=1: disjoint active sets at once,
    strided sets, the whole job, host arrays and stream-ordered calls."""
    code = ("import oracle\n"
            "d = shm.malloc_device(1 << 20); s = shm.malloc_device(1 << 20)\n"
            "ok = True\n"
            "for rnd in range(20):\n"
            "    n = 1000 + 37 * rnd\n"
            "    xs = [np.random.default_rng(rnd * 10 + p).random(n) for p in range(npes)]\n"
            "    shm.put(s, xs[me]); shm.barrier_all()\n"
            "    sets = [(0, 0, 2), (2, 0, 2)] if rnd % 3 == 0 else [(me % 2, 1, 2)] if rnd % 3 == 1 else [(0, 0, 4)]\n"
            "    st = [t for t in sets if me in [t[0] + i * (1 << t[1]) for i in range(t[2])]][0]\n"
            "    mem = [st[0] + i * (1 << st[1]) for i in range(st[2])]\n"
            "    if rnd % 4 == 3:\n"
            "        q = shm.stream_create(); shm.to_all_on_stream('sum', 'double', d, s, n, *st, q)\n"
            "        shm.stream_sync(q); shm.stream_destroy(q)\n"
            "    else:\n"
            "        shm.to_all('sum', 'double', d, s, n, *st)\n"
            "    got = shm.get(d, n, 'double')\n"
            "    want = oracle.reduce_pe('sum', 'double', [xs[p] for p in mem], mem.index(me))\n"
            "    ok &= bool((got.view(np.uint64) == want.view(np.uint64)).all())\n"
            "print('OK', ok, flush=True)\nshm.finalize()\n")
    rcs, outs, _ = spawn(4, code, extra={"SHMEM_DEBUG": "1"})
    for rc, out in zip(rcs, outs):
        assert rc == 0 and "OK True" in out, out[-2000:]


def test_settings_must_agree_at_init():
    rcs, outs, _ = spawn(2, "print('INIT-RETURNED', flush=True)\nshm.finalize()\n",
                         per_pe={1: {"SHMEM_REDUCE_ORDER": "pe_start"}})
    assert all(rc != 0 for rc in rcs) and not any("INIT-RETURNED" in o for o in outs), outs
    assert any("SHMEM_REDUCE_ORDER differs between PEs" in o for o in outs), outs

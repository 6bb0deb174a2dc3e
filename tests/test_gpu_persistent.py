"""GPU: the opt-in persistent fused server (SHMEM_PERSISTENT=1; reduce.c,
fused.hip fused_server). PE processes sharing the one test GPU run scripted
sequences of blocking reductions (tests/persistent_worker.py), each result
checked bit-exact against the oracle's result for that PE; the stats show
that a resident server served the calls. Scripts: bursts of every kind of
call the server takes (one-shot/two-shot, in place, offsets, ordered pairs);
bursts interrupted by operations that stop it (a larger multi-launch call,
another op, a broadcast, a stream-ordered call); gaps longer than its idle
time; gaps around the idle time (a call rung as the server leaves); a call
after GPU work the caller queued and then completed (it sees that work's
result)."""
import json
import os
import subprocess
import sys
import uuid

import pytest

from test_gpu_multipe import oshrun_queues

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = [pytest.mark.gpu, pytest.mark.multipe]


def run(npes, script, seed=1, extra=None, timeout=300):
    env = dict(os.environ)
    env.update({"SHMEM_NPES": str(npes), "SHMEM_JOB_ID": uuid.uuid4().hex[:12], "SHMEM_DEVICE": "0",
                "SHMEM_DEVICE_HEAP_SIZE": "32M", "SHMEM_DEVICE_SCRATCH_SIZE": "384K",
                "SHMEM_DEVICE_ORDER_SIZE": "4M", "SHMEM_BARRIER_TIMEOUT": "60", "SHMEM_PEER_ACQUIRE": "1",
                "SHMEM_PERSISTENT": "1"})
    env.update(oshrun_queues(npes, env))
    env.update(extra or {})
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "persistent_worker.py"), script, str(seed)],
                              env=dict(env, SHMEM_PE=str(pe)), stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True) for pe in range(npes)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    stats = []
    for pe, (rc, out) in enumerate(outs):
        assert rc == 0, f"PE {pe} exited {rc}:\n{out[-3000:]}"
        stats.append(json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1]))
    return stats


@pytest.mark.parametrize("npes", [1, 2, 3])
def test_bursts_served_bit_exact(npes):
    # one PE: the identity copy, served by a one-member server (in-place calls move nothing)
    st = run(npes, "burst", seed=npes)
    for s in st:
        assert s["checked"] == 192
        # most calls of a batch are served by a resident server (restarted
        # when a call is more than 4x the size it was started for)
        assert s["served"] >= (90 if npes == 1 else 120) and s["launched"] >= 6, s


def test_interrupted_bursts():
    # fused path up to 256 KiB: the 1 MiB call takes the multi-launch schedule (device barriers)
    st = run(3, "mixed", seed=5, extra={"SHMEM_FUSED_MAX_BYTES": "262144"})
    for s in st:
        assert s["checked"] == 3 * 46 and s["served"] >= 40 and s["launched"] >= 12, s


def test_order_switched_inside_a_burst():
    """shmemx_set_reduce_order between two calls of a burst: the calls after it
    deliver the new order on every PE (the resident server, started for the
    old order, is stopped by the switch; server_matches also compares it)."""
    st = run(2, "orderflip", seed=3)
    for s in st:
        assert s["checked"] == 4 * 16 and s["served"] >= 16 and s["launched"] >= 8, s


def test_gaps_longer_than_idle():
    st = run(2, "idle", seed=7, extra={"SHMEM_PERSISTENT_IDLE_US": "300"})
    for s in st:
        assert s["checked"] == 90 and s["launched"] >= 10, s


def test_call_rung_as_the_server_leaves():
    st = run(2, "race", seed=11, extra={"SHMEM_PERSISTENT_IDLE_US": "60"})
    for s in st:
        assert s["checked"] == 400 and s["launched"] >= 10 and s["served"] >= 10, s


@pytest.mark.parametrize("npes", [1, 2])
def test_call_after_the_callers_queued_work(npes):
    # the caller completes its queued null-stream work (hipStreamSynchronize)
    # before the call: no hang, and the call reduces the new data
    st = run(npes, "ordered", seed=13)
    for s in st:
        assert s["checked"] == 4 and s["launched"] >= 1, s

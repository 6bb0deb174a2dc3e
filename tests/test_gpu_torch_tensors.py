"""PyTorch tensors as *_to_all target/source at 2 PEs (sharing the test
GPU): the members map each other's caching-allocator segments for the call
(extmap.c) -- no staging copies -- and every PE gets the reference's result
for itself; a view off 16-byte alignment makes every member stage instead."""
import json
import os
import subprocess
import sys
import uuid

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = [pytest.mark.gpu, pytest.mark.multipe]


def run_workers(script, npes=2):
    env = dict(os.environ, SHMEM_NPES=str(npes), SHMEM_JOB_ID=uuid.uuid4().hex[:12], SHMEM_DEVICE="0",
               SHMEM_DEVICE_HEAP_SIZE="64M", SHMEM_DEVICE_SCRATCH_SIZE="3M", SHMEM_BARRIER_TIMEOUT="120",
               SHMEM_PEER_ACQUIRE="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, script)],
                              env=dict(env, SHMEM_PE=str(pe)), stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True) for pe in range(npes)]
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append(out)
    for pe, (p, out) in enumerate(zip(procs, outs)):
        assert p.returncode == 0, f"PE {pe} failed:\n{out[-4000:]}"
    return [json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1]) for out in outs]


def test_torch_tensors_mapped_between_pes():
    for rec in run_workers("_torch_tensor_worker.py"):
        for name, sched in rec["schedules"].items():
            assert sched.startswith("mapped-") == ("unaligned" not in name), (rec["pe"], name, sched)
        mapped, opened, closed = rec["map_stats"]
        assert opened >= 1 and closed == 0, rec


def test_torch_stream_and_graph():
    """Symmetric-heap torch tensors with the stream-ordered reduction between
    torch kernels on one torch stream, eager and captured by torch.cuda.graph
    (5 replays = 5 collectives), bit-exact against the oracle."""
    for rec in run_workers("_torch_graph_worker.py"):
        assert rec["ok"] and rec["replays"] == 5, rec

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


def test_torch_tensors_mapped_between_pes():
    env = dict(os.environ, SHMEM_NPES="2", SHMEM_JOB_ID=uuid.uuid4().hex[:12], SHMEM_DEVICE="0",
               SHMEM_DEVICE_HEAP_SIZE="64M", SHMEM_DEVICE_SCRATCH_SIZE="3M", SHMEM_BARRIER_TIMEOUT="120",
               SHMEM_PEER_ACQUIRE="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "_torch_tensor_worker.py")],
                              env=dict(env, SHMEM_PE=str(pe)), stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                              text=True) for pe in range(2)]
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
    for out in outs:
        rec = json.loads([ln for ln in out.splitlines() if ln.startswith("{")][-1])
        for name, sched in rec["schedules"].items():
            assert sched.startswith("mapped-") == ("unaligned" not in name), (rec["pe"], name, sched)
        mapped, opened, closed = rec["map_stats"]
        assert opened >= 1 and closed == 0, rec

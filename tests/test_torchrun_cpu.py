"""CPU, world_size 2 under torch.distributed.run (gloo): the library's N > 1
host path -- PE identity and bootstrap under torchrun's environment, exactly
as bench.py is launched for N > 1 -- and the P2P schedule's shard
decomposition checked against the oracle (tests/_torchrun_worker.py)."""
import os
import socket
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_under_torchrun_gloo(tmp_path):
    env = dict(os.environ, SHMEM_BOOTSTRAP_ONLY="1", SHMEM_BARRIER_TIMEOUT="60", OMP_NUM_THREADS="1")
    for k in ("SHMEM_PE", "SHMEM_NPES", "SHMEM_JOB_ID"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
                        os.path.join(HERE, "_torchrun_worker.py")],
                       env=env, capture_output=True, text=True, timeout=240, cwd=str(tmp_path))
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.count(" ok") >= 2, out[-4000:]

"""One rank of tests/test_torchrun_cpu.py (launched by torch.distributed.run,
gloo backend, no GPU). Checks, across real torchrun ranks:
  - the library's PE identity and bootstrap segment under torchrun's env
    (RANK/WORLD_SIZE, segment named from the agent pid + MASTER_PORT);
  - the P2P schedule's decomposition: every rank folds its own shard
    (mi355_shard_bounds) of all members' sources in member order (the oracle
    on the shard), the shards are all-gathered over gloo, and the assembled
    array equals the oracle's full fold on PE_start, bit for bit.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch.distributed as dist  # noqa: E402

import oracle  # noqa: E402
import shmem_reduce  # noqa: E402
from _inputs import source  # noqa: E402


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    shm = shmem_reduce.Shmem()
    shm.init()
    assert (shm.my_pe(), shm.n_pes()) == (rank, world), (shm.my_pe(), shm.n_pes(), rank, world)
    shm.barrier_all()
    cases = [("sum", "double", 100003), ("prod", "float", 777), ("xor", "int", 4099), ("min", "longlong", 64),
             ("sum", "complexd", 1000), ("max", "short", 5), ("sum", "longdouble", 333), ("and", "long", 0)]
    for k, (op, dtype, n) in enumerate(cases):
        srcs = [source(op, dtype, n, 4242 + k, pe) for pe in range(world)]
        es = np.dtype(oracle.NP[dtype]).itemsize
        lo, hi = shmem_reduce.shard_bounds(shm.lib, n, es, world, rank)
        mine = oracle.reduce_pe(op, dtype, [s[lo:hi] for s in srcs], 0) if hi > lo else srcs[0][:0]
        parts = [None] * world
        dist.all_gather_object(parts, (lo, hi, mine.tobytes()))
        full = np.zeros(n, dtype=oracle.NP[dtype])
        covered = np.zeros(n, dtype=np.int64)
        for lo_i, hi_i, b in parts:
            full[lo_i:hi_i] = np.frombuffer(b, dtype=oracle.NP[dtype])
            covered[lo_i:hi_i] += 1
            assert lo_i == hi_i or (lo_i * es) % 256 == 0, (lo_i, es)
        assert (covered == 1).all(), f"{op}/{dtype}: shards do not tile [0, {n})"
        want = oracle.reduce_pe(op, dtype, srcs, 0)
        assert oracle.as_value_bytes(full, dtype).tobytes() == oracle.as_value_bytes(want, dtype).tobytes(), \
            f"{op}/{dtype}: sharded fold differs from the PE_start fold"
    shm.barrier_all()
    shm.finalize()
    dist.barrier()
    dist.destroy_process_group()
    print(f"rank {rank} ok", flush=True)


if __name__ == "__main__":
    main()

"""One PE of tests/test_gpu_torch_tensors.py::test_torch_stream_and_graph:
symmetric-heap torch tensors (Shmem.heap_tensor), the stream-ordered
reduction enqueued on a torch stream between torch kernels with no host
wait, then the same step captured with torch.cuda.graph and replayed --
every replay one more collective -- checked bit for bit against the oracle
replaying the same float64 arithmetic."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (HERE, os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle  # noqa: E402
import shmem_reduce  # noqa: E402
from _compare import assert_match  # noqa: E402
from _inputs import source  # noqa: E402


def main():
    shm = shmem_reduce.Shmem()
    shm.init()
    me, npes = shm.my_pe(), shm.n_pes()
    torch.cuda.set_device(shm.lib.shmemx_device_id())
    n, replays = 70001, 5
    srcs = [source("sum", "double", n, 31, pe) for pe in range(npes)]
    x = shm.heap_tensor(n, torch.float64)
    out = shm.heap_tensor(n, torch.float64)
    acc = shm.heap_tensor(n, torch.float64)
    s = torch.cuda.Stream()

    def step():
        x.add_(1.0)
        shm.to_all_on_stream("sum", "double", out.data_ptr(), x.data_ptr(), n, 0, 0, npes, s.cuda_stream)
        acc.add_(out)

    # eager: torch kernels and the reduction queued on one torch stream, no host wait in between
    with torch.cuda.stream(s):
        x.copy_(torch.from_numpy(srcs[me]).cuda())
        acc.zero_()
        step()
    s.synchronize()
    xs = [v + 1.0 for v in srcs]
    want_acc = np.zeros(n) + oracle.reduce_pe("sum", "double", xs, me)
    assert_match(acc.cpu().numpy(), want_acc, "sum", "double", ctx=f"PE {me} eager:")

    # the same step captured once and replayed
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s, capture_error_mode="relaxed"):
        step()
    # capture does not run the step: acc, x unchanged
    for _ in range(replays):
        g.replay()
        xs = [v + 1.0 for v in xs]
        want_acc = want_acc + oracle.reduce_pe("sum", "double", xs, me)
    torch.cuda.synchronize()
    assert_match(acc.cpu().numpy(), want_acc, "sum", "double", ctx=f"PE {me} after {replays} graph replays:")
    shm.barrier_all()
    del g
    for t in (acc, out, x):
        shm.free_device(t.data_ptr())
    print(json.dumps({"pe": me, "replays": replays, "ok": True}), flush=True)
    shm.finalize()


if __name__ == "__main__":
    main()

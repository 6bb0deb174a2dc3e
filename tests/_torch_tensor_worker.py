"""One PE of tests/test_gpu_torch_tensors.py: shmem_<T>_<op>_to_all on
PyTorch tensors (the caching allocator's device memory, outside the
symmetric heap) -- whole tensors, views at an offset into a larger one, in
place, and a view 4 bytes off alignment -- checked against the oracle's
result for this PE. Prints one JSON line of the schedules the library ran."""
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
    cases = [("sum", "double", 100003, "whole"), ("max", "float", 5000, "whole"), ("and", "longlong", 70000, "whole"),
             ("min", "short", 999, "whole"), ("prod", "complexd", 3000, "whole"), ("sum", "double", 300000, "view"),
             ("xor", "int", 40000, "view"), ("sum", "float", 20000, "inplace"), ("sum", "double", 8192, "unaligned"),
             ("max", "int", 123457, "unaligned")]
    scheds = {}
    for k, (op, dtype, n, kind) in enumerate(cases):
        srcs = [source(op, dtype, n, 900 + k, pe) for pe in range(npes)]
        x = torch.from_numpy(srcs[me]).cuda()
        if kind == "whole":
            src, dst = x, torch.empty_like(x)
        elif kind == "view":      # both 4 KiB into larger tensors
            big_s = torch.zeros(n + 4096, dtype=x.dtype, device="cuda")
            big_d = torch.zeros(n + 4096, dtype=x.dtype, device="cuda")
            off = 4096 // x.element_size()
            big_s[off:off + n] = x
            src, dst = big_s[off:off + n], big_d[off:off + n]
        elif kind == "inplace":
            src = dst = x
        else:                     # one element in: 4 or 8 bytes off 16-byte alignment, every PE stages
            big_s = torch.zeros(n + 1, dtype=x.dtype, device="cuda")
            big_d = torch.zeros(n + 1, dtype=x.dtype, device="cuda")
            big_s[1:] = x
            src, dst = big_s[1:], big_d[1:]
        shm.to_all(op, dtype, dst.data_ptr(), src.data_ptr(), n, 0, 0, npes)
        scheds[f"{op}_{dtype}_{kind}"] = shm.last_call_info()["schedule"]
        got = dst.cpu().numpy()
        want = oracle.reduce_pe(op, dtype, srcs, me)
        assert_match(got, want, op, dtype, ctx=f"PE {me} {op}/{dtype} {kind}:")
    # the tensor form of the call (shmem_reduce.Shmem.to_all_tensors)
    for k, (op, tdt) in enumerate([("sum", torch.float64), ("min", torch.int16), ("xor", torch.int64),
                                   ("prod", torch.complex64), ("max", torch.float32), ("or", torch.int32)]):
        name = shmem_reduce.TORCH_DTYPES[str(tdt).replace("torch.", "")]
        n = 10007 + 999 * k
        srcs = [source(op, name, n, 1700 + k, pe) for pe in range(npes)]
        x = torch.from_numpy(srcs[me]).cuda()
        out = torch.empty_like(x)
        shm.to_all_tensors(op, out, x)
        assert shm.last_call_info()["schedule"].startswith("mapped-")
        assert_match(out.cpu().numpy(), oracle.reduce_pe(op, name, srcs, me), op, name,
                     ctx=f"PE {me} to_all_tensors {op}/{tdt}:")
    shm.barrier_all()
    print(json.dumps({"pe": me, "schedules": scheds, "map_stats": shm.external_map_stats()}), flush=True)
    shm.finalize()


if __name__ == "__main__":
    main()

"""GPU: stream-ordered reductions (shmemx_<T>_<op>_to_all_on_stream) and the
device barrier (shmemx_barrier_on_stream) across PE processes on one GPU.

Each case enqueues a chain buf[i+1] <- reduce(buf[i]) on a HIP stream with no
host wait between the calls, so every cross-PE step of the chain is ordered by
device-side flags alone (fused kernel or device barriers). The expected chain
is computed with the oracle: step 1 gives member q the reference's result
for q (its own source first, the default result order), step i+1 reduces the
members' step-i results the same way (with order "pe_start": PE_start's
result on every member, so step i+1 folds size copies of it).
"""
import numpy as np
import pytest

import oracle
from _compare import assert_match
from _inputs import source
from test_gpu_multipe import members, run_pes

pytestmark = [pytest.mark.gpu, pytest.mark.multipe]


def chain_want(op, dtype, n, seed, mem, k, pe, order="reference"):
    """Step results 1..k on member `pe` of `mem`."""
    def step(xs):
        return [oracle.reduce_pe(op, dtype, xs, i if order == "reference" else 0) for i in range(len(mem))]
    ys = []
    y = step([source(op, dtype, n, seed, q) for q in mem])
    ys.append(y[mem.index(pe)])
    for _ in range(k - 1):
        y = step(y)
        ys.append(y[mem.index(pe)])
    return ys


def stream_case(cid, op, dtype, n, sets, chain=3, **kw):
    c = {"id": cid, "kind": "stream", "op": op, "dtype": dtype, "n": n, "sets": sets, "chain": chain,
         "seed": 500 + cid}
    c.update(kw)
    return c


def check_stream(results, cases):
    for c in cases:
        op, dtype, n, k = c["op"], c["dtype"], c["n"], c["chain"]
        for s in c["sets"]:
            mem = members(*s)
            for pe in mem:
                res = results[pe]
                order = c.get("order", "reference")
                if c.get("graph"):
                    for r in range(c["graph"]):
                        want = chain_want(op, dtype, n, c["seed"] + r, mem, k, pe, order)[-1]
                        assert_match(res[f"{c['id']}_r{r}"], want, op, dtype,
                                     ctx=f"case {c['id']} graph replay {r} set {s} PE {pe}:")
                    continue
                for i, want in enumerate(chain_want(op, dtype, n, c["seed"], mem, k, pe, order), start=1):
                    assert_match(res[f"{c['id']}_{i}"], want, op, dtype,
                                 ctx=f"case {c['id']} step {i} set {s} PE {pe}:")
                if c.get("mixed"):
                    want = oracle.reduce_pe(op, dtype, [source(op, dtype, n, c["seed"] + 1, q) for q in mem],
                                            mem.index(pe) if order == "reference" else 0)
                    assert_match(res[f"{c['id']}_host"], want, op, dtype, ctx=f"case {c['id']} host call PE {pe}:")


SOME = [("sum", "double"), ("prod", "float"), ("xor", "int"), ("max", "longlong"), ("min", "short"),
        ("sum", "complexd"), ("prod", "longdouble")]


def test_stream_chains_fused_and_multi_launch(tmp_path):
    """Small messages (one fused launch per call) and large ones (fold and
    gather between device barriers), aligned and not, with device barriers
    interleaved, on 4 PEs; two disjoint sets at once; a one-PE set; n = 0."""
    cases, cid = [], 0
    for op, dtype in SOME:
        cases.append(stream_case(cid, op, dtype, 1000, [[0, 0, 4]])); cid += 1
        cases.append(stream_case(cid, op, dtype, 70000, [[0, 0, 4]])); cid += 1   # > 256 KiB fused limit below
        cases.append(stream_case(cid, op, dtype, 3001, [[0, 0, 4]], offset=1, barriers=True)); cid += 1
    cases.append(stream_case(cid, "sum", "double", 5000, [[0, 1, 2], [1, 1, 2]])); cid += 1
    cases.append(stream_case(cid, "sum", "double", 70000, [[0, 1, 2], [1, 1, 2]])); cid += 1
    cases.append(stream_case(cid, "and", "long", 777, [[2, 0, 1]])); cid += 1
    cases.append(stream_case(cid, "sum", "double", 0, [[0, 0, 4]], barriers=True)); cid += 1
    cases.append(stream_case(cid, "sum", "float", 1, [[1, 0, 3]])); cid += 1
    # PE_start order on every member
    cases.append(stream_case(cid, "sum", "double", 1000, [[0, 0, 4]], order="pe_start")); cid += 1
    cases.append(stream_case(cid, "max", "float", 70000, [[0, 0, 4]], order="pe_start")); cid += 1
    # every member's order through version areas too small for one round
    cases.append(stream_case(cid, "sum", "float", 90001, [[0, 0, 4]])); cid += 1
    results = run_pes(4, cases, tmp_path, extra_env={"SHMEM_FUSED_MAX_BYTES": "256K",
                                                     "SHMEM_DEVICE_ORDER_SIZE": "512K"})
    check_stream(results, cases)


def test_stream_graph_replay(tmp_path):
    """The chain captured once into a HIP graph and replayed with new inputs:
    the device pair counts advance on every replay."""
    cases = [stream_case(0, "sum", "double", 4096, [[0, 0, 4]], chain=2, graph=3),
             stream_case(1, "max", "int", 100000, [[0, 0, 4]], chain=2, graph=3),
             stream_case(2, "xor", "short", 333, [[0, 0, 4]], chain=3, graph=2, barriers=True)]
    results = run_pes(4, cases, tmp_path, extra_env={"SHMEM_FUSED_MAX_BYTES": "64K"})
    check_stream(results, cases)


def test_stream_and_host_calls_interleaved(tmp_path):
    """A host-side call issued while a stream chain is still in flight (the
    host fused kernel must queue behind it: they share the pair counts)."""
    cases = [stream_case(0, "sum", "double", 2000, [[0, 0, 3]], chain=4, mixed=True),
             stream_case(1, "prod", "complexf", 60000, [[0, 0, 3]], chain=2, mixed=True),
             stream_case(2, "min", "double", 500, [[0, 0, 3]], chain=2, mixed=True)]
    results = run_pes(3, cases, tmp_path)
    check_stream(results, cases)

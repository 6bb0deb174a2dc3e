"""GPU: put/get, broadcast, fcollect and collect across PE processes
(SURVEY.md 8f rows 3-4), checked against the oracle's restatement of the
reference semantics (oracle.broadcast / fcollect / collect)."""
import numpy as np
import pytest

import oracle
from pe_worker import dm_source
from test_gpu_multipe import members, run_pes

pytestmark = [pytest.mark.gpu, pytest.mark.multipe]


def case(cid, kind, bits, n, sets, **kw):
    c = {"id": cid, "kind": kind, "bits": bits, "n": n, "sets": sets, "seed": 500 + cid, "cap": 4096,
         "op": "sum", "dtype": "long"}  # op/dtype only size the worker's buffers
    c.update(kw)
    return c


def check_dm(results, cases):
    for c in cases:
        dt = np.int32 if c["bits"] == 32 else np.int64
        for s in c["sets"]:
            mem = members(*s)
            srcs = [dm_source(c, pe) for pe in mem]
            cap = c["cap"]
            sentinel = np.full(cap, -7, dtype=dt)
            if c["kind"] == "broadcast":
                want = oracle.broadcast([x for x in srcs], c["root"], [sentinel[:len(srcs[0])]] * len(mem))
                for i, pe in enumerate(mem):
                    got = results[pe][str(c["id"])]
                    assert (got[:len(want[i])] == want[i]).all(), (c, pe)
                    assert (got[len(want[i]):] == -7).all(), (c, pe)
            elif c["kind"] in ("fcollect", "collect"):
                want = (oracle.fcollect if c["kind"] == "fcollect" else oracle.collect)(srcs)
                for i, pe in enumerate(mem):
                    got = results[pe][str(c["id"])]
                    assert (got[:len(want[i])] == want[i]).all(), (c, pe)
                    assert (got[len(want[i]):] == -7).all(), (c, pe)
            elif c["kind"] == "putget":
                n, size = c["n"], len(mem)
                for i, pe in enumerate(mem):
                    got = results[pe][str(c["id"])]
                    prv = (i - 1) % size
                    assert (got[prv * n:(prv + 1) * n] == srcs[prv]).all(), (c, pe)
                    assert (results[pe][str(c["id"]) + "_get"] == srcs[prv]).all(), (c, pe)


def test_host_heap_objects_three_pes(tmp_path):
    """the symmetric objects in shmem_malloc's default host
    heap (every PE's segment mapped by every PE, csrc/hostheap.c, as the
    reference's segment exchange makes them reachable, comms-inline.h:766-845):
    shmem_getmem / putmem (putget.c:249-256) with device, page-locked and
    pageable local sides, broadcast from every root (broadcast-linear.c:61-82),
    fcollect (fcollect-linear.c:60-93) and collect into device, host-heap and
    pageable targets, on 3 PEs; every PE's result against the oracle."""
    cases = []
    cid = 0
    for bits in (32, 64):
        for root in (0, 1, 2):
            cases.append(case(cid, "broadcast", bits, 300, [[0, 0, 3]], root=root, source="host")); cid += 1
        for tk in ("device", "host", "pageable"):
            cases.append(case(cid, "broadcast", bits, 129, [[0, 0, 3]], root=1, source="host", target=tk)); cid += 1
            cases.append(case(cid, "fcollect", bits, 200, [[0, 0, 3]], source="host", target=tk)); cid += 1
            cases.append(case(cid, "collect", bits, 5, [[0, 0, 3]], source="host", target=tk)); cid += 1
        cases.append(case(cid, "fcollect", bits, 33, [[1, 0, 2]], source="host")); cid += 1
        cases.append(case(cid, "broadcast", bits, 40, [[2, 0, 1]], root=0, source="host")); cid += 1
        for pf in ("device", "host", "pageable"):
            cases.append(case(cid, "putget", bits, 100, [[0, 0, 3]], source="host", put_from=pf)); cid += 1
        cases.append(case(cid, "putget", bits, 51, [[0, 0, 3]], source="host", target="host")); cid += 1
    results = run_pes(3, cases, tmp_path)
    check_dm(results, cases)


@pytest.mark.parametrize("fused", ["fused", "barrier_copy_barrier"])
def test_collectives_four_pes(tmp_path, fused):
    """Small broadcast/fcollect run as one fused pull launch by default;
    SHMEM_FUSED_MAX_BYTES=0 keeps them on device barrier + copy kernel +
    device barrier (the path for messages above the fused limit)."""
    cases = []
    cid = 0
    for bits in (32, 64):
        for root in (0, 2, 3):
            cases.append(case(cid, "broadcast", bits, 300, [[0, 0, 4]], root=root)); cid += 1
        cases.append(case(cid, "broadcast", bits, 257, [[0, 1, 2], [1, 1, 2]], root=1)); cid += 1
        cases.append(case(cid, "broadcast", bits, 0, [[0, 0, 4]], root=1)); cid += 1
        cases.append(case(cid, "broadcast", bits, 129, [[0, 0, 4]], root=1, target="host")); cid += 1
        cases.append(case(cid, "fcollect", bits, 200, [[0, 0, 4]])); cid += 1
        cases.append(case(cid, "fcollect", bits, 33, [[1, 0, 3]])); cid += 1
        cases.append(case(cid, "fcollect", bits, 100, [[0, 0, 4]], target="host")); cid += 1
        for tk in ("pageable", "mixed"):  # target the kernel cannot write: scratch + copy out
            cases.append(case(cid, "broadcast", bits, 77, [[0, 0, 4]], root=3, target=tk)); cid += 1
            cases.append(case(cid, "fcollect", bits, 45, [[0, 0, 4]], target=tk)); cid += 1
        for tk in ("device", "pageable"):  # one-member active sets (PEs 2 and 3 alone)
            cases.append(case(cid, "broadcast", bits, 40, [[2, 0, 1], [3, 0, 1]], root=0, target=tk)); cid += 1
            cases.append(case(cid, "fcollect", bits, 41, [[2, 0, 1], [3, 0, 1]], target=tk)); cid += 1
        cases.append(case(cid, "collect", bits, 4, [[0, 0, 4]])); cid += 1  # PE 0 contributes nothing
        cases.append(case(cid, "collect", bits, 3, [[0, 1, 2], [1, 1, 2]])); cid += 1
        cases.append(case(cid, "putget", bits, 100, [[0, 0, 4]])); cid += 1
        cases.append(case(cid, "putget", bits, 64, [[0, 0, 4]], target="host")); cid += 1
        for pf in ("host", "pageable"):  # put from host memory (kernel over PCIe / DMA)
            cases.append(case(cid, "putget", bits, 51, [[0, 0, 4]], put_from=pf)); cid += 1
    results = run_pes(4, cases, tmp_path, extra_env=None if fused == "fused" else {"SHMEM_FUSED_MAX_BYTES": "0"})
    check_dm(results, cases)


def test_collectives_eight_pes(tmp_path):
    """Broadcast and fcollect over 8 PE processes (one fused pull launch below
    the fused limit, barrier + copy kernel + barrier above it), and over two
    interleaved strided sets of 4."""
    cases = []
    cid = 0
    for n in (100, 40000):  # 800 B / 320 KB per PE (fcollect: 8x that into every PE)
        cases.append(case(cid, "broadcast", 64, n, [[0, 0, 8]], root=5, cap=40960)); cid += 1
        cases.append(case(cid, "fcollect", 64, n // 8, [[0, 0, 8]], cap=40960)); cid += 1
        cases.append(case(cid, "fcollect", 32, n // 8, [[0, 1, 4], [1, 1, 4]], cap=40960)); cid += 1
    results = run_pes(8, cases, tmp_path)
    check_dm(results, cases)


def test_mixed_collectives_stress(tmp_path):
    """200 back-to-back calls on 4 PEs mixing reductions (fused and multi-launch
    sizes), broadcast, fcollect, collect and put/get with random sizes, targets
    and active sets: every collective kind advances the same per-pair counts
    of the signal region, so a kind that miscounted would deadlock or let a
    PE read a buffer too early here."""
    from test_gpu_multipe import check as check_red
    rng = np.random.default_rng(4242)
    sets_choices = [[[0, 0, 4]], [[0, 1, 2], [1, 1, 2]], [[1, 0, 3]], [[0, 0, 2], [2, 0, 2]]]
    cases = []
    for cid in range(200):
        sets = sets_choices[rng.integers(len(sets_choices))]
        k = int(rng.integers(6))
        if k <= 1:
            op, dtype = oracle.PAIRS[rng.integers(len(oracle.PAIRS))]
            cases.append({"id": cid, "op": op, "dtype": dtype, "n": int(rng.choice([1, 100, 3000, 40000])),
                          "sets": sets, "mode": str(rng.choice(["dev", "inplace", "host"])),
                          "algorithm": "p2p", "seed": 9000 + cid})
            continue
        bits = int(rng.choice([32, 64]))
        tgt = str(rng.choice(["device", "device", "host", "pageable"]))
        if k == 2:
            size = sets[0][2]
            cases.append(case(cid, "broadcast", bits, int(rng.choice([0, 5, 300, 3000])), sets,
                              root=int(rng.integers(size)), target=tgt))
        elif k == 3:
            cases.append(case(cid, "fcollect", bits, int(rng.choice([1, 50, 900])), sets, target=tgt))
        elif k == 4:
            cases.append(case(cid, "collect", bits, 5, sets))
        else:
            cases.append(case(cid, "putget", bits, int(rng.choice([3, 64, 500])), [[0, 0, 4]]))
    results = run_pes(4, cases, tmp_path, extra_env={"SHMEM_DEVICE_HEAP_SIZE": "64M",
                                                     "SHMEM_DEVICE_SCRATCH_SIZE": "3M"})
    check_red(results, [c for c in cases if "op" in c and "kind" not in c])
    check_dm(results, [c for c in cases if "kind" in c])

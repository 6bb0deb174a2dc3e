"""GPU: the collectives across several PE processes (P2P and EXACT schedules).

The box has one MI355X, so the PEs share it: each PE is its own process with
its own device heap, peers are mapped through hipIpcOpenMemHandle exactly as
across GPUs (the xGMI case differs only in where the bytes travel). Each run
starts N pe_worker.py processes from this (not yet GPU-initialised) pytest
process, then checks every PE's target against the oracle:

  P2P   member i's result == the reference's result on member i
        (bit-exact, NaN payloads aside): the default result order
        (SHMEM_REDUCE_ORDER=reference) folds every member's order for the
        order-sensitive pairs; with order "pe_start" every member's result
        == the reference's result on PE_start
  EXACT member i's result == the reference's result on member i
"""
import itertools
import json
import os
import subprocess
import sys
import uuid

import numpy as np
import pytest

import oracle
from _compare import assert_match
from _inputs import source

HERE = os.path.dirname(os.path.abspath(__file__))
pytestmark = [pytest.mark.gpu, pytest.mark.multipe]


def oshrun_queues(npes, env):
    """tools/oshrun's hardware-queue policy for PEs sharing one GPU."""
    import importlib.machinery
    import importlib.util
    path = os.path.join(os.path.dirname(HERE), "tools", "oshrun")
    loader = importlib.machinery.SourceFileLoader("oshrun", path)
    spec = importlib.util.spec_from_loader("oshrun", loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod.hw_queue_env(npes, True, env)


def run_pes(npes, cases, tmp_path, extra_env=None, timeout=600, per_pe_env=None):
    spec = tmp_path / "spec.json"
    spec.write_text(json.dumps({"cases": cases}))
    env = dict(os.environ)
    env.update({"SHMEM_NPES": str(npes), "SHMEM_JOB_ID": uuid.uuid4().hex[:12], "SHMEM_DEVICE": "0",
                "SHMEM_DEVICE_HEAP_SIZE": "96M", "SHMEM_DEVICE_SCRATCH_SIZE": "384K",
                "SHMEM_BARRIER_TIMEOUT": "120",
                # the multi-GPU layout queues a system-scope acquire before every read of peers'
                # buffers (peers on other GPUs); the PEs here share one GPU, so force it on
                "SHMEM_PEER_ACQUIRE": "1"})
    # PEs sharing the one test GPU: the job's hardware queues kept at 16, the
    # same policy as tools/oshrun (8 processes x the default 4 oversubscribe
    # the GPU's queue slots and every call then waits ~34 ms for a time slice;
    # DESIGN.md section 5)
    env.update(oshrun_queues(npes, env))
    env.update(extra_env or {})
    procs = []
    for pe in range(npes):
        e = dict(env, SHMEM_PE=str(pe))
        e.update((per_pe_env or {}).get(pe, {}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "pe_worker.py"), str(spec), str(tmp_path)],
                                      env=e, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        outs.append((p.returncode, out))
    for pe, (rc, out) in enumerate(outs):
        assert rc == 0, f"PE {pe} exited {rc}:\n{out[-3000:]}"
    return [np.load(tmp_path / f"pe{pe}.npz") for pe in range(npes)]


def members(start, logstride, size):
    return [start + i * (1 << logstride) for i in range(size)]


def check(results, cases):
    for c in cases:
        op, dtype, n = c["op"], c["dtype"], c["n"]
        for s in c["sets"]:
            mem = members(*s)
            srcs = [source(op, dtype, n, c["seed"], pe) for pe in mem]
            per_pe = c.get("algorithm") == "exact" or c.get("order", "reference") == "reference"
            for i, pe in enumerate(mem):
                got = results[pe][str(c["id"])]
                want = oracle.reduce_pe(op, dtype, srcs, i if per_pe else 0)
                assert_match(got, want, op, dtype, ctx=f"case {c['id']} {c['mode']} {c.get('algorithm')} "
                                                        f"{c.get('order', 'reference')} set {s} PE {pe}:")


def make_cases(pairs, n, sets, mode, algorithm, start_id, seed=11, order="reference"):
    out = []
    for k, (op, dtype) in enumerate(pairs):
        out.append({"id": start_id + k, "op": op, "dtype": dtype, "n": n, "sets": sets, "mode": mode,
                    "algorithm": algorithm, "seed": seed + start_id + k, "order": order})
    return out


SOME = [("sum", "double"), ("sum", "float"), ("xor", "int"), ("and", "longlong"), ("max", "float"),
        ("min", "short"), ("prod", "complexd"), ("sum", "longdouble")]


@pytest.mark.parametrize("fused_max,oneshot_max", [("1M", "64K"), ("2M", "0"), ("0", "0")],
                         ids=["fused-oneshot", "fused-twoshot-2M", "multi-launch"])
def test_four_pes_all_44_pairs_p2p_and_exact(tmp_path, fused_max, oneshot_max):
    """Every pair on 4 PEs, through the one-launch fused kernel (messages up to
    1 MiB; one-shot fold up to 64 KiB, reduce-scatter + all-gather above) and
    through the multi-launch shard schedule (fused path disabled)."""
    cases = []
    cases += make_cases(oracle.PAIRS, 1000, [[0, 0, 4]], "dev", "p2p", 0)
    cases += make_cases(oracle.PAIRS, 257, [[0, 0, 4]], "dev", "exact", 100)
    cases += make_cases(oracle.PAIRS, 1000, [[0, 0, 4]], "inplace", "p2p", 200)  # in place: never one-shot
    cases += make_cases(SOME, 9, [[0, 0, 4]], "dev", "p2p", 300)      # less than one 16-byte vector per element type
    cases += make_cases(SOME, 4099, [[1, 0, 3]], "dev", "p2p", 400)  # several blocks and an element tail
    cases += make_cases(oracle.PAIRS, 1000, [[0, 0, 4]], "dev", "p2p", 500, order="pe_start")
    cases += make_cases(SOME, 4099, [[0, 0, 4]], "inplace", "p2p", 600, order="pe_start")
    results = run_pes(4, cases, tmp_path, extra_env={"SHMEM_FUSED_MAX_BYTES": fused_max,
                                                     "SHMEM_ONESHOT_MAX_BYTES": oneshot_max})
    check(results, cases)


GOLDEN_ROWS = json.load(open(os.path.join(HERE, "golden", "manifest.json")))["cases"]
NAN_ROWS = json.load(open(os.path.join(HERE, "golden", "manifest.json")))["nan_cases"]


@pytest.mark.parametrize("fused_max,oneshot_max", [("1M", "64K"), ("2M", "0"), ("0", "0")],
                         ids=["fused-oneshot", "fused-twoshot-2M", "multi-launch"])
def test_golden_fixtures_on_every_pe(tmp_path, fused_max, oneshot_max):
    """The committed golden vectors (outputs of the reference's own compiled
    operators in each member's fold order, NaN / +-0 / Inf / x87 encodings
    included) through the public entry points on 2-8 PE processes: member i's
    target must equal the fixture's row i for every one of the 44 pairs, on the
    one-shot, two-shot and multi-launch schedules."""
    import gen_golden  # noqa: F401  (same fixtures as tests/golden)
    cases, cid = [], 0
    for op, dtype in oracle.PAIRS:
        for k, row in enumerate(GOLDEN_ROWS[f"{op}_{dtype}"]):
            if row["npes"] < 2 or row["n"] == 0:
                continue
            cases.append({"id": cid, "op": op, "dtype": dtype, "n": row["n"], "sets": [[0, 0, row["npes"]]],
                          "mode": "dev", "algorithm": "p2p", "seed": 0, "golden": k})
            cid += 1
    results = run_pes(8, cases, tmp_path, extra_env={"SHMEM_FUSED_MAX_BYTES": fused_max,
                                                     "SHMEM_ONESHOT_MAX_BYTES": oneshot_max})
    for c in cases:
        g = np.load(os.path.join(HERE, "golden", f"golden_{c['op']}_{c['dtype']}.npz"))
        outs = g[f"out_{c['golden']}"]
        for i in range(c["sets"][0][2]):
            assert_match(results[i][str(c["id"])], outs[i], c["op"], c["dtype"],
                         ctx=f"golden {c['op']}/{c['dtype']} case {c['golden']} PE {i}:")


@pytest.mark.parametrize("fused_max,oneshot_max", [("1M", "64K"), ("2M", "0"), ("0", "0")],
                         ids=["fused-oneshot", "fused-twoshot-2M", "multi-launch"])
def test_nan_payload_fixtures_on_every_pe(tmp_path, fused_max, oneshot_max):
    """The NaN-payload families (tests/golden/golden_nan_*: float, double and
    complex sum/prod on operands full of NaNs of every sign, payload and kind,
    infinities and overflowing values, outputs from the reference's compiled
    operators) on 2-9 PE processes through the public entry points: every PE's
    target must equal its fixture row bit for bit, NaN payloads included."""
    cases, cid = [], 0
    for key, rows in NAN_ROWS.items():
        op, dtype = key.split("_")
        for k, row in enumerate(rows):
            # two members: also in place, host arrays, unaligned and outside the heap (the two-member
            # schedule folds each shard in its owner's order and NaN-patches the gather, reduce.c nan_pair)
            modes = ["dev"] + (["inplace", "host", "unaligned", "devmap_offset", "overlap_up"]
                               if row["npes"] == 2 else [])
            for mode in modes:
                cases.append({"id": cid, "op": op, "dtype": dtype, "n": row["n"], "sets": [[0, 0, row["npes"]]],
                              "mode": mode, "algorithm": "p2p", "seed": 0, "golden": k, "family": "nan_"})
                cid += 1
    results = run_pes(9, cases, tmp_path, extra_env={"SHMEM_FUSED_MAX_BYTES": fused_max,
                                                     "SHMEM_ONESHOT_MAX_BYTES": oneshot_max})
    for c in cases:
        g = np.load(os.path.join(HERE, "golden", f"golden_nan_{c['op']}_{c['dtype']}.npz"))
        outs = g[f"out_{c['golden']}"]
        for i in range(c["sets"][0][2]):
            assert_match(results[i][str(c["id"])], outs[i], c["op"], c["dtype"], strict=True,
                         ctx=f"nan golden {c['op']}/{c['dtype']} case {c['golden']} PE {i}:")


def two_member_nan_sequence(tmp_path, extra_env):
    """A sequence on one pair alternating NaN-rich calls (golden_nan rows),
    NaN-free ones and tiny ones whose second shard is empty (no fold on PE 1:
    it only clears the next call's NaN word), in place and not; every call
    checked bit-exact on both PEs."""
    cases, cid = [], 0
    for rep in range(2):
        for op in ("sum", "prod"):
            for dtype in ("double", "float"):
                for mode in ("dev", "inplace"):
                    cases.append({"id": cid, "op": op, "dtype": dtype, "n": NAN_ROWS[f"{op}_{dtype}"][0]["n"],
                                  "sets": [[0, 0, 2]], "mode": mode, "algorithm": "p2p", "seed": 0, "golden": 0,
                                  "family": "nan_"})
                    cid += 1
                    cases.append({"id": cid, "op": op, "dtype": dtype, "n": 70001 + cid, "sets": [[0, 0, 2]],
                                  "mode": mode, "algorithm": "p2p", "seed": 900 + cid})
                    cid += 1
                    cases.append({"id": cid, "op": op, "dtype": dtype, "n": 3 + rep, "sets": [[0, 0, 2]],
                                  "mode": mode, "algorithm": "p2p", "seed": 950 + cid})
                    cid += 1
    results = run_pes(2, cases, tmp_path, extra_env=extra_env)
    for c in cases:
        if "golden" in c:
            g = np.load(os.path.join(HERE, "golden", f"golden_nan_{c['op']}_{c['dtype']}.npz"))
            outs = g["out_0"]
        else:
            xs = [source(c["op"], c["dtype"], c["n"], c["seed"], pe) for pe in range(2)]
            outs = [oracle.reduce_pe(c["op"], c["dtype"], xs, pe) for pe in range(2)]
        for i in range(2):
            assert_match(results[i][str(c["id"])], outs[i], c["op"], c["dtype"], strict=True,
                         ctx=f"case {c['id']} {c['mode']} {c['op']}/{c['dtype']} PE {i}:")


@pytest.mark.parametrize("fused_max", ["0", "2M"], ids=["multi-launch", "fused"])
def test_two_member_calls_alternating_nan_and_finite(tmp_path, fused_max):
    """The two-member float/double schedule (reduce.c nan_pair): the owner's
    fold sets a per-call NaN word (parity of the call number with that
    partner) and the other member patches its gather only when it is set;
    alternating NaN-rich and NaN-free calls take each parity's word from set
    to clear and back."""
    two_member_nan_sequence(tmp_path, {"SHMEM_FUSED_MAX_BYTES": fused_max})


def test_two_member_nan_calls_without_signal_regions(tmp_path):
    """The same sequence when PE 1 cannot map its peer's signal region
    (SHMEM_TEST_IPC_FAIL=sig): host barriers, and no NaN word to read -- the
    gather patches unconditionally (reduce.c nan_word_ok) instead of loading
    through a NULL mapping."""
    two_member_nan_sequence(tmp_path, {"SHMEM_TEST_IPC_FAIL": "sig"})


def test_pe_start_order_within_stated_fp_tolerance(tmp_path):
    """SHMEM_REDUCE_ORDER=pe_start gives every PE PE_start's result. For FP
    sum/prod on PE p != PE_start that differs from the reference's own result
    by rounding only: |r - ref_p| <= 2 (N-1) u sum|x_i| (sum) and
    <= 2 (N-1) u |prod x_i| (prod), u = 2^-53 / 2^-24,
    wherever every input is finite and normal and neither result overflowed;
    where an input is NaN both results must be NaN."""
    pairs = [("sum", "double"), ("sum", "float"), ("prod", "double"), ("prod", "float")]
    cases = make_cases(pairs, 20000, [[0, 0, 5]], "dev", "p2p", 0, order="pe_start")
    cases += make_cases(pairs, 300, [[0, 0, 5]], "dev", "p2p", 100, order="pe_start")
    results = run_pes(5, cases, tmp_path)
    for c in cases:
        op, dtype, n = c["op"], c["dtype"], c["n"]
        srcs = [source(op, dtype, n, c["seed"], pe) for pe in range(5)]
        x = np.stack(srcs).astype(np.float64)
        u = 2.0 ** -53 if dtype == "double" else 2.0 ** -24
        with np.errstate(all="ignore"):
            bound = 2 * 4 * u * (np.abs(x).sum(axis=0) if op == "sum" else np.abs(np.prod(x, axis=0)))
        finite_in = np.isfinite(x).all(axis=0)
        # subnormal inputs round relative to the subnormal grid, not to u
        normal_in = ((np.abs(x) >= np.finfo(oracle.NP[dtype]).tiny) | (x == 0)).all(axis=0)
        differs = 0
        for p in range(5):
            got = results[p][str(c["id"])].astype(np.float64)
            ref = oracle.reduce_pe(op, dtype, srcs, p).astype(np.float64)
            both = finite_in & normal_in & np.isfinite(got) & np.isfinite(ref)
            err = np.abs(got - ref)
            assert (err[both] <= bound[both]).all(), f"{op}/{dtype} PE {p}: error above the stated bound"
            # a NaN input makes the result NaN in every order (an Inf may give Inf or NaN by order)
            nan_in = np.isnan(x).any(axis=0)
            assert (np.isnan(got[nan_in]) & np.isnan(ref[nan_in])).all(), f"{op}/{dtype} PE {p}"
            differs += int((got[both] != ref[both]).sum())
        if n > 1000:
            assert differs > 0, "inputs too benign: no PE's result differed from PE_start's"


@pytest.mark.parametrize("fused_max", ["1M", "0"], ids=["fused", "multi-launch"])
def test_four_pes_modes_and_active_sets(tmp_path, fused_max):
    cases = []
    cid = 1000
    for mode, alg in itertools.product(["inplace", "overlap_up", "overlap_down", "host", "unaligned"],
                                       ["p2p", "exact"]):
        cases += make_cases(SOME, 515, [[0, 0, 4]], mode, alg, cid)
        cid += 100
    # two disjoint strided sets running at once, a 3-PE set, and a set of one
    cases += make_cases(SOME, 515, [[0, 1, 2], [1, 1, 2]], "dev", "p2p", cid); cid += 100
    cases += make_cases(SOME, 515, [[1, 0, 3]], "dev", "p2p", cid); cid += 100
    cases += make_cases(SOME, 515, [[2, 0, 1]], "dev", "p2p", cid); cid += 100
    # multi-chunk staging (scratch is 3 x 128 KiB): 100k doubles from host memory
    cases += make_cases([("sum", "double"), ("max", "int")], 100000, [[0, 0, 4]], "host", "p2p", cid); cid += 100
    cases += make_cases([("sum", "double")], 100000, [[0, 0, 4]], "host", "exact", cid); cid += 100
    # edge sizes: nothing, one element, fewer elements than PEs x alignment
    for n in (0, 1, 3, 64):
        cases += make_cases([("sum", "double"), ("or", "short")], n, [[0, 0, 4]], "dev", "p2p", cid); cid += 100
    results = run_pes(4, cases, tmp_path, extra_env={"SHMEM_FUSED_MAX_BYTES": fused_max})
    check(results, cases)


@pytest.mark.parametrize("npes", [2, 3])
def test_two_and_three_pes(tmp_path, npes):
    cases = make_cases(SOME, 4099, [[0, 0, npes]], "dev", "p2p", 0)
    cases += make_cases(SOME, 333, [[0, 0, npes]], "inplace", "exact", 100)
    results = run_pes(npes, cases, tmp_path)
    check(results, cases)


@pytest.mark.parametrize("npes", [9, 12])
def test_more_than_eight_pes_one_gpu(tmp_path, npes):
    """9-12 PEs: the fused kernel's batched fold goes past its first batch of
    8 members' vectors (one-shot and reduce-scatter, element tails), the
    every-member-order fold of more than 8 sources runs one fold per member,
    and 9-12 spin-waiting grids share the GPU (co-residency cap)."""
    pairs = [("sum", "double"), ("max", "float"), ("xor", "int"), ("prod", "complexf")]
    cases = make_cases(pairs, 1001, [[0, 0, npes]], "dev", "p2p", 0)            # fused one-shot (< 64 KiB)
    cases += make_cases(pairs, 20003, [[0, 0, npes]], "dev", "p2p", 100)        # fused two-shot
    cases += make_cases(pairs, 20003, [[0, 0, npes]], "inplace", "p2p", 200)    # two-shot in place
    cases += make_cases(pairs[:2], 200001, [[0, 0, npes]], "dev", "p2p", 300)   # multi-launch
    cases += make_cases(pairs[:2], 20003, [[0, 0, npes]], "dev", "p2p", 400, order="pe_start")
    results = run_pes(npes, cases, tmp_path, extra_env={"SHMEM_DEVICE_HEAP_SIZE": "32M",
                                                        "SHMEM_DEVICE_ORDER_SIZE": "16M"})
    check(results, cases)


def test_reduction_while_another_kernel_holds_every_cu(tmp_path):
    """PE 0 enters each collective right after queueing, on a stream of its
    own, a kernel that fills every CU for 300 ms (the helper returns once all
    of its blocks are resident): its spin-waiting grid (fused one-launch, or
    the device barriers of the multi-launch schedule) starts block by block as
    that kernel drains -- or, when the GPU's scheduler time-slices the busy
    queue out (seen on some boxes: the call then returns in ~0.1 ms), at once
    -- while its peers already wait in theirs. Every call must complete with
    the right result, well inside the barrier timeout."""
    cases = make_cases([("sum", "double")], 8000, [[0, 0, 3]], "dev", "p2p", 0)        # fused one-shot
    cases += make_cases([("max", "float")], 100000, [[0, 0, 3]], "dev", "p2p", 100)   # fused two-shot
    cases += make_cases([("sum", "double")], 300000, [[0, 0, 3]], "dev", "p2p", 200)  # multi-launch
    for c in cases:
        c["busy_ms"] = 300
    results = run_pes(3, cases, tmp_path, extra_env={"SHMEM_BARRIER_TIMEOUT": "60"})
    check(results, cases)
    for c in cases:
        t = float(results[0][str(c["id"]) + "_seconds"][0])
        assert t < 10.0, f"case {c['id']}: {t:.3f} s from the busy launch to the call's return"
        print(f"case {c['id']}: {t * 1e3:.1f} ms from the busy grid holding every CU to the call's return")


def test_largest_messages(tmp_path):
    """nreduce up to INT_MAX (the `int nreduce` of shmem.h:1507-1743): 2^31-1
    shorts (4 GiB) on one PE, the identity checked whole; and 2^29 floats
    (2 GiB per PE) on 2 PEs through max_to_all, whose every-member order needs
    several rounds of the default 256 MiB version area, NaN and +-0 planted,
    checked on a million samples per PE against the oracle's result for that
    PE. (The reference's own byte count `int snred = sizeof(Type)*nreduce`,
    reduce-op.c:190, overflows above 2 GiB; this build counts in size_t.)"""
    one = [{"id": 0, "kind": "big", "op": "sum", "dtype": "short", "n": (1 << 31) - 1, "sets": [[0, 0, 1]],
            "seed": 3}]
    res = run_pes(1, one, tmp_path, extra_env={"SHMEM_DEVICE_HEAP_SIZE": "8400M"}, timeout=900)
    assert int(res[0]["0_bad"][0]) == 0
    two = [{"id": 1, "kind": "big", "op": "max", "dtype": "float", "n": 1 << 29, "sets": [[0, 0, 2]], "seed": 5},
           {"id": 2, "kind": "big", "op": "sum", "dtype": "int", "n": (1 << 29) + 3, "sets": [[0, 0, 2]], "seed": 6}]
    res = run_pes(2, two, tmp_path, extra_env={"SHMEM_DEVICE_HEAP_SIZE": "4200M"}, timeout=900)
    for pe in range(2):
        for c in two:
            assert int(res[pe][f"{c['id']}_bad"][0]) == 0, (pe, c["id"])


def test_eight_pes_one_gpu(tmp_path):
    cases = make_cases([("sum", "double"), ("and", "longlong"), ("max", "float")], 20000, [[0, 0, 8]],
                       "dev", "p2p", 0)
    cases += make_cases([("sum", "double")], 20000, [[0, 1, 4], [1, 1, 4]], "dev", "p2p", 100)
    # above the fused limit: the multi-launch schedule, in the same run
    cases += make_cases([("sum", "double"), ("xor", "int")], 300000, [[0, 0, 8]], "dev", "p2p", 200)
    results = run_pes(8, cases, tmp_path)
    check(results, cases)


FORTRAN_PAIRS = [(op, dt) for op, dt in oracle.PAIRS if dt != "longlong"]


def test_fortran_binding_three_pes(tmp_path):
    """The 37 Fortran-callable reductions (csrc/fortran.c, reference
    fortran.c:1218-1256) on 3 PEs: by-reference arguments, INTEGER pSync,
    fused and multi-launch schedules, a strided set; same parity bar as C."""
    assert len(FORTRAN_PAIRS) == 37
    cases = make_cases(FORTRAN_PAIRS, 300, [[0, 0, 3]], "dev", "p2p", 0)
    cases += make_cases(FORTRAN_PAIRS, 70000, [[0, 0, 3]], "inplace", "p2p", 100)
    cases += make_cases([p for p in SOME if p[1] != "longlong"], 515, [[0, 1, 2]], "host", "exact", 200)
    for c in cases:
        c["api"] = "fortran"
    results = run_pes(3, cases, tmp_path, extra_env={"SHMEM_FUSED_MAX_BYTES": "256K"})
    check(results, cases)


def test_bad_active_set_aborts_every_pe(tmp_path):
    """A PE outside the active set fails loudly and its peers do not hang."""
    cases = [{"id": 0, "op": "sum", "dtype": "double", "n": 10, "sets": [[0, 0, 2]], "mode": "dev",
              "algorithm": "p2p", "seed": 1},
             # PE 1 calls with a set that excludes it -> fatal; PE 0 waits in a barrier
             {"id": 1, "op": "sum", "dtype": "double", "n": 10, "sets": [[0, 0, 1], [1, 0, 1]], "mode": "dev",
              "algorithm": "p2p", "seed": 2, "bad_for_pe1": True}]
    spec = tmp_path / "spec.json"
    bad = dict(cases[1])
    bad["sets"] = [[0, 0, 2]]
    spec.write_text(json.dumps({"cases": [cases[0], bad]}))
    env = dict(os.environ, SHMEM_NPES="2", SHMEM_JOB_ID=uuid.uuid4().hex[:12], SHMEM_DEVICE="0",
               SHMEM_DEVICE_HEAP_SIZE="32M", SHMEM_DEVICE_SCRATCH_SIZE="384K", SHMEM_BARRIER_TIMEOUT="60")
    code = ("import sys,os; sys.path[:0]=[%r,%r,%r]\n" % (HERE, os.path.join(os.path.dirname(HERE), "osss-gasnet_amd"),
                                                          os.path.join(os.path.dirname(HERE), "oracle")) +
            "import shmem_reduce\nshm=shmem_reduce.Shmem(); shm.init(); d=shm.malloc_device(1024)\n"
            "pe=shm.my_pe()\n"
            "shm.to_all('sum','double',d,d,10,0,0,2)\n"
            "if pe==1: shm.to_all('sum','double',d,d,10,0,0,1)\n"
            "else: shm.to_all('sum','double',d,d,10,0,0,2)\n")
    procs = [subprocess.Popen([sys.executable, "-c", code], env=dict(env, SHMEM_PE=str(pe)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for pe in range(2)]
    outs = [p.communicate(timeout=120) for p in procs]
    assert procs[1].returncode != 0 and "not in the active set" in outs[1][0]
    assert procs[0].returncode != 0 and "aborting" in outs[0][0]


def test_rccl_init_is_bounded_on_a_shared_gpu(tmp_path):
    """shmemx_rccl_init (non-blocking RCCL bring-up with a deadline): with two
    PEs on ONE GPU, which RCCL does not support, it must come back on both PEs
    (ready or not, the same answer) instead of hanging or aborting the job, and
    the P2P schedule must still work afterwards. bench.py relies on this before
    timing its RCCL comparison leg."""
    env = dict(os.environ, SHMEM_NPES="2", SHMEM_JOB_ID=uuid.uuid4().hex[:12], SHMEM_DEVICE="0",
               SHMEM_DEVICE_HEAP_SIZE="32M", SHMEM_DEVICE_SCRATCH_SIZE="384K", SHMEM_BARRIER_TIMEOUT="60")
    code = ("import sys,os,time; sys.path[:0]=[%r,%r]\n" % (HERE, os.path.join(os.path.dirname(HERE), "osss-gasnet_amd")) +
            "import numpy as np, shmem_reduce\nshm=shmem_reduce.Shmem(); shm.init()\n"
            "t0=time.time(); rc=shm.lib.shmemx_rccl_init(15.0); dt=time.time()-t0\n"
            "d=shm.malloc_device(1024); shm.put(d, np.full(16, 1.0 + shm.my_pe()))\n"
            "shm.to_all('sum','double',d,d,16,0,0,2)\n"
            "ok=(shm.get(d,16,'double')==3.0).all()\n"
            "print('rc', rc, 'dt %.1f' % dt, 'p2p', ok, flush=True)\nshm.finalize()\n")
    procs = [subprocess.Popen([sys.executable, "-c", code], env=dict(env, SHMEM_PE=str(pe)),
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for pe in range(2)]
    outs = [p.communicate(timeout=100)[0] for p in procs]
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out[-2000:]
        assert "p2p True" in out, out[-2000:]
    rcs = [int(o.split("rc ")[1].split()[0]) for o in outs]
    assert rcs[0] == rcs[1], outs


def test_small_host_arrays_one_launch_and_mixed(tmp_path):
    """Host arrays (shmem_malloc, page-locked) up to 64 KiB take the one-launch
    path with in-kernel staging; odd PEs use plain numpy arrays (staged
    copies) in the same collectives: both forms must meet and agree. Sizes
    around the 64 KiB limit and the multi-chunk path above it."""
    cases = []
    cid = 0
    for mode in ("host", "host_mixed"):
        for n in (1, 3, 515, 8191, 8192, 8193, 100000):
            cases += make_cases([("sum", "double"), ("max", "int"), ("xor", "short"), ("prod", "complexf")],
                                n, [[0, 0, 4]], mode, "p2p", cid)
            cid += 100
    cases += make_cases(SOME, 515, [[0, 1, 2], [1, 1, 2]], "host_mixed", "p2p", cid)
    results = run_pes(4, cases, tmp_path, extra_env={"SHMEM_DEVICE_SCRATCH_SIZE": "3M"})
    check(results, cases)


def test_non_symmetric_device_buffers(tmp_path):
    """Plain hipMalloc buffers (a framework's tensors): small messages go
    through the fused kernel staging them itself, larger ones through the
    scratch staging path; odd PEs passing page-locked host arrays in the same
    calls (_mixed) must meet them."""
    cases = []
    cid = 0
    for mode in ("devother", "devother_mixed"):
        for n in (1, 515, 8192, 100000, 300000):
            cases += make_cases([("sum", "double"), ("min", "int"), ("and", "longlong")], n, [[0, 0, 4]], mode,
                                "p2p", cid)
            cid += 100
    results = run_pes(4, cases, tmp_path, extra_env={"SHMEM_DEVICE_SCRATCH_SIZE": "3M"})
    check(results, cases)


MAPPED_PAIRS = [("sum", "double"), ("max", "float"), ("and", "longlong"), ("prod", "complexd"),
                ("sum", "longdouble"), ("min", "short")]


def test_external_device_buffers_mapped(tmp_path):
    """hipMalloc buffers at 3 PEs: the members map each other's allocations for
    the call (extmap.c) and run the heap schedules on them -- fused one-shot,
    two-shot and the multi-launch shards -- in place, at per-PE offsets into
    the allocations and with the target in the heap; every PE's result is the
    reference's for it, the schedule says "mapped-", and the peers' mappings
    are opened once and reused."""
    cases = []
    cid = 0
    for mode in ("devother", "devmap_inplace", "devmap_offset", "devmap_symtarget"):
        for n in (515, 8192, 60000, 300000):
            cases += make_cases(MAPPED_PAIRS, n, [[0, 0, 3]], mode, "p2p", cid)
            cid += 100
    cases += make_cases(MAPPED_PAIRS[:3], 5000, [[0, 1, 2]], "devother", "p2p", cid)  # strided set {0, 2}
    cases += make_cases(MAPPED_PAIRS, 20000, [[0, 0, 3]], "devother", "exact", cid + 100)  # EXACT schedule
    cases += make_cases(MAPPED_PAIRS, 200000, [[0, 0, 3]], "devmap_offset", "p2p", cid + 200, order="pe_start")
    results = run_pes(3, cases, tmp_path, extra_env={"SHMEM_DEVICE_SCRATCH_SIZE": "3M"})
    check(results, cases)
    for c in cases:
        for s in c["sets"]:
            for pe in members(*s):
                sched = str(results[pe][str(c["id"]) + "_schedule"][0])
                assert sched.startswith("mapped-"), f"case {c['id']} {c['mode']} PE {pe}: schedule {sched}"
    for pe in range(3):
        mapped, opened, closed = (int(v) for v in results[pe]["external_map_stats"])
        # two hipMalloc allocations per peer, each opened once for all the calls
        assert opened <= 4 and closed == 0 and mapped == opened, (pe, mapped, opened, closed)
        # exports are cached per allocation: no file descriptor per call
        fd0, fd1 = (int(v) for v in results[pe]["fd_count"])
        assert fd1 - fd0 <= 8, (pe, fd0, fd1)


def test_external_device_buffers_fallbacks(tmp_path):
    """Where one member cannot share its buffers (PE 1 8 bytes off 16-byte
    alignment) every member stages and the results stay exact; buffers
    re-allocated before every call get new handles (no stale mapping); a
    cache of one mapping closes and reopens as the calls alternate."""
    cases = []
    cases += make_cases(MAPPED_PAIRS, 5000, [[0, 0, 3]], "devmap_unaligned_pe1", "p2p", 0)
    cases += make_cases(MAPPED_PAIRS, 70000, [[0, 0, 3]], "devmap_unaligned_pe1", "p2p", 100)
    cases += make_cases(MAPPED_PAIRS * 2, 3000, [[0, 0, 3]], "devmap_realloc", "p2p", 200)
    cases += make_cases(MAPPED_PAIRS, 40000, [[0, 0, 3]], "devother", "p2p", 300)
    results = run_pes(3, cases, tmp_path, extra_env={"SHMEM_DEVICE_SCRATCH_SIZE": "3M",
                                                     "SHMEM_EXTERNAL_MAP_CACHE": "1"})
    check(results, cases)
    for c in cases:
        for pe in range(3):
            sched = str(results[pe][str(c["id"]) + "_schedule"][0])
            assert sched.startswith("mapped-") == (c["mode"] != "devmap_unaligned_pe1"), (c["id"], pe, sched)
    for pe in range(3):
        mapped, opened, closed = (int(v) for v in results[pe]["external_map_stats"])
        assert opened >= 2 * 12 and closed >= opened - 4, (pe, mapped, opened, closed)
    # mapping off: the same calls staged
    off = make_cases(MAPPED_PAIRS, 70000, [[0, 0, 3]], "devother", "p2p", 400)
    results = run_pes(3, off, tmp_path, extra_env={"SHMEM_DEVICE_SCRATCH_SIZE": "3M", "SHMEM_EXTERNAL_MAP": "0"})
    check(results, off)
    for c in off:
        assert not str(results[0][str(c["id"]) + "_schedule"][0]).startswith("mapped-")
        assert tuple(int(v) for v in results[0]["external_map_stats"]) == (0, 0, 0)


def test_external_buffer_open_failure_stages_the_call(tmp_path):
    """A member that cannot open a peer's exported buffer (simulated on PE 1,
    SHMEM_TEST_IPC_FAIL=extopen; HIP refuses the handle of an allocation its
    owner has freed; profiles/r04/ipc_reopen_probe.json) does not abort the job: after the
    second round of the record exchange every member stages the call, and the
    results stay exact on every PE, fused and multi-launch sizes alike."""
    cases = make_cases(MAPPED_PAIRS, 5000, [[0, 0, 3]], "devother", "p2p", 0)
    cases += make_cases(MAPPED_PAIRS, 200000, [[0, 0, 3]], "devmap_offset", "p2p", 100)
    results = run_pes(3, cases, tmp_path, extra_env={"SHMEM_DEVICE_SCRATCH_SIZE": "3M",
                                                     "SHMEM_TEST_IPC_FAIL": "extopen"})
    check(results, cases)
    for c in cases:
        for pe in range(3):
            assert not str(results[pe][str(c["id"]) + "_schedule"][0]).startswith("mapped-"), (c["id"], pe)


def test_external_buffer_open_failure_recovers(tmp_path):
    """after ONE failed open (SHMEM_TEST_IPC_FAIL=extopen1, PE 1's
    first hipIpcOpenMemHandle) the call stages, every member drops its cached
    exports of the call's buffers, and the next calls on the same buffers map
    again: exactly one staged fallback on every PE, every later call
    "mapped-*", the results exact."""
    cases = make_cases(MAPPED_PAIRS[:4], 5000, [[0, 0, 3]], "devother", "p2p", 0)
    cases += make_cases(MAPPED_PAIRS[:4], 200000, [[0, 0, 3]], "devmap_offset", "p2p", 100)
    results = run_pes(3, cases, tmp_path, extra_env={"SHMEM_DEVICE_SCRATCH_SIZE": "3M",
                                                     "SHMEM_TEST_IPC_FAIL": "extopen1"})
    check(results, cases)
    for pe in range(3):
        assert int(results[pe]["external_map_fallbacks"][0]) == 1, pe
        scheds = [str(results[pe][str(c["id"]) + "_schedule"][0]) for c in cases]
        assert not scheds[0].startswith("mapped-"), scheds[0]
        assert all(s.startswith("mapped-") for s in scheds[1:]), (pe, scheds)
        mapped, opened, closed = (int(v) for v in results[pe]["external_map_stats"])
        assert opened >= 2, (pe, opened)


@pytest.mark.parametrize("npes", [1, 3])
def test_mixed_memory_kinds(tmp_path, npes):
    """Target and source of different kinds on every PE (heap target + host
    source, host target + heap source, host target + hipMalloc source), in
    one and several scratch chunks: staged, every PE's result exact."""
    cases = []
    cid = 0
    for mode in ("mixed_heapdst_hostsrc", "mixed_hostdst_heapsrc", "mixed_hostdst_devsrc"):
        for n in (1, 1000, 300000):
            cases += make_cases([("sum", "double"), ("max", "float"), ("or", "long")], n, [[0, 0, npes]], mode,
                                "p2p", cid)
            cid += 100
    results = run_pes(npes, cases, tmp_path, extra_env={"SHMEM_DEVICE_SCRATCH_SIZE": "3M"})
    check(results, cases)


@pytest.mark.parametrize("npes", [1, 2])
def test_overlapping_buffers_outside_the_heap(tmp_path, npes):
    """Target 5 elements above / below source in host arrays and in hipMalloc
    memory, over several scratch chunks: the result is the fold of the
    original sources (the reference's temporary target, reduce-op.c:174-215),
    whatever order the staging copies run in."""
    cases = []
    cid = 0
    for mode in ("host_overlap_up", "host_overlap_down", "devother_overlap_up", "devother_overlap_down"):
        for n in (1000, 300000):
            cases += make_cases([("sum", "double"), ("max", "int"), ("xor", "short")], n, [[0, 0, npes]], mode,
                                "p2p", cid)
            cid += 100
    results = run_pes(npes, cases, tmp_path, extra_env={"SHMEM_DEVICE_SCRATCH_SIZE": "3M"})
    check(results, cases)


@pytest.mark.parametrize("persistent", ["0", "1"], ids=["launched", "persistent-server"])
def test_random_sequence_stress_outside_heap(tmp_path, persistent):
    """200 back-to-back reductions on buffers outside the heap -- hipMalloc
    memory mapped by the peers (whole, at per-PE offsets, in place, heap
    target, one PE unaligned), host arrays, overlapping targets -- with random
    op/type, size and active set, including two disjoint sets at once: the
    per-call record exchange and the staging paths stay in step; with the
    opt-in persistent server too (heap calls served, the others stop it)."""
    rng = np.random.default_rng(int(os.environ.get("SHMEM_TEST_STRESS_SEED", "2027")))
    sets_choices = [[[0, 0, 4]], [[0, 1, 2], [1, 1, 2]], [[1, 0, 3]], [[0, 0, 2], [2, 0, 2]]]
    modes = ["devother", "devmap_offset", "devmap_inplace", "devmap_symtarget", "devmap_unaligned_pe1", "host",
             "devother_mixed", "host_overlap_up", "devother_overlap_up", "devother_overlap_down", "dev"]
    cases = []
    for cid in range(int(os.environ.get("SHMEM_TEST_STRESS_CALLS", "200"))):
        op, dtype = oracle.PAIRS[rng.integers(len(oracle.PAIRS))]
        n = int(rng.choice([0, 1, 7, 1000, 8192, 40000, 150000, 300000]))
        cases.append({"id": cid, "op": op, "dtype": dtype, "n": n, "sets": sets_choices[rng.integers(4)],
                      "mode": str(rng.choice(modes)), "algorithm": str(rng.choice(["p2p", "p2p", "exact"])),
                      "seed": 9000 + cid})
    results = run_pes(4, cases, tmp_path, extra_env={"SHMEM_DEVICE_HEAP_SIZE": "64M",
                                                     "SHMEM_DEVICE_SCRATCH_SIZE": "3M",
                                                     "SHMEM_DEVICE_ORDER_SIZE": "256K",
                                                     "SHMEM_EXTERNAL_MAP_CACHE": "3",
                                                     "SHMEM_PERSISTENT": persistent})
    check(results, cases)


def test_signal_region_mapping_failure_falls_back(tmp_path):
    """One PE cannot map the peers' signal regions (SHMEM_TEST_IPC_FAIL=sig
    on PE 1): init must not abort; every PE agrees to run without device-side
    flags (no fused kernel, host barriers) and the results stay exact."""
    cases = make_cases(SOME, 1000, [[0, 0, 3]], "dev", "p2p", 0)
    cases += make_cases(SOME[:3], 200000, [[0, 0, 3]], "dev", "p2p", 100)
    results = run_pes(3, cases, tmp_path, extra_env={"SHMEM_TEST_IPC_FAIL": "sig"})
    check(results, cases)


def test_random_sequence_stress(tmp_path):
    """300 back-to-back reductions with random op/type, size (0 .. 300k elements,
    across the fused/multi-launch threshold), buffer mode, schedule and active
    set -- including two disjoint sets running at once -- on 4 PEs. Catches
    races between consecutive calls (a PE racing ahead into the next call)."""
    rng = np.random.default_rng(int(os.environ.get("SHMEM_TEST_STRESS_SEED", "2026")))
    sets_choices = [[[0, 0, 4]], [[0, 1, 2], [1, 1, 2]], [[1, 0, 3]], [[0, 0, 2], [2, 0, 2]], [[0, 0, 4]]]
    cases = []
    for cid in range(int(os.environ.get("SHMEM_TEST_STRESS_CALLS", "300"))):
        op, dtype = oracle.PAIRS[rng.integers(len(oracle.PAIRS))]
        n = int(rng.choice([0, 1, 7, 64, 1000, 8191, 40000, 150000, 300000]))
        mode = str(rng.choice(["dev", "dev", "inplace", "host", "host_mixed"]))
        alg = str(rng.choice(["p2p", "p2p", "p2p", "exact"]))
        sets = sets_choices[rng.integers(len(sets_choices))]
        cases.append({"id": cid, "op": op, "dtype": dtype, "n": n, "sets": sets, "mode": mode,
                      "algorithm": alg, "seed": 7000 + cid})
    # version areas of 128 KiB per channel: order-sensitive calls above ~160 KiB
    # run the multi-launch schedule in several rounds
    results = run_pes(4, cases, tmp_path, extra_env={"SHMEM_DEVICE_HEAP_SIZE": "64M",
                                                     "SHMEM_DEVICE_SCRATCH_SIZE": "3M",
                                                     "SHMEM_DEVICE_ORDER_SIZE": "256K"})
    check(results, cases)


def test_random_sequence_stress_eight_pes(tmp_path):
    """The random sequence on 8 PEs (the driver's largest job size): whole-job
    sets (every-member fold of 8 sources in registers), halves, strided
    quarters (logPE_stride 2: PEs {q, q+4}), a 7-member set starting at PE 1,
    several disjoint sets at once; heap, in place, host and mapped hipMalloc
    buffers; fused one-shot / two-shot, multi-launch (in rounds) and EXACT."""
    rng = np.random.default_rng(int(os.environ.get("SHMEM_TEST_STRESS_SEED", "2028")))
    sets_choices = [[[0, 0, 8]], [[0, 0, 4], [4, 0, 4]], [[0, 2, 2], [1, 2, 2], [2, 2, 2], [3, 2, 2]],
                    [[1, 0, 7]], [[0, 1, 4], [1, 1, 4]], [[0, 0, 8]]]
    cases = []
    for cid in range(int(os.environ.get("SHMEM_TEST_STRESS_CALLS", "120"))):
        op, dtype = oracle.PAIRS[rng.integers(len(oracle.PAIRS))]
        n = int(rng.choice([0, 1, 7, 1000, 8192, 40000, 150000, 300000]))
        cases.append({"id": cid, "op": op, "dtype": dtype, "n": n, "sets": sets_choices[rng.integers(len(sets_choices))],
                      "mode": str(rng.choice(["dev", "dev", "inplace", "host", "devother", "devmap_offset"])),
                      "algorithm": str(rng.choice(["p2p", "p2p", "p2p", "exact"])), "seed": 11000 + cid})
    results = run_pes(8, cases, tmp_path, extra_env={"SHMEM_DEVICE_HEAP_SIZE": "64M",
                                                     "SHMEM_DEVICE_SCRATCH_SIZE": "3M",
                                                     "SHMEM_DEVICE_ORDER_SIZE": "1M"})
    check(results, cases)


# The RCCL schedule (SHMEM_REDUCE_ALGORITHM=rccl, csrc/rccl.c) with more than
# one rank. RCCL refuses two ranks on one GPU of one host ("Duplicate GPU
# detected"), and the test box has one GPU, so each PE announces a host of its
# own (NCCL_HOSTID): RCCL then connects the ranks through its socket network
# transport over loopback instead of xGMI. The transport is not what is under
# test -- the library's glue is: communicator bring-up through the bootstrap
# segment, the type/operator mapping, short widened to int32 and truncated,
# complex sum as 2n reals, staging of host arrays, in place.
RCCL_PAIRS = [("sum", "double"), ("sum", "float"), ("prod", "double"), ("sum", "int"), ("prod", "long"),
              ("max", "longlong"), ("min", "int"), ("sum", "short"), ("prod", "short"), ("max", "short"),
              ("sum", "complexd"), ("sum", "complexf"), ("max", "double"), ("min", "float")]


def rccl_multi_rank(npes, cases, tmp_path):
    per_pe = {pe: {"NCCL_HOSTID": f"shmem-rccl-test-pe{pe}"} for pe in range(npes)}
    return run_pes(npes, cases, tmp_path, per_pe_env=per_pe,
                   extra_env={"NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1", "SHMEM_DEVICE_SCRATCH_SIZE": "3M"})


def check_rccl(results, cases, npes):
    """RCCL's own reduction order: integers bit-exact; at 2 PEs FP sum/prod
    too (a + b and a * b commute in IEEE arithmetic); at 3 PEs FP sums and
    products within DESIGN.md's bounds 2 (N-1) u sum|x_i| and 2 (N-1) u
    |prod x_i| of the reference's result for the PE;
    FP min/max equal as values where no input is NaN (RCCL's NaN and +-0
    selects are not the reference's -- one reason RCCL is opt-in)."""
    for c in cases:
        op, dtype, n = c["op"], c["dtype"], c["n"]
        srcs = [source(op, dtype, n, c["seed"], pe) for pe in range(npes)]
        for pe in range(npes):
            got = results[pe][str(c["id"])]
            want = oracle.reduce_pe(op, dtype, srcs, pe)
            ctx = f"rccl case {c['id']} {c['mode']} PE {pe}:"
            fp = dtype in ("float", "double", "complexf", "complexd")
            if not fp or (op in ("sum", "prod") and npes == 2):
                assert_match(got, want, op, dtype, ctx=ctx)
                continue
            x = np.stack(srcs)
            if op in ("min", "max"):
                ok = ~np.isnan(x).any(axis=0)
                assert (got[ok] == want[ok]).all(), f"{ctx} {op}/{dtype} differs from the reference's value"
                continue
            g, w, xs = (np.asarray(a).astype(np.complex128 if dtype.startswith("complex") else np.float64)
                        for a in (got, want, x))
            u = 2.0 ** -53 if dtype in ("double", "complexd") else 2.0 ** -24
            tiny = np.finfo(np.float64 if dtype in ("double", "complexd") else np.float32).tiny
            parts = (xs.real, xs.imag) if dtype.startswith("complex") else (xs,)
            # subnormal inputs round relative to the subnormal grid, not to u
            normal = np.logical_and.reduce([((np.abs(q) >= tiny) | (q == 0)).all(axis=0) for q in parts])
            with np.errstate(all="ignore"):
                fin = np.isfinite(xs).all(axis=0) & np.isfinite(g) & np.isfinite(w) & normal
                mag = np.abs(xs).sum(axis=0) if op == "sum" else np.abs(np.prod(xs, axis=0))
                bound = 2 * (npes - 1) * u * mag * (2 if dtype.startswith("complex") else 1)
                err = np.abs(g - w)
            bad = np.nonzero(fin & (err != 0) & ~(err <= bound))[0]  # a NaN bound: Inf x 0 among the inputs
            assert len(bad) == 0, (f"{ctx} {op}/{dtype}: {len(bad)} elements above the stated bound; first at "
                                   f"{bad[0]}: got {g[bad[0]]!r} want {w[bad[0]]!r} inputs {xs[:, bad[0]]!r}")


@pytest.mark.parametrize("npes", [2, 3])
def test_rccl_schedule_multi_rank(tmp_path, npes):
    cases = make_cases(RCCL_PAIRS, 4099, [[0, 0, npes]], "dev", "rccl", 0)
    cases += make_cases(RCCL_PAIRS, 1001, [[0, 0, npes]], "inplace", "rccl", 100)
    cases += make_cases(RCCL_PAIRS[:4] + [("sum", "short")], 100000, [[0, 0, npes]], "host", "rccl", 200)
    # pairs RCCL does not have, and a sub-set of the PEs: the P2P schedule
    cases += make_cases([("xor", "int"), ("prod", "complexd")], 515, [[0, 0, npes]], "dev", "rccl", 300)
    cases += make_cases([("sum", "double")], 515, [[0, 0, npes - 1]], "dev", "rccl", 400)
    results = rccl_multi_rank(npes, cases, tmp_path)
    check_rccl(results, cases[:-3], npes)
    check(results, cases[-3:])


def test_peer_heap_mapping_failure_runs_rccl_pairs(tmp_path):
    """One PE cannot map the peers' heaps (SHMEM_TEST_IPC_FAIL=heap on PE 1):
    every PE agrees at init that the P2P schedules cannot run, and the pairs
    RCCL has then go through RCCL whatever schedule is selected (here the
    default) -- with RCCL's own order, as test_rccl_schedule_multi_rank."""
    cases = make_cases(RCCL_PAIRS, 4099, [[0, 0, 3]], "dev", "auto", 0)
    cases += make_cases(RCCL_PAIRS[:4], 100000, [[0, 0, 3]], "host", "auto", 100)
    per_pe = {pe: {"NCCL_HOSTID": f"shmem-rccl-test-pe{pe}"} for pe in range(3)}
    results = run_pes(3, cases, tmp_path, per_pe_env=per_pe,
                      extra_env={"NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1", "SHMEM_TEST_IPC_FAIL": "heap",
                                 "SHMEM_DEVICE_SCRATCH_SIZE": "3M"})
    check_rccl(results, cases, 3)


def test_peer_heap_mapping_failure_other_pairs_abort_cleanly(tmp_path):
    """With the peers' heaps unmapped (SHMEM_TEST_IPC_FAIL=heap on PE 1), a
    pair RCCL does not have (int xor), small or large, device or host arrays,
    must end the job with the library's message on every PE -- no PE may take
    a kernel path that reads a peer's heap."""
    for n, mode in ((16, "dev"), (16, "host"), (300000, "dev")):
        env = dict(os.environ, SHMEM_NPES="3", SHMEM_JOB_ID=uuid.uuid4().hex[:12], SHMEM_DEVICE="0",
                   SHMEM_DEVICE_HEAP_SIZE="32M", SHMEM_DEVICE_SCRATCH_SIZE="3M", SHMEM_BARRIER_TIMEOUT="60",
                   SHMEM_TEST_IPC_FAIL="heap", NCCL_SOCKET_IFNAME="lo", NCCL_IB_DISABLE="1")
        code = ("import sys,os; sys.path[:0]=[%r,%r]\n" % (HERE, os.path.join(os.path.dirname(HERE), "osss-gasnet_amd")) +
                "import numpy as np, shmem_reduce\nshm=shmem_reduce.Shmem(); shm.init()\n"
                f"n={n}\n"
                + ("d=shm.malloc_device(8*n); s=d\n" if mode == "dev" else
                   "a=np.ones(n,dtype=np.int32); d=a.ctypes.data; s=d\n") +
                "shm.to_all('xor','int',d,s,n,0,0,3)\nprint('CALL-RETURNED', flush=True)\nshm.finalize()\n")
        procs = [subprocess.Popen([sys.executable, "-c", code],
                                  env=dict(env, SHMEM_PE=str(pe), NCCL_HOSTID=f"shmem-rccl-test-pe{pe}"),
                                  stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True) for pe in range(3)]
        outs = [p.communicate(timeout=120)[0] for p in procs]
        for p, out in zip(procs, outs):
            assert p.returncode != 0 and "CALL-RETURNED" not in out, out[-2000:]
        assert any("only the RCCL pairs" in o for o in outs), outs

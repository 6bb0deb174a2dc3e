"""GPU: bench.py's contract with the driver, on a short run -- exactly one
JSON line on stdout (rank 0), the metric/config of BASELINE.json, a bit-exact
check, and the roofline / cpu_baseline / op_coverage records. The N = 2 run
shares the one test GPU and forces the RCCL comparison, which then fails
(RCCL refuses two ranks on one device): the line must still come out, with
the comparison marked as skipped and the target re-checked on the default
schedule. At N = 2 the line must also carry the same-run CPU baseline (2
cores), the roofline of the kernel the library's trace says it ran, with the
bytes recomputed from that schedule, the opt-in persistent leg and the
coherence self-test."""
import json
import os
import re
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu
METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run(cmd, timeout=240, env=None):
    # the bench sizes its own device heap (the in-process tests' fixture sets a small one in os.environ)
    # and calibrates its thresholds at init as the driver's run does
    env = {k: v for k, v in (env or os.environ).items()
           if k not in ("SHMEM_DEVICE_HEAP_SIZE", "SHMEM_DEVICE_SCRATCH_SIZE", "SHMEM_THRESHOLD_CALIBRATE")}
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def fractions(d, path=""):
    """Every roofline fraction the line prints: (path, value) for keys named
    frac / *_frac / frac_* (the VALU-floor ratio and the PCIe ratio are
    bounded separately)."""
    if isinstance(d, dict):
        for k, v in d.items():
            p = f"{path}.{k}"
            if (k == "frac" or k.endswith("_frac") or k.startswith("frac_")) and k not in ("valu_frac", "pcie_frac"):
                yield p, v
            else:
                yield from fractions(v, p)
    elif isinstance(d, list):
        for i, v in enumerate(d):
            yield from fractions(v, f"{path}[{i}]")


def common(d, n):
    # no fraction of a roofline above 1 anywhere in the line (a bound the run
    # exceeded is reported as refuted or not applicable, never as a fraction > 1)
    fr = list(fractions(d))
    assert fr and all(v is None or (isinstance(v, (int, float)) and 0 < v <= 1.0) for _, v in fr), \
        [x for x in fr if x[1] is not None and not 0 < x[1] <= 1.0]
    assert "legs_s" in d and d["legs_s"]["total_before_print"] > 0, d.get("legs_s")
    pc = d["per_call"]
    assert 0 < pc["p10_us"] <= pc["median_us"] <= pc["p90_us"] <= pc["max_us"] and pc["calls"] == d["steps"], pc
    assert d["small_call"]["per_call"]["median_us"] > 0, d["small_call"]
    assert d["metric"] == METRIC and d["unit"] == "GiB/s" and d["n_gpus"] == n
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["check"].startswith("bit-exact"), d["check"]
    r = d["roofline"]
    if n == 1:
        assert r["bound"] == "hbm" and r["peak"] == 8000.0 and 0 < r["frac"] <= 1.0 and r["achieved"] > 0
    else:
        # N > 1: the reduce-scatter fold's remote reads against the links into the GPU; here
        # (PEs sharing the test GPU) its local-HBM view, the link view kept aside
        assert r["xgmi_view"] is None and "not applicable" in r["xgmi_view_note"], r
        assert r["bound"] == "hbm" and r["peak"] == 8000.0 and 0 < r["frac"] <= 1.0
        assert 0 < r["per_launch_frac"] <= 1.0, r
    # every element of every PE's target, headline and both op-coverage calls
    assert d["check"].startswith("bit-exact, every element, every PE"), d["check"]
    assert len(d["target_sha256_pe0"]) == 16, d["target_sha256_pe0"]
    for name in ("float_max", "longlong_and"):
        assert d["op_coverage"][name]["check"].startswith("bit-exact, every element, every PE"), d["op_coverage"]
    # BASELINE config 1's call through the library, host and device heap, beside the CPU's
    c1 = d["config1_call"]
    for kind in ("host_heap", "device_heap"):
        assert c1[kind]["check"].startswith("bit-exact") and c1[kind]["us_per_call"] > 0, c1
    assert c1["cpu_us_per_call"] is None or c1["cpu_us_per_call"] > 0, c1
    assert d["small_call"]["us_per_call"] > 0
    g = d["small_call_graph"]
    assert g["us_per_call"] > 0 and g["check"].startswith("bit-exact") and g["calls"] == 4096, g
    assert g["schedule"] == ("stream-identity" if n == 1 else "stream-fused-oneshot"), g


def test_bench_one_gpu_line():
    d = run([sys.executable, "bench.py", "--steps", "5", "--warmup", "2", "--cpu-seconds", "1", "--kernel-reps", "5"])
    common(d, 1)
    cb = d["cpu_baseline"]
    # the headline's shape: 1 PE on 1 core; the other PE counts as sub-records
    assert cb["kind"] == "port" and cb["cores"] == 1 and cb["value"] > 0 and "one_pe" not in cb
    assert cb["two_pe"]["cores"] == 2 and cb["config1"]["us_per_call"] > 0 and cb["host"]["nproc"] >= 1
    assert d["vs_baseline"] is None and d["vs_cpu_baseline"] > 0
    assert cb["eight_pe"]["cores"] == 8 and cb["eight_pe"]["value"] > 0 and cb["config5"]["us_per_call"] > 0
    assert d["config"]["bytes_per_pe"] == 256 << 20
    r = d["roofline"]
    assert r["kernel"] == "void mi355k::copy_segments<4, 1>(mi355k::SegParams<1>)", r
    assert r["call"]["schedule"] == "identity" and r["alg_bytes_per_launch"] == 2 * (256 << 20), r
    # the HBM-only figure: the same call over disjoint pairs taken in turn, >= 2 GiB of footprint
    hr = d["headline_rotating"]
    assert hr["check"].startswith("bit-exact") and hr["footprint_MiB"] >= 2048 and hr["kernel"] == r["kernel"], hr
    assert 0 < hr["frac"] <= 1.0 and r["hbm_only_frac"] == hr["frac"] and "Infinity Cache" in r["attribution"]
    assert r["hbm_only_kernel_avg_us"] == hr["kernel_avg_us"] and r["call_schedule"] == "identity", r
    # a target one element off the source's 16-byte phase: unaligned-load copy, not 8-byte words
    ot = d["headline_offset_target"]
    assert ot["check"].startswith("bit-exact") and ot["kernel"].startswith("void mi355k::copy_segments_shift"), ot
    assert 0.4 < ot["frac"] <= 1.0 and ot["target_offset_bytes"] == 8, ot
    assert ot["traffic"] is None or ot["traffic_over_alg"] < 1.03, ot   # PMC profile of this build, when committed
    assert d["coherence_selftest"] is None
    # north_star's host-memory rate: page-locked host arrays, staged over PCIe in each call
    hs = d["host_staged"]
    # copy-in and copy-out overlap: a staged call takes less than the two
    # copies one after the other (round 5: 6.2 ms against 9.4; 10.1 ms when the
    # staging streams shared a hardware queue); the rate itself is reported
    assert hs["check"].startswith("bit-exact") and hs["value"] > 0 and 0 < hs["pcie_frac"] < 1.2, hs
    assert hs["ms_per_call"] < 0.9 * hs["serial_copies_ms"] and hs["overlap"] > 1.1, hs
    assert hs["pcie"]["both_GB_s_each_direction"] > 0, hs
    k = d["kernels"]
    for name in ("fold_k2_double_sum", "fold_k8_double_sum", "rs_shard_n8_double_sum", "fold_k8_float_max",
                 "fold_k8_longlong_and", "rs_shard_n8_float_max", "rs_shard_n8_longdouble_sum",
                 "rs_shard_n8_longdouble_prod", "rs_shard_n8_complexf_prod", "rs_shard_n8_longlong_and",
                 "rs_shard_n8_float_max_2mib", "rs_shard_n8_double_sum_8mib", "rs_shard_n8_float_max_nan_rich"):
        assert k[name]["check"].startswith("bit-exact"), (name, k[name])
        assert 0 < k[name]["frac"] <= 1.0 and k[name]["kernel_avg_us"] > 0, (name, k[name])
        assert 0 < k[name]["cold"]["frac"] <= 1.0 and k[name]["cold"]["footprint_MiB"] >= 2048, (name, k[name])
        assert 0 < k[name]["warm_aligned"]["frac"] <= 1.0, (name, k[name])
    # the every-member folds' per-launch fixed cost, fitted from two shard sizes each
    fc = k["fixed_cost_fit"]
    for kn in ("combine_orders_vec<max,float,8>", "combine_orders_vec<sum,double,8>"):
        assert fc[kn]["stream_GB_s"] > 0 and 0 < fc[kn]["stream_frac"] <= 1.0, fc
    # the x87 sum's own roofline: VALU issue, from this build's instruction stream
    ls = k["rs_shard_n8_longdouble_sum"]
    assert ls["bound"] == "valu" and 0.3 < ls["valu_frac"] < 1.05 and ls["valu_per_element_wave"] > 1000, ls
    lp = k["rs_shard_n8_longdouble_prod"]
    assert lp["bound"] in ("valu", "hbm") and 0.3 < lp["valu_frac"] < 1.05 and lp["hbm_floor_us"] > 0, lp
    f = d["fused_same_gpu"]
    assert "error" not in f, f
    for leg in f["legs"].values():
        assert leg["check"].startswith("bit-exact") and leg["us_per_call"] > 0 and leg["kernel_avg_us"] > 0, leg
    fp = d["fused_same_gpu_persistent"]
    assert "error" not in fp, fp
    for leg in fp["legs"].values():
        assert leg["check"].startswith("bit-exact") and leg["us_per_call"] > 0, leg
    sp = d["small_call_persistent"]
    assert sp["us_per_call"] > 0 and sp["served"] >= sp["calls"] - 16 and sp["servers_launched"] >= 1, sp


@pytest.mark.multipe
def test_bench_two_ranks_line_with_failed_rccl_comparison(tmp_path):
    log = tmp_path / "trace.log"
    env = dict(os.environ, SHMEM_LOG_LEVELS="REDUCTION", SHMEM_LOG_FILE=str(log))
    d = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
             "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--steps",
             "5", "--warmup", "2", "--force-rccl-compare", "--cpu-seconds", "2"], env=env)
    common(d, 2)
    assert "error" in d["rccl_compare"], d["rccl_compare"]
    assert d["xgmi"]["busbw_GB_s_per_pe"] > 0
    # the same-run CPU baseline at N = 2: 2 PE processes on 2 pinned cores
    cb = d["cpu_baseline"]
    assert cb["cores"] == 2 and cb["value"] > 0 and cb["kind"] == "port" and cb["host"]["nproc"] >= 2
    # the roofline kernel is the one the library ran: the trace's schedule
    # line for the 256 MiB calls says which fold (a 2-member double sum: each
    # owner folds its shard in its own order, the plain fold with one output,
    # and the other member gathers it NaN-patched -- where both operands are
    # NaNs SSE keeps the first, reduce.c nan_pair)
    S = d["config"]["bytes_per_pe"]
    n = S // 8
    lines = [ln for ln in open(log).read().splitlines() if "schedule:" in ln and f"({n} elements" in ln]
    assert lines, "no schedule trace line for the 256 MiB calls"
    assert all("P2P shards, device barriers, each member's reference order (own-order fold, NaN-patched gather)"
               in ln for ln in lines), lines[:3]
    r = d["roofline"]
    assert re.fullmatch(r"void mi355k::combine_vec<0, double, 2, \d, \d, false>\(mi355k::CombineParams\)", r["kernel"]), r
    shard = S // 2
    assert r["call"]["schedule"] == "p2p" and r["call"]["sources"] == 2 and r["call"]["outputs"] == 1, r
    assert r["alg_bytes_per_launch"] == 3 * shard, r
    # both PEs' folds share this GPU's HBM: the device rate counts both PEs' bytes over the call's
    # wall time (a window holding both launches), so it cannot pass the peak
    assert r["pes_on_gpu"] == 2 and 0 < r["frac"] <= 1.0, r
    assert abs(r["achieved"] - 2 * r["alg_bytes_per_launch"] / (d["ms_per_step"] * 1e-3) / 1e9) < 0.01 * r["achieved"], r
    assert "2 PEs share each GPU" in d["config"]["workload"], d["config"]
    # the opt-in persistent server at N > 1 (a child job of one PE per rank)
    sp = d["small_call_persistent"]
    assert "error" not in sp, sp
    # (a host pause longer than SHMEM_PERSISTENT_IDLE_US lets a server idle out: the next call is launched and
    # restarts it, so a few of the 4096 calls may be launched ones)
    assert sp["opt_in"] and sp["check"].startswith("bit-exact") and sp["served"] >= sp["calls"] - 16, sp
    assert sp["schedule"] == "persistent" and "fused_server<0, double>" in sp["kernel"], sp
    # the init coherence test ran on the real layout (here: one GPU) and passed
    c = d["coherence_selftest"]
    assert c["ran"] and c["passed"], c
    # round 4: the caller's producer path (plain stores in a null-stream kernel), both orderings,
    # all three ways of reading; the fused kernel skips its acquires only with fused_sysload
    pp = c["producer_path"]
    assert pp["ran"] and all(pp[k] for k in ("fused_sysload", "fused_after_acquire", "host_after_acquire")), pp
    assert c["fused_acquires_skipped"] == (c["sysload_fresh"] and pp["fused_sysload"]), c
    # fused vs multi-launch and one-shot vs two-shot per size, schedules as forced, results exact
    ts = d["threshold_sweep"]
    assert ts["check"].startswith("bit-exact") and len(ts["fused_vs_multi_launch"]) == 6, ts
    # the thresholds in force came from shmem_init's measurement on this layout
    cal = ts["calibrated_at_init"]
    assert cal is not None and cal["fused_max"] == ts["defaults"]["fused_max"], ts
    fm = [b for b, f, m in cal["fused_vs_multi_launch_us"]]
    assert cal["fused_max"] == 0 or cal["fused_max"] in fm, cal
    for b, f, m in cal["fused_vs_multi_launch_us"]:
        if b <= cal["fused_max"]:
            assert 0 < f <= m, cal
    for r in ts["fused_vs_multi_launch"]:
        assert r["fused_schedule"].startswith("fused") and r["multi_launch_schedule"] == "p2p", r
    for r in ts["oneshot_vs_twoshot"]:
        assert r["oneshot_schedule"] == "fused-oneshot" and r["twoshot_schedule"] == "fused-twoshot", r
    # broadcast / fcollect beside the reduction
    co = d["collectives"]
    assert co["check"] == "bit-exact on every PE" and co[str(4 << 20)]["fcollect64"]["GB_s_into_each_pe"] > 0, co
    # the fused small calls' results, every element on every PE
    assert d["small_call"]["check"].startswith("bit-exact"), d["small_call"]
    # every leg's wall time, and no optional leg failed
    assert d["legs_s"]["headline"] > 0 and d["legs_s"]["cpu_baseline"] > 0, d["legs_s"]
    assert not any(isinstance(v, dict) and "error" in v and k != "rccl_compare" for k, v in d.items()), d
    # the xGMI legs need one GPU per PE: here they say why they did not run
    assert "not_applicable" in d["xgmi_ceiling"] and "not_applicable" in d["peer_fold_shapes"], d
    assert d["xgmi"]["frac"] is None and d["xgmi"]["frac_one_direction"] is None, d["xgmi"]
    assert d["config1_call"]["layout"].startswith("PEs 0 and 1"), d["config1_call"]
    # the same call on plain hipMalloc buffers: mapped by the peers, not staged
    e = d["external_buffers"]
    assert e["schedule"] == "mapped-p2p" and e["check"].startswith("bit-exact") and e["mappings_opened"] >= 1, e
    assert e["fallbacks"] == 0 and e["over_heap_buffers"] > 0, e
    # PE 0's one-peer-at-a-time get/put rates (local HBM copies on this layout)
    lp = d["link_probe"]
    assert lp["check"] == "bit-exact" and lp["from_pe0"]["1"]["get_GB_s"] > 0 and lp["from_pe0"]["1"]["put_GB_s"] > 0, lp
    assert "share ONE GPU" in lp["note"], lp
    # those three legs ran in the child job (tools/extra_legs.py), before the rank touched the GPU
    assert d["legs_s"]["extra_legs_child"] > 0, d["legs_s"]


@pytest.mark.multipe
def test_bench_line_survives_a_dying_extra_legs_job():
    """The N > 1 legs that had never run with one GPU per PE run in a child
    job (tools/extra_legs.py) so that a fatal error there cannot cost the
    driver its line: with every child PE aborting after init (as a fatal
    library error ends a PE), rank 0 still prints one line, with an error
    entry under exactly those three legs and the headline intact."""
    env = dict(os.environ, SHMEM_TEST_EXTRA_LEGS_ABORT="1")
    d = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
             "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "2", "--steps",
             "5", "--warmup", "2", "--no-cpu-baseline", "--no-small", "--no-ops", "--no-threshold-sweep",
             "--no-rccl-compare"], env=env)
    assert d["value"] > 0 and d["check"].startswith("bit-exact"), d
    legs = ("external_buffers", "link_probe", "collectives", "xgmi_ceiling", "peer_fold_shapes")
    # (--no-small: no config-1 leg either)
    assert d["config1_call"] is None, d["config1_call"]
    for leg in legs:
        assert set(d[leg]) == {"error"} and "child job" in d[leg]["error"], (leg, d[leg])
    assert not any(isinstance(v, dict) and "error" in v for k, v in d.items() if k not in legs), d


@pytest.mark.multipe
def test_bench_xgmi_legs_rehearsal_four_ranks():
    """The legs that only mean something with one GPU per PE -- the measured
    all-peers pull ceiling (xgmi_ceiling) and the every-member fold's launch
    shapes with N-1 peer sources (peer_fold_shapes) -- forced on with four
    ranks sharing the test GPU (--force-xgmi-legs): their code path runs
    (peer mappings, copy kernel, copy engines, the probe library's shapes),
    every variant's outputs equal the library's, and the figures stay out of
    the roofline (a rehearsal, marked so)."""
    d = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "4",
             "--master-addr", "127.0.0.1", "--master-port", str(free_port()), "bench.py", "--gpus", "4", "--steps",
             "5", "--warmup", "2", "--mib", "64", "--force-xgmi-legs", "--no-cpu-baseline", "--no-small", "--no-ops",
             "--no-threshold-sweep", "--no-rccl-compare", "--no-external", "--no-link-probe", "--no-collectives"],
            timeout=400)
    assert d["check"].startswith("bit-exact, every element, every PE"), d["check"]
    xc = d["xgmi_ceiling"]
    assert xc["check"].startswith("bit-exact") and xc["rehearsal_same_gpu"] > 0, xc
    assert xc["kernel_GB_s_into_each_pe"] > 0 and xc["sdma_GB_s_into_each_pe"] > 0, xc
    assert xc["bytes_into_each_pe"] == 3 * ((64 << 20) // 4), xc
    ps = d["peer_fold_shapes"]
    assert ps["rehearsal_same_gpu"] and ps["sources"] == 4 and ps["peer_sources"] == 3, ps
    assert len(ps["rows"]) >= 4 and all(r["same_outputs"] and r["kernel_avg_us"] > 0 for r in ps["rows"]), ps
    # the rehearsal feeds no bound: the roofline stays the shared-GPU HBM view
    assert d["roofline"]["bound"] == "hbm" and d["xgmi"]["peak_measured_GB_s"] is None, d["roofline"]

"""GPU: bench.py's contract with the driver, on a short run -- exactly one
JSON line on stdout (rank 0), the metric/config of BASELINE.json, a bit-exact
check, and the roofline / cpu_baseline / op_coverage records. The N = 2 run
shares the one test GPU and forces the RCCL comparison, which then fails
(RCCL refuses two ranks on one device): the line must still come out, with
the comparison marked as skipped and the target re-checked on the default
schedule."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu
METRIC = json.load(open(os.path.join(ROOT, "BASELINE.json")))["metric"]


def run(cmd, timeout=240):
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout[-3000:]
    return json.loads(lines[0])


def common(d, n):
    assert d["metric"] == METRIC and d["unit"] == "GiB/s" and d["n_gpus"] == n
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["check"].startswith("bit-exact"), d["check"]
    r = d["roofline"]
    if n == 1:
        assert r["bound"] == "hbm" and r["peak"] == 8000.0 and 0 < r["frac"] < 1.2 and r["achieved"] > 0
    else:
        # N > 1: the reduce-scatter fold's remote reads against the links into the GPU
        assert r["bound"] == "xgmi" and r["peak"] == (n - 1) * 153.0 and r["achieved"] > 0
        assert r["alg_bytes_per_launch"] == (n - 1) * (d["config"]["bytes_per_pe"] // n)
        assert r["hbm"]["peak"] == 8000.0 and r["hbm"]["achieved"] > 0
    for name in ("float_max", "longlong_and"):
        assert d["op_coverage"][name]["check"].startswith("bit-exact"), d["op_coverage"]
    assert d["small_call"]["us_per_call"] > 0


def test_bench_one_gpu_line():
    d = run([sys.executable, "bench.py", "--steps", "5", "--warmup", "2", "--cpu-seconds", "1", "--kernel-reps", "5"])
    common(d, 1)
    cb = d["cpu_baseline"]
    assert cb["kind"] == "port" and cb["cores"] == 2 and cb["value"] > 0
    assert cb["one_pe"]["cores"] == 1 and cb["config1"]["us_per_call"] > 0 and cb["host"]["nproc"] >= 1
    assert cb["eight_pe"]["cores"] == 8 and cb["eight_pe"]["value"] > 0 and cb["config5"]["us_per_call"] > 0
    assert d["config"]["bytes_per_pe"] == 256 << 20
    k = d["kernels"]
    for name in ("fold_k2_double_sum", "fold_k8_double_sum", "rs_shard_n8_double_sum", "fold_k8_float_max",
                 "fold_k8_longlong_and", "rs_shard_n8_float_max"):
        assert k[name]["check"].startswith("bit-exact"), (name, k[name])
        assert 0 < k[name]["frac"] < 1.2 and k[name]["kernel_avg_us"] > 0, (name, k[name])
    f = d["fused_same_gpu"]
    assert "error" not in f, f
    for leg in f["legs"].values():
        assert leg["check"].startswith("bit-exact") and leg["us_per_call"] > 0 and leg["kernel_avg_us"] > 0, leg
    fp = d["fused_same_gpu_persistent"]
    assert "error" not in fp, fp
    for leg in fp["legs"].values():
        assert leg["check"].startswith("bit-exact") and leg["us_per_call"] > 0, leg
    sp = d["small_call_persistent"]
    assert sp["us_per_call"] > 0 and sp["served"] >= sp["calls"] - 2 and sp["servers_launched"] >= 1, sp


@pytest.mark.multipe
def test_bench_two_ranks_line_with_failed_rccl_comparison():
    d = run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
             "--master-addr", "127.0.0.1", "--master-port", "29563", "bench.py", "--gpus", "2", "--steps", "5",
             "--warmup", "2", "--force-rccl-compare"])
    common(d, 2)
    assert d["cpu_baseline"] is None and d["small_call_persistent"] is None
    assert "error" in d["rccl_compare"], d["rccl_compare"]
    assert d["xgmi"]["busbw_GB_s_per_pe"] > 0

#!/usr/bin/env python3
"""Run a few reduction cases on N PE processes sharing this GPU (debugging
aid): repro_pes.py NPES 'op,dtype,n,mode[,order]' ... ; prints per case
whether every PE matched the oracle and, on failure, each PE's output tail."""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "osss-gasnet_amd")]
import pathlib  # noqa: E402

from test_gpu_multipe import check, make_cases, run_pes  # noqa: E402

npes = int(sys.argv[1])
cases = []
for k, spec in enumerate(sys.argv[2:]):
    f = spec.split(",")
    cases += make_cases([(f[0], f[1])], int(f[2]), [[0, 0, npes]], f[3], "p2p", 100 * k,
                        order=f[4] if len(f) > 4 else "reference")
env = json.loads(os.environ.get("REPRO_ENV", "{}"))
with tempfile.TemporaryDirectory() as d:
    try:
        res = run_pes(npes, cases, pathlib.Path(d), extra_env=env, timeout=float(os.environ.get("REPRO_TIMEOUT", 120)))
        check(res, cases)
        print("ok", flush=True)
    except AssertionError as e:
        print("FAILED", str(e)[-4000:], flush=True)
        sys.exit(1)

#!/usr/bin/env python3
"""The reference algorithm (restated in C, oracle/reduce_oracle.c) timed on the
host: npes forked processes, shared-memory transport (shmem_getmem = memcpy
from the peer's source, shmem_barrier = process-shared pthread barrier), one
PE per process. Median per call, max over PEs. Prints one JSON line per case.
Configs from BASELINE.md section 3 (double sum at 256 MiB and 64 KiB, 1/2/8 PEs).
"""
import json
import os
import platform
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle  # noqa: E402


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


for npes, nbytes, warm, reps in [(1, 256 << 20, 2, 10), (2, 256 << 20, 1, 5), (8, 256 << 20, 1, 3),
                                 (2, 4096, 50, 2000), (8, 64 << 10, 20, 500)]:
    n = nbytes // 8
    t = oracle.cpu_baseline_double_sum(npes, n, warm, reps)
    print(json.dumps({"npes": npes, "bytes_per_pe": nbytes, "s_per_call": t,
                      "gib_s_per_pe": nbytes / t / 2**30, "gib_s_total": npes * nbytes / t / 2**30,
                      "reps": reps, "nproc": os.cpu_count(), "cpu": cpu_model()}), flush=True)

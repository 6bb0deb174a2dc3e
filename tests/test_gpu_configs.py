"""GPU: the BASELINE.json configs at their full sizes, as parity cases.

Inputs follow SURVEY.md §8(d) (tests/_configs.py); PEs share this box's one
GPU (8 PE processes for the 8-GPU configs: same kernels and IPC mappings,
without xGMI). Every PE's whole target is compared with the oracle's result
for THAT PE (the reference's own-source-first order, which the default result
order delivers) through a SHA-256 of its bytes, with a strided sample kept for
diagnostics.
"""
import numpy as np
import pytest

import _configs
import oracle
from test_gpu_multipe import run_pes

pytestmark = [pytest.mark.gpu, pytest.mark.multipe]


def want_digest(config, n, npes, slot=0, pe=0):
    op, dtype = _configs.CONFIGS[config]
    srcs = [_configs.source(config, n, p, slot) for p in range(npes)]
    return _configs.digest(oracle.reduce_pe(op, dtype, srcs, pe))


def check(results, c, npes):
    for k in range(c.get("slots", 1)):
        for pe in range(npes):
            h, sample = want_digest(c["config"], c["n"], npes, k, pe)
            got_h = bytes(results[pe][f"{c['id']}_{k}_sha"]).hex()
            if got_h != h:
                got = results[pe][f"{c['id']}_{k}_sample"]
                nbad = int((got.view(np.uint8).reshape(len(got), -1) !=
                            sample.view(np.uint8).reshape(len(sample), -1)).any(axis=1).sum())
                raise AssertionError(f"{c['config']} slot {k} PE {pe}: digest differs from the oracle "
                                     f"({nbad} of {len(sample)} sampled elements differ)")


def test_config1_int_sum_2pes(tmp_path):
    c = {"id": 0, "kind": "config", "config": "c1", "n": 1024, "calls": 3}
    results = run_pes(2, [c], tmp_path)
    check(results, c, 2)


def test_config3_double_sum_256mib_8pes(tmp_path):
    c = {"id": 0, "kind": "config", "config": "c3", "n": 1 << 25}
    results = run_pes(8, [c], tmp_path, extra_env={"SHMEM_DEVICE_HEAP_SIZE": "640M",
                                                   "SHMEM_DEVICE_SCRATCH_SIZE": "3M"})
    check(results, c, 8)


def test_config4_float_max_and_longlong_and_64mib_8pes(tmp_path):
    cases = [{"id": 0, "kind": "config", "config": "c4f", "n": 1 << 24},
             {"id": 1, "kind": "config", "config": "c4l", "n": 1 << 23}]
    results = run_pes(8, cases, tmp_path, extra_env={"SHMEM_DEVICE_HEAP_SIZE": "256M",
                                                     "SHMEM_DEVICE_SCRATCH_SIZE": "3M"})
    for c in cases:
        check(results, c, 8)


def test_config5_4096_calls_of_64kib_8pes(tmp_path):
    """4096 calls of 64 KiB back to back on 8 PEs (fused one-launch path),
    cycling over 8 distinct source/target pairs."""
    c = {"id": 0, "kind": "config", "config": "c5", "n": 8192, "slots": 8, "calls": 4096}
    results = run_pes(8, [c], tmp_path, extra_env={"SHMEM_DEVICE_SCRATCH_SIZE": "3M"})
    check(results, c, 8)

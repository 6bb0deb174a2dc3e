"""CPU: bench.py's child jobs turn a failing child into "error" entries of
the line instead of ending the bench rank. Here there is no GPU, so the
child PE's shmem_init fails: that is the failure being reported."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_extra_legs_child_failure_becomes_error_entries(monkeypatch):
    monkeypatch.setenv("SHMEM_BOOTSTRAP_TIMEOUT", "5")
    d = bench.extra_legs_child(0, 1, 1, 2, "auto", ["--no-link-probe"])
    assert set(d) == {"external_buffers", "collectives", "xgmi_ceiling", "peer_fold_shapes", "config1_call"}, d
    for k, v in d.items():
        assert set(v) == {"error"} and "child job" in v["error"], (k, v)


def test_extra_legs_child_nothing_to_run():
    assert bench.extra_legs_child(0, 2, 1, 2, "auto", ["--no-external", "--no-link-probe", "--no-collectives",
                                                        "--no-xgmi-legs", "--no-config1"]) == {}

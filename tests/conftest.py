"""Test configuration.

Markers:
  gpu  -- needs an MI355X (run on the GPU box with `pytest -m gpu`); everything
          else runs on the CPU container (`pytest -m "not gpu"`).
GPU tests that launch several PE processes are ordered first, so they start
before the pytest process itself initialises HIP for the in-process tests.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "osss-gasnet_amd"), os.path.join(ROOT, "oracle"), os.path.dirname(__file__)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (run with -m gpu)")
    config.addinivalue_line("markers", "multipe: spawns several PE processes on the GPU")


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=lambda it: 0 if it.get_closest_marker("multipe") else 1)


_SHM = None

# Up to 12 PE processes share the test GPU. With HIP's default of 4 hardware
# queues each, more than 4 of them exceed what the GPU schedules together and
# the library (runtime.c device_wait_test) would run host barriers instead of
# the device-side waits these tests are meant to cover; 2 queues each keeps up
# to 8 PEs on the device path (the spawned PE processes inherit this).
os.environ.setdefault("GPU_MAX_HW_QUEUES", "2")
# the suite's multi-PE jobs keep the default thresholds (deterministic
# schedules); the init-time calibration is tested on its own
# (test_gpu_checks.py) and runs in the bench lines (test_gpu_bench.py)
os.environ.setdefault("SHMEM_THRESHOLD_CALIBRATE", "0")


@pytest.fixture(scope="session")
def shm():
    """This pytest process as PE 0 of 1 on cuda:0 (initialised once)."""
    global _SHM
    if _SHM is None:
        os.environ.setdefault("SHMEM_DEVICE_HEAP_SIZE", "1600M")
        os.environ.setdefault("SHMEM_DEVICE_SCRATCH_SIZE", "3M")  # small: forces chunked staging
        os.environ.pop("SHMEM_PE", None)
        os.environ.pop("SHMEM_NPES", None)
        import shmem_reduce
        _SHM = shmem_reduce.Shmem()
        _SHM.init()
    yield _SHM

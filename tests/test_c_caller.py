"""C programs build and link against libshmem_reduce.so (CPU) and run on 1
and 3 PEs (GPU): one written against the reference's API, one using the
stream-ordered extension with HIP streams and graphs, and a C++ caller
(std::complex through COMPLEXIFY, long double)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "osss-gasnet_amd", "lib")


def build(tmp_path):
    exe = str(tmp_path / "reduce_example")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "reduce_example.c"), "-L", LIBDIR, "-lshmem_reduce",
                    f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def build_stream(tmp_path):
    exe = str(tmp_path / "stream_example")
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-D__HIP_PLATFORM_AMD__", "-I",
                    os.path.join(ROOT, "include"), "-I", "/opt/rocm/include",
                    os.path.join(ROOT, "examples", "stream_example.c"), "-L", LIBDIR, "-lshmem_reduce",
                    "-L", "/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib",
                    "-o", exe], check=True)
    return exe


def build_cpp(tmp_path):
    exe = str(tmp_path / "reduce_example_cpp")
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "examples", "reduce_example.cpp"), "-L", LIBDIR, "-lshmem_reduce",
                    f"-Wl,-rpath,{LIBDIR}", "-o", exe], check=True)
    return exe


def test_cpp_program_compiles_and_links(tmp_path):
    exe = build_cpp(tmp_path)
    out = subprocess.check_output(["nm", "-u", exe], text=True)
    assert "shmem_complexd_prod_to_all" in out and "shmem_longdouble_sum_to_all" in out


def test_c_stream_program_compiles_and_links(tmp_path):
    exe = build_stream(tmp_path)
    out = subprocess.check_output(["nm", "-u", exe], text=True)
    assert "shmemx_long_sum_to_all_on_stream" in out


def test_c_program_compiles_and_links(tmp_path):
    exe = build(tmp_path)
    out = subprocess.check_output(["nm", "-u", exe], text=True)
    assert "shmem_int_sum_to_all" in out and "shmem_double_max_to_all" in out


def oshrun_module():
    import importlib.machinery
    import importlib.util
    loader = importlib.machinery.SourceFileLoader("oshrun", os.path.join(ROOT, "tools", "oshrun"))
    spec = importlib.util.spec_from_loader("oshrun", loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    return mod


def test_oshrun_hardware_queue_policy():
    """More than 4 PEs on one GPU: at most 16 hardware queues for the job,
    also over the box's preset GPU_MAX_HW_QUEUES=4; opt-out kept."""
    q = oshrun_module().hw_queue_env
    assert q(8, True, {"GPU_MAX_HW_QUEUES": "4"}) == {"GPU_MAX_HW_QUEUES": "2"}
    assert q(8, True, {}) == {"GPU_MAX_HW_QUEUES": "2"}
    assert q(12, True, {}) == {"GPU_MAX_HW_QUEUES": "1"}
    assert q(12, True, {"GPU_MAX_HW_QUEUES": "1"}) == {}
    assert q(4, True, {"GPU_MAX_HW_QUEUES": "4"}) == {}
    assert q(8, False, {"GPU_MAX_HW_QUEUES": "4"}) == {}          # one GPU per PE
    assert q(8, True, {"GPU_MAX_HW_QUEUES": "4", "SHMEM_KEEP_HW_QUEUES": "1"}) == {}


@pytest.mark.gpu
@pytest.mark.multipe
@pytest.mark.parametrize("npes", [1, 3, 8])
def test_c_program_runs(tmp_path, npes):
    """1, 3 and 8 PEs (8: tools/oshrun's hardware-queue cap for PEs sharing the
    one test GPU, over the box's preset GPU_MAX_HW_QUEUES)."""
    exe = build(tmp_path)
    env = dict(os.environ, SHMEM_DEVICE_HEAP_SIZE="16M", SHMEM_DEVICE_SCRATCH_SIZE="3M")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "oshrun"), "-np", str(npes), "--same-device",
                        exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(": ok") == npes, r.stdout


@pytest.mark.gpu
@pytest.mark.multipe
@pytest.mark.parametrize("npes", [1, 3])
def test_c_stream_program_runs(tmp_path, npes):
    exe = build_stream(tmp_path)
    env = dict(os.environ, SHMEM_DEVICE_HEAP_SIZE="16M", SHMEM_DEVICE_SCRATCH_SIZE="3M")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "oshrun"), "-np", str(npes), "--same-device",
                        exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(": ok") == npes, r.stdout


@pytest.mark.gpu
@pytest.mark.multipe
@pytest.mark.parametrize("npes", [1, 3])
def test_cpp_program_runs(tmp_path, npes):
    exe = build_cpp(tmp_path)
    env = dict(os.environ, SHMEM_DEVICE_HEAP_SIZE="16M", SHMEM_DEVICE_SCRATCH_SIZE="3M")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "oshrun"), "-np", str(npes), "--same-device",
                        exe], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count(": ok") == npes, r.stdout

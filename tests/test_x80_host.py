"""CPU: the GPU's x87 long double arithmetic (osss-gasnet_amd/csrc/x80.h, its
fast and general paths) compiled for the host and checked bit for bit against
the host x87's own long double + and * on 8 x 500 000 pairs
(tests/native/x80_host_check.cpp). The GPU-side checks of the same code are
test_gpu_combine.py::test_longdouble_add_mul_paths and
::test_longdouble_random_encodings."""
import os
import platform
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


@pytest.mark.skipif(platform.machine() != "x86_64", reason="needs the x87 long double of x86-64")
def test_x80_matches_host_x87(tmp_path):
    exe = tmp_path / "x80_host_check"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "osss-gasnet_amd", "csrc"),
                           os.path.join(HERE, "native", "x80_host_check.cpp"), "-o", str(exe)])
    out = subprocess.run([str(exe), "500000"], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "4000000 pairs, 0 mismatches" in out.stdout, out.stdout
    assert "compare: 500000 pairs, 0 mismatches" in out.stdout, out.stdout
    assert "general: 500000 pairs, 0 mismatches" in out.stdout, out.stdout

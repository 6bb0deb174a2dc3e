"""Host-code AddressSanitizer + UBSan (GPU ASan is not available on this
pool): the C runtime built instrumented (`make asan`) and driven through
tools/asan_driver.c -- staged host arrays, device symmetric arrays (fused and
multi-launch), in place, overlapping, hipMalloc memory, stream-ordered calls,
a strided set, broadcast/fcollect/collect/put/get -- on 1 and 3 PEs."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "tools", "asan_check.sh")


def test_asan_build(tmp_path):
    subprocess.run([SCRIPT, "build"], check=True, capture_output=True, timeout=600)
    assert os.path.exists(os.path.join(ROOT, "osss-gasnet_amd", "lib", "asan", "asan_driver"))


@pytest.mark.gpu
@pytest.mark.multipe
def test_asan_run_1_and_3_pes():
    subprocess.run([SCRIPT, "build"], check=True, capture_output=True, timeout=600)
    r = subprocess.run([SCRIPT, "run"], capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert out.count(": ok") == 4, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]

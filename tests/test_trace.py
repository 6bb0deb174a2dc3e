"""The trace facility (csrc/trace.c; reference src/utils/trace.c): levels from
SHMEM_LOG_LEVELS, lines appended to SHMEM_LOG_FILE in the reference's
"[elapsed] PE n: LEVEL: message" format; SHMEM_INFO lists the environment.

CPU: PEs brought up without a GPU (SHMEM_BOOTSTRAP_ONLY=1). GPU: the
reduction's own trace lines (buffer kinds, overlap, schedule) on 1 PE.
"""
import os
import re
import subprocess
import sys
import textwrap

import numpy as np
import pytest

from test_bootstrap import spawn

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINE = re.compile(r"^\[\d+\.\d+\s*\] PE (\d+): ([A-Z]+): (.*)$")


def read_lines(path):
    out = []
    for line in open(path).read().splitlines():
        m = LINE.match(line)
        assert m, f"bad trace line: {line!r}"
        out.append((int(m.group(1)), m.group(2), m.group(3)))
    return out


def test_levels_file_and_format(tmp_path):
    log = tmp_path / "trace.log"
    body = """
    p = shm.malloc(4096)
    shm.barrier_all()
    shm.free(p)
    shm.finalize()
    print('ok')
    """
    res = spawn(2, body, tmp_path, extra={"SHMEM_LOG_LEVELS": "memory:barrier", "SHMEM_LOG_FILE": str(log)})
    for rc, out in res:
        assert rc == 0, out
    lines = read_lines(log)
    assert {pe for pe, _, _ in lines} == {0, 1}
    assert {lvl for _, lvl, _ in lines} == {"MEMORY", "BARRIER"}
    for pe in (0, 1):
        msgs = [m for p, lvl, m in lines if p == pe and lvl == "MEMORY"]
        assert any(re.match(r"shmem_malloc\(4096\) = 0x[0-9a-f]+ \(symmetric host heap\)", m) for m in msgs), msgs
        assert sum(1 for p, lvl, m in lines if p == pe and m == "shmem_barrier_all") >= 3


def test_disabled_by_default_and_unknown_names_ignored(tmp_path):
    log = tmp_path / "trace.log"
    res = spawn(1, "shm.finalize()\nprint('ok')\n", tmp_path,
                extra={"SHMEM_LOG_LEVELS": "no_such_level", "SHMEM_LOG_FILE": str(log)})
    assert res[0][0] == 0, res[0][1]
    assert not log.exists() or log.read_text() == ""


def test_info_lists_environment(tmp_path):
    log = tmp_path / "trace.log"
    res = spawn(1, "shm.finalize()\nprint('ok')\n", tmp_path, extra={"SHMEM_INFO": "1", "SHMEM_LOG_FILE": str(log)})
    assert res[0][0] == 0, res[0][1]
    text = log.read_text()
    for var in ("SHMEM_LOG_LEVELS", "SHMEM_REDUCE_ALGORITHM", "SHMEM_DEVICE_HEAP_SIZE", "SHMEM_FUSED_MAX_BYTES"):
        assert var in text, var
    assert all(lvl == "INFO" for _, lvl, _ in read_lines(log))


@pytest.mark.gpu
def test_reduction_trace_one_pe(tmp_path):
    """Buffer kinds, the overlap verdict and the chosen schedule, per call."""
    log = tmp_path / "trace.log"
    code = textwrap.dedent(f"""
        import sys, numpy as np
        sys.path.insert(0, {os.path.join(ROOT, 'osss-gasnet_amd')!r})
        import shmem_reduce
        shm = shmem_reduce.Shmem(); shm.init()
        a, b = shm.malloc_device(8 << 10), shm.malloc_device(8 << 10)
        shm.put(a, np.arange(1024.0))
        shm.to_all("sum", "double", b, a, 1024, 0, 0, 1)
        shm.to_all("sum", "double", a, a, 1024, 0, 0, 1)
        shm.to_all("sum", "double", a + 64, a, 512, 0, 0, 1)
        assert (shm.get(a + 64, 512, "double") == np.arange(512.0)).all()
        shm.finalize()
    """)
    env = dict(os.environ, SHMEM_LOG_LEVELS="reduction,init", SHMEM_LOG_FILE=str(log),
               SHMEM_DEVICE_HEAP_SIZE="64M", SHMEM_DEVICE_SCRATCH_SIZE="3M")
    for k in ("SHMEM_PE", "SHMEM_NPES"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    msgs = [m for _, lvl, m in read_lines(log) if lvl == "REDUCTION"]
    text = "\n".join(msgs)
    assert "shmem_double_sum_to_all: nreduce 1024" in text
    assert "(device heap)" in text
    assert "do not overlap" in text and "are the same buffer" in text and "overlap, using temporary target" in text
    assert "schedule: 1-PE identity, one copy of 8192 bytes" in text
    assert "schedule: 1-PE identity in place" in text
    assert "schedule: overlapping target" in text
    inits = [m for _, lvl, m in read_lines(log) if lvl == "INIT"]
    assert any("PE 0 of 1 on GPU" in m for m in inits), inits

"""The Fortran-callable binding (osss-gasnet_amd/csrc/fortran.c, declared in
include/shmem_fortran.h): reference src/fortran/fortran.c:1218-1256 (37
REDUCIFY wrappers), :95-134 and :636-645 (runtime calls).

CPU: every name is exported, shmem_*_ weak over pshmem_*_ strong, and the set
of (kind, op) pairs is exactly the reference's. GPU (1 PE, in-process): each
wrapper reaches its C entry point with the right element type (identity on a
1-PE set, bit-exact). Multi-PE parity: tests/test_gpu_multipe.py::
test_fortran_binding_three_pes.
"""
import ctypes
import re
import subprocess

import numpy as np
import pytest

import gen_golden
import oracle
import shmem_reduce
from pe_worker import FORTRAN_KIND

# the reference's REDUCIFY list (fortran.c:1218-1256), as (op, kind)
REF_PAIRS = ([(op, k) for op in ("sum", "prod", "max", "min")
              for k in ("int2", "int4", "int8", "real4", "real8", "real16")]
             + [(op, k) for op in ("and", "or", "xor") for k in ("int2", "int4", "int8")]
             + [(op, k) for op in ("sum", "prod") for k in ("comp4", "comp8")])
RUNTIME = ["start_pes_", "shmem_init_", "shmem_finalize_", "shmem_global_exit_", "my_pe_", "num_pes_",
           "shmem_my_pe_", "shmem_n_pes_", "shmem_barrier_all_", "shmem_barrier_", "shmem_quiet_"]


def _nm():
    out = subprocess.check_output(["nm", "-D", "--defined-only", shmem_reduce.LIB_PATH], text=True)
    return {line.split()[-1]: line.split()[-2] for line in out.splitlines() if len(line.split()) >= 2}


def test_fortran_names_exported_weak_over_strong():
    kinds = _nm()
    names = [f"shmem_{k}_{op}_to_all_" for op, k in REF_PAIRS] + RUNTIME
    assert len(REF_PAIRS) == 37
    for n in names:
        assert kinds.get(n) == "W", n
        assert kinds.get("p" + n) == "T", "p" + n


def test_fortran_pairs_match_reference_list():
    kinds = _nm()
    got = sorted(m.groups() for m in (re.match(r"^shmem_(\w+?)_(sum|prod|and|or|xor|max|min)_to_all_$", n)
                                      for n in kinds) if m)
    assert got == sorted((k, op) for op, k in REF_PAIRS)


def test_kind_map_covers_c_pairs():
    """every Fortran pair is a C pair under the kind -> C type map"""
    inv = {v: k for k, v in FORTRAN_KIND.items()}
    for op, k in REF_PAIRS:
        assert (op, inv[k]) in oracle.PAIRS


@pytest.mark.gpu
@pytest.mark.parametrize("op,kind", REF_PAIRS)
def test_fortran_entry_one_pe(shm, op, kind):
    dtype = {v: k for k, v in FORTRAN_KIND.items()}[kind]
    n = 515
    es = np.dtype(oracle.NP[dtype]).itemsize
    x = gen_golden.values(np.random.default_rng(5), op, dtype, n)
    ds, dt = shm.malloc_device(n * es), shm.malloc_device(n * es)
    shm.put(ds, x)
    f = getattr(shm.lib, f"shmem_{kind}_{op}_to_all_")
    f.restype = None
    psync = np.full(shmem_reduce.SHMEM_REDUCE_SYNC_SIZE, -1, dtype=np.int32)
    args = [ctypes.c_int(v) for v in (n, 0, 0, 1)]
    f(ctypes.c_void_p(dt), ctypes.c_void_p(ds), *[ctypes.byref(a) for a in args], None,
      ctypes.c_void_p(psync.ctypes.data))
    got = shm.get(dt, n, dtype)
    assert (oracle.as_value_bytes(got, dtype) == oracle.as_value_bytes(x, dtype)).all()
    assert (psync == -1).all()
    shm.free_device(dt)
    shm.free_device(ds)


def test_fortran_include_constants_match_c_header(tmp_path):
    """include/shmem.fh declares the collectives' work-array sizes in default
    INTEGERs: twice the C header's `long` counts (reference src/shmem.fh:71-95
    against src/shmem.h's values), the same SHMEM_SYNC_VALUE; and every
    statement is valid fixed-form (column 7 on, no continuation)."""
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fh = open(os.path.join(root, "include", "shmem.fh")).read().splitlines()
    vals = {}
    for line in fh:
        if line.startswith("!") or not line.strip():
            continue
        assert line.startswith("      ") and not line[5].strip() and len(line) <= 72, line
        m = re.match(r"\s+parameter \((\w+) = (-?\d+)\)$", line)
        if m:
            vals[m.group(1)] = int(m.group(2))
    names = ["SHMEM_BCAST_SYNC_SIZE", "SHMEM_BARRIER_SYNC_SIZE", "SHMEM_REDUCE_SYNC_SIZE",
             "SHMEM_REDUCE_MIN_WRKDATA_SIZE", "SHMEM_COLLECT_SYNC_SIZE", "SHMEM_SYNC_VALUE"]
    src = tmp_path / "c.c"
    src.write_text('#include <stdio.h>\n#include "shmem.h"\nint main(void){printf("%ld %ld %ld %ld %ld %ld\\n",'
                   + ",".join(f"(long){n}" for n in names) + ");return 0;}\n")
    exe = tmp_path / "c"
    subprocess.check_call(["gcc", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)])
    cvals = [int(x) for x in subprocess.check_output([str(exe)], text=True).split()]
    scale = ctypes.sizeof(ctypes.c_long) // ctypes.sizeof(ctypes.c_int)
    for name, c in zip(names, cvals):
        want = c if name == "SHMEM_SYNC_VALUE" else c * scale
        assert vals[name] == want, (name, vals[name], c)
    assert vals["SHMEM_REDUCE_SYNC_SIZE"] == 256 and vals["SHMEM_REDUCE_MIN_WRKDATA_SIZE"] == 128

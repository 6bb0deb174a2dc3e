"""CPU: the C-ABI library loads and exports every symbol include/*.h declares.

No compute calls here (there is no GPU in the CPU container): only symbol
resolution and the host-only helpers.
"""
import ctypes
import os
import re
import subprocess

import pytest

import shmem_reduce

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = ["shmem.h", "pshmem.h", "shmemx.h", "mi355_reduce.h", "shmem_fortran.h"]


def declared_functions(header):
    text = open(os.path.join(ROOT, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\(", text)
    skip = {"COMPLEXIFY", "sizeof", "defined", "SHMEM_INTERNAL_F2C_SCALE"}
    decl = set()
    for m in re.finditer(r"^\s*(?:void|int|double|size_t|long|void\s*\*)\s*\*?\s*([A-Za-z_][A-Za-z0-9_]*)\s*\(",
                         text, flags=re.M):
        decl.add(m.group(1))
    return sorted(n for n in decl if n not in skip)


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(shmem_reduce.LIB_PATH):
        pytest.fail(f"{shmem_reduce.LIB_PATH} not built (run __graft_entry__.build())")
    return ctypes.CDLL(shmem_reduce.LIB_PATH)


@pytest.mark.parametrize("header", HEADERS)
def test_every_declared_symbol_is_exported(lib, header):
    names = declared_functions(header)
    assert names, header
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, f"{header}: not exported: {missing}"


def test_44_reductions_in_both_namespaces():
    names = declared_functions("shmem.h")
    red = [n for n in names if n.endswith("_to_all")]
    assert len(red) == 44
    pnames = declared_functions("pshmem.h")
    assert sorted("p" + n for n in red) == sorted(n for n in pnames if n.endswith("_to_all"))


def test_shmem_names_are_weak_aliases():
    out = subprocess.check_output(["nm", "-D", shmem_reduce.LIB_PATH], text=True)
    kinds = {line.split()[-1]: line.split()[-2] for line in out.splitlines() if len(line.split()) >= 2}
    assert kinds["shmem_double_sum_to_all"] == "W"
    assert kinds["pshmem_double_sum_to_all"] == "T"
    assert kinds["shmem_init"] == "W"


def test_dtype_sizes_and_op_matrix(lib):
    L = shmem_reduce.load()
    sizes = [L.mi355_dtype_size(i) for i in range(9)]
    assert sizes == [2, 4, 8, 8, 4, 8, 16, 8, 16]
    import oracle
    for op in range(7):
        for t in range(9):
            want = (oracle.OPS[op], oracle.DTYPES[t]) in oracle.PAIRS
            assert bool(L.mi355_op_supported(op, t)) == want


def test_shard_bounds_partition():
    L = shmem_reduce.load()
    for n in [0, 1, 63, 64, 1000, 33554432, 2**31 - 1]:
        for es in [2, 4, 8, 16]:
            for k in [1, 2, 3, 7, 8]:
                prev = 0
                for i in range(k):
                    lo, hi = shmem_reduce.shard_bounds(L, n, es, k, i)
                    assert lo == prev and lo <= hi <= n
                    if lo < n:
                        assert (lo * es) % 256 == 0
                    prev = hi
                assert prev == n


def test_constants_match_reference_values():
    text = open(os.path.join(ROOT, "include", "shmem.h")).read()
    assert "#define SHMEM_REDUCE_SYNC_SIZE          (256L / SHMEM_INTERNAL_F2C_SCALE)" in text
    assert "#define SHMEM_REDUCE_MIN_WRKDATA_SIZE   (128L / SHMEM_INTERNAL_F2C_SCALE)" in text
    assert "#define SHMEM_SYNC_VALUE (-1L)" in text


def test_kernel_code_hash_reads_the_fatbin():
    """bench.py ties PMC traffic to the library's gfx950 code objects
    (shmem_reduce.kernel_code_hash, the .hip_fatbin section): present, and
    the same value on every read."""
    import shmem_reduce
    h = shmem_reduce.kernel_code_hash()
    assert len(h) == 16 and int(h, 16) >= 0 and h == shmem_reduce.kernel_code_hash()

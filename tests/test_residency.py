"""CPU: the build-time co-residency guard (tools/check_residency.py).

The spin-waiting grids (fused.hip) are capped at min(occupancy API,
MI355_FUSED_RESIDENT_PER_CU) - 1 blocks per CU; the API ignores the SGPR
admission limit of 256-thread blocks (MI355X_MICROARCH.md "Residency"), so
the build reads every such kernel's register use from the code object and
fails when the cap could exceed what the hardware admits (the failure would
be a hang, round 2's test_more_than_eight_pes_one_gpu[9])."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "check_residency.py")


def run(obj, header=None):
    cmd = [sys.executable, TOOL, obj] + (["--header", header] if header else [])
    return subprocess.run(cmd, capture_output=True, text=True)


def test_library_spin_kernels_fit_the_grid_cap():
    obj = os.path.join(ROOT, "osss-gasnet_amd", "lib", "fused.o")
    r = run(obj)
    assert r.returncode == 0, r.stdout + r.stderr
    rows = [ln for ln in r.stdout.splitlines() if "fused_" in ln and not ln.startswith("check_residency")]
    # every (op, type) instantiation of the fused kernel and its server, plus fused_pull
    assert sum("fused_allreduce<" in ln for ln in rows) == 37, r.stdout
    assert sum("fused_server<" in ln for ln in rows) == 37, r.stdout
    assert any("fused_pull" in ln for ln in rows)
    for ln in rows:
        admit, planned = (int(x) for x in ln.split()[-2:])
        assert planned <= admit, ln
    # the table the build writes next to the library
    assert os.path.exists(os.path.join(ROOT, "osss-gasnet_amd", "lib", "residency.txt"))


def test_register_heavy_variant_trips_the_check(tmp_path):
    obj = str(tmp_path / "probe.o")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-c",
                    os.path.join(ROOT, "tests", "native", "residency_probe.hip"), "-o", obj], check=True,
                   cwd=str(tmp_path))
    ok = run(obj)  # the library's constant (6): 108 SGPRs still admit 6 blocks
    assert ok.returncode == 0, ok.stdout + ok.stderr
    hdr = tmp_path / "residency.h"
    hdr.write_text("#define MI355_FUSED_RESIDENT_PER_CU 7\n")
    bad = run(obj, str(hdr))
    assert bad.returncode == 1
    fails = [ln for ln in bad.stderr.splitlines() if "FAIL" in ln]
    assert len(fails) == 1 and "fused_allreduce_heavy" in fails[0] and "admits 6" in fails[0], bad.stderr


def test_library_kernels_use_no_scratch():
    """Round 4: no kernel of the library has a private
    segment -- the complex-product fused kernels had 1,264 B per lane (call
    frames of non-inlined helpers), the x87 every-member fold 24 B."""
    lib = os.path.join(ROOT, "osss-gasnet_amd", "lib")
    objs = ["combine.o", "fused.o"] + sorted(f for f in os.listdir(lib) if f.startswith("combine_t_"))
    for o in objs:
        r = subprocess.run([sys.executable, TOOL, "--no-scratch", os.path.join(lib, o)], capture_output=True,
                           text=True)
        assert r.returncode == 0, o + ": " + r.stdout + r.stderr
        assert ", 0 with scratch" in r.stdout, r.stdout


def test_scratch_kernel_trips_the_no_scratch_check(tmp_path):
    obj = str(tmp_path / "scratch_probe.o")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O2", "-c",
                    os.path.join(ROOT, "tests", "native", "scratch_probe.hip"), "-o", obj], check=True,
                   cwd=str(tmp_path))
    r = subprocess.run([sys.executable, TOOL, "--no-scratch", obj], capture_output=True, text=True)
    assert r.returncode == 1
    fails = [ln for ln in r.stderr.splitlines() if "FAIL" in ln]
    assert len(fails) == 1 and "with_scratch" in fails[0], r.stderr

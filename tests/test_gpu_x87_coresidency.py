"""GPU: the x87 long double arithmetic (osss-gasnet_amd/csrc/x80.h, the
reference's reduce-op.c:99,158 long double sum/prod on the 387) in waves that
SHARE a SIMD with other waves -- the condition of round 2's nondeterministic
errors (profiles/r04/x80/).

tools/x80_lane_probe folds three operand arrays, (a op b) op c, with x80.h's
general path in every lane (`general`), the library's per-wave choice between
fast and general paths (`vote`) and a per-lane choice (`lane`), and compares
every element with the host's own x87. Grid 2048 x 256 on 200 000 elements
puts two to four waves on each SIMD; grid 2048 with 96 KiB of dynamic LDS per
block admits one block per CU (every wave alone on its SIMD).

The round-2 header (tools/x80_round2/x80.h, built into x80_lane_probe_r2) is
the control: its general kernels returned wrong x87 products and sums only
in waves that shared a SIMD with an older wave -- never with one block per
CU -- which is what the assertions on today's header rule out. The control's
counts are reported (they depend on the hardware's interleaving, so they are
not asserted)."""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOLS = os.path.join(ROOT, "tools")

pytestmark = pytest.mark.gpu


def probe(binary, grid, lds, kernels):
    exe = os.path.join(TOOLS, binary)
    if not os.path.exists(exe):
        pytest.fail(f"{exe} is not built: run `make -C tools x80probes` (__graft_entry__.build())")
    r = subprocess.run([exe, "200000", "2", str(grid), "none", kernels, "-", str(lds)], capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    counts = {}
    for op in ("add", "mul"):
        m = re.search(r"^  %s: (.*)$" % op, r.stdout, re.M)
        assert m, r.stdout[-2000:]
        for k, bad, first in re.findall(r"(\w+) (\d+)/(\d+)", m.group(1)):
            counts[(op, k)] = int(bad)
    return counts, r.stdout


@pytest.mark.parametrize("grid,lds", [(2048, 0), (512, 0), (2048, 98304)],
                         ids=["waves-share-simds", "two-blocks-per-cu", "one-block-per-cu"])
def test_x87_general_paths_exact_when_waves_share_a_simd(grid, lds):
    counts, out = probe("x80_lane_probe_now", grid, lds, "gvl")
    control = None
    if os.path.exists(os.path.join(TOOLS, "x80_lane_probe_r2")):
        control, _ = probe("x80_lane_probe_r2", grid, lds, "g")
    bad = {k: v for k, v in counts.items() if v}
    assert not bad, f"today's x80.h differs from the host x87 (grid {grid}, LDS {lds}): {bad}; " \
                    f"round-2 control: {control}\n{out[-1500:]}"
    print(f"grid {grid} LDS {lds}: today's header 0 mismatches in {sorted(counts)}; "
          f"round-2 control (general kernels): {control}")

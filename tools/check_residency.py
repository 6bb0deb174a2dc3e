#!/usr/bin/env python3
"""Build-time guard for the co-residency of the spin-waiting grids.

Every block of a fused_allreduce / fused_server / fused_pull grid waits for
the others (fused.hip), so a launch is capped at
min(occupancy API, MI355_FUSED_RESIDENT_PER_CU) - 1 blocks per CU
(coresident_grid, csrc/residency.h). The occupancy API ignores the SGPR
admission limit of 256-thread blocks, floor(800 / (ceil(sgpr/16)*16 + 16))
per CU (MI355X_MICROARCH.md "Residency"); a kernel that grows past it would
make the cap too high, and the symptom is a hang, not an error. This reads
the compiled code object's kernel metadata (.sgpr_count, .vgpr_count,
.agpr_count, LDS bytes), prints the per-kernel admission table and exits 1
when, for any matched kernel, the blocks per CU the runtime may plan --
min(constant, the occupancy API's view: VGPRs, LDS, 8) -- exceed what the
hardware admits (the same, and the SGPR limit).

usage: check_residency.py OBJECT [--header residency.h] [--kernels REGEX] [--quiet]
       check_residency.py --no-scratch OBJECT
OBJECT: a hipcc -c output (its .hip_fatbin section is unbundled) or a code object.

--no-scratch (round 4): every kernel of OBJECT must have a private segment of
0 bytes and no dynamic stack -- no scratch memory per lane. Scratch in a
kernel with several blocks per CU was the suspect of round 2's x87 errors
(the probe of profiles/r04 ruled it out there), and in the
spin-waiting grids it is a cost on every launch: the 1,264 bytes per lane of
the complex-product fused kernels were the call frames of non-inlined
helpers, the 24 bytes of the x87 every-member fold a copy of the kernel
arguments' pointer array indexed by a rolled loop. A kernel that must keep
scratch is listed in SCRATCH_ALLOWED with its reason.
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
MAX_PER_CU = 8           # blocks of 256 threads per CU (MI355X_MICROARCH.md)
VGPRS_PER_LANE = 512     # per SIMD, unified VGPR + AGPR budget (gfx950)
LDS_PER_CU = 160 * 1024


def code_object(path, tmp):
    """The gfx950 code object inside a hipcc object file (or the file itself)."""
    with open(path, "rb") as f:
        if f.read(4) != b"\x7fELF":
            sys.exit(f"{path}: not an ELF file")
    fat = os.path.join(tmp, "fatbin")
    r = subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", path,
                        os.path.join(tmp, "stripped.o")], capture_output=True, text=True)
    if r.returncode != 0:
        return path  # no fat binary section: already a device code object
    co = os.path.join(tmp, "device.co")
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    f"--targets={TARGET}", f"--output={co}"], check=True)
    return co


def kernels(co):
    """Kernel records of amdhsa.kernels: an entry starts at '  - .key:', its
    fields sit at four spaces ('    .key: value'); deeper lines are .args."""
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True,
                           check=True).stdout
    out, cur, inside = [], None, False
    for line in notes.splitlines():
        if line.startswith("amdhsa.kernels:"):
            inside = True
            continue
        if inside and line and not line.startswith(" "):
            inside = False
        if not inside:
            continue
        if line.startswith("  - ."):
            cur = {}
            out.append(cur)
            line = "    " + line[4:]
        m = re.match(r"^ {4}\.(\w+):\s*(\S+)$", line)
        if m and cur is not None:
            cur[m.group(1)] = m.group(2)
    return [k for k in out if "name" in k and "sgpr_count" in k]


def demangle(names):
    """c++filt (binutils; the ROCm image has no llvm-cxxfilt); the mangled names if it is missing"""
    try:
        r = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True)
    except OSError:
        return names
    out = r.stdout.splitlines()
    return out if r.returncode == 0 and len(out) == len(names) else names


def admitted(k):
    sgpr = int(k["sgpr_count"])
    vgpr = int(k.get("vgpr_count", 0)) + int(k.get("agpr_count", 0))
    lds = int(k.get("group_segment_fixed_size", 0))
    by_sgpr = 800 // ((sgpr + 15) // 16 * 16 + 16)
    by_vgpr = VGPRS_PER_LANE // max(8, (vgpr + 7) // 8 * 8)   # waves per SIMD = blocks per CU
    by_lds = LDS_PER_CU // lds if lds else MAX_PER_CU
    return min(MAX_PER_CU, by_sgpr, by_vgpr, by_lds), by_sgpr, by_vgpr, by_lds


SCRATCH_ALLOWED = {}   # demangled-name regex -> why the scratch is needed (none today)


def no_scratch(path):
    with tempfile.TemporaryDirectory() as tmp:
        ks = kernels(code_object(path, tmp))
    names = demangle([k["name"] for k in ks])
    bad = []
    for k, dn in zip(ks, names):
        ps = int(k.get("private_segment_fixed_size", 0))
        dyn = k.get("uses_dynamic_stack", "false") == "true"
        if (ps or dyn) and not any(re.search(rx, dn) for rx in SCRATCH_ALLOWED):
            bad.append((dn, ps, dyn))
    for dn, ps, dyn in bad:
        print(f"check_residency: FAIL {dn}: {ps} bytes of scratch per lane{' + a dynamic stack' if dyn else ''} "
              f"(private_segment_fixed_size); inline the callees / index register arrays with constants, or "
              f"justify it in SCRATCH_ALLOWED", file=sys.stderr)
    print(f"check_residency --no-scratch: {len(ks)} kernels in {os.path.basename(path)}, {len(bad)} with scratch")
    return 1 if bad else 0


def header_constant(path):
    m = re.search(r"#define\s+MI355_FUSED_RESIDENT_PER_CU\s+(\d+)", open(path).read())
    if not m:
        sys.exit(f"{path}: MI355_FUSED_RESIDENT_PER_CU not found")
    return int(m.group(1))


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--no-scratch":
        sys.exit(no_scratch(sys.argv[2]))
    here = os.path.dirname(os.path.abspath(__file__))
    ap = argparse.ArgumentParser()
    ap.add_argument("object")
    ap.add_argument("--header", default=os.path.join(here, "..", "osss-gasnet_amd", "csrc", "residency.h"))
    ap.add_argument("--kernels", default=r"fused_allreduce|fused_server|fused_pull")
    ap.add_argument("--quiet", action="store_true", help="print only violations and the summary")
    args = ap.parse_args()
    need = header_constant(args.header)
    with tempfile.TemporaryDirectory() as tmp:
        ks = kernels(code_object(args.object, tmp))
    names = demangle([k["name"] for k in ks])
    rows, bad = [], []
    for k, dn in zip(ks, names):
        if not re.search(args.kernels, dn):
            continue
        adm, s_, v_, l_ = admitted(k)
        planned = min(need, MAX_PER_CU, v_, l_)   # coresident_grid before its margin of one
        row = (dn, int(k["sgpr_count"]), int(k.get("vgpr_count", 0)) + int(k.get("agpr_count", 0)),
               int(k.get("group_segment_fixed_size", 0)), s_, v_, l_, adm, planned)
        rows.append(row)
        if planned > adm:
            bad.append(row)
    if not rows:
        sys.exit(f"check_residency: no kernel matching /{args.kernels}/ in {args.object}")
    fmt = "{:<72} {:>5} {:>5} {:>6} {:>7} {:>7} {:>6} {:>6} {:>7}"
    if not args.quiet:
        print(fmt.format("kernel", "sgpr", "vgpr", "lds", "by_sgpr", "by_vgpr", "by_lds", "admit", "planned"))
        for r in rows:
            print(fmt.format(r[0][:72], *r[1:]))
    slack = min(r[7] - r[8] for r in rows)
    print(f"check_residency: {len(rows)} spin-waiting kernels, MI355_FUSED_RESIDENT_PER_CU = {need}; "
          f"least slack between blocks admitted and planned per CU: {slack} (256-thread blocks per CU = "
          f"min(8, floor(800 / (ceil(sgpr/16)*16 + 16)), VGPR, LDS), MI355X_MICROARCH.md)")
    if bad:
        for r in bad:
            print(f"check_residency: FAIL {r[0]}: {r[1]} SGPRs / {r[2]} VGPRs / {r[3]} B LDS: the hardware admits "
                  f"{r[7]} blocks per CU, coresident_grid would plan {r[8]} (MI355_FUSED_RESIDENT_PER_CU = {need}): "
                  f"its grids could not all be resident (a hang); lower the constant in residency.h or the "
                  f"kernel's SGPR use", file=sys.stderr)
        sys.exit(1)


if __name__ == "__main__":
    main()

#!/usr/bin/env python3
"""Turn two rocprofv3 --pmc runs (FETCH_SIZE pass, WRITE_SIZE pass) into HBM
bytes per launch of the bench's dominant kernel, with the gfx950 correction
of MI355X_MICROARCH.md (HBM section): FETCH_SIZE counts half the bytes of a
wide (16 B/lane) coalesced streaming read, so it is doubled; WRITE_SIZE is
exact for 16-B streaming stores. Both counters are in KB (1024 B). Each
entry records the hash of the gfx950 code objects it was taken from
(shmem_reduce.kernel_code_hash): bench.py reports an entry's traffic only
for a library with the same machine code.

usage: pmc_traffic.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR MIN_GRID[:MAX_GRID][@MIN_B:MAX_B] KEY [out.json]
(grid in threads: launches of one kernel at different sizes told apart; a
kernel launched with one grid at several sizes is told apart by @MIN_B:MAX_B,
the dispatch's own bytes in each pass -- FETCH_SIZE doubled, WRITE_SIZE)
"""
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "osss-gasnet_amd"))
import shmem_reduce  # noqa: E402  (kernel_code_hash only; the library is read, not loaded)


def per_dispatch(d, counter, kname, min_grid, max_grid=1 << 62):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
            if kname in r["Kernel_Name"] and min_grid <= grid <= max_grid and r["Counter_Name"] == counter:
                key = r["Dispatch_Id"]
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def in_bytes(vals, scale, brange):
    """Dispatches whose counter, as bytes (x scale), lies in brange."""
    return [v for v in vals if brange[0] <= v * scale <= brange[1]]


def main():
    fdir, wdir, kname, grid, key = sys.argv[1:6]
    out = sys.argv[6] if len(sys.argv) > 6 else None
    grid, _, bsel = grid.partition("@")
    lo, _, hi = grid.partition(":")
    rng = (int(lo), int(hi) if hi else 1 << 62)
    f = per_dispatch(fdir, "FETCH_SIZE", kname, *rng)
    w = per_dispatch(wdir, "WRITE_SIZE", kname, *rng)
    if bsel:
        blo, _, bhi = bsel.partition(":")
        brange = (int(blo), int(bhi) if bhi else 1 << 62)
        f = in_bytes(f, 2 * 1024, brange)
        w = in_bytes(w, 1024, brange)
    if not f or not w:
        sys.exit(f"no dispatches of {kname}: fetch {len(f)} write {len(w)}")
    fetch = sorted(f)[len(f) // 2] * 1024
    write = sorted(w)[len(w) // 2] * 1024
    res = {"fetch_size_bytes_raw": fetch, "write_size_bytes": write,
           "hbm_bytes_per_launch": 2 * fetch + write,
           "kernel_code_sha": shmem_reduce.kernel_code_hash(),
           "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), median of {len(f)}/{len(w)} "
                     f"dispatches of {kname}; FETCH_SIZE x2 (gfx950 wide-read correction)"}
    print(json.dumps({key: res}, indent=1))
    if out:
        data = json.load(open(out)) if os.path.exists(out) else {}
        data[key] = res
        json.dump(data, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()

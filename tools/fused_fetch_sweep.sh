#!/bin/bash
# Where the fused one-shot's extra fetch bytes come from: two PE
# processes of tools/fused_bench.py on the GPU, one-shot calls of 8/16/32/64 KiB
# (grids of 2/4/8/16 blocks), PE 0 under rocprofv3: FETCH_SIZE and
# SQ_INSTS_VMEM_RD (+ SQ_WAVES) per dispatch, in separate passes. A fit of
# FETCH_SIZE against the message size separates the bytes that scale with the
# sources (the fold's loads) from a per-dispatch constant.
# usage (GPU box, repo root): tools/fused_fetch_sweep.sh r03
set -uo pipefail
R=${1:-r03}
OUT=gpurun_out/prof_fetch_sweep_$R
DST=gpurun_out/profiles/$R/fused
mkdir -p "$OUT" "$DST"
export TMPDIR=/tmp SHMEM_NPES=2 SHMEM_DEVICE=0
SIZES="8192 16384 32768 65536"
run_pair () {
    local name=$1; shift
    local job="fs$name$$"
    SHMEM_PE=0 SHMEM_JOB_ID=$job timeout -k 10 240 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- \
        python3 tools/fused_bench.py 1024 $SIZES > "$OUT/$name.pe0.log" 2>&1 &
    local p0=$!
    SHMEM_PE=1 SHMEM_JOB_ID=$job timeout -k 10 240 python3 tools/fused_bench.py 1024 $SIZES > "$OUT/$name.pe1.log" 2>&1 &
    local p1=$!
    wait $p0; local r0=$?
    wait $p1; local r1=$?
    echo "$name: PE0 rc $r0, PE1 rc $r1"
    [ $r0 -eq 0 ] && [ $r1 -eq 0 ]
}
run_pair fetch --pmc FETCH_SIZE || exit 1
run_pair vmem --pmc SQ_INSTS_VMEM_RD SQ_WAVES || exit 1
python3 - "$OUT" "$DST" <<'PY'
import csv, glob, json, os, sys
out, dst = sys.argv[1], sys.argv[2]
per = {}
for counter, d in (("FETCH_SIZE", "fetch"), ("SQ_INSTS_VMEM_RD", "vmem"), ("SQ_WAVES", "vmem")):
    f = glob.glob(os.path.join(out, d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        if "fused_allreduce<0, double>" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            vals.setdefault(int(r["Grid_Size"]), []).append(float(r["Counter_Value"]) * (1024 if counter == "FETCH_SIZE" else 1))
    for g, v in vals.items():
        v.sort()
        per.setdefault(g, {})[counter] = v[len(v) // 2]
rows = []
for g in sorted(per):
    nbytes = g // 256 * 256 * 16  # one-shot grid: one 16-byte vector per thread
    rows.append({"grid_threads": g, "message_bytes": nbytes, "source_bytes_read": 2 * nbytes, **per[g]})
xs = [r["source_bytes_read"] for r in rows]
ys = [r["FETCH_SIZE"] for r in rows]
n = len(xs)
mx, my = sum(xs) / n, sum(ys) / n
slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sum((x - mx) ** 2 for x in xs)
res = {"kernel": "fused_allreduce<sum,double>, one-shot, PE 0 of 2 sharing the GPU (medians per dispatch)",
       "rows": rows, "fetch_fit": {"bytes_per_source_byte": round(slope, 4), "per_dispatch_bytes": round(my - slope * mx)},
       "note": "FETCH_SIZE raw (MI355X_MICROARCH.md: 16-B/lane streaming reads tallied at half their bytes)"}
json.dump(res, open(os.path.join(dst, "fetch_sweep_oneshot.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
PY

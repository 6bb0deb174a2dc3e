#!/bin/bash
# rocprofv3 evidence for the fused one-launch kernel (fused_allreduce), on the GPU box from the repo
# root: tools/profile_fused.sh r02
# Two PE processes of tools/fused_bench.py share the GPU; PE 0 runs under rocprofv3 (the program
# itself after --), PE 1 plainly. Passes: kernel trace + stats, FETCH_SIZE, WRITE_SIZE. Output under
# gpurun_out/profiles/$R/fused/.
set -uo pipefail
R=${1:-r02}
OUT=gpurun_out/prof_fused_$R
DST=gpurun_out/profiles/$R/fused
mkdir -p "$OUT" "$DST"
export TMPDIR=/tmp SHMEM_NPES=2 SHMEM_DEVICE=0
CALLS=2048
run_pair () {  # $1 = pass name, rest = rocprofv3 options
    local name=$1; shift
    local job="pf$name$$"
    SHMEM_PE=0 SHMEM_JOB_ID=$job timeout -k 10 240 rocprofv3 "$@" --output-format csv -d "$OUT/$name" -o run -- \
        python3 tools/fused_bench.py $CALLS > "$OUT/$name.pe0.log" 2>&1 &
    local p0=$!
    SHMEM_PE=1 SHMEM_JOB_ID=$job timeout -k 10 240 python3 tools/fused_bench.py $CALLS > "$OUT/$name.pe1.log" 2>&1 &
    local p1=$!
    wait $p0; local r0=$?
    wait $p1; local r1=$?
    echo "$name: PE0 rc $r0, PE1 rc $r1"
    [ $r0 -eq 0 ] && [ $r1 -eq 0 ]
}
run_pair trace --kernel-trace --stats || exit 1
run_pair fetch --pmc FETCH_SIZE || exit 1
run_pair write --pmc WRITE_SIZE || exit 1
# VMEM read instructions per dispatch: the fold's loads are known, the rest
# are flag polls (one wave instruction each, one small uncached request):
# separates the fetch bytes of polling from the sources'
run_pair vmem --pmc SQ_INSTS_VMEM_RD SQ_WAVES || exit 1
cp "$(find "$OUT/trace" -name '*kernel_stats.csv' -print -quit)" "$DST/rocprof_kernel_stats_fused_pe0.csv"
grep '^{' "$OUT/trace.pe0.log" > "$DST/fused_bench_under_rocprof.json" || true
for sz in 65536 1048576; do :; done
python3 - "$OUT" "$DST" <<'PY'
import csv, glob, json, os, sys
out, dst = sys.argv[1], sys.argv[2]
res = {}
for counter, d in (("FETCH_SIZE", "fetch"), ("WRITE_SIZE", "write"), ("SQ_INSTS_VMEM_RD", "vmem"),
                   ("SQ_WAVES", "vmem")):
    f = glob.glob(os.path.join(out, d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if "fused_allreduce<0, double>" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            scale = 1024 if counter.endswith("_SIZE") else 1
            per.setdefault(int(r["Grid_Size"]), []).append(float(r["Counter_Value"]) * scale)
    for g, v in per.items():
        v.sort()
        key = "median_bytes" if counter.endswith("_SIZE") else "median"
        res.setdefault(str(g), {})[counter] = {key: v[len(v) // 2], "dispatches": len(v)}
json.dump({"kernel": "fused_allreduce<sum,double> on PE 0 of 2 sharing the GPU, keyed by grid size (threads)",
           "by_grid": res, "note": "FETCH_SIZE raw (double it for wide streaming reads, MI355X_MICROARCH.md); "
           "the one-shot fold reads both PEs' whole sources, the two-shot reads both shards and the peer's shard"},
          open(os.path.join(dst, "pmc_fused_pe0.json"), "w"), indent=1)
PY
head -n 6 "$DST/rocprof_kernel_stats_fused_pe0.csv"

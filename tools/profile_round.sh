#!/bin/bash
# Refresh the judged profiles for one round, on the GPU box, from the repo root:
#   tools/profile_round.sh r01
# 1. rocprofv3 --kernel-trace --stats of bench.py (N = 1, 256 MiB, no small-call or op-coverage
#    leg, so the dominant kernel's average is the 256 MiB copy's)
# 2. two separate --pmc passes (FETCH_SIZE, WRITE_SIZE) of the same command,
#    turned into HBM bytes per launch by tools/pmc_traffic.py
#    (profiles/pmc_traffic.json, which bench.py reports as roofline.traffic)
# Everything lands under gpurun_out/profiles/ (what gpurun brings back); copy
# it over profiles/ and commit.
set -euo pipefail
R=${1:-r01}
OUT=gpurun_out/prof_$R
DST=gpurun_out/profiles/$R
mkdir -p "$OUT" "$DST/pmc"
export TMPDIR=/tmp
BENCH=(bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-small --no-ops)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "${BENCH[@]}" \
    > "$OUT/bench_trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "${BENCH[@]}" --no-check \
    > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "${BENCH[@]}" --no-check \
    > "$OUT/bench_write.log" 2>&1
python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" copy_segments 1000 n1_256mib gpurun_out/profiles/pmc_traffic.json
cp "$(find "$OUT/trace" -name '*kernel_stats.csv' -print -quit)" "$DST/rocprof_kernel_stats_bench_n1.csv"
cp "$(find "$OUT/trace" -name '*kernel_trace.csv' -print -quit)" "$DST/rocprof_kernel_trace_bench_n1.csv"
cp "$(find "$OUT/fetch" -name '*counter_collection.csv' -print -quit)" "$DST/pmc/fetch_size_counter_collection.csv"
cp "$(find "$OUT/write" -name '*counter_collection.csv' -print -quit)" "$DST/pmc/write_size_counter_collection.csv"
grep "^{\"metric\"" "$OUT/bench_trace.log" > "$DST/bench_n1_under_rocprof.json"
head -n 3 "$DST/rocprof_kernel_stats_bench_n1.csv"

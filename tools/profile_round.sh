#!/bin/bash
# Refresh the judged profiles for one round, on the GPU box, from the repo root:
#   tools/profile_round.sh r02
# 1. rocprofv3 --kernel-trace --stats of bench.py (N = 1, 256 MiB; no small-call or op-coverage
#    leg, so the copy's average is the 256 MiB headline calls'; the kernel legs run: the fold
#    kernels k = 2 / 8 and config 3 / 4's per-GPU reduce-scatter shapes)
# 2. separate --pmc passes of the same command: FETCH_SIZE, WRITE_SIZE (turned into HBM bytes per
#    launch per kernel by tools/pmc_traffic.py -> profiles/pmc_traffic.json, which bench.py reports
#    as roofline.traffic and kernels.*.traffic), then TCC_HIT/TCC_MISS + TA_BUSY
# Everything lands under gpurun_out/profiles/$R (what gpurun brings back); copy it over profiles/
# and commit.
set -euo pipefail
R=${1:-r02}
OUT=gpurun_out/prof_$R
DST=gpurun_out/profiles/$R
mkdir -p "$OUT" "$DST/pmc"
export TMPDIR=/tmp
BENCH=(bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-small --no-ops --no-rotating)
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "${BENCH[@]}" \
    > "$OUT/bench_trace.log" 2>&1
# the HBM-only headline (bench.py headline_rotating): its copy_segments<4,1>
# dispatches come after the headline's 620 (20 warm-up + 3 x 200); the last
# 200 are its event-stamped pass
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_rot" -o run -- python3 bench.py \
    --steps 200 --warmup 20 --no-cpu-baseline --no-small --no-ops --no-kernels --no-host-staged \
    > "$OUT/bench_trace_rot.log" 2>&1
python3 tools/trace_split.py "$OUT/trace_rot" "copy_segments<4, 1>" 200 620 > "$DST/rocprof_rotating_split.json"
grep "^{\"metric\"" "$OUT/bench_trace_rot.log" > "$DST/bench_n1_rotating_under_rocprof.json"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 "${BENCH[@]}" --no-check \
    > "$OUT/bench_fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 "${BENCH[@]}" --no-check \
    > "$OUT/bench_write.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr --output-format csv -d "$OUT/tcc" -o run -- \
    python3 "${BENCH[@]}" --no-check > "$OUT/bench_tcc.log" 2>&1 || echo "TCC/TA pass failed (see $OUT/bench_tcc.log)"
J=gpurun_out/profiles/pmc_traffic.json
cp profiles/pmc_traffic.json "$J" 2>/dev/null || true
# key, kernel-name substring (~ = space), minimum grid (threads) of the launches to count
# (since round 6 the 8-source every-member folds run a grid of one or two blocks per CU at
# every size: their legs are told apart by their bytes per pass -- double sum 256 MiB read +
# 256 MiB written vs 64 + 64, float max 64 + 64 vs 16 + 16)
while read -r key sub grid; do
    python3 tools/pmc_traffic.py "$OUT/fetch" "$OUT/write" "${sub//\~/ }" "$grid" "$key" "$J" > /dev/null
done <<'EOF'
n1_256mib copy_segments<4,~1> 1000
offset_target_copy_shift copy_segments_shift<4,~1> 1000
kernel_fold_k2_double_sum combine_vec<0,~double,~2, 1000
kernel_fold_k8_double_sum combine_vec<0,~double,~8, 1000
kernel_rs_shard_n8_double_sum combine_orders_vec<0,~double,~8, 1000@134217729
kernel_rs_shard_n8_double_sum_8mib combine_orders_vec<0,~double,~8, 1000@1:134217728
kernel_fold_k8_float_max combine_vec<6,~float,~8, 1000
kernel_fold_k8_longlong_and combine_vec<2,~long,~8, 300000
kernel_rs_shard_n8_longlong_and combine_vec<2,~long,~8, 1000:300000
kernel_rs_shard_n8_float_max combine_orders_vec<6,~float,~8, 1000@33554433
kernel_rs_shard_n8_float_max_nan_rich combine_orders_vec<6,~float,~8, 1000@33554433
kernel_rs_shard_n8_float_max_2mib combine_orders_vec<6,~float,~8, 1000@1:33554432
kernel_rs_shard_n8_longdouble_sum combine_orders_vec<0,~x80,~8, 1000
kernel_rs_shard_n8_longdouble_prod combine_orders_vec<1,~x80,~8, 1000
kernel_rs_shard_n8_complexf_prod combine_orders_vec<1,~mi355::cplxf,~8, 1000
EOF
cp "$(find "$OUT/trace" -name '*kernel_stats.csv' -print -quit)" "$DST/rocprof_kernel_stats_bench_n1.csv"
cp "$(find "$OUT/fetch" -name '*counter_collection.csv' -print -quit)" "$DST/pmc/fetch_size_counter_collection.csv"
cp "$(find "$OUT/write" -name '*counter_collection.csv' -print -quit)" "$DST/pmc/write_size_counter_collection.csv"
f=$(find "$OUT/tcc" -name '*counter_collection.csv' -print -quit 2>/dev/null || true)
[ -n "$f" ] && cp "$f" "$DST/pmc/tcc_ta_counter_collection.csv"
grep "^{\"metric\"" "$OUT/bench_trace.log" > "$DST/bench_n1_under_rocprof.json"
head -n 12 "$DST/rocprof_kernel_stats_bench_n1.csv"

#!/bin/bash
# Round 4, first GPU call: (1) the mechanism of round 2's x87 nondeterminism
# (tools/x80_lane_probe.hip: grid 2048 vs 256, register scrub before each
# kernel), round-2 header (_r2) and today's (_now); (2) 16-byte system-coherent
# loads in the fold (tools/fold_probe S). Every step under its own time limit.
set -o pipefail
mkdir -p gpurun_out/r04
O=gpurun_out/r04
P=tools/x80_lane_probe
timeout -k 10 120 $P'_r2' 200000 3 2048 none gvlah > $O/x80_r2_g2048_none.txt &&
timeout -k 10 120 $P'_r2' 200000 3 256 none gh > $O/x80_r2_g256_none.txt &&
timeout -k 10 120 $P'_r2' 200000 3 2048 ones gh > $O/x80_r2_g2048_ones.txt &&
timeout -k 10 120 $P'_r2' 200000 3 2048 zero gh > $O/x80_r2_g2048_zero.txt &&
timeout -k 10 120 $P'_r2' 200000 3 2048 a5 gvlah > $O/x80_r2_g2048_a5.txt &&
timeout -k 10 120 $P'_r2' 200000 3 256 ones gh > $O/x80_r2_g256_ones.txt &&
timeout -k 10 120 $P'_now' 200000 3 2048 none gvlah > $O/x80_now_g2048_none.txt &&
timeout -k 10 120 $P'_now' 200000 3 2048 ones gvlah > $O/x80_now_g2048_ones.txt &&
timeout -k 10 120 $P'_now' 200000 3 2048 a5 gvlah > $O/x80_now_g2048_a5.txt &&
timeout -k 10 300 tools/fold_probe S > $O/fold_probe_sysload16.txt
rc=$?
grep -h "SUMMARY\|^  add:\|^  mul:\|hwid kernel" $O/x80_*.txt
cat $O/fold_probe_sysload16.txt | tail -60
exit $rc

#!/bin/bash
# Round 4: which instruction class of the round-2 general x87 kernels has its
# result consumed too early under co-residency? tools/x80_isa_variants.py code
# objects (s_nop inserted after a class of instructions), each run by
# x80_lane_probe_r2 at grid 2048 (several waves per SIMD) on the general kernels.
# usage: r04_x80_isa.sh <tag> <variant>...
set -o pipefail
mkdir -p gpurun_out/r04
tag=$1; shift
O=gpurun_out/r04/x80_isa_$tag.txt
: > $O
for v in "$@"; do
    timeout -k 10 120 tools/x80_lane_probe_r2 200000 4 2048 none g tools/x80_isa/general_$v.hsaco > gpurun_out/r04/x80_isa_${tag}_$v.txt || exit $?
    echo "== $v" >> $O
    grep -A2 SUMMARY gpurun_out/r04/x80_isa_${tag}_$v.txt >> $O
done
cat $O

#!/bin/bash
# Round 4: co-residency vs dispatch order. The round-2 general x87 kernels at
# grid 2048 with 96 KiB of dynamic LDS per block (one block per CU: every wave
# alone on its SIMD, blocks >= 256 start only as earlier ones finish), against
# the same launch without it, and at grid 512 (two blocks per CU).
set -o pipefail
mkdir -p gpurun_out/r04
O=gpurun_out/r04/x80_lds.txt
: > $O
run() {
    tag=$1; shift
    timeout -k 10 120 tools/x80_lane_probe_r2 "$@" > gpurun_out/r04/x80_lds_$tag.txt || exit $?
    echo "== $tag: $*" >> $O
    grep -A3 SUMMARY gpurun_out/r04/x80_lds_$tag.txt >> $O
}
run builtin_nolds 200000 4 2048 none gh - 0
run builtin_lds96k 200000 4 2048 none gh - 98304
run orig_lds96k 200000 4 2048 none g tools/x80_isa/general_orig.hsaco 98304
run builtin_grid512 200000 4 512 none gh - 0
run builtin_grid512_lds96k 200000 4 512 none gh - 98304
cat $O

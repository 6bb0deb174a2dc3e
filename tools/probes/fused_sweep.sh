#!/bin/bash
# Fused one-launch kernel vs the multi-launch P2P schedule at mid sizes, with
# PEs sharing this GPU (tools/fused_bench.py, one process per PE), run from
# the repo root on the GPU box:
#   tools/probes/fused_sweep.sh OUTDIR [npes...]
# For each PE count: the default thresholds (fused up to SHMEM_FUSED_MAX_BYTES
# = 1 MiB, multi-launch above) and every size forced onto the fused kernel
# (SHMEM_FUSED_MAX_BYTES=64M). One JSON line per run in OUTDIR/fused_sweep.jsonl.
set -uo pipefail
OUT=${1:?outdir}
shift
mkdir -p "$OUT"
SIZES="262144 1048576 2097152 4194304 8388608 16777216 33554432"
export SHMEM_DEVICE_HEAP_SIZE=$((80 << 20)) SHMEM_DEVICE_SCRATCH_SIZE=3M SHMEM_DEVICE_ORDER_SIZE=64M SHMEM_DEVICE=0
for np in "${@:-2}"; do
    for mode in default fused; do
        if [ "$mode" = fused ]; then export SHMEM_FUSED_MAX_BYTES=64M; else unset SHMEM_FUSED_MAX_BYTES; fi
        job="fs$$-$np-$mode"
        pids=()
        for ((pe = 0; pe < np; pe++)); do
            SHMEM_PE=$pe SHMEM_NPES=$np SHMEM_JOB_ID=$job timeout -k 10 240 python3 tools/fused_bench.py 200 $SIZES \
                > "$OUT/pe$pe.out" 2> "$OUT/pe$pe.err" &
            pids+=($!)
        done
        rc=0
        for p in "${pids[@]}"; do wait "$p" || rc=$?; done
        if [ $rc -ne 0 ]; then
            echo "npes $np $mode failed rc $rc" >&2
            tail -5 "$OUT"/pe*.err >&2
            exit $rc
        fi
        python3 -c "import json,sys; d=json.loads([l for l in open('$OUT/pe0.out') if l.startswith('{')][-1]); d['mode']='$mode'; print(json.dumps(d))" \
            >> "$OUT/fused_sweep.jsonl"
        echo "npes $np $mode done"
    done
done

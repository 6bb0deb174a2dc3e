#!/bin/bash
# tools/fused_phases.py on PEs sharing this GPU (from the repo root, on the GPU
# box, after `make -C osss-gasnet_amd/csrc probe`): tools/fused_phases.sh OUTDIR [npes...]
set -uo pipefail
OUT=${1:?outdir}
shift
mkdir -p "$OUT"
export SHMEM_REDUCE_LIBDIR="$PWD/osss-gasnet_amd/lib/probe" SHMEM_DEVICE=0 SHMEM_FUSED_MAX_BYTES=4M \
    SHMEM_DEVICE_HEAP_SIZE=$((16 << 20)) SHMEM_DEVICE_SCRATCH_SIZE=3M SHMEM_DEVICE_ORDER_SIZE=16M
for np in "${@:-2}"; do
    pids=()
    for ((pe = 0; pe < np; pe++)); do
        SHMEM_PE=$pe SHMEM_NPES=$np SHMEM_JOB_ID="fp$$-$np" timeout -k 10 180 python3 tools/fused_phases.py \
            65536 262144 1048576 2097152 4194304 > "$OUT/pe$pe.out" 2> "$OUT/pe$pe.err" &
        pids+=($!)
    done
    rc=0
    for p in "${pids[@]}"; do wait "$p" || rc=$?; done
    if [ $rc -ne 0 ]; then echo "npes $np failed rc $rc" >&2; tail -5 "$OUT"/pe*.err >&2; exit $rc; fi
    grep '^{' "$OUT/pe0.out" >> "$OUT/fused_phases.jsonl"
    echo "npes $np done"
done

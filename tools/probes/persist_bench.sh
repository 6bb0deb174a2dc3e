#!/bin/bash
# Same-GPU fused calls with and without the persistent server (SHMEM_PERSISTENT),
# PEs of tools/fused_bench.py sharing the one GPU; one JSON line per run.
set -o pipefail
mkdir -p gpurun_out
run() {  # npes persistent
    local pids=() job=pb$$_$1_$2
    for ((pe = 0; pe < $1; pe++)); do
        SHMEM_NPES=$1 SHMEM_PE=$pe SHMEM_JOB_ID=$job SHMEM_DEVICE=0 SHMEM_PERSISTENT=$2 \
            timeout -k 5 120 python tools/fused_bench.py 4096 8192 65536 1048576 > gpurun_out/pb_$1_$2_$pe.out 2>&1 &
        pids+=($!)
    done
    for p in "${pids[@]}"; do wait $p || return 1; done
    echo "{\"npes\": $1, \"persistent\": $2, \"result\": $(grep '^{' gpurun_out/pb_$1_$2_0.out)}"
}
for np in 2 3 4; do
    run $np 0 && run $np 1 || exit 1
done

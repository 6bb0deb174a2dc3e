#!/bin/bash
# Round 4: the fused kernel's variants (tools/build_fused_variants.sh) on this
# GPU: NPES fused_bench.py processes sharing it, 4096 calls of 64 KiB and 1 MiB,
# per-call time, kernel duration and a bit-exact check (PE 0's JSON line).
set -o pipefail
mkdir -p gpurun_out/r04
O=gpurun_out/r04/fused_variants.jsonl
: > $O
for rep in 1 2; do
for v in "$@"; do
  for np in 2 4; do
    job=fv$RANDOM$RANDOM
    pids=()
    for pe in $(seq 0 $((np - 1))); do
      SHMEM_REDUCE_LIBDIR=$PWD/osss-gasnet_amd/lib/variants/$v SHMEM_PE=$pe SHMEM_NPES=$np SHMEM_JOB_ID=$job \
        SHMEM_DEVICE=0 timeout -k 10 120 python tools/fused_bench.py 4096 65536 1048576 \
        > gpurun_out/r04/fv_${v}_${np}_$pe.out 2>&1 &
      pids+=($!)
    done
    for p in "${pids[@]}"; do wait $p || { echo "variant $v np $np failed"; cat gpurun_out/r04/fv_${v}_${np}_*.out | tail -20; exit 1; }; done
    line=$(grep '^{' gpurun_out/r04/fv_${v}_${np}_0.out | tail -1)
    echo "{\"variant\": \"$v\", \"npes\": $np, \"rep\": $rep, \"result\": $line}" >> $O
  done
done
done
python3 - <<'PY'
import json
for ln in open("gpurun_out/r04/fused_variants.jsonl"):
    d = json.loads(ln)
    r = d["result"]["legs"]
    print(d["variant"], d["npes"], d["rep"], " ".join(f"{k}: {v['us_per_call']} us/call kernel {v['kernel_avg_us']} {v['check'][:9]}" for k, v in r.items()))
PY

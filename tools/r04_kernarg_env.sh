#!/bin/bash
mkdir -p gpurun_out/r04
for v in unset 0 1; do
  if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
  for rep in 1 2; do
    job=ka$RANDOM
    for pe in 0 1; do SHMEM_PE=$pe SHMEM_NPES=2 SHMEM_JOB_ID=$job SHMEM_DEVICE=0 timeout -k 5 120 python tools/fused_bench.py 4096 65536 1048576 > gpurun_out/r04/ka_${v}_${rep}_$pe.out 2>&1 & done
    wait
    echo "HIP_FORCE_DEV_KERNARG=$v rep $rep: $(grep '^{' gpurun_out/r04/ka_${v}_${rep}_0.out | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k:(v["us_per_call"], v["kernel_avg_us"]) for k,v in d["legs"].items()})')"
  done
done

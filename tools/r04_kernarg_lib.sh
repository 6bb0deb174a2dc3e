#!/bin/bash
# Round 4: the library's own HIP_FORCE_DEV_KERNARG default (set in shmem_init) against SHMEM_DEV_KERNARG=0
mkdir -p gpurun_out/r04
unset HIP_FORCE_DEV_KERNARG
for v in 1 0 1 0; do
  SHMEM_DEV_KERNARG=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernels --no-ops --no-host-staged > gpurun_out/r04/kal_bench_$v.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r04/kal_bench_$v.json'))
print('SHMEM_DEV_KERNARG=$v', d['value'], d['ms_per_step'], d['per_call']['median_us'], d['roofline']['kernel_avg_us'], 'small', d['small_call']['us_per_call'], d['small_call']['per_call']['median_us'], 'persist', d['small_call_persistent']['us_per_call'], 'graph', d['small_call_graph']['us_per_call'], 'fused', {k:v['us_per_call'] for k,v in d['fused_same_gpu']['legs'].items()})"
done

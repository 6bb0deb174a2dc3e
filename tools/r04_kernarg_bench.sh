#!/bin/bash
# Round 4: HIP_FORCE_DEV_KERNARG (kernel arguments in device memory) on the N = 1 line
mkdir -p gpurun_out/r04
for v in unset 1 unset 1; do
  if [ $v = unset ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$v; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-kernels --no-ops --no-host-staged > gpurun_out/r04/ka_bench_$v.json 2>/dev/null || exit 1
  python3 -c "
import json; d=json.load(open('gpurun_out/r04/ka_bench_$v.json'))
print('HIP_FORCE_DEV_KERNARG=$v', d['value'], d['ms_per_step'], d['per_call']['median_us'], d['roofline']['kernel_avg_us'], 'small', d['small_call']['us_per_call'], d['small_call']['per_call']['median_us'], 'persist', d['small_call_persistent']['us_per_call'], 'graph', d['small_call_graph']['us_per_call'], 'fused', {k:v['us_per_call'] for k,v in d['fused_same_gpu']['legs'].items()})"
done

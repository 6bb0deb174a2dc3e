#!/bin/bash
# Round 6: the blocking N = 1 call's fixed cost under HIP runtime settings
# (kernel-argument placement). One short bench line per setting.
set -o pipefail
R=${1:-r06fc}
mkdir -p gpurun_out/$R
B=(bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-kernels --no-fused --no-host-staged --no-rotating --no-ops)
for v in default 1 0; do
  if [ $v = default ]; then
    timeout -k 10 200 python -u "${B[@]}" > gpurun_out/$R/n1_$v.json 2> gpurun_out/$R/n1_$v.err || exit 1
  else
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 200 python -u "${B[@]}" > gpurun_out/$R/n1_$v.json 2> gpurun_out/$R/n1_$v.err || exit 1
  fi
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/$R/n1_$v.json').read()); print('$v', d['ms_per_step'], d['roofline']['kernel_avg_us'], d['fixed_cost'], d['small_call']['us_per_call'])"
done

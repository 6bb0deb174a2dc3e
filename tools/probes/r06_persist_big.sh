#!/bin/bash
# Round 6: the N = 1 headline call served by the opt-in persistent server
# (SHMEM_PERSISTENT=1, fused_max raised so a 256 MiB identity copy is
# servable) against the launched copy kernel. Timed region only.
set -o pipefail
R=${1:-r06pb}
mkdir -p gpurun_out/$R
B=(bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-kernels --no-fused --no-host-staged --no-rotating --no-ops --no-small)
timeout -k 10 200 python -u "${B[@]}" > gpurun_out/$R/launched.json 2> gpurun_out/$R/launched.err || exit 1
SHMEM_PERSISTENT=1 SHMEM_FUSED_MAX_BYTES=1G timeout -k 10 200 python -u "${B[@]}" > gpurun_out/$R/persistent.json 2> gpurun_out/$R/persistent.err || exit 1
for v in launched persistent; do
  python3 -c "import json; d=json.loads(open('gpurun_out/$R/$v.json').read()); print('$v', d['ms_per_step'], d['roofline']['kernel'], d['roofline']['kernel_avg_us'], d['roofline']['call_schedule'], d['per_call']['median_us'], d['check'][:20])"
done

#!/bin/bash
# Round-6 mid-round GPU check: the bench tests, an N = 1 bench line and the
# same-GPU N = 4 rehearsal with the xGMI legs forced on. Output under gpurun_out/$1.
set -o pipefail
R=${1:-r06a}
mkdir -p gpurun_out/$R
timeout -k 10 700 python -u -m pytest -x -v --timeout 400 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_bench.py > gpurun_out/$R/tests.log 2>&1
rc=$?
tail -12 gpurun_out/$R/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/$R/bench_n1.json 2> gpurun_out/$R/bench_n1.err || { echo "bench n1 failed"; tail -20 gpurun_out/$R/bench_n1.err; exit 1; }
echo "bench n1 ok"
GPU_MAX_HW_QUEUES=2 timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
  --master-port 29534 bench.py --gpus 4 --steps 50 --warmup 5 --force-xgmi-legs > gpurun_out/$R/bench_n4.json 2> gpurun_out/$R/bench_n4.err || { echo "bench n4 failed"; tail -20 gpurun_out/$R/bench_n4.err; exit 1; }
echo "bench n4 ok"

#!/bin/bash
# Round-6 mid-round GPU check: the tests touched this round, an N = 1 bench
# line and the same-GPU N = 2 rehearsal line. Output under gpurun_out/$1.
set -o pipefail
R=${1:-r06a}
mkdir -p gpurun_out/$R
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  "tests/test_gpu_checks.py::test_thresholds_calibrated_at_init" \
  "tests/test_gpu_checks.py::test_calibration_settings_must_agree" \
  tests/test_gpu_bench.py > gpurun_out/$R/tests.log 2>&1
rc=$?
tail -30 gpurun_out/$R/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/$R/bench_n1.json 2> gpurun_out/$R/bench_n1.err || { echo "bench n1 failed"; tail -20 gpurun_out/$R/bench_n1.err; exit 1; }
echo "bench n1 ok"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 > gpurun_out/$R/bench_n2.json 2> gpurun_out/$R/bench_n2.err || { echo "bench n2 failed"; tail -20 gpurun_out/$R/bench_n2.err; exit 1; }
echo "bench n2 ok"

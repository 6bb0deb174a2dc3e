#!/bin/bash
# Round-6 full GPU pass: the whole GPU suite, smoke, then N = 1 and the
# same-GPU N = 2 bench lines. Output under gpurun_out/$1.
set -o pipefail
R=${1:-r06c}
mkdir -p gpurun_out/$R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider \
    > gpurun_out/$R/gputest.log 2>&1 || { echo "GPU suite failed"; grep -E "FAILED|Error|error" gpurun_out/$R/gputest.log | tail -20; tail -30 gpurun_out/$R/gputest.log; exit 1; }
tail -1 gpurun_out/$R/gputest.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke.log 2>&1 \
    || { echo "smoke failed"; cat gpurun_out/$R/smoke.log; exit 1; }
tail -1 gpurun_out/$R/smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/$R/bench_n1.json 2> gpurun_out/$R/bench_n1.err || { echo "bench n1 failed"; tail -20 gpurun_out/$R/bench_n1.err; exit 1; }
echo "bench n1 ok"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 > gpurun_out/$R/bench_n2.json 2> gpurun_out/$R/bench_n2.err || { echo "bench n2 failed"; tail -20 gpurun_out/$R/bench_n2.err; exit 1; }
echo "bench n2 ok"

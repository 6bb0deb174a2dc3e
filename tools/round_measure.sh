#!/bin/bash
# One GPU call's worth of round-end measurements, run from the repo root on
# the GPU box: tools/round_measure.sh r05
#   1. tools/profile_round.sh: rocprofv3 kernel trace + stats of bench.py (and
#      of its HBM-only headline), FETCH_SIZE / WRITE_SIZE / TCC passes
#   2. the bench lines: N = 1, and N = 2 / 4 with the PEs sharing this GPU
# Every step has its own time limit; the first failure ends the script.
set -euo pipefail
R=${1:-r05}
mkdir -p gpurun_out/bench_$R
timeout -k 10 900 bash tools/profile_round.sh "$R" > gpurun_out/profile_round_$R.log 2>&1
# the bench lines below report the traffic just profiled (same code objects)
cp gpurun_out/profiles/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$R/bench_n1.json 2> gpurun_out/bench_$R/bench_n1.err
# N = 4 also rehearses the one-GPU-per-PE legs (--force-xgmi-legs); 2 hardware
# queues per PE keep 4 PEs' device-side waits off the time-sliced path
for n in 2 4; do
    extra=()
    [ $n = 4 ] && extra=(--force-xgmi-legs)
    GPU_MAX_HW_QUEUES=2 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $((29640 + n)) bench.py --gpus $n --steps 50 --warmup 5 "${extra[@]}" \
        > gpurun_out/bench_$R/bench_n${n}_same_gpu.json 2> gpurun_out/bench_$R/bench_n${n}_same_gpu.err
done

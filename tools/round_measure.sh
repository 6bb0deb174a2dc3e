#!/bin/bash
# One GPU call's worth of round-end measurements (tools/profile_round.sh and
# tools/profile_fused.sh for the profiles, then the bench lines), run from the
# repo root on the GPU box: tools/round_measure.sh r03
# Every step has its own time limit; the first failure ends the script.
set -euo pipefail
R=${1:-r03}
mkdir -p gpurun_out/bench_$R
timeout -k 10 600 bash tools/profile_round.sh "$R" > gpurun_out/profile_round_$R.log 2>&1
# the bench lines below report the traffic just profiled (same code objects)
cp gpurun_out/profiles/pmc_traffic.json profiles/pmc_traffic.json
timeout -k 10 300 bash tools/profile_fused.sh "$R" > gpurun_out/profile_fused_$R.log 2>&1
timeout -k 10 300 python3 bench.py > gpurun_out/bench_$R/bench_n1.json 2> gpurun_out/bench_$R/bench_n1.err
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29641 bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/bench_$R/bench_n2_same_gpu.json \
    2> gpurun_out/bench_$R/bench_n2_same_gpu.err

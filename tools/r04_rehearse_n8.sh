#!/bin/bash
# Round 4: the driver's 8-rank bench command, rehearsed on
# this one GPU with the same-GPU hardware-queue policy (GPU_MAX_HW_QUEUES =
# 16 / 8 when 8 PEs share one GPU): every leg of the N > 1 line
# at 8 ranks, per-leg wall times in legs_s, total wall time beside it.
set -o pipefail
mkdir -p gpurun_out/r04
t0=$(date +%s.%N)
GPU_MAX_HW_QUEUES=2 timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 \
    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 8 --steps 20 --warmup 5 \
    > gpurun_out/r04/bench_n8_same_gpu.json 2> gpurun_out/r04/bench_n8_same_gpu.err
rc=$?
t1=$(date +%s.%N)
echo "{\"rc\": $rc, \"wall_s\": $(python3 -c "print(round($t1 - $t0, 1))")}" > gpurun_out/r04/bench_n8_same_gpu.wall
cat gpurun_out/r04/bench_n8_same_gpu.wall
exit $rc

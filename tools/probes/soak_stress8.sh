# Randomized stress on 8 PEs sharing the GPU box's one GPU (from the repo root):
# the default sequence, then two more seeds with 300 calls each.
set -o pipefail
mkdir -p gpurun_out/soak8
timeout -k 10 400 python -u -m pytest tests/test_gpu_multipe.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "stress_eight_pes" > gpurun_out/soak8/default.log 2>&1 || { echo "default failed"; tail -30 gpurun_out/soak8/default.log; exit 1; }
tail -1 gpurun_out/soak8/default.log
for seed in 41 42; do
  SHMEM_TEST_STRESS_SEED=$seed SHMEM_TEST_STRESS_CALLS=300 timeout -k 10 400 python -u -m pytest tests/test_gpu_multipe.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "stress_eight_pes" > gpurun_out/soak8/seed$seed.log 2>&1 || { echo "seed $seed failed"; tail -30 gpurun_out/soak8/seed$seed.log; exit 1; }
  echo "seed $seed ok"; tail -1 gpurun_out/soak8/seed$seed.log
done

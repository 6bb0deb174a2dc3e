# Randomized stress soak on the GPU box (from the repo root): the two random-sequence stress tests
# (on and outside the heap, launched and persistent server) with three more seeds, 600 calls each.
set -o pipefail
mkdir -p gpurun_out/soak
for seed in 31 32 33; do
  SHMEM_TEST_STRESS_SEED=$seed SHMEM_TEST_STRESS_CALLS=600 timeout -k 10 400 python -u -m pytest tests/test_gpu_multipe.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider -k "random_sequence_stress" > gpurun_out/soak/seed$seed.log 2>&1 || { echo "seed $seed failed"; exit 1; }
  echo "seed $seed ok"; tail -1 gpurun_out/soak/seed$seed.log
done

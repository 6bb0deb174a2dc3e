set -o pipefail
export SHMEM_NPES=2 SHMEM_JOB_ID=dbg$$ SHMEM_DEVICE=0 SHMEM_DEVICE_HEAP_SIZE=16M SHMEM_DEVICE_SCRATCH_SIZE=384K SHMEM_DEVICE_ORDER_SIZE=4M SHMEM_BARRIER_TIMEOUT=60 SHMEM_PEER_ACQUIRE=1 SHMEM_PERSISTENT=1 SHMEM_PERSISTENT_IDLE_US=200000 SHMEM_LOG_LEVELS=REDUCTION
mkdir -p gpurun_out
SHMEM_PE=0 SHMEM_LOG_FILE=gpurun_out/trace_pe0.log timeout -k 5 120 python tests/persistent_worker.py burst 2 > gpurun_out/dbg0.out 2>&1 &
p0=$!
SHMEM_PE=1 SHMEM_LOG_FILE=gpurun_out/trace_pe1.log timeout -k 5 120 python tests/persistent_worker.py burst 2 > gpurun_out/dbg1.out 2>&1
r1=$?
wait $p0
r0=$?
echo rc $r0 $r1

set -u
export SHMEM_NPES=1 SHMEM_PE=0 SHMEM_JOB_ID=diag$$ SHMEM_DEVICE=0 SHMEM_DEVICE_HEAP_SIZE=32M SHMEM_DEVICE_SCRATCH_SIZE=384K SHMEM_DEVICE_ORDER_SIZE=4M SHMEM_BARRIER_TIMEOUT=20 SHMEM_PERSISTENT=1 SHMEM_LOG_LEVELS=REDUCTION SHMEM_LOG_FILE=gpurun_out/diag_trace.log
timeout -k 5 60 python3 -u tests/persistent_worker.py burst 1 > gpurun_out/diag_burst.log 2>&1
echo "burst rc $?" >> gpurun_out/diag_burst.log

#!/bin/bash
# Host-code AddressSanitizer + UBSan run (GPU ASan is not available on this
# pool): the C runtime instrumented (make asan), tools/asan_driver.c built
# instrumented against it, run on 1 and 3 PEs sharing the GPU.
#   build (CPU container):  tools/asan_check.sh build
#   run   (GPU box):        tools/asan_check.sh run
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
LIB=$ROOT/osss-gasnet_amd/lib/asan
EXE=$LIB/asan_driver
case "${1:-run}" in
build)
    make -C "$ROOT/osss-gasnet_amd/csrc" asan -j8
    gcc -std=c99 -g -O1 -fsanitize=address,undefined -fno-omit-frame-pointer -D__HIP_PLATFORM_AMD__ \
        -I"$ROOT/include" -I/opt/rocm/include "$ROOT/tools/asan_driver.c" -L"$LIB" -lshmem_reduce \
        -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,"$LIB" -Wl,-rpath,/opt/rocm/lib -o "$EXE"
    ;;
run)
    export ASAN_OPTIONS=detect_leaks=0:abort_on_error=1
    export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
    export SHMEM_DEVICE_HEAP_SIZE=64M SHMEM_DEVICE_SCRATCH_SIZE=3M
    for n in 1 3; do
        timeout -k 10 300 python3 "$ROOT/tools/oshrun" -np $n --same-device "$EXE"
    done
    ;;
esac

#!/bin/bash
# Measurement builds of the library with fused.hip variants (round 4):
#   inl{0,1}  MI355_FUSED_INLINE_HELPERS (protocol helpers force-inlined or not)
#   buf{0,1}  MI355_FUSED_BUFFER_LOADS   (folds' 16-byte buffer sc0 sc1 loads or 2 x 8-byte atomics)
# into osss-gasnet_amd/lib/variants/<name>/ (libshmem_reduce.so + libshmem_bench.so);
# run with SHMEM_REDUCE_LIBDIR=<that dir> (tools/r04_fused_variants.sh).
set -e
cd "$(dirname "$0")/../osss-gasnet_amd/csrc"
make -s ../lib/libshmem_reduce.so >/dev/null
OBJS=$(ls ../lib/*.o | grep -v '/fused.o$')
for v in "$@"; do
    inl=${v:3:1}; buf=${v:8:1}
    d=../lib/variants/$v
    mkdir -p $d
    ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 -I../../include \
        -DMI355_FUSED_INLINE_HELPERS=$inl -DMI355_FUSED_BUFFER_LOADS=$buf -c fused.hip -o $d/fused.o &&
      /opt/rocm/bin/hipcc $OBJS $d/fused.o -shared -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lamdhip64 -lrccl -lrt \
        -lpthread -o $d/libshmem_reduce.so &&
      cc -std=c11 -O2 -fPIC -shared -Wall -I../../include -I/opt/rocm/include bench_loop.c -L$d -lshmem_reduce \
        -Wl,-rpath,'$ORIGIN' -o $d/libshmem_bench.so && rm -f $d/fused.o && echo "built $v" ) &
done
wait

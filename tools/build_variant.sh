#!/bin/bash
# A measurement build of the library with some fold translation units compiled
# with extra defines (combine_kernels.h's build-time switches):
#   tools/build_variant.sh NAME "-DMI355_CPLX_VOTE=1" complexf complexd
# -> osss-gasnet_amd/lib/variants/NAME/libshmem_reduce.so; run a tool with
# SHMEM_REDUCE_LIBDIR=<that dir> (e.g. tools/orders_sweep.py). Objects that
# would need scratch memory fail the build, as in the library's own Makefile.
set -e
cd "$(dirname "$0")/../osss-gasnet_amd/csrc"
name=$1; defs=$2; shift 2
make -s ../lib/libshmem_reduce.so >/dev/null
d=../lib/variants/$name
mkdir -p $d
OBJS=$(ls ../lib/*.o)
for t in "$@"; do
    OBJS=$(echo "$OBJS" | grep -v "/combine_t_$t.o$")
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 -I../../include $defs \
        -c combine_t_$t.hip -o $d/combine_t_$t.o &
done
wait
for t in "$@"; do python3 ../../tools/check_residency.py --no-scratch $d/combine_t_$t.o; done
/opt/rocm/bin/hipcc $OBJS $(for t in "$@"; do echo $d/combine_t_$t.o; done) -shared -L/opt/rocm/lib \
    -Wl,-rpath,/opt/rocm/lib -lamdhip64 -lrccl -lrt -lpthread -o $d/libshmem_reduce.so
rm -f $d/*.o
echo "built $name"

#!/bin/bash
# Measurement builds of the library with the long double every-member fold's
# build-time forms (combine_kernels.h, round 4), named s<S>e<E>w<W>n<N>[m<M>]:
#   S  MI355_X80_SERIAL_CHAINS  1: chains kept one after the other, 0: free to interleave
#   E  MI355_X80_EARLY_STORE    1: each member's output stored when its chain ends
#   W  MI355_X80_WAVES          occupancy floor (waves per SIMD) of the orders kernels, 0: none
#   N  MI355_X80_NT_LOADS       1: non-temporal source loads
#   M  MI355_X80_MUL128         1: the significand product from 32-bit limbs (x80.h mul64x64)
# into osss-gasnet_amd/lib/variants/<name>/ (libshmem_reduce.so); run with
# SHMEM_REDUCE_LIBDIR=<that dir> (tools/x80_variant_time.py). A variant whose
# kernels need scratch memory is reported and not built.
set -e
cd "$(dirname "$0")/../osss-gasnet_amd/csrc"
make -s ../lib/libshmem_reduce.so >/dev/null
OBJS=$(ls ../lib/*.o | grep -v '/combine_t_longdouble.o$')
for v in "$@"; do
    s=${v:1:1}; e=${v:3:1}; w=${v:5:1}; p=${v:7:1}; m=${v:9:1}
    d=../lib/variants/$v
    mkdir -p $d
    ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 -I../../include \
        -DMI355_X80_SERIAL_CHAINS=$s -DMI355_X80_EARLY_STORE=$e -DMI355_X80_WAVES=$w -DMI355_X80_NT_LOADS=${p:-0} -DMI355_X80_MUL128=${m:-0} \
        -c combine_t_longdouble.hip -o $d/combine_t_longdouble.o &&
      python3 ../../tools/check_residency.py --no-scratch $d/combine_t_longdouble.o &&
      python3 - $d/combine_t_longdouble.o $v <<'PY' &&
import sys, tempfile
sys.path.insert(0, "../../tools")
import check_residency as cr
with tempfile.TemporaryDirectory() as t:
    ks = cr.kernels(cr.code_object(sys.argv[1], t))
    for k, name in zip(ks, cr.demangle([k["name"] for k in ks])):
        if "combine_orders_vec<0, x80, 8, 1, 1, true>" in name or "combine_orders_vec<1, x80, 8, 1, 1, true>" in name:
            print(sys.argv[2], name.split("<")[1].split(",")[0], "vgpr", k["vgpr_count"], "sgpr", k["sgpr_count"])
PY
      /opt/rocm/bin/hipcc $OBJS $d/combine_t_longdouble.o -shared -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib \
        -lamdhip64 -lrccl -lrt -lpthread -o $d/libshmem_reduce.so &&
      rm -f $d/combine_t_longdouble.o && echo "built $v" ) || echo "variant $v: not built" &
done
wait

#!/bin/bash
# PMC passes over tools/probes/orders_stall_pmc.py (round 6). Run on the GPU box from the repo root.
set -e
cd "$(dirname "$0")/../.."
out=gpurun_out/r06s
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/probes/orders_stall_pmc.py > $out/plain.jsonl
timeout -s KILL 60 rocprofv3 -L > $out/counters.txt 2>&1 || true
pass() {
    name=$1; shift
    timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex 'combine_orders|copy_segments' -d $out/$name -o pmc \
        --output-format csv -- python3 tools/probes/orders_stall_pmc.py > $out/$name.log 2>&1
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT
pass ta TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_TA_BUSY_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum \
    SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE
pass lvl TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE

#!/bin/bash
# Issue / wait split of k_step (two SQ passes).  Run through gpurun.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/sqq_${1:-x}
mkdir -p $OUT
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/p1 -o p1 -- $B > $OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS --output-format csv -d $OUT/p2 -o p2 -- $B > $OUT/p2.log 2>&1
echo done

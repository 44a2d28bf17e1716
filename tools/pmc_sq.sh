#!/bin/bash
# SQ counters of k_step (issue / wait / fetch breakdown).  Run through gpurun.
export TMPDIR=/tmp
OUT=gpurun_out/pmc_sq_${1:-r01}
mkdir -p $OUT
rocprofv3 -L > $OUT/avail.txt 2>&1 || true
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d $OUT/p1 -o p1 -- $B > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_BRANCH --output-format csv -d $OUT/p2 -o p2 -- $B > $OUT/p2.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_IFETCH_LEVEL --output-format csv -d $OUT/p3 -o p3 -- $B > $OUT/p3.log 2>&1
echo done

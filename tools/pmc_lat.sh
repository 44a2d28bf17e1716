#!/bin/bash
# Memory-latency counters of k_step (Little's law: INST_LEVEL_x / INSTS_x = mean latency in cycles).
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/pmc_lat_$TAG
mkdir -p $OUT
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_WAVE_CYCLES --output-format csv -d $OUT/p1 -o p1 -- $B > $OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum --output-format csv -d $OUT/p2 -o p2 -- $B > $OUT/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_FLAT SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_FMA_F32 SQ_THREAD_CYCLES_VALU --output-format csv -d $OUT/p3 -o p3 -- $B > $OUT/p3.log 2>&1
echo done

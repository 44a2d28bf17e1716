#!/bin/bash
# SQ counters of k_step (issue / wait / fetch breakdown) + the stage profile.  Run through gpurun.
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/pmc_sq_$TAG
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES --output-format csv -d $OUT/p1 -o p1 -- $B > $OUT/p1.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_IFETCH SQ_INSTS_BRANCH --output-format csv -d $OUT/p2 -o p2 -- $B > $OUT/p2.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_IFETCH_LEVEL --output-format csv -d $OUT/p3 -o p3 -- $B > $OUT/p3.log 2>&1
echo "[pmc_sq] stage profile"
timeout -k 10 300 python tools/stage_profile.py --steps 200 --out $OUT/stage_200.json > $OUT/stage.log 2>&1
if grep -q "SQC_ICACHE_MISSES" $OUT/avail.txt; then
  echo "[pmc_sq] icache"
  timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $OUT/p4 -o p4 -- $B > $OUT/p4.log 2>&1
fi
echo done

#!/bin/bash
# SQ_INST_LEVEL_* calibration (tools/mb/waitlvl.hip) and the same counters over k_step:
#   tools/gpu_waitlvl.sh TAG     (through gpurun; the summary is tools/summarize_profiles.py waitlvl TAG)
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
C="SQ_WAVES SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM"
timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $OUT/wl_cal -o wl -- tools/mb/waitlvl > $OUT/wl_cal.log 2>&1
grep chain $OUT/wl_cal.log
B3="bench.py --steps 3 --warmup 1 --preroll 20 --no-cpu-baseline --no-parity --no-config2"
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/wl_kstep -o wl -- python $B3 > $OUT/wl_kstep.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU --output-format csv -d $OUT/wl_kstep2 -o wl -- python $B3 > $OUT/wl_kstep2.log 2>&1
echo "[waitlvl] done"

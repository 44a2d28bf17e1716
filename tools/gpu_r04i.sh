#!/bin/bash
# r04i: stage profiles (random, DAPG) of the current kernel + LDS / cache counters of k_step
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04i
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
timeout -k 10 300 python tools/stage_profile.py --steps 20 --out $OUT/stage_profile.json > $OUT/stage.log 2>&1
timeout -k 10 300 python tools/stage_profile.py --steps 20 --policy dapg --out $OUT/stage_profile_dapg.json > $OUT/stage_dapg.log 2>&1
echo "[r04i] stage ok"
B3="bench.py --steps 3 --warmup 1 --preroll 20 --no-cpu-baseline --no-parity --no-config2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --output-format csv -d $OUT/sq3 -o sq3 -- python $B3 > $OUT/sq3.log 2>&1
echo "[r04i] sq ok"
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_fetch -o cf -- ./tools/mb/calib > $OUT/cal_fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cal_write -o cw -- ./tools/mb/calib > $OUT/cal_write.log 2>&1
echo "[r04i] calibration ok"

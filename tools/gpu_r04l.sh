#!/bin/bash
# r04l: main (MPR midphase + bit-sliced scans) vs mpr vs HEAD~ base; GPU suite; stage profiles;
# the wait-class split (SQ_INST_LEVEL_* per instruction class)
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04l
mkdir -p $OUT
bash tools/ab.sh base mpr main > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg base mpr main > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rA --timeout 500 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || true
tail -n 1 $OUT/pytest_gpu.log
timeout -k 10 300 python tools/stage_profile.py --steps 20 --out $OUT/stage_profile.json > $OUT/stage.log 2>&1
timeout -k 10 300 python tools/stage_profile.py --steps 20 --policy dapg --out $OUT/stage_profile_dapg.json > $OUT/stage_dapg.log 2>&1
B3="bench.py --steps 3 --warmup 1 --preroll 20 --no-cpu-baseline --no-parity --no-config2"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM --output-format csv -d $OUT/sql -o sql -- python $B3 > $OUT/sql.log 2>&1
echo "[r04l] done"

#!/bin/bash
# r03r: grouped G-column chains + 2-chain pair columns (g4); + block-split Newton factor when hand
# and objects are uncoupled (spl); hammer parity on spl; A/B against main (r03q).
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03r
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_spl.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_spl.txt 2>&1 || { tail -30 $OUT/pytest_spl.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_spl.txt | tail -8
bash tools/ab.sh main g4 spl > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg main g4 spl > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

#!/bin/bash
# r03o: LDL' Newton factor with unmasked substitutions (ldl) parity on hammer; A/B of main,
# m3 (LL' + med3 pivot + LDS matvec), pk (m3 + packed trailing update), ldl.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03o
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_ldl.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_ldl.txt 2>&1 || { tail -30 $OUT/pytest_ldl.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_ldl.txt | tail -8
bash tools/ab.sh main m3 pk ldl > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg main m3 pk ldl > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

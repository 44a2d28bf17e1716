#!/bin/bash
# r03ze: noslip pair coupling G = Jd Xd' on the matrix cores (nsmf, on crb2) against crb2; hammer
# parity on nsmf first.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03ze
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_nsmf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer or smooth" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_nsmf.txt 2>&1 || { tail -30 $OUT/pytest_nsmf.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_nsmf.txt | tail -8
bash tools/ab.sh -p dapg crb2 nsmf > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
bash tools/ab.sh crb2 nsmf > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt

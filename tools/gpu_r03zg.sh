#!/bin/bash
# r03zg: noslip xd = inv(M) Jd' on the matrix cores (nsx = -DAW_NS_X_MFMA on HEAD) against main
# (HEAD); hammer parity on nsx first.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03zg
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_nsx.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer or smooth" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_nsx.txt 2>&1 || { tail -30 $OUT/pytest_nsx.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_nsx.txt | tail -8
bash tools/ab.sh -p dapg main nsx > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
bash tools/ab.sh main nsx > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt

#!/bin/bash
# r03n: A/B of the shorter dependency chains (lat: pivot-folded substitution, 4-way dot products,
# med3 pivot clamp) against main; hammer parity on lat.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03n
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_lat.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_lat.txt 2>&1 || { tail -30 $OUT/pytest_lat.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_lat.txt | tail -8
bash tools/ab.sh main lat > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg main lat > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

#!/bin/bash
# r03j: row-space noslip (nsr) parity on hammer + A/B against main; MFMA Hessian (hmf) vs its
# base (opq) under DAPG.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03j
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_nsr.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_nsr.txt 2>&1 || { tail -30 $OUT/pytest_nsr.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_nsr.txt | tail -12
bash tools/ab.sh main nsr nsm > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg main nsr nsm opq hmf > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
echo done

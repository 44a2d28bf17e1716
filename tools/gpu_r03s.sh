#!/bin/bash
# r03s: block-split Newton factor (sp), + y-tracking noslip sweep (yt), + merged hand/object dof steps (mg),
# + uniform per-env row pointers (up), + preloaded spill K-steps in the MFMA Hessian (pf), stacked,
# against main (r03q); hammer parity on pf.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03s
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_pf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_pf.txt 2>&1 || { tail -30 $OUT/pytest_pf.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_pf.txt | tail -8
bash tools/ab.sh main sp yt mg up pf > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg main sp yt mg up pf > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

#!/bin/bash
# r04k: MPR-class midphase (mpr), + broadphase loads up front (bp) against the abs-noise Newton
# floor (main) and r04h's best (ni2); parity of bp with the f32-model sensitivity classifier
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04k
mkdir -p $OUT
bash tools/ab.sh ni2 main mpr bp > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg ni2 main mpr bp > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
AW_LIB=mj_envs_amd/libadroit_hip_bp.so timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 500 --timeout-method thread > $OUT/pytest_gpu_bp.log 2>&1 || true
tail -n 1 $OUT/pytest_gpu_bp.log

#!/bin/bash
# r04j: per-dof Newton noise floor over the terms' magnitudes (4e-6 main / 1.6e-5 nf16) vs the
# magnitude-of-sums floor (ni2 = r04h's best), HEAD~ base; parity of both
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04j
mkdir -p $OUT
bash tools/ab.sh base ni2 main nf16 > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg base ni2 main nf16 > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
for v in main nf16; do
  LIB=mj_envs_amd/libadroit_hip_$v.so; [ $v = main ] && LIB=mj_envs_amd/libadroit_hip.so
  AW_LIB=$LIB timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 500 --timeout-method thread -k "teacher_forced or c3 or one_env_step" > $OUT/pytest_parity_$v.log 2>&1 || true
  tail -n 1 $OUT/pytest_parity_$v.log
done

#!/bin/bash
# A/B of library variants + their oracle parity (run through gpurun):
#   tools/gpu_ab_parity.sh TAG "variants"    (main = mj_envs_amd/libadroit_hip.so)
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
bash tools/ab.sh $2 > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg $2 > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
for v in $2; do
  [ $v = main ] && continue
  AW_LIB=mj_envs_amd/libadroit_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 500 --timeout-method thread -k "teacher_forced or c3 or one_env_step" > $OUT/pytest_parity_$v.log 2>&1 || true
  echo "$v: $(tail -n 1 $OUT/pytest_parity_$v.log)"
done

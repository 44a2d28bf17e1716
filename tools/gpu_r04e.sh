#!/bin/bash
# r04e: capsule-box on 16-lane rows (main) vs HEAD (base); per-dof Newton noise floor at 8e-6 / 3.2e-5
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04e
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_colliders.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest_colliders.log 2>&1
tail -n 2 $OUT/pytest_colliders.log
for v in main ntn8 ntn32; do
  LIB=mj_envs_amd/libadroit_hip_$v.so; [ $v = main ] && LIB=mj_envs_amd/libadroit_hip.so
  AW_LIB=$LIB timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 500 --timeout-method thread -k "teacher_forced or c3 or one_env_step" > $OUT/pytest_parity_$v.log 2>&1 || true
  tail -n 1 $OUT/pytest_parity_$v.log
done
bash tools/ab.sh base main ntn8 ntn32 > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg base main ntn8 ntn32 > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

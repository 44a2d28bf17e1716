#!/bin/bash
# r04f: capsule-box midphase + 16-lane rows (main) vs HEAD (base); Newton termination variants
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04f
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_colliders.py -m gpu -v --timeout 200 --timeout-method thread > $OUT/pytest_colliders.log 2>&1
tail -n 1 $OUT/pytest_colliders.log
bash tools/ab.sh base main nti ntni ntn > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg base main nti ntni ntn > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
for v in main nti ntni ntn; do
  LIB=mj_envs_amd/libadroit_hip_$v.so; [ $v = main ] && LIB=mj_envs_amd/libadroit_hip.so
  AW_LIB=$LIB timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 500 --timeout-method thread -k "teacher_forced or c3 or one_env_step" > $OUT/pytest_parity_$v.log 2>&1 || true
  tail -n 1 $OUT/pytest_parity_$v.log
done

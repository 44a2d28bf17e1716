#!/bin/bash
# r04d: Newton termination A/B -- norm-wide fp32 noise floor (main) vs per-dof (ntn): misses,
# their attribution and the cost in k_step time
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04d
mkdir -p $OUT
for v in main ntn; do
  LIB=mj_envs_amd/libadroit_hip_$v.so; [ $v = main ] && LIB=mj_envs_amd/libadroit_hip.so
  AW_LIB=$LIB timeout -k 10 300 python -u tools/diag_tf.py relocate-v0 random 1 256 3 > $OUT/diag_relocate0_$v.log 2>&1
  AW_LIB=$LIB timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 500 --timeout-method thread -k "teacher_forced or c3" > $OUT/pytest_parity_$v.log 2>&1 || true
  tail -n 2 $OUT/pytest_parity_$v.log
done
bash tools/ab.sh main ntn > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg main ntn > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

#!/bin/bash
# r04g: Newton termination -- accurate improvement (nti) with no fp32 noise-floor exit (ntx) or a
# per-dof floor at 8e-6 / 3.2e-5 (ntni8 / ntni32)
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04g
mkdir -p $OUT
bash tools/ab.sh main nti ntx ntni8 ntni32 > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg main nti ntx ntni8 ntni32 > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
for v in ntx ntni8 ntni32; do
  AW_LIB=mj_envs_amd/libadroit_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 500 --timeout-method thread -k "teacher_forced or c3 or one_env_step" > $OUT/pytest_parity_$v.log 2>&1 || true
  tail -n 1 $OUT/pytest_parity_$v.log
done

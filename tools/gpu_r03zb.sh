#!/bin/bash
# r03zb: block-split Newton factor (sp, on top of ueo: scalar env index + opaque env-level lane
# ids) and + mass-matrix rows from an MFMA product P = B C' in CRB (crb) against ueo; hammer
# parity (incl. the constraint-free smooth-dynamics test) on sp and crb first.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03zb
mkdir -p $OUT
for v in sp crb; do
  AW_LIB=$PWD/mj_envs_amd/libadroit_hip_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer or smooth" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_$v.txt 2>&1 || { tail -30 $OUT/pytest_$v.txt; exit 1; }
  grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_$v.txt | tail -8
done
bash tools/ab.sh ueo sp crb > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg ueo sp crb > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

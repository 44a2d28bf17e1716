#!/bin/bash
# r03zc: mass-matrix rows from an MFMA product P = B C' in CRB (crb, on top of sp) against sp;
# hammer parity (incl. the constraint-free smooth-dynamics test) on crb first.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03zc
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_crb.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer or smooth" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_crb.txt 2>&1 || { tail -30 $OUT/pytest_crb.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_crb.txt | tail -8
bash tools/ab.sh sp crb > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg sp crb > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

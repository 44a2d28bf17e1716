#!/bin/bash
# r03p: stacked A/B on the LDL' base (ldl): + prefetched MFMA Hessian and unrolled J'f (hm),
# + ballot noslip setup (ns), + pointer-jumping kinematics (kn), + pointer-jumping RNE (rn),
# + unrolled subtree sums (all); hammer parity on all.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03p
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_all.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_all.txt 2>&1 || { tail -30 $OUT/pytest_all.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_all.txt | tail -8
bash tools/ab.sh ldl hm ns kn rn all > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg ldl hm ns kn rn all > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

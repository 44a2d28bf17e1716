#!/bin/bash
# r04h: GPU suite on the new defaults (per-dof Newton floor + row-wise improvement, box-box /
# plane midphase), relocate C3 miss attribution, A/B against HEAD~ (base)
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04h
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rA --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && rc=0 || rc=$?
tail -n 3 $OUT/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest rc $rc: stopping"; exit $rc;; esac
timeout -k 10 400 python -u tools/diag_tf.py relocate-v0 random 200 256 6 > $OUT/diag_relocate_c3.log 2>&1
grep "outside tolerance\|misses per step" $OUT/diag_relocate_c3.log
bash tools/ab.sh base main ni2 blk > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg base main ni2 blk > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

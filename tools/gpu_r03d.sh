#!/bin/bash
# Round-3 GPU pass: full GPU suite, hammer C3 miss attribution, A/B of variants.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03d}
mkdir -p $OUT
echo "[gpu] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rA --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1 && rc=0 || rc=$?
tail -3 $OUT/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest rc $rc: stopping"; exit $rc;; esac
echo "[gpu] diag"
timeout -k 10 600 python -u tools/diag_tf.py hammer-v0 random 200 256 20 > $OUT/diag.log 2>&1
cp gpurun_out/diag_hammer_random.json $OUT/
echo "[gpu] ab"
bash tools/ab.sh main base tftz tla2 tnsb ftz flat > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg main base tnsb > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
echo "[gpu] done"

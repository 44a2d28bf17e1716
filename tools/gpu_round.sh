#!/bin/bash
# One GPU-box pass (run through gpurun): gpu tests, smoke, bench.  Every GPU step has its own
# time limit; the first failure ends the script.
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/$TAG
mkdir -p $OUT
echo "[gpu_round] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1 && rc=0 || rc=$?
tail -3 $OUT/pytest_gpu.log
# a failing test is a result; a time-out / crash (124, 134, 137, 139) ends the GPU work here
case $rc in 0|1) ;; *) echo "pytest rc $rc: stopping"; exit $rc;; esac
echo "[gpu_round] smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
echo "[gpu_round] bench"
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo "[gpu_round] done"

#!/bin/bash
# Quick GPU check (through gpurun): selected GPU tests (PYTEST_ARGS), then the headline bench line
# and BASELINE config 3's relocate line, into gpurun_out/<tag>.  Each GPU step has its own limit;
# a crash / time-out ends the script.
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-quick}
OUT=gpurun_out/$TAG
mkdir -p $OUT
echo "[quick] tests: ${PYTEST_ARGS:-tests -m gpu}"
timeout -k 10 ${PYTEST_TIMEOUT:-600} python -u -m pytest ${PYTEST_ARGS:-tests -m gpu} -v -s -rA --timeout 400 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && rc=0 || rc=$?
tail -5 $OUT/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest rc $rc: stopping"; exit $rc;; esac
if [ -z "$NO_BENCH" ]; then
echo "[quick] bench"
timeout -k 10 300 python bench.py --steps 100 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo "[quick] config 3 relocate"
timeout -k 10 200 python bench.py --env relocate-v0 --envs-per-gpu 16384 --steps 200 --no-cpu-baseline > $OUT/bench_relocate.json 2> $OUT/bench_relocate.err
cat $OUT/bench_relocate.json
fi
echo "[quick] done"

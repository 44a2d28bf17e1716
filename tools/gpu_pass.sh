#!/bin/bash
# GPU pass A (run through gpurun): GPU test suite, smoke, the headline bench line, the DAPG
# closed-loop line, BASELINE config 3 (door / pen / relocate at 16 384 envs) and config 5 (depth)
# lines, into gpurun_out/<tag>.  Every GPU step has its own time limit; a crash / time-out ends it.
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r03}
OUT=gpurun_out/$TAG
mkdir -p $OUT
echo "[pass] tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rA --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $OUT/pytest_gpu.log 2>&1 && rc=0 || rc=$?
tail -3 $OUT/pytest_gpu.log
case $rc in 0|1) ;; *) echo "pytest rc $rc: stopping"; exit $rc;; esac
echo "[pass] smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
echo "[pass] bench"
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo "[pass] bench dapg"
timeout -k 10 300 python bench.py --policy dapg --steps 200 --no-cpu-baseline --no-config2 > $OUT/bench_dapg.json 2> $OUT/bench_dapg.err
echo "[pass] config 3"
for e in door-v0 pen-v0 relocate-v0; do
  timeout -k 10 200 python bench.py --env $e --envs-per-gpu 16384 --steps 200 --no-cpu-baseline >> $OUT/bench_config3.jsonl 2>> $OUT/bench_config3.err
done
echo "[pass] config 5"
timeout -k 10 200 python bench.py --depth --steps 200 --no-cpu-baseline > $OUT/bench_depth.json 2> $OUT/bench_depth.err
echo "[pass] done"

#!/bin/bash
# One GPU-box pass (run through gpurun): gpu tests, smoke, bench, kernel trace, HBM PMC.
# Every GPU step has its own time limit; the first failure ends the script.
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
echo "[gpu_round] tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -3 $OUT/pytest_gpu.log
echo "[gpu_round] smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
echo "[gpu_round] bench"
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
echo "[gpu_round] kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o kt -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-config2 > $OUT/trace.log 2>&1
echo "[gpu_round] pmc fetch"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pf -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config2 > $OUT/pmc_fetch.log 2>&1
echo "[gpu_round] pmc write"
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pw -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config2 > $OUT/pmc_write.log 2>&1
echo "[gpu_round] done"

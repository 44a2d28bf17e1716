#!/bin/bash
# r04a: the launcher path on hardware (one RCCL rank) + the headline line through the launcher
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04a
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_distributed.py -m gpu -v -s --timeout 500 --timeout-method thread > $OUT/pytest_launch.log 2>&1
tail -3 $OUT/pytest_launch.log
timeout -k 10 400 python bench.py --gpus 1 --launch --steps 200 --no-cpu-baseline --no-config2 > $OUT/bench_launch.json 2> $OUT/bench_launch.err
cat $OUT/bench_launch.json

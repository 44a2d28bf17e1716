#!/bin/bash
# r03zi: config 4's 262 144 hammer envs on ONE GPU and the closed loop with the on-device random-init
# MLP policy at 65 536 envs, on the current kernel (DESIGN quoted round-1 numbers for both).
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03zi
mkdir -p $OUT
timeout -k 10 400 python bench.py --envs-per-gpu 262144 --steps 50 --no-cpu-baseline --no-config2 > $OUT/bench_config4_1gpu.json 2> $OUT/bench_config4_1gpu.err
cat $OUT/bench_config4_1gpu.json
timeout -k 10 300 python bench.py --policy random-mlp --steps 200 --no-cpu-baseline --no-config2 > $OUT/bench_mlp.json 2> $OUT/bench_mlp.err
cat $OUT/bench_mlp.json

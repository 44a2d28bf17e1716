#!/bin/bash
# BASELINE config 3: door / pen / relocate at 16 384 envs each on one GPU (run through gpurun)
set -e -o pipefail
mkdir -p gpurun_out
for e in door-v0 pen-v0 relocate-v0; do
  timeout -k 10 200 python bench.py --env $e --envs-per-gpu 16384 --steps 200 --no-cpu-baseline > gpurun_out/bench_$e.json
  cat gpurun_out/bench_$e.json
done

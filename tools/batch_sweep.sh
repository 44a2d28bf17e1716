#!/bin/bash
# Throughput against batch size on one GPU (run through gpurun): the headline bench (hammer-v0,
# random policy, staggered phases, auto-reset) at 1 024 ... 262 144 envs.  Prints envs, env-steps/s,
# ms per env-step and k_step ms per size.
set -e -o pipefail
OUT=gpurun_out/${1:-batch}
mkdir -p $OUT
for n in 1024 2048 4096 8192 16384 32768 65536 131072 262144; do
  steps=200; [ $n -ge 131072 ] && steps=60
  timeout -k 10 300 python bench.py --envs-per-gpu $n --steps $steps --warmup 5 --no-cpu-baseline --no-config2 --no-parity \
    > $OUT/b_$n.json 2> $OUT/b_$n.err
  python -c "import json;d=json.load(open('$OUT/b_$n.json'));print($n, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
done

#!/bin/bash
# A/B bench of library variants in the closed-loop DAPG regime (run through gpurun):
#   tools/ab_policy.sh name1 name2 ...
set -e -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  AW_LIB=mj_envs_amd/libadroit_hip_$v.so timeout -k 10 200 python bench.py --steps 100 --policy dapg --no-cpu-baseline --no-parity --no-config2 > gpurun_out/abd_$v.json 2> gpurun_out/abd_$v.err
  python -c "import json;d=json.load(open('gpurun_out/abd_$v.json'));print('dapg $v', d['value'], d['roofline']['kernel_ms'], d['episodes']['success_pct'])"
done

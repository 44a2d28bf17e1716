#!/bin/bash
# A/B bench of library variants (run through gpurun): tools/ab.sh name1 name2 ...
set -e -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  AW_LIB=mj_envs_amd/libadroit_hip_$v.so timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', d['value'], d['roofline']['kernel_ms'])"
done

#!/bin/bash
# A/B bench of library variants (run through gpurun): tools/ab.sh [-p dapg] name1 name2 ...
# Each variant runs twice, interleaved (A B A B), on the headline workload (random policy) or
# with -p dapg in the closed-loop DAPG regime; prints env-steps/s, k_step ms and the bench's
# same-run parity on the headline handle.  BENCH_ARGS adds bench.py arguments (another env / size).
set -e -o pipefail
mkdir -p gpurun_out/ab
POL=none
if [ "$1" = "-p" ]; then POL=$2; shift 2; fi
for rep in 1 2; do
  for v in "$@"; do
    LIB=mj_envs_amd/libadroit_hip_$v.so
    [ "$v" = "main" ] && LIB=mj_envs_amd/libadroit_hip.so
    AW_LIB=$LIB timeout -k 10 200 python bench.py --steps 200 --policy $POL --no-cpu-baseline --no-config2 $BENCH_ARGS \
      > gpurun_out/ab/${POL}_${v}_$rep.json 2> gpurun_out/ab/${POL}_${v}_$rep.err
    python -c "import json;d=json.load(open('gpurun_out/ab/${POL}_${v}_$rep.json'));p=d.get('parity_one_step',{});print('$POL $v rep$rep', d['value'], d['roofline']['kernel_ms'], 'parity', p.get('frac_within_tol'), 'success', d['episodes']['success_pct'], 'wide', d.get('wide_tier_envs'), 'overflow', d.get('overflow_envs'))"
  done
done

#!/bin/bash
# r03w: which round-3 change moved the one-step oracle misses on DAPG states (r03h 46, main 69 of 8192)?
# Same saved states, one variant per numerics change reverted.
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_noslip.py save 16384 > gpurun_out/diag_ns_save.log 2>&1
for v in wl r03h nsp llt hv lvl crbv; do
  AW_LIB=$PWD/mj_envs_amd/libadroit_hip_$v.so timeout -k 10 300 python tools/diag_noslip.py $v 8192 > gpurun_out/diag_ns_$v.log 2>&1
  python -c "
import json; d=json.load(open('gpurun_out/diag_ns_$v.json')); print('$v', d['misses'], d['frac'], (d.get('vs_main') or {}).get('max_dq'), (d.get('vs_main') or {}).get('n_dq_gt_1e4'))"
done

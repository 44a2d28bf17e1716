#!/bin/bash
# r03v: noslip row saves by v_writelane + start/end sweep improvement (wl) against crb; one-step
# oracle parity at scale on the same DAPG states for the r03h kernel, main (r03q) and wl.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03v
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_wl.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_wl.txt 2>&1 || { tail -30 $OUT/pytest_wl.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_wl.txt | tail -8
timeout -k 10 300 python tools/diag_noslip.py save 16384 > gpurun_out/diag_ns_save.log 2>&1
timeout -k 10 300 python tools/diag_noslip.py main 8192 > gpurun_out/diag_ns_main.log 2>&1
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_r03h.so timeout -k 10 300 python tools/diag_noslip.py r03h 8192 > gpurun_out/diag_ns_r03h.log 2>&1
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_wl.so timeout -k 10 300 python tools/diag_noslip.py wl 8192 > gpurun_out/diag_ns_wl.log 2>&1
for t in r03h main wl; do python -c "
import json; d=json.load(open('gpurun_out/diag_ns_$t.json')); print('$t', d['misses'], d['frac'], (d.get('vs_main') or {}).get('max_dq'), (d.get('vs_main') or {}).get('n_dq_gt_1e4'))"; done
bash tools/ab.sh crb wl > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg crb wl > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

#!/bin/bash
# r03t: one-step oracle parity at scale on DAPG steady-state states (16 384 stepped, 4 096
# checked): main (r03q) vs sp (block-split factor) vs up (+ y-tracking noslip, merged dof steps,
# uniform row pointers).
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_noslip.py save 16384 > gpurun_out/diag_ns_save.log 2>&1
timeout -k 10 300 python tools/diag_noslip.py main 4096 > gpurun_out/diag_ns_main.log 2>&1
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_sp.so timeout -k 10 300 python tools/diag_noslip.py sp 4096 > gpurun_out/diag_ns_sp.log 2>&1
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_up.so timeout -k 10 300 python tools/diag_noslip.py up 4096 > gpurun_out/diag_ns_up.log 2>&1
for t in main sp up; do python -c "
import json; d=json.load(open('gpurun_out/diag_ns_$t.json')); print('$t', d['misses'], d['frac'], d.get('vs_main'))"; done

#!/bin/bash
# r03k: one-step oracle parity of main vs the row-space noslip (nsr) on the same 16 384 DAPG
# steady-state states (4 096 checked), with the noslip pair counts of the misses.
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/diag_noslip.py save 16384 > gpurun_out/diag_ns_save.log 2>&1
timeout -k 10 300 python tools/diag_noslip.py main 4096 > gpurun_out/diag_ns_main.log 2>&1
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_nsr.so timeout -k 10 300 python tools/diag_noslip.py nsr 4096 > gpurun_out/diag_ns_nsr.log 2>&1
tail -2 gpurun_out/diag_ns_main.log | cut -c1-600
tail -2 gpurun_out/diag_ns_nsr.log | cut -c1-1500

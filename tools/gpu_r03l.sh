#!/bin/bash
# r03l: A/B of the pair-column setup from the transpose buffer (nsx) against nsr; DAPG one-step
# parity diagnostic with the oracle's noslip sweep counts (nsx).
set -e -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r03l
timeout -k 10 300 python tools/diag_noslip.py save 16384 > gpurun_out/diag_ns_save.log 2>&1
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_nsx.so timeout -k 10 300 python tools/diag_noslip.py nsx 4096 > gpurun_out/diag_ns_nsx.log 2>&1
tail -1 gpurun_out/diag_ns_nsx.log | cut -c1-3000
bash tools/ab.sh main nsr nsx > gpurun_out/r03l/ab_random.txt 2>&1
cat gpurun_out/r03l/ab_random.txt
bash tools/ab.sh -p dapg main nsr nsx > gpurun_out/r03l/ab_dapg.txt 2>&1
cat gpurun_out/r03l/ab_dapg.txt

#!/bin/bash
# r03g: A/B of the pair-space noslip sweep (nsg) and constant-address model reads (as4) against
# main, then the parity suite on the nsg build.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03g
mkdir -p $OUT
bash tools/ab.sh main as4 nsg > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg main nsg > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_nsg.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_nsg.txt 2>&1
tail -5 $OUT/pytest_nsg.txt

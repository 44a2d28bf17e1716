#!/bin/bash
# r03x: uniform env-loop exits + global-address state rows (ua), + opaque env-level lane ids (uao:
# 84 B/lane scratch) against wl; hammer parity on uao; then the r03w one-step miss attribution.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03x
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_uao.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_uao.txt 2>&1 || { tail -30 $OUT/pytest_uao.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_uao.txt | tail -8
bash tools/ab.sh wl ua uao > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg wl ua uao > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
bash tools/gpu_r03w.sh

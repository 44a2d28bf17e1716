#!/bin/bash
# r03y: noslip pair columns on MFMA (nsmf, on top of uao: uniform env-loop exits, global-address
# state rows, opaque env-level lane ids) against wl and uao; hammer parity on nsmf; then the
# one-step miss attribution over numerics variants (r03w).
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03y
mkdir -p $OUT
AW_LIB=$PWD/mj_envs_amd/libadroit_hip_nsmf.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_closed_loop.py -k "hammer" -x -q --timeout 300 --timeout-method thread -s > $OUT/pytest_nsmf.txt 2>&1 || { tail -30 $OUT/pytest_nsmf.txt; exit 1; }
grep -E "teacher-forced|headline|passed|failed" $OUT/pytest_nsmf.txt | tail -8
bash tools/ab.sh wl uao nsmf > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg wl uao nsmf > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
sed -i 's/for v in wl r03h nsp llt hv lvl crbv; do/for v in wl r03h nsp llt hv lvl crbv nsmf; do/' tools/gpu_r03w.sh
bash tools/gpu_r03w.sh

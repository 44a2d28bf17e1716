#!/bin/bash
# r04c: attribute the teacher-forced misses (relocate step 0 in C3, hammer under DAPG) with
# tools/diag_tf.py, then the parity tests with the fp32-action fix
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r04c
mkdir -p $OUT
timeout -k 10 300 python -u tools/diag_tf.py relocate-v0 random 1 256 8 > $OUT/diag_relocate_step0.log 2>&1
timeout -k 10 300 python -u tools/diag_tf.py hammer-v0 dapg 80 64 10 > $OUT/diag_hammer_dapg.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -v -s --timeout 500 --timeout-method thread -k "teacher_forced or c3" > $OUT/pytest_parity.log 2>&1 || true
tail -3 $OUT/pytest_parity.log

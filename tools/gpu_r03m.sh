#!/bin/bash
# r03m: full GPU suite on the row-space noslip build + packed-FMA issue-rate microbenchmark.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03m
mkdir -p $OUT
timeout -k 10 60 ./tools/mb/pk_fma > $OUT/pk_fma.txt 2>&1
cat $OUT/pk_fma.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s -rA --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 && rc=0 || rc=$?
tail -3 $OUT/pytest_gpu.log
grep -E "teacher-forced|headline config" $OUT/pytest_gpu.log | cut -c1-200
exit $rc

#!/bin/bash
# GPU-box profiling recipe (run through gpurun), into the same gpurun_out/<tag> directory as
# tools/gpu_round.sh so tools/summarize_profiles.py <tag> finds both.  Counters are collected in
# their own passes with --pmc only (no sys/runtime traces), one counter group per pass.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02}
mkdir -p $OUT
B="bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --no-config2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o kt -- python $B > $OUT/trace.log 2>&1
echo "[prof_round] trace ok"
B3="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-config2"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pf -- python $B3 > $OUT/pmc_fetch.log 2>&1
echo "[prof_round] fetch ok"
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pw -- python $B3 > $OUT/pmc_write.log 2>&1
echo "[prof_round] done"

#!/bin/bash
# GPU-box profiling recipe (run through gpurun). Writes under gpurun_out/.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/prof_${1:-r01}
mkdir -p $OUT
timeout -k 10 300 python bench.py --steps ${2:-200} > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o kt -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-config2 > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pf -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config2 > $OUT/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pw -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-config2 > $OUT/pmc_write.log 2>&1
echo done

#!/bin/bash
# End-of-round GPU pass (run through gpurun): tools/gpu_round.sh (tests, smoke, headline bench),
# the DAPG closed-loop bench line, tools/prof_round.sh (rocprof kernel trace + HBM PMC) and the
# stage profiles under both policies, all into gpurun_out/<tag>.  Each GPU step has its own
# time limit; the first failure ends the script.
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r02}
OUT=gpurun_out/$TAG
bash tools/gpu_round.sh $TAG
echo "[gpu_final] bench --policy dapg"
timeout -k 10 300 python bench.py --policy dapg --steps 200 --no-cpu-baseline --no-config2 > $OUT/bench_dapg.json 2> $OUT/bench_dapg.err
bash tools/prof_round.sh $TAG
echo "[gpu_final] stage profiles"
timeout -k 10 300 python tools/stage_profile.py --steps 20 --out $OUT/stage_profile.json > $OUT/stage.log 2>&1
timeout -k 10 300 python tools/stage_profile.py --steps 20 --policy dapg --out $OUT/stage_profile_dapg.json > $OUT/stage_dapg.log 2>&1
echo "[gpu_final] done"

#!/bin/bash
# Final round-3 GPU pass (run through gpurun) on the in-tree libraries: the GPU test suite, smoke,
# the headline bench line, DAPG closed loop, BASELINE config 3 / config 5 lines, the rocprof
# kernel trace + HBM PMC passes, SQ counter passes and the stage profiles under both policies,
# all into gpurun_out/<tag>.  Every GPU step has its own time limit; the first failure ends it.
set -e -o pipefail
export TMPDIR=/tmp
TAG=${1:-r03zf}
OUT=gpurun_out/$TAG
bash tools/gpu_pass.sh $TAG
bash tools/prof_round.sh $TAG
bash tools/pmc_sq_quick.sh $TAG
echo "[final] stage profiles"
timeout -k 10 300 python tools/stage_profile.py --steps 20 --out $OUT/stage_profile.json > $OUT/stage.log 2>&1
timeout -k 10 300 python tools/stage_profile.py --steps 20 --policy dapg --out $OUT/stage_profile_dapg.json > $OUT/stage_dapg.log 2>&1
echo "[final] done"

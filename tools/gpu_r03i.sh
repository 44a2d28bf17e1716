#!/bin/bash
# r03i: A/B of opaque env-level lane ids (opq: scratch 272 -> 152 B/lane) against main under both
# policies, then the stage profiles of main (random + DAPG).
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03i
mkdir -p $OUT
bash tools/ab.sh main opq > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg main opq > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
timeout -k 10 300 python tools/stage_profile.py --steps 20 --out $OUT/stage_profile.json > $OUT/stage.log 2>&1
timeout -k 10 300 python tools/stage_profile.py --steps 20 --policy dapg --out $OUT/stage_profile_dapg.json > $OUT/stage_dapg.log 2>&1
echo done

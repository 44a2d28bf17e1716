#!/bin/bash
# A/B pass (run through gpurun): tools/gpu_ab.sh TAG "variants random" "variants dapg"
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
bash tools/ab.sh $2 > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
if [ -n "$3" ]; then
  bash tools/ab.sh -p dapg $3 > $OUT/ab_dapg.txt 2>&1
  cat $OUT/ab_dapg.txt
fi

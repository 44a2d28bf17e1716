#!/bin/bash
# r03zd: MFMA CRB without the split factor (crb2, on ueo) against ueo, and the Newton factor's
# look-ahead depth on crb2 (la1, la4; default 2).
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03zd
mkdir -p $OUT
bash tools/ab.sh ueo crb2 la1 la4 > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg ueo crb2 la1 la4 > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt

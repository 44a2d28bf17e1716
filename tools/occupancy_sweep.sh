#!/bin/bash
# Latency-hiding curve of k_step (run through gpurun): the headline bench with the persistent grid
# forced to G workgroups (AW_STEP_GRID; one workgroup = one wave = one env at a time).  1 024 = one
# wave per SIMD on 256 CUs, 2 048 = two (the default, the LDS / VGPR limit), 1 536 = half the SIMDs
# with two.  Each variant twice, interleaved; prints env-steps/s and k_step ms.
set -e -o pipefail
OUT=gpurun_out/${1:-occ}
mkdir -p $OUT
for rep in 1 2; do
  for g in 1024 1536 2048; do
    AW_STEP_GRID=$g timeout -k 10 200 python bench.py --steps 200 ${POLICY:+--policy $POLICY} --no-cpu-baseline --no-config2 --no-parity \
      > $OUT/occ_${POLICY:-none}_${g}_$rep.json 2> $OUT/occ_${POLICY:-none}_${g}_$rep.err
    python -c "import json;d=json.load(open('$OUT/occ_${POLICY:-none}_${g}_$rep.json'));print('grid $g rep$rep', d['value'], d['roofline']['kernel_ms'])"
  done
done

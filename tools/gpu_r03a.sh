#!/bin/bash
# Round-3 first GPU pass (run through gpurun): hammer C3 miss attribution (tools/diag_tf.py) and
# the SQ issue / wait split of k_step (separate --pmc passes, program directly after --).
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03a}
mkdir -p $OUT
echo "[r03a] diag"
timeout -k 10 600 python -u tools/diag_tf.py hammer-v0 random 200 256 40 > $OUT/diag.log 2>&1
cp gpurun_out/diag_hammer_random.json $OUT/
echo "[r03a] counters list"
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1
B="bench.py --steps 3 --warmup 1 --preroll 20 --no-cpu-baseline --no-parity --no-config2"
echo "[r03a] sq1"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/sq1 -o sq1 -- python $B > $OUT/sq1.log 2>&1
echo "[r03a] sq2"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS --output-format csv -d $OUT/sq2 -o sq2 -- python $B > $OUT/sq2.log 2>&1
echo "[r03a] sq3"
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_IFETCH SQ_IFETCH_LEVEL --output-format csv -d $OUT/sq3 -o sq3 -- python $B > $OUT/sq3.log 2>&1
echo "[r03a] done"

#!/bin/bash
# GPU pass B (run through gpurun): rocprofv3 kernel trace + stats of the headline bench, HBM PMC
# (FETCH_SIZE, WRITE_SIZE in separate passes), the SQ issue / wait split (three passes of <= 8 SQ
# counters), and the stage profiles under both policies, into gpurun_out/<tag>.  Counters run
# with --pmc only; the program follows -- directly.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03}
mkdir -p $OUT
# the counter-calibration programs (git-ignored binaries; built here when absent)
for p in calib waitlvl; do
  [ -x tools/mb/$p ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o tools/mb/$p tools/mb/$p.hip
done
B="bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity --no-config2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o kt -- python $B > $OUT/trace.log 2>&1
echo "[prof] trace ok"
B3="bench.py --steps 3 --warmup 1 --preroll 20 --no-cpu-baseline --no-parity --no-config2"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o pf -- python $B3 > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o pw -- python $B3 > $OUT/pmc_write.log 2>&1
# FETCH_SIZE / WRITE_SIZE calibration for k_step's 4 B/lane row pattern (known-byte kernels)
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_fetch -o cf -- tools/mb/calib > $OUT/cal_fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/cal_write -o cw -- tools/mb/calib > $OUT/cal_write.log 2>&1
echo "[prof] hbm ok"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS --output-format csv -d $OUT/sq1 -o sq1 -- python $B3 > $OUT/sq1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAIT_INST_LDS --output-format csv -d $OUT/sq2 -o sq2 -- python $B3 > $OUT/sq2.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_IFETCH SQ_IFETCH_LEVEL --output-format csv -d $OUT/sq3 -o sq3 -- python $B3 > $OUT/sq3.log 2>&1
echo "[prof] sq ok"
C="SQ_WAVES SQ_WAVE_CYCLES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_SMEM"
timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d $OUT/wl_cal -o wl -- tools/mb/waitlvl > $OUT/wl_cal.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/wl_kstep -o wl -- python $B3 > $OUT/wl_kstep.log 2>&1
echo "[prof] wait levels ok"
timeout -k 10 300 python tools/stage_profile.py --steps 20 --out $OUT/stage_profile.json > $OUT/stage.log 2>&1
timeout -k 10 300 python tools/stage_profile.py --steps 20 --policy dapg --out $OUT/stage_profile_dapg.json > $OUT/stage_dapg.log 2>&1
echo "[prof] done"

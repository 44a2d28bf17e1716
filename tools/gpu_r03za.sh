#!/bin/bash
# r03za: env index kept scalar (readfirstlane claim: ue) and + opaque env-level lane ids (ueo)
# against main (HEAD); HBM FETCH / WRITE passes on ue.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r03za
mkdir -p $OUT
bash tools/ab.sh main ue ueo > $OUT/ab_random.txt 2>&1
cat $OUT/ab_random.txt
bash tools/ab.sh -p dapg main ue ueo > $OUT/ab_dapg.txt 2>&1
cat $OUT/ab_dapg.txt
B3="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity --no-config2"
for v in ue ueo; do
  AW_LIB=$PWD/mj_envs_amd/libadroit_hip_$v.so timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$v -o pf -- python $B3 > $OUT/pmc_fetch_$v.log 2>&1
  AW_LIB=$PWD/mj_envs_amd/libadroit_hip_$v.so timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$v -o pw -- python $B3 > $OUT/pmc_write_$v.log 2>&1
done
echo done

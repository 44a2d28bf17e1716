#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of k_step per library variant (run through gpurun after an A/B):
#   tools/gpu_pmc_ab.sh TAG "variants"    (main = mj_envs_amd/libadroit_hip.so)
# one --pmc counter per pass (MI355X_MICROARCH.md HBM section), each pass under its own time limit
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/$1
mkdir -p $OUT
B3="bench.py --steps 3 --warmup 1 --preroll 20 --no-cpu-baseline --no-parity --no-config2"
for v in $2; do
  LIB=mj_envs_amd/libadroit_hip_$v.so
  [ "$v" = "main" ] && LIB=mj_envs_amd/libadroit_hip.so
  AW_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf_$v -o pf -- python $B3 > $OUT/pf_$v.log 2>&1
  AW_LIB=$LIB timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw_$v -o pw -- python $B3 > $OUT/pw_$v.log 2>&1
  python - $OUT $v <<'PY'
import csv, re, sys, statistics
out, v = sys.argv[1], sys.argv[2]
def ks(path, c):
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if re.search(r"\bk_step(?![A-Za-z0-9_])", r["Kernel_Name"]) and r["Counter_Name"] == c]
f = ks(f"{out}/pf_{v}/pf_counter_collection.csv", "FETCH_SIZE")
w = ks(f"{out}/pw_{v}/pw_counter_collection.csv", "WRITE_SIZE")
n = 65536
print(f"{v}: k_step launches {len(f)}/{len(w)}  fetch {statistics.mean(f) * 1024 / n:.1f} B/env-step  "
      f"write {statistics.mean(w) * 1024 / n:.1f} B/env-step")
PY
done

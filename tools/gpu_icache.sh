#!/bin/bash
# Instruction-cache behaviour of k_step (run through gpurun): the SQC instruction-cache counters over
# the headline bench (3 timed steps after a 20-step pre-roll), one --pmc pass, plus the list of the
# counters this box offers.
set -e -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-icache}
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
B3="bench.py --steps 3 --warmup 1 --preroll 20 --no-cpu-baseline --no-parity --no-config2"
timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d $OUT/ic -o ic -- python $B3 > $OUT/ic.log 2>&1
python - $OUT <<'PY'
import csv, re, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f"{out}/ic/ic_counter_collection.csv")):
    if re.search(r"\bk_step(?![A-Za-z0-9_])", r["Kernel_Name"]):
        agg[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
per = {c: sum(d.values()) / len(d) for c, d in agg.items()}
print({c: f"{v:.4g}" for c, v in per.items()})
if "SQC_ICACHE_REQ" in per and per["SQC_ICACHE_REQ"]:
    print("miss rate", per.get("SQC_ICACHE_MISSES", 0) / per["SQC_ICACHE_REQ"],
          "hit rate", per.get("SQC_ICACHE_HITS", 0) / per["SQC_ICACHE_REQ"])
PY

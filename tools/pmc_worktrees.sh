#!/bin/bash
# HBM traffic and time of k_step across revisions (run through gpurun): each argument is a tree --
# "." (the current one) or a git worktree under wt/ with its own built library -- whose bench runs
# from that tree: FETCH_SIZE and WRITE_SIZE in separate --pmc passes (3 timed steps after a 20-step
# pre-roll) and a 200-step timing run.  Prints bytes per env-step (raw) and k_step ms per tree.
set -e -o pipefail
export TMPDIR=/tmp
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/pmcwt
mkdir -p $OUT
B3="bench.py --steps 3 --warmup 1 --preroll 20 --no-cpu-baseline --no-parity --no-config2"
for t in "$@"; do
  n=$(echo $t | tr '/.' '__')
  (cd $ROOT/$t && timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pf_$n -o pf -- python $B3 > $OUT/pf_$n.log 2>&1)
  (cd $ROOT/$t && timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pw_$n -o pw -- python $B3 > $OUT/pw_$n.log 2>&1)
  (cd $ROOT/$t && timeout -k 10 200 python bench.py --steps 200 --no-cpu-baseline --no-config2 --no-parity > $OUT/time_$n.json 2> $OUT/time_$n.err)
  python - $OUT $n <<'PY'
import csv, json, re, sys, statistics
out, n = sys.argv[1], sys.argv[2]
def ks(path, c):
    return [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if re.search(r"\bk_step(?![A-Za-z0-9_])", r["Kernel_Name"]) and r["Counter_Name"] == c]
f = ks(f"{out}/pf_{n}/pf_counter_collection.csv", "FETCH_SIZE")
w = ks(f"{out}/pw_{n}/pw_counter_collection.csv", "WRITE_SIZE")
d = json.load(open(f"{out}/time_{n}.json"))
E = 65536
print(f"{n}: k_step launches {len(f)}/{len(w)}  fetch {statistics.mean(f) * 1024 / E:.1f} B/env-step  "
      f"write {statistics.mean(w) * 1024 / E:.1f} B/env-step  k_step {d['roofline']['kernel_ms']} ms  {d['value']:.4g} env-steps/s")
PY
done

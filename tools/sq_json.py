"""profiles/<tag>_sq_kstep.json from a tools/pmc_sq_quick.sh pass (gpurun_out/sqq_<tag>/p*/).

    python tools/sq_json.py <tag> [envs] [frame_skip] [first] [last]

Per-dispatch means over the k_step launches [first, last) (default 150..205: the headline
handle's steady state -- 200-step pre-roll, warmup, 3 timed steps, the parity step -- before the
bench's 4 096-env config-2 leg), per wave-substep figures (÷ envs × frame_skip: one
env per wave) and the issue / wait fractions of the wave's cycles.
"""
import collections
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
envs = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
fs = int(sys.argv[3]) if len(sys.argv) > 3 else 5
first = int(sys.argv[4]) if len(sys.argv) > 4 else 150
last = int(sys.argv[5]) if len(sys.argv) > 5 else 205
acc = collections.defaultdict(list)
for p in sorted(glob.glob(os.path.join(REPO, "gpurun_out", f"sqq_{tag}", "p*", "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(p)):
        if "k_step" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
per = {k: sum(v[first:last]) / len(v[first:last]) for k, v in sorted(acc.items())}
pws = {k: round(v / (envs * fs), 1) for k, v in per.items()}
wc = per["SQ_WAVE_CYCLES"]
fr = dict(active_inst_any=per["SQ_ACTIVE_INST_ANY"] / wc, active_valu=per["SQ_ACTIVE_INST_VALU"] / wc,
          active_lds=per["SQ_ACTIVE_INST_LDS"] / wc, wait_any=per["SQ_WAIT_ANY"] / wc,
          wait_inst_any=per["SQ_WAIT_INST_ANY"] / wc)
if "SQ_WAIT_INST_LDS" in per:
    fr["wait_inst_lds"] = per["SQ_WAIT_INST_LDS"] / wc
out = dict(tag=tag, dispatches=[first, last], kernel="k_step (hammer-v0, 65 536 envs, persistent grid)", per_dispatch=per,
           per_wave_substep=pws, fractions_of_wave_cycles={k: round(v, 4) for k, v in fr.items()},
           note="SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles (x4 = shader cycles); "
                "WAIT_ANY = parked on s_waitcnt, WAIT_INST_ANY = issue stall on a dependency, "
                "ACTIVE_INST_ANY = issuing (MI355X_MICROARCH.md PMC section)")
path = os.path.join(REPO, "profiles", f"{tag}_sq_kstep.json")
json.dump(out, open(path, "w"), indent=1)
print(path, json.dumps(out["fractions_of_wave_cycles"]), pws.get("SQ_INSTS_VALU"))

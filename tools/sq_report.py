"""Per-wave SQ counter summary of k_step from a tools/pmc_sq_quick.sh pass."""
import collections, csv, glob, sys
d = sys.argv[1]
acc = collections.defaultdict(list)
for p in sorted(glob.glob(f"{d}/p*/p*_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        if "k_step" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
w = acc["SQ_WAVES"][-1] if "SQ_WAVES" in acc else 65536
wc = acc["SQ_WAVE_CYCLES"][-1]
for k, v in sorted(acc.items()):
    x = v[-1]
    print(f"{k:24s} {x:16.0f} per-wave {x / w:12.1f}" + (f"  {x / wc * 100:5.1f}% of wave cycles" if k.startswith(("SQ_WAIT", "SQ_ACTIVE", "SQ_BUSY")) else ""))

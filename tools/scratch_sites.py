"""Scratch stores / loads of k_step<0> by loop nesting (run tools/spill_report.py first: /tmp/isa/one.s).

Prints each scratch op outside the kernel-entry block with its source line and the loop
header it sits in, so per-launch, per-env and per-substep spill traffic can be told apart."""
import re
import sys

lines = open("/tmp/isa/one.s").readlines()
fmap = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
    if m:
        fmap[m.group(1)] = m.group(2).split("/")[-1]
s = next(i for i, l in enumerate(lines) if l.startswith("_Z6k_stepILi0"))
e = next(i for i in range(s + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
cur, loop, n = None, "entry", 0
for i in range(s, e):
    l = lines[i]
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m:
        cur = f"{fmap.get(m.group(1))}:{m.group(2)}"
        continue
    t = l.strip()
    if t.endswith(":") or (":" in t and "Loop" in t and t.startswith(".LBB")):
        mm = re.search(r"(Header=BB\S+ Depth=\d+|Loop Header: Depth=\d+|Parent Loop BB\S+ Depth=\d+)", l)
        loop = mm.group(1) if mm else ("entry" if loop == "entry" else "-")
        continue
    if not t or t.startswith((".", ";")):
        continue
    n += 1
    if "scratch_" in t and (len(sys.argv) < 2 or loop != "entry"):
        print(n, loop, cur, t.split(";")[0][:60])

"""Attribute scratch (spill) instructions of k_step<TASK> to source lines (debug .s build)."""
import collections, re, subprocess, sys
task = sys.argv[1] if len(sys.argv) > 1 else "0"   # task kind (hammer 0)
src = "mj_envs_amd/csrc/adroit_wave.hip"
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from __graft_entry__ import HIPCC_FLAGS  # noqa: E402  (the product build's flags)
os.makedirs("/tmp/isa", exist_ok=True)
flags = [f for f in HIPCC_FLAGS if f not in ("-shared", "-fPIC")]
subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-g", "-S", "--cuda-device-only",
                f"-DAW_ONLY_TASK={task}", *sys.argv[2:], "-o", "/tmp/isa/one.s", src], check=True)
lines = open("/tmp/isa/one.s").readlines()
fmap = {}
for l in lines:
    m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
    if m: fmap[m.group(1)] = m.group(2)
s = next(i for i, l in enumerate(lines) if l.startswith(f"_Z6k_stepILi{task}"))
e = next(i for i in range(s + 1, len(lines)) if lines[i].startswith(".Lfunc_end"))
cur = None; cnt = collections.Counter(); n = 0
for l in lines[s:e]:
    m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
    if m: cur = (fmap.get(m.group(1)), int(m.group(2))); continue
    t = l.strip()
    if not t or t.startswith((".", ";")) or t.endswith(":"): continue
    n += 1
    if "scratch_" in t: cnt[cur] += 1
print("k_step instructions", n, "scratch ops", sum(cnt.values()))
for k, c in cnt.most_common(25): print(c, k)
print([l.strip() for l in lines[e:e+400] if "vgpr_count" in l or "private_segment" in l or "vgpr_spill" in l][:6])

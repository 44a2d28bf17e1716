"""Static instruction mix of k_step<TASK> per source function (debug-line attribution).

    python tools/isa_regions.py [task_kind] [extra hipcc flags...]

Compiles the device code with -g, attributes every instruction of k_step<TASK> to its source
line (.loc; inlined code keeps its own file / line) and sums the counts per enclosing function of
mj_envs_amd/csrc/*.h / adroit_wave.hip: VALU, SALU, LDS, VMEM, scratch, readlane / writelane and
s_nop.  Together with the stage profile (cycles per stage) it says which stages are issue-heavy
and which are latency-bound.
"""
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from __graft_entry__ import HIPCC_FLAGS, HIP_SRC  # noqa: E402

FUNC = re.compile(r"^(?:template\s*<[^>]*>\s*)?(?:AW_DEV|__global__|static)[^;{]*?\b(\w+)\s*\(", re.M)


def functions(path):
    """(name, first line, last line) of the top-level functions of one source file"""
    lines = open(path).read().splitlines()
    starts = []
    for i, l in enumerate(lines):
        m = re.match(r"^(?:AW_DEV|__global__|template|static)[^;]*?\b(\w+)\s*\(", l)
        if m and not l.rstrip().endswith(";"):
            # the declaration may continue; the name is the identifier before the first '('
            starts.append((i + 1, m.group(1)))
    out = []
    for k, (ln, name) in enumerate(starts):
        end = starts[k + 1][0] - 1 if k + 1 < len(starts) else len(lines)
        out.append((name, ln, end))
    return out


def classify(op):
    if op.startswith("scratch_") or op.startswith("buffer_"):
        return "scratch"
    if "readlane" in op:
        return "readlane"
    if "writelane" in op:
        return "writelane"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "flat_")):
        return "vmem"
    if op.startswith("s_nop"):
        return "s_nop"
    if op.startswith("s_waitcnt"):
        return "waitcnt"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    task = sys.argv[1] if len(sys.argv) > 1 else "0"
    extra = sys.argv[2:]
    out = "/tmp/isa_regions.s"
    flags = [f for f in HIPCC_FLAGS if f not in ("-shared", "-fPIC")]
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-g", "-S", "--cuda-device-only", f"-DAW_ONLY_TASK={task}", *extra,
                    "-o", out, HIP_SRC], check=True)
    text = open(out).read().splitlines()
    files = {}
    for l in text:
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]+)"', l)
        if m:
            files[m.group(1)] = os.path.join(m.group(2), m.group(3))
    s = next(i for i, l in enumerate(text) if l.startswith(f"_Z6k_stepILi{task}"))
    e = next(i for i in range(s + 1, len(text)) if text[i].startswith(".Lfunc_end"))
    csrc = os.path.join(REPO, "mj_envs_amd", "csrc")
    spans = {}
    for f in os.listdir(csrc):
        spans[f] = functions(os.path.join(csrc, f))
    counts = collections.defaultdict(collections.Counter)
    cur = None
    for l in text[s:e]:
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", l)
        if m:
            cur = (os.path.basename(files.get(m.group(1), "?")), int(m.group(2)))
            continue
        t = l.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        fn = "?"
        if cur and cur[0] in spans:
            for name, a, b in spans[cur[0]]:
                if a <= cur[1] <= b:
                    fn = f"{cur[0]}:{name}"
                    break
        elif cur:
            fn = cur[0]
        counts[fn][classify(t.split()[0])] += 1
    cols = ["valu", "salu", "lds", "vmem", "scratch", "readlane", "writelane", "s_nop", "waitcnt"]
    tot = collections.Counter()
    rows = sorted(counts.items(), key=lambda kv: -sum(kv[1].values()))
    print(f"{'function':44s} {'total':>6s} " + " ".join(f"{c:>9s}" for c in cols))
    for fn, c in rows:
        tot.update(c)
        print(f"{fn[:44]:44s} {sum(c.values()):6d} " + " ".join(f"{c[k]:9d}" for k in cols))
    print(f"{'TOTAL':44s} {sum(tot.values()):6d} " + " ".join(f"{tot[k]:9d}" for k in cols))


if __name__ == "__main__":
    main()

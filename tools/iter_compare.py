"""Per-state solver iteration counts: HIP path (fp32) vs oracle (fp64) on identical states.

    python tools/iter_compare.py [--env hammer-v0] [--n 64] [--steps 50]   # GPU box
"""
import argparse
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env", default="hammer-v0")
    ap.add_argument("--n", type=int, default=64)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from test_gpu_parity import _sim, _t, contact_states
    m, o, P, st = contact_states(a.env, a.n, a.steps, seed=3)
    _, sim = _sim(a.env, a.n)
    sim.set_state(_t(st["qpos"]), _t(st["qvel"]), _t(st["warm"]), _t(P))
    rows = []
    for e in range(a.n):
        d = sim.forward_dump(e)
        o.forward1(P[e], st["qpos"][e], st["qvel"][e], st["warm"][e])
        sc = o.get("scalars")
        qa = o.get("qacc")
        rows.append(dict(env=e, ncon=d["ncon"], ncon_ref=int(sc[0]), nefc=d["nefc"], nefc_ref=int(sc[1]),
                         newton=d["solver_iter"], newton_ref=int(sc[2]), noslip=d["noslip_iter"],
                         noslip_ref=int(sc[3]),
                         qacc_rel=float(np.abs(d["qacc"] - qa).max() / (np.abs(qa).max() + 1e-9))))
    R = {k: float(np.mean([r[k] for r in rows])) for k in ("newton", "newton_ref", "noslip", "noslip_ref")}
    res = dict(env=a.env, n=a.n, mean=R, rows=rows)
    txt = json.dumps(res, indent=1)
    print(json.dumps(R))
    for r in rows:
        print(r)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()

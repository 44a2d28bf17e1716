"""One forward at large geom margins, GPU vs oracle (GPU box diagnostic).

    python tools/diag_margin.py [env_id] [margin] [n_envs]

With every geom margin at `margin` (the tests' "margin=X" pseudo-variation), n envs are reset and
stepped 3 times; then for the env whose next mj_step differs most, one forward from that identical
state is compared field by field (tools/diag_tf.analyse_case: contacts, rows, Newton iterations and
exit reason, qacc, row forces).
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "tools"))
from conftest import make_oracle  # noqa: E402
from diag_tf import analyse_case, pair_geoms  # noqa: E402
from mj_envs_amd import _native  # noqa: E402


def main(env_id="hammer-v0", margin=0.04, n=64):
    m, o = make_oracle(env_id, f"margin={margin}")
    sim = _native.Sim(m.to_blob(), n)
    obs, rew = sim.empty(n, sim.obs_dim), sim.empty(n)
    done, goal = sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    sim.reset(obs, seed=5)
    act = sim.empty(n, sim.nu)
    for k in range(3):
        sim.random_actions(act, 3, k)
        sim.step(act, obs, rew, done, goal)
    q, v, w, p = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv), sim.empty(n, sim.nparam)
    sim.get_state(q, v, w, p)
    sim.random_actions(act, 3, 3)
    torch.cuda.synchronize()
    st = dict(qpos=q.cpu().numpy().astype(np.float64), qvel=v.cpu().numpy().astype(np.float64),
              warm=w.cpu().numpy().astype(np.float64), params=p.cpu().numpy().astype(np.float64))
    a = act.cpu().numpy().astype(np.float64)
    m1 = make_oracle(env_id, f"margin={margin}")[0]
    m1.dims["task_frame_skip"] = 1
    one = _native.Sim(m1.to_blob(), n)
    one.set_state(q, v, w, p)
    one.step(act, obs, rew, done, goal)
    v1 = one.empty(n, one.nv)
    one.get_state(qvel=v1)
    torch.cuda.synchronize()
    ctrl = m.task_act_mid + np.clip(a, -1, 1) * m.task_act_rng
    errs = []
    for j in range(n):
        qq, vv, ww = st["qpos"][j].copy(), st["qvel"][j].copy(), st["warm"][j].copy()
        o.mjstep1(st["params"][j], qq, vv, ww, ctrl[j], 1)
        errs.append(np.abs(v1[j].cpu().numpy() - vv).max() / (np.abs(vv - st["qvel"][j]).max() + 1e-6))
    order = np.argsort(errs)[::-1]
    print("worst envs", [(int(j), round(float(errs[j]), 4)) for j in order[:6]], flush=True)
    single = _native.Sim(m.to_blob(), 1)
    for j in order[:2]:
        pre = {k2: st[k2][j] for k2 in st}
        rec = analyse_case(m, o, single, 1, pair_geoms(m), 0, int(j), pre, a[j], 0.0, float(errs[j]))
        for sub in rec["substeps"]:
            print(json.dumps({k2: v2 for k2, v2 in sub.items() if k2 != "state"})[:6000], flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "hammer-v0", float(a[1]) if len(a) > 1 else 0.04, int(a[2]) if len(a) > 2 else 64)

"""Fast vs wide tier on identical inputs (GPU box): where do the results differ?"""
import faulthandler
import os
import sys

import numpy as np
import torch

faulthandler.dump_traceback_later(100, exit=True)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mj_envs_amd import _native  # noqa: E402
from mj_envs_amd.tasks import attach_task, load_model  # noqa: E402

env_id = sys.argv[1] if len(sys.argv) > 1 else "hammer-v0"
n = 64
m = attach_task(load_model(env_id), env_id)
res = {}
for mode in (0, 1):
    sim = _native.Sim(m.to_blob(), n)
    sim.set_tier(mode)
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, seed=3)
    o0 = obs.clone()
    act = sim.empty(n, sim.nu)
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    outs = []
    for k in range(5):
        sim.random_actions(act, 5, k)
        sim.step(act, obs, rew, done, goal)
        q, v = sim.empty(n, sim.nq), sim.empty(n, sim.nv)
        sim.get_state(q, v)
        outs.append((obs.clone(), q, v))
    torch.cuda.synchronize()
    res[mode] = (o0, outs)
    sim.close()
d0 = (res[0][0] - res[1][0]).abs()
print("reset obs: max diff", float(d0.max()), "envs differing", int((d0.max(1).values > 0).sum()))
if float(d0.max()) > 0:
    e = int(d0.max(1).values.argmax())
    cols = torch.nonzero(d0[e] > 0).flatten().tolist()
    print(" env", e, "cols", cols[:20], "fast", res[0][0][e, cols[:6]].tolist(), "wide", res[1][0][e, cols[:6]].tolist())
for k in range(5):
    (oa, qa, va), (ob, qb, vb) = res[0][1][k], res[1][1][k]
    dq, dv, do = (qa - qb).abs(), (va - vb).abs(), (oa - ob).abs()
    print(f"step {k}: max |dq| {float(dq.max()):.3e} |dv| {float(dv.max()):.3e} |dobs| {float(do.max()):.3e} "
          f"envs differing {int((dq.max(1).values > 0).sum())}", flush=True)
    if float(dq.max()) > 0 and k == 0:
        e = int(dq.max(1).values.argmax())
        print("  env", e, "dofs", torch.nonzero(dq[e] > 0).flatten().tolist()[:20])
print("ok")

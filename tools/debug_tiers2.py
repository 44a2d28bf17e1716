"""Determinism probe (GPU box): the same relocate / pen rollout through the fast tier with one
workgroup per env, through the fast tier with 8 persistent workgroups (AW_STEP_GRID=8: each slot
steps 8 envs in turn), and through the wide tier; prints where they part."""
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

env_id = sys.argv[1] if len(sys.argv) > 1 else "relocate-v0"
n = 64
m = attach_task(load_model(env_id), env_id)


def run(mode, grid):
    if grid:
        os.environ["AW_STEP_GRID"] = str(grid)
    else:
        os.environ.pop("AW_STEP_GRID", None)
    sim = _native.Sim(m.to_blob(), n)
    sim.set_tier(mode)
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, seed=3)
    act = sim.empty(n, sim.nu)
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    qs = []
    for k in range(6):
        sim.random_actions(act, 5, k)
        sim.step(act, obs, rew, done, goal)
        q, v = sim.empty(n, sim.nq), sim.empty(n, sim.nv)
        sim.get_state(q, v)
        qs.append(torch.cat([q, v], 1))
    torch.cuda.synchronize()
    print(f"mode {mode} grid {sim.grid}", flush=True)
    sim.close()
    return qs


ref = run(0, 0)
for mode, grid in ((0, 0), (0, 8), (0, 1), (1, 0)):
    qs = run(mode, grid)
    for k in range(6):
        d = (qs[k] - ref[k]).abs()
        if float(d.max()) > 0:
            e = int(d.max(1).values.argmax())
            print(f"  mode {mode} grid {grid}: first difference at step {k}, max {float(d.max()):.3e}, envs "
                  f"{torch.nonzero(d.max(1).values > 0).flatten().tolist()[:10]}, env {e} cols "
                  f"{torch.nonzero(d[e] > 0).flatten().tolist()[:12]}", flush=True)
            break
    else:
        print(f"  mode {mode} grid {grid}: bitwise equal to mode 0 / one workgroup per env", flush=True)
print("ok")

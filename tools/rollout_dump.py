"""Deterministic rollouts for bitwise A/B of library variants (GPU box):

    AW_LIB=... python tools/rollout_dump.py OUT.npz

hammer-v0 / relocate-v0, 4 096 envs: 40 env-steps under random actions and 40 in the DAPG closed loop,
with auto-reset; saves the final states and every step's obs.  Two variants whose files are equal
array for array compute the same arithmetic."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from mj_envs_amd import _native  # noqa: E402
from mj_envs_amd.policy import GaussianMLP  # noqa: E402
from mj_envs_amd.tasks import attach_task, load_model  # noqa: E402

out = {}
for env_id in ("hammer-v0", "relocate-v0"):
    for pol in ("random", "dapg"):
        n = 4096
        sim = _native.Sim(attach_task(load_model(env_id), env_id).to_blob(), n)
        obs, act = sim.empty(n, sim.obs_dim), sim.empty(n, sim.nu)
        rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
        sim.reset(obs, seed=3)
        p = GaussianMLP.from_npz(os.path.join(REPO, "tests", "golden", f"dapg_{env_id.split('-')[0]}.npz"),
                                 device=0) if pol == "dapg" else None
        obs_all = []
        for k in range(40):
            if p is not None:
                p.act(obs, out=act)
            else:
                sim.random_actions(act, 4, k)
            sim.step(act, obs, rew, done, goal, autoreset=True, seed=3)
            obs_all.append(obs.cpu().numpy().copy())
        q, v = sim.empty(n, sim.nq), sim.empty(n, sim.nv)
        sim.get_state(q, v)
        torch.cuda.synchronize()
        out[f"{env_id}_{pol}_obs"] = np.stack(obs_all)
        out[f"{env_id}_{pol}_qpos"] = q.cpu().numpy()
        out[f"{env_id}_{pol}_qvel"] = v.cpu().numpy()
        sim.close()
np.savez_compressed(sys.argv[1], **out)
print("saved", sys.argv[1])

"""Diagnostic (GPU box): teacher-forced per-step GPU vs oracle errors along a GPU rollout."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mj_envs_amd import _native  # noqa: E402
from mj_envs_amd.tasks import attach_task, load_model, sample_params  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402

env_id = sys.argv[1] if len(sys.argv) > 1 else "pen-v0"
n, steps = 64, 40
m = attach_task(load_model(env_id), env_id)
o = Oracle(m.to_blob())
o.set_option(max_con=32, max_efc=128)
sim = _native.Sim(m.to_blob(), n)
P = sample_params(env_id, m, np.random.default_rng(11), n)
t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device="cuda")
obs = sim.empty(n, sim.obs_dim)
sim.reset(obs, params=t(P))
rew = sim.empty(n)
done, goal = sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
q, v, w = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv)
fl = sim.empty(n, dtype=torch.int32)
rng = np.random.default_rng(13)
for k in range(steps):
    sim.get_state(q, v, w)
    torch.cuda.synchronize()
    st = dict(qpos=q.cpu().numpy().astype(np.float64), qvel=v.cpu().numpy().astype(np.float64),
              warm=w.cpu().numpy().astype(np.float64), params=np.asarray(P, np.float64))
    q0 = st["qpos"].copy()
    act = rng.uniform(-1, 1, (n, sim.nu))
    sim.step(t(act), obs, rew, done, goal)
    sim.get_state(q, v)
    sim.status(fl)
    torch.cuda.synchronize()
    _, r_ref, _, _, ost = o.step(st, act, nthreads=8)
    qg, vg = q.cpu().numpy(), v.cpu().numpy()
    eq = np.abs(qg - st["qpos"]) - (2e-5 + 1e-5 * np.abs(st["qpos"]))
    ev = np.abs(vg - st["qvel"]) - 5e-3 * (1 + np.abs(st["qvel"]))
    bad = (eq > 0).any(1) | (ev > 0).any(1)
    if bad.any():
        e = int(np.where(bad)[0][0])
        jq, jv = int(np.argmax(eq[e])), int(np.argmax(ev[e]))
        print(f"step {k:2d} bad {bad.sum():2d}/{n} env {e} q-dof {jq} dq {abs(qg[e,jq]-st['qpos'][e,jq]):.2e} "
              f"v-dof {jv} dv {abs(vg[e,jv]-st['qvel'][e,jv]):.2e} |v| {abs(st['qvel'][e,jv]):.2f} "
              f"gpu-status {int(fl[e])} orc-status {int(ost[e])} obj-z {q0[e, -4] if env_id=='pen-v0' else 0:.3f}")
    else:
        print(f"step {k:2d} ok")

"""Diagnostic (GPU box): for the teacher-forced cases outside tolerance, which oracle solver
iteration cap reproduces the GPU's step best (Newton early stop vs other causes)."""
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
n, steps = 64, 30
m = attach_task(load_model(env_id), env_id)
o = Oracle(m.to_blob())
o.set_option(max_con=32, max_efc=128)
sim = _native.Sim(m.to_blob(), n)
sim.set_option(disableflags=int(os.environ.get("AW_DSBL", "0"), 0))   # e.g. AW_DSBL=0x10000: fp32 MPR
P = sample_params(env_id, m, np.random.default_rng(11), n)
t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device="cuda")
obs = sim.empty(n, sim.obs_dim)
sim.reset(obs, params=t(P))
rew = sim.empty(n)
done, goal = sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
q, v, w = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv)
rng = np.random.default_rng(13)
caps = (1, 2, 3, 4, 5, 6, 8, 20)
hist = {}
nbad = 0
for k in range(steps):
    sim.get_state(q, v, w)
    torch.cuda.synchronize()
    st = dict(qpos=q.cpu().numpy().astype(np.float64), qvel=v.cpu().numpy().astype(np.float64),
              warm=w.cpu().numpy().astype(np.float64), params=np.asarray(P, np.float64))
    act = rng.uniform(-1, 1, (n, sim.nu))
    sim.step(t(act), obs, rew, done, goal)
    sim.get_state(q, v)
    torch.cuda.synchronize()
    vg = v.cpu().numpy()
    errs = {}
    for c in caps:
        s2 = {kk: vv.copy() for kk, vv in st.items()}
        o.set_option(iterations=c)
        o.step(s2, act, nthreads=8)
        errs[c] = (np.abs(vg - s2["qvel"]) / (5e-3 * (1 + np.abs(s2["qvel"])))).max(1)
    o.set_option(iterations=20)
    bad = errs[20] > 1
    for e in np.where(bad)[0]:
        nbad += 1
        best = min(caps, key=lambda c: errs[c][e])
        hist[best] = hist.get(best, 0) + 1
        if nbad <= 25:
            print(f"step {k} env {e}: err@20 {errs[20][e]:.2f} " + " ".join(f"{c}:{errs[c][e]:.2f}" for c in caps))
print("bad", nbad, "of", n * steps, "best-matching cap histogram", dict(sorted(hist.items())))

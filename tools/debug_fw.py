"""Diagnostic (GPU box): at the first teacher-forced mismatch, compare one forward pass
(contacts, constraint rows, qacc) of the GPU and the oracle on the same pre-step state."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mj_envs_amd import _native  # noqa: E402
from mj_envs_amd.tasks import attach_task, load_model, sample_params  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402

np.set_printoptions(precision=5, suppress=True, linewidth=160)
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
rng = np.random.default_rng(13)
names = m.names["geom"]
for k in range(steps):
    sim.get_state(q, v, w)
    torch.cuda.synchronize()
    st = dict(qpos=q.cpu().numpy().astype(np.float64), qvel=v.cpu().numpy().astype(np.float64),
              warm=w.cpu().numpy().astype(np.float64), params=np.asarray(P, np.float64))
    pre = {kk: vv.copy() for kk, vv in st.items()}
    act = rng.uniform(-1, 1, (n, sim.nu))
    sim.step(t(act), obs, rew, done, goal)
    sim.get_state(q, v)
    torch.cuda.synchronize()
    o.step(st, act, nthreads=8)
    qg, vg = q.cpu().numpy(), v.cpu().numpy()
    ev = np.abs(vg - st["qvel"]) - 5e-3 * (1 + np.abs(st["qvel"]))
    bad = (ev > 0).any(1)
    if bad.sum() >= 5:
        e = int(np.where(bad)[0][0])
        print("step", k, "env", e)
        # single substep comparison from the pre-step state
        ctrl = m.task_act_mid + np.clip(act[e], -1, 1) * m.task_act_rng
        sim.set_state(t(pre["qpos"]), t(pre["qvel"]), t(pre["warm"]), t(pre["params"]))
        d = sim.forward_dump(e, ctrl=t(ctrl))
        o.forward1(pre["params"][e], pre["qpos"][e], pre["qvel"][e], pre["warm"][e], ctrl)
        sc = o.get("scalars")
        print("ncon gpu", d["ncon"], "orc", int(sc[0]), " nefc gpu", d["nefc"], "orc", int(sc[1]),
              " newton it gpu", d["solver_iter"], "orc", int(sc[2]), "noslip", d["noslip_iter"], int(sc[3]))
        c = o.get("contact").reshape(-1, 23)
        for i in range(max(d["ncon"], len(c))):
            if i < len(c):
                g1, g2 = int(c[i, 13]), int(c[i, 14])
                print(" orc", i, names[g1], names[g2], "dist %.6f" % c[i, 0], "pos", c[i, 1:4], "n", c[i, 4:7])
            if i < d["ncon"]:
                print(" gpu", i, "pair", int(d["con_pair"][i]), "dist %.6f" % d["con_dist"][i], "pos", d["con_pos"][i],
                      "n", d["con_frame"][i][:3])
        print("qacc gpu", d["qacc"][-6:])
        print("qacc orc", o.get("qacc")[-6:])
        print("efc_force gpu", d["efc_force"][:d["nefc"]][-16:])
        print("efc_force orc", o.get("efc_force")[-16:])
        break

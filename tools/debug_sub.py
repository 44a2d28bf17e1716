"""Diagnostic (GPU box): substep-by-substep GPU vs oracle for one env (frame_skip forced to 1)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mj_envs_amd import _native  # noqa: E402
from mj_envs_amd.tasks import attach_task, load_model, sample_params  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402

np.set_printoptions(precision=5, suppress=True, linewidth=180)
env_id = sys.argv[1] if len(sys.argv) > 1 else "pen-v0"
n, steps = 64, 12
m = attach_task(load_model(env_id), env_id)
o = Oracle(m.to_blob())
o.set_option(max_con=32, max_efc=128)
sim = _native.Sim(m.to_blob(), n)
m1 = attach_task(load_model(env_id), env_id)
m1.dims["task_frame_skip"] = 1
sim1 = _native.Sim(m1.to_blob(), n)
P = sample_params(env_id, m, np.random.default_rng(11), n)
t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device="cuda")
obs = sim.empty(n, sim.obs_dim)
sim.reset(obs, params=t(P))
rew = sim.empty(n)
done, goal = sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
q, v, w = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv)
rng = np.random.default_rng(13)
names = m.names["geom"]
fs = sim.frame_skip
for k in range(steps):
    sim.get_state(q, v, w)
    torch.cuda.synchronize()
    pre = dict(qpos=q.cpu().numpy().astype(np.float64), qvel=v.cpu().numpy().astype(np.float64),
               warm=w.cpu().numpy().astype(np.float64))
    act = rng.uniform(-1, 1, (n, sim.nu))
    sim.step(t(act), obs, rew, done, goal)
    sim.get_state(q, v)
    torch.cuda.synchronize()
    qg, vg = q.cpu().numpy(), v.cpu().numpy()
    bad_envs = []
    for e in range(n):
        qq, vv, ww = pre["qpos"][e].copy(), pre["qvel"][e].copy(), pre["warm"][e].copy()
        ctrl = m.task_act_mid + np.clip(act[e], -1, 1) * m.task_act_rng
        o.mjstep1(P[e], qq, vv, ww, ctrl, nstep=fs)
        if not ((np.abs(vg[e] - vv) <= 5e-3 * (1 + np.abs(vv))).all()):
            bad_envs.append(e)
    print("step", k, "bad", len(bad_envs))
    if len(bad_envs) >= 5:
        e = bad_envs[0]
        ctrl = m.task_act_mid + np.clip(act[e], -1, 1) * m.task_act_rng
        # substep by substep: GPU (frame_skip 1 sim, env 0 slot used for all) vs oracle
        qq, vv, ww = pre["qpos"][e].copy(), pre["qvel"][e].copy(), pre["warm"][e].copy()
        Q = np.tile(qq, (n, 1)); V = np.tile(vv, (n, 1)); W = np.tile(ww, (n, 1)); PP = np.tile(P[e], (n, 1))
        sim1.set_state(t(Q), t(V), t(W), t(PP))
        A = np.tile(act[e], (n, 1))
        for sub in range(fs):
            # GPU forward on the current substep state, then one substep
            d = sim1.forward_dump(0, ctrl=t(ctrl))
            o.forward1(P[e], qq, vv, ww, ctrl)
            sc = o.get("scalars")
            c = o.get("contact").reshape(-1, 23)
            print(f" sub {sub}: ncon {d['ncon']}/{int(sc[0])} nefc {d['nefc']}/{int(sc[1])} it {d['solver_iter']}/{int(sc[2])} "
                  f"ns {d['noslip_iter']}/{int(sc[3])} |dqacc| {np.abs(d['qacc']-o.get('qacc')).max():.3e} "
                  f"|qacc| {np.abs(o.get('qacc')).max():.3e}")
            if np.abs(d['qacc'] - o.get('qacc')).max() > 1e-2 * (1 + np.abs(o.get('qacc')).max()):
                for i in range(max(d["ncon"], len(c))):
                    if i < len(c):
                        print("   orc", i, names[int(c[i, 13])], names[int(c[i, 14])], "dist %.6f" % c[i, 0], "pos", c[i, 1:4], "n", c[i, 4:7])
                    if i < d["ncon"]:
                        print("   gpu", i, "pair", int(d["con_pair"][i]), "dist %.6f" % d["con_dist"][i], "pos", d["con_pos"][i],
                              "n", d["con_frame"][i][:3])
                print("   qacc gpu", d["qacc"]); print("   qacc orc", o.get("qacc"))
                print("   force gpu", d["efc_force"]); print("   force orc", o.get("efc_force"))
                print("   type", d["efc_type"])
            sim1.step(t(A), obs, rew, done, goal)
            o.mjstep1(P[e], qq, vv, ww, ctrl, nstep=1)
            sim1.get_state(q, v, w)
            torch.cuda.synchronize()
            # continue the oracle from the GPU state (teacher forcing per substep)
            qq, vv, ww = (q[0].cpu().numpy().astype(np.float64), v[0].cpu().numpy().astype(np.float64),
                          w[0].cpu().numpy().astype(np.float64))
        break

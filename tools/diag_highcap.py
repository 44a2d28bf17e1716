"""Wide-tier accuracy against the fast tier in the same regime (GPU box diagnostic).

    python tools/diag_highcap.py [env_id] [margins...]

For each geom margin (the tests' "margin=X" pseudo-variation: more contacts and rows than the
reference's regimes), 64 envs take 10 random-action env-steps, each teacher-forced against the
oracle on the same model; prints, separately for the env-steps the fast tier finished and those it
handed to the wide tier, the fraction within the one-step tolerance and the p50 / p99 errors.
"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import make_oracle  # noqa: E402
from mj_envs_amd import _native  # noqa: E402


def run(env_id, margin, n=64, steps=10):
    m, o = make_oracle(env_id, f"margin={margin}")
    sim = _native.Sim(m.to_blob(), n)
    obs, rew = sim.empty(n, sim.obs_dim), sim.empty(n)
    done, goal = sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    sim.reset(obs, seed=5)
    q, v, w, p = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv), sim.empty(n, sim.nparam)
    last = sim.empty(n, dtype=torch.int32)
    act = sim.empty(n, sim.nu)
    rec = {"fast": [], "wide": []}
    for k in range(steps):
        sim.get_state(q, v, w, p)
        torch.cuda.synchronize()
        st = dict(qpos=q.cpu().numpy().astype(np.float64), qvel=v.cpu().numpy().astype(np.float64),
                  warm=w.cpu().numpy().astype(np.float64), params=p.cpu().numpy().astype(np.float64))
        sim.random_actions(act, 3, k)
        sim.step(act, obs, rew, done, goal)
        sim.get_state(q, v)
        sim.status(last)
        torch.cuda.synchronize()
        o.step(st, act.cpu().numpy().astype(np.float64), nthreads=8)
        dq = np.abs(q.cpu().numpy() - st["qpos"])
        dv = np.abs(v.cpu().numpy() - st["qvel"])
        ok = (dq <= 2e-5 + 1e-5 * np.abs(st["qpos"])).all(1) & (dv <= 5e-3 * (1 + np.abs(st["qvel"]))).all(1)
        wide = (last.cpu().numpy() & _native.ST_WIDE) != 0
        for j in range(n):
            rec["wide" if wide[j] else "fast"].append((ok[j], dq[j].max(), (dv[j] / (1 + np.abs(st["qvel"][j]))).max()))
    for tier, r in rec.items():
        if not r:
            print(f"{env_id} margin {margin}: {tier}: no env-steps", flush=True)
            continue
        a = np.array(r, dtype=float)
        print(f"{env_id} margin {margin}: {tier}: {len(r)} env-steps, {a[:, 0].mean():.4f} within tolerance, "
              f"|dqpos| p50 {np.percentile(a[:, 1], 50):.2e} p99 {np.percentile(a[:, 1], 99):.2e}, "
              f"|dqvel|/(1+|v|) p50 {np.percentile(a[:, 2], 50):.2e} p99 {np.percentile(a[:, 2], 99):.2e}", flush=True)


if __name__ == "__main__" and not os.environ.get("ONE_SUBSTEP"):
    a = sys.argv[1:]
    env = a[0] if a else "hammer-v0"
    for mg in (a[1:] or ["0.0005", "0.02", "0.03", "0.04", "0.05"]):
        run(env, float(mg))


def one_substep(env_id, margin, n=64, warm_steps=3):
    """one mj_step from identical fp32 states (a frame_skip-1 handle), GPU vs oracle: the relative
    error of the velocity change, per tier"""
    m, o = make_oracle(env_id, f"margin={margin}")
    sim = _native.Sim(m.to_blob(), n)
    obs, rew = sim.empty(n, sim.obs_dim), sim.empty(n)
    done, goal = sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    sim.reset(obs, seed=5)
    act = sim.empty(n, sim.nu)
    for k in range(warm_steps):
        sim.random_actions(act, 3, k)
        sim.step(act, obs, rew, done, goal)
    q, v, w, p = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv), sim.empty(n, sim.nparam)
    sim.get_state(q, v, w, p)
    sim.random_actions(act, 3, warm_steps)
    torch.cuda.synchronize()
    st = dict(qpos=q.cpu().numpy().astype(np.float64), qvel=v.cpu().numpy().astype(np.float64),
              warm=w.cpu().numpy().astype(np.float64), params=p.cpu().numpy().astype(np.float64))
    a = act.cpu().numpy().astype(np.float64)
    m.dims["task_frame_skip"] = 1
    one = _native.Sim(m.to_blob(), n)
    one.set_state(q, v, w, p)
    one.clear_status()
    one.step(act, obs, rew, done, goal)
    q1, v1 = one.empty(n, one.nq), one.empty(n, one.nv)
    last = one.empty(n, dtype=torch.int32)
    one.get_state(q1, v1)
    one.status(last)
    torch.cuda.synchronize()
    ctrl = m.task_act_mid + np.clip(a, -1, 1) * m.task_act_rng
    errs = {"fast": [], "wide": []}
    wide = (last.cpu().numpy() & _native.ST_WIDE) != 0
    for j in range(n):
        qq, vv, ww = st["qpos"][j].copy(), st["qvel"][j].copy(), st["warm"][j].copy()
        o.mjstep1(st["params"][j], qq, vv, ww, ctrl[j], 1)
        dvo = vv - st["qvel"][j]
        e = np.abs(v1[j].cpu().numpy() - vv).max() / (np.abs(dvo).max() + 1e-6)
        errs["wide" if wide[j] else "fast"].append(e)
    for tier, e in errs.items():
        if e:
            e = np.array(e)
            print(f"{env_id} margin {margin} one substep: {tier}: {len(e)} envs, |dv error| / max|dv| "
                  f"p50 {np.percentile(e, 50):.2e} p90 {np.percentile(e, 90):.2e} max {e.max():.2e}", flush=True)


if __name__ == "__main__" and os.environ.get("ONE_SUBSTEP"):
    for mg in (sys.argv[2:] or ["0.03", "0.04", "0.06", "0.08"]):
        one_substep(sys.argv[1] if len(sys.argv) > 1 else "hammer-v0", float(mg))

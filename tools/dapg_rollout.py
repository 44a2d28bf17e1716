"""Closed-loop DAPG rollouts on the CPU oracle at the reference's capacities (behavioural pin).

Drives the fp64 oracle with the reference's pretrained DAPG policies (tests/golden/dapg_*.npz,
extracted by tests/golden/make_dapg.py) using the policy mean, exactly as the reference's
evaluation does (``algos/baselines.py:82-86`` ``get_action(o)[1]['evaluation']``), and logs
  * the success rate (``evaluate_success``: > 25 goal steps, pen > 20; ``hammer_v0.py:167-175``),
  * overflow at MuJoCo's capacities nconmax 100 / njmax 500 (``DAPG_assets.xml:4``).
(The DAPG regime's per-substep work counts come from tools/work_counts.py ... dapg.)
Output: profiles/dapg_oracle_<task>.json
    python tools/dapg_rollout.py [env_id|all] [n_envs] [seed]
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mj_envs_amd.tasks import TASKS, attach_task, load_model, sample_params  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402


def load_policy(env_id):
    return dict(np.load(os.path.join(REPO, "tests", "golden", f"dapg_{env_id.split('-')[0]}.npz")))


def policy_mean(p, obs):
    """mjrl FCNetwork.forward (fp64 restatement): the DAPG evaluation action."""
    x = (obs - p["in_shift"]) / (p["in_scale"] + 1e-8)
    x = np.tanh(x @ p["W0"].T + p["b0"])
    x = np.tanh(x @ p["W1"].T + p["b1"])
    x = x @ p["W2"].T + p["b2"]
    return x * p["out_scale"] + p["out_shift"]


def rollout(env_id, n=32, seed=0, counts=False, max_con=100, max_efc=500):
    m = attach_task(load_model(env_id), env_id)
    o = Oracle(m.to_blob())
    o.set_option(max_con=max_con, max_efc=max_efc)
    pol = load_policy(env_id)
    rng = np.random.default_rng(seed)
    P = sample_params(env_id, m, rng, n)
    st, obs = o.reset(P)
    spec = TASKS[env_id]
    goals = np.zeros(n, int)
    alive = np.ones(n, bool)
    rows = []
    status = np.zeros(n, np.uint32)
    for t in range(spec.horizon):
        act = policy_mean(pol, obs)
        if counts:
            for e in range(n):
                ctrl = m.task_act_mid + np.clip(act[e], -1, 1) * m.task_act_rng
                q, v, w = st["qpos"][e].copy(), st["qvel"][e].copy(), st["warm"][e].copy()
                for _ in range(o.frame_skip):
                    status[e] |= o.mjstep1(P[e], q, v, w, ctrl, 1)
                    ncon, nefc, it, nsit, _ = o.get("scalars")
                    nden = int(np.sum(o.get("efc_type") >= 4))
                    rows.append((ncon, nefc, nden, it, nsit))
        obs, rew, done, goal, stt = o.step(st, act, nthreads=8)
        status |= stt
        goals += goal & alive
        alive &= ~done        # pen: the reference's trainers stop an episode at done
    succ = float(np.mean(goals > spec.success_steps) * 100)
    out = dict(env_id=env_id, n_envs=n, horizon=spec.horizon, seed=seed, policy="DAPG pretrained (mean action)",
               caps=dict(max_con=max_con, max_efc=max_efc), success_pct=succ,
               goal_steps_mean=float(goals.mean()), overflow_envs=int(np.sum((status & 24) != 0)))
    if rows:
        r = np.array(rows, float)
        out.update(substeps=len(rows),
                   avg=dict(ncon=r[:, 0].mean(), nefc=r[:, 1].mean(), ndense=r[:, 2].mean(),
                            newton_iter=r[:, 3].mean(), noslip_iter=r[:, 4].mean()),
                   max=dict(ncon=int(r[:, 0].max()), nefc=int(r[:, 1].max()), ndense=int(r[:, 2].max())),
                   p999=dict(ncon=float(np.quantile(r[:, 0], 0.999)), nefc=float(np.quantile(r[:, 1], 0.999)),
                             ndense=float(np.quantile(r[:, 2], 0.999))))
    return out


def main(which="all", n=32, seed=0):
    envs = list(TASKS) if which == "all" else [which]
    for env_id in envs:
        t0 = time.time()
        out = rollout(env_id, n, seed)
        out["wall_s"] = round(time.time() - t0, 1)
        path = os.path.join(REPO, "profiles", f"dapg_oracle_{env_id.split('-')[0]}.json")
        with open(path, "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "all", int(a[1]) if len(a) > 1 else 32, int(a[2]) if len(a) > 2 else 0)

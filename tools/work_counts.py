"""Log per-substep work counts from the CPU oracle (counts come from the oracle).

Output: profiles/work_counts_<task>.json (random policy) or work_counts_<task>_dapg.json (the
reference's pretrained DAPG policy, mean action: algos/baselines.py:82-86) -- average ncon, nefc,
dense rows, Newton iterations, line-search derivative evaluations per Newton iteration and noslip
sweeps per substep, at MuJoCo's capacities (nconmax 100 / njmax 500) -- consumed by
mj_envs_amd/perfmodel.py to price the bench's algorithmic FLOPs for the matching --policy.

    python tools/work_counts.py [env_id] [n_envs] [steps] [random|dapg]
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mj_envs_amd.tasks import attach_task, load_model, sample_params  # noqa: E402
from oracle.pyoracle import Oracle, build  # noqa: E402


def policy_mean(p, obs):
    """mjrl FCNetwork.forward (fp64 restatement): the DAPG evaluation action"""
    x = (obs - p["in_shift"]) / (p["in_scale"] + 1e-8)
    x = np.tanh(x @ p["W0"].T + p["b0"])
    x = np.tanh(x @ p["W1"].T + p["b1"])
    return (x @ p["W2"].T + p["b2"]) * p["out_scale"] + p["out_shift"]


def counts(env_id="hammer-v0", n=32, steps=200, policy="random", seed=0, threads=8):
    build()
    m = attach_task(load_model(env_id), env_id)
    o = Oracle(m.to_blob())
    rng = np.random.default_rng(seed)
    P = sample_params(env_id, m, rng, n)
    st, obs = o.reset(P, nthreads=threads)
    pol = None
    if policy == "dapg":
        pol = dict(np.load(os.path.join(REPO, "tests", "golden", f"dapg_{env_id.split('-')[0]}.npz")))
    tot = np.zeros(12, np.int64)
    mx = np.zeros(3, np.int64)
    over = 0
    t0 = time.time()
    for _ in range(steps):
        act = policy_mean(pol, obs) if pol is not None else rng.uniform(-1, 1, (n, o.nu))
        obs, _, _, _, s = o.step_stats(st, act, nthreads=threads)
        tot += s.sum(axis=0)
        mx = np.maximum(mx, s[:, :3].max(axis=0))
        over += int(((s[:, 7] & 24) != 0).sum())
    sub = float(tot[6])
    avg = dict(ncon=tot[8] / sub, nefc=tot[9] / sub, ndense=tot[10] / sub, newton_iter=tot[3] / sub,
               noslip_iter=tot[5] / sub, ls_iter=tot[4] / max(tot[3], 1), boxbox_substep_frac=tot[11] / sub)
    return dict(env_id=env_id, n_envs=n, steps=steps, seed=seed, substeps=int(sub),
                policy="iid U(-1,1) actions" if pol is None else "DAPG pretrained (mean action)",
                caps=dict(max_con=o.max_con, max_efc=o.max_efc), overflow_env_steps=over,
                avg={k: float(v) for k, v in avg.items()},
                ls_iter_note="line-search derivative evaluations per Newton iteration (incl. the one at alpha = 0), "
                             "logged by the oracle's mj_solNewton line search (oracle/solver.cc line_search)",
                max=dict(ncon=int(mx[0]), nefc=int(mx[1]), ndense=int(mx[2])), wall_s=round(time.time() - t0, 1))


def main(env_id="hammer-v0", n=32, steps=200, policy="random"):
    out = counts(env_id, n, steps, policy)
    suffix = "_dapg" if policy == "dapg" else ""
    path = os.path.join(REPO, "profiles", f"work_counts_{env_id.split('-')[0]}{suffix}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "hammer-v0", int(a[1]) if len(a) > 1 else 32, int(a[2]) if len(a) > 2 else 200,
         a[3] if len(a) > 3 else "random")

"""Log per-substep work counts from the CPU oracle on a random-policy trajectory.

Output: profiles/work_counts_<task>.json (average ncon, nefc, dense rows, Newton / noslip
iterations) consumed by mj_envs_amd/perfmodel.py to price the bench's algorithmic FLOPs.
    python tools/work_counts.py [env_id] [n_envs] [steps]
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mj_envs_amd.tasks import attach_task, load_model, sample_params  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402


def main(env_id="hammer-v0", n=32, steps=200, seed=0):
    m = attach_task(load_model(env_id), env_id)
    o = Oracle(m.to_blob())
    rng = np.random.default_rng(seed)
    P = sample_params(env_id, m, rng, n)
    st, _ = o.reset(P)
    rows = []
    for t in range(steps):
        act = rng.uniform(-1, 1, (n, o.nu))
        for e in range(n):
            ctrl = m.task_act_mid + np.clip(act[e], -1, 1) * m.task_act_rng
            q, v, w = st["qpos"][e], st["qvel"][e], st["warm"][e]
            for _ in range(o.frame_skip):
                o.mjstep1(P[e], q, v, w, ctrl, 1)
                ncon, nefc, it, nsit, _ = o.get("scalars")
                ty = o.get("efc_type")
                nden = int(np.sum(ty >= 4))
                rows.append((ncon, nefc, nden, it, nsit))
    r = np.array(rows, float)
    avg = dict(ncon=r[:, 0].mean(), nefc=r[:, 1].mean(), ndense=r[:, 2].mean(),
               newton_iter=r[:, 3].mean(), noslip_iter=r[:, 4].mean(), ls_iter=6.0)
    out = dict(env_id=env_id, n_envs=n, steps=steps, seed=seed, substeps=len(rows),
               policy="iid U(-1,1) actions", avg=avg,
               max=dict(ncon=int(r[:, 0].max()), nefc=int(r[:, 1].max()), ndense=int(r[:, 2].max())))
    path = os.path.join(REPO, "profiles", f"work_counts_{env_id.split('-')[0]}.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "hammer-v0", int(a[1]) if len(a) > 1 else 32, int(a[2]) if len(a) > 2 else 200)

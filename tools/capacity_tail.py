"""Tail of the per-env constraint work under the reference's caps (nconmax 100 / njmax 500,
DAPG_assets.xml:4): how many envs of a random-policy run exceed the fast k_step tier's
capacities (aw_common.h MAXCON / MAXEFC / MAXDENSE) at some substep.

    python tools/capacity_tail.py [env_id] [n_envs] [steps] [threads]

Runs the fp64 oracle (OpenMP over envs, oracle.step_stats) from the reference reset
distribution with i.i.d. U(-1, 1) actions and prints the distribution of each env's maximum
ncon / nefc / dense rows and the envs past each cap.
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

FAST_CAPS = dict(ncon=48, nefc=192, ndense=128)


def main(env_id="relocate-v0", n=4096, steps=200, threads=8, seed=0):
    build()
    m = attach_task(load_model(env_id), env_id)
    o = Oracle(m.to_blob())
    rng = np.random.default_rng(seed)
    P = sample_params(env_id, m, rng, n)
    st, _ = o.reset(P, nthreads=threads)
    mx = np.zeros((n, 3), np.int64)
    t0 = time.time()
    for t in range(steps):
        act = rng.uniform(-1, 1, (n, o.nu))
        _, _, _, _, s = o.step_stats(st, act, nthreads=threads)
        mx = np.maximum(mx, s[:, :3])   # per env: max ncon, nefc, dense rows of the env-step
    keys = ("ncon", "nefc", "ndense")
    out = dict(env_id=env_id, n_envs=n, steps=steps, seed=seed, wall_s=round(time.time() - t0, 1),
               caps_oracle=dict(ncon=o.max_con, nefc=o.max_efc), fast_caps=FAST_CAPS,
               max={k: int(mx[:, i].max()) for i, k in enumerate(keys)},
               p999={k: float(np.percentile(mx[:, i], 99.9)) for i, k in enumerate(keys)},
               envs_past_fast_cap={k: int((mx[:, i] > FAST_CAPS[k]).sum()) for i, k in enumerate(keys)},
               envs_past_any_fast_cap=int(((mx[:, 0] > FAST_CAPS["ncon"]) | (mx[:, 1] > FAST_CAPS["nefc"])
                                           | (mx[:, 2] > FAST_CAPS["ndense"])).sum()),
               top_envs=[dict(env=int(e), **{k: int(mx[e, i]) for i, k in enumerate(keys)})
                         for e in np.argsort(-mx[:, 2])[:12]])
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "relocate-v0", int(a[1]) if len(a) > 1 else 4096, int(a[2]) if len(a) > 2 else 200,
         int(a[3]) if len(a) > 3 else 8)

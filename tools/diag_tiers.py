"""Where do the fast and the forced-wide tier first differ?  (GPU box)

    python tools/diag_tiers.py [env_id] [n] [steps]

Runs the same reset + random actions through a fast-tier handle and a forced-wide handle and prints,
per env-step, the number of envs whose state differs and the largest difference."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from mj_envs_amd import _native  # noqa: E402
from mj_envs_amd.tasks import attach_task, load_model  # noqa: E402

env_id = sys.argv[1] if len(sys.argv) > 1 else "relocate-v0"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 256
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 20
sims = []
for mode in (0, 1):
    sim = _native.Sim(attach_task(load_model(env_id), env_id).to_blob(), n)
    sim.set_tier(mode)
    sims.append(sim)
bufs = [(s.empty(n, s.obs_dim), s.empty(n), s.empty(n, dtype=torch.uint8), s.empty(n, dtype=torch.uint8)) for s in sims]
acts = [s.empty(n, s.nu) for s in sims]
for s, b in zip(sims, bufs):
    s.reset(b[0], seed=4)
print("reset obs equal:", torch.equal(bufs[0][0], bufs[1][0]))
for k in range(steps):
    qs = []
    for s, b, a in zip(sims, bufs, acts):
        s.random_actions(a, 2, k)
        s.step(a, *b)
        q, v = s.empty(n, s.nq), s.empty(n, s.nv)
        s.get_state(q, v)
        qs.append((q, v))
    torch.cuda.synchronize()
    dq = (qs[0][0] - qs[1][0]).abs().max(1).values.cpu().numpy()
    dv = (qs[0][1] - qs[1][1]).abs().max(1).values.cpu().numpy()
    bad = np.nonzero((dq > 0) | (dv > 0))[0]
    print(f"step {k}: {len(bad)} envs differ, max |dq| {dq.max():.3e} |dv| {dv.max():.3e}, first envs {bad[:5].tolist()}",
          flush=True)
    if len(bad):
        e = int(bad[0])
        dd = (qs[0][1][e] - qs[1][1][e]).abs().cpu().numpy()
        print("   env", e, "dofs with |dv| > 0:", np.nonzero(dd)[0].tolist(), "max at dof", int(dd.argmax()))
        ob = (bufs[0][0][e] - bufs[1][0][e]).abs().cpu().numpy()
        print("   obs entries differing:", np.nonzero(ob)[0].tolist()[:20])
        break

"""First fast/wide difference in the tier-equality test's rollout (GPU box), with the work counts of
the env-step that differs (aw_forward_dump of its pre-step state)."""
import faulthandler
import os
import sys

import numpy as np
import torch

faulthandler.dump_traceback_later(200, exit=True)
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mj_envs_amd import _native  # noqa: E402
from mj_envs_amd.tasks import attach_task, load_model  # noqa: E402

env_id = sys.argv[1] if len(sys.argv) > 1 else "pen-v0"
auto = int(sys.argv[2]) if len(sys.argv) > 2 else 1
n, steps = 512, 30
m = attach_task(load_model(env_id), env_id)
sims, bufs = [], []
for mode in (0, 1):
    sim = _native.Sim(m.to_blob(), n)
    sim.set_tier(mode)
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, seed=3)
    if auto:
        sim.set_episode(ep_len=torch.from_numpy(np.arange(n, dtype=np.int32) % sim.horizon).cuda())
    sims.append(sim)
    bufs.append((obs, sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)))
act = sims[0].empty(n, sims[0].nu)
for k in range(steps):
    sims[0].random_actions(act, 5, k)
    pre = []
    for sim in sims:
        q, v, w, p = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv), sim.empty(n, sim.nparam)
        sim.get_state(q, v, w, p)
        pre.append((q, v, w, p))
    for sim, b in zip(sims, bufs):
        sim.step(act, *b, autoreset=bool(auto), seed=3)
    st = []
    for sim in sims:
        q, v = sim.empty(n, sim.nq), sim.empty(n, sim.nv)
        sim.get_state(q, v)
        st.append(torch.cat([q, v], 1))
    torch.cuda.synchronize()
    pre_eq = all(torch.equal(a, b) for a, b in zip(pre[0], pre[1]))
    d = (st[0] - st[1]).abs().max(1).values
    if float(d.max()) > 0 or not torch.equal(bufs[0][0], bufs[1][0]):
        envs = torch.nonzero(d > 0).flatten().tolist()
        do = (bufs[0][0] - bufs[1][0]).abs().max(1).values
        oenvs = torch.nonzero(do > 0).flatten().tolist()
        print(f"step {k}: pre-step states equal: {pre_eq}; state differs in envs {envs[:10]} (max {float(d.max()):.3e}); "
              f"obs differs in envs {oenvs[:10]}; done {bufs[0][2][oenvs[:5]].tolist() if oenvs else []}", flush=True)
        for e in (envs or oenvs)[:3]:
            one = _native.Sim(m.to_blob(), 1)
            q, v, w, p = (x[e:e + 1].clone() for x in pre[0])
            one.set_state(q, v, w, p)
            ctrl = torch.tensor(m.task_act_mid + np.clip(act[e].cpu().numpy(), -1, 1) * m.task_act_rng,
                                dtype=torch.float32, device="cuda")
            dd = one.forward_dump(0, ctrl)
            print(f"  env {e}: ncon {dd['ncon']} nefc {dd['nefc']} nsparse {dd['nsparse']} ndense {dd['ndense']} "
                  f"newton {dd['solver_iter']} ({dd['solver_exit']}) noslip {dd['noslip_iter']} status {dd['status']}",
                  flush=True)
        break
else:
    print("no difference", flush=True)
print("ok")

"""One-step parity of the current library on DAPG steady-state (grasp-regime) states, at scale,
with the noslip workload of every miss (GPU box diagnostic).

    python tools/diag_noslip.py save [n_envs] [n_check]     # pre-roll like bench.py --policy dapg,
                                                            # save pre-step states + actions
    python tools/diag_noslip.py TAG [n_check]               # step the saved states with this library
                                                            # (AW_LIB), compare with the fp64 oracle

The saved states (gpurun_out/diag_ns_states.npz) let two libraries (AW_LIB) step identical
pre-step states; each run writes its post-step states to gpurun_out/diag_ns_<TAG>.npz and prints
the miss count, the misses' noslip pair counts (pyramidal rows / 2 from aw_forward_dump) and the
pair-count histogram of the checked envs.
"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mj_envs_amd import _native  # noqa: E402
from mj_envs_amd.dist import stagger_phases  # noqa: E402
from mj_envs_amd.policy import GaussianMLP  # noqa: E402
from mj_envs_amd.tasks import attach_task, load_model  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402

ENV = "hammer-v0"
OUT = os.path.join(REPO, "gpurun_out")
STATES = os.path.join(OUT, "diag_ns_states.npz")


def main():
    os.makedirs(OUT, exist_ok=True)
    tag = sys.argv[1]
    m = attach_task(load_model(ENV), ENV)
    blob = m.to_blob()
    if tag == "save":
        n = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
        sim = _native.Sim(blob, n)
        obs, act = sim.empty(n, sim.obs_dim), sim.empty(n, sim.nu)
        rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
        sim.reset(obs, seed=1)
        sim.set_episode(ep_len=torch.from_numpy(stagger_phases(n, 0, sim.horizon)).cuda())
        pol = GaussianMLP.from_npz(os.path.join(REPO, "tests", "golden", "dapg_hammer.npz"), device=0)
        for k in range(sim.horizon + 20):
            pol.act(obs, out=act, sample=False, seed=2, step=k)
            sim.step(act, obs, rew, done, goal, autoreset=True, seed=1)
        q, v, w, p = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv), sim.empty(n, sim.nparam)
        sim.get_state(q, v, w, p)
        sim.random_actions(act, 12345, 0)
        torch.cuda.synchronize()
        np.savez(STATES, qpos=q.cpu().numpy(), qvel=v.cpu().numpy(), warm=w.cpu().numpy(),
                 params=p.cpu().numpy(), act=act.cpu().numpy())
        print("saved", n, "states", flush=True)
        return
    ncheck = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    S = np.load(STATES)
    n = S["qpos"].shape[0]
    t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device="cuda")
    sim = _native.Sim(blob, n)
    obs = sim.empty(n, sim.obs_dim)
    sim.set_state(t(S["qpos"]), t(S["qvel"]), t(S["warm"]), t(S["params"]), obs)
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    sim.step(t(S["act"]), obs, rew, done, goal)
    q2, v2 = sim.empty(n, sim.nq), sim.empty(n, sim.nv)
    sim.get_state(q2, v2)
    torch.cuda.synchronize()
    q2, v2 = q2.cpu().numpy(), v2.cpu().numpy()
    np.savez(os.path.join(OUT, f"diag_ns_{tag}.npz"), qpos=q2, qvel=v2)
    idx = np.unique(np.linspace(0, n - 1, min(ncheck, n)).round().astype(int))
    st = {k: S[k][idx].astype(np.float64) for k in ("qpos", "qvel", "warm", "params")}
    o = Oracle(blob)
    t0 = time.perf_counter()
    o.step(st, S["act"][idx].astype(np.float64), nthreads=16)
    okq = (np.abs(q2[idx] - st["qpos"]) <= 2e-5 + 1e-5 * np.abs(st["qpos"])).all(axis=1)
    okv = (np.abs(v2[idx] - st["qvel"]) <= 5e-3 * (1 + np.abs(st["qvel"]))).all(axis=1)
    ok = okq & okv
    print(f"{tag}: {int((~ok).sum())} misses of {len(idx)} ({ok.mean():.4f} within tolerance), oracle "
          f"{time.perf_counter() - t0:.1f} s", flush=True)
    # noslip workload (first substep's forward) of every checked env
    one = _native.Sim(blob, 1)
    ctrl = m.task_act_mid + np.clip(S["act"][idx], -1, 1) * m.task_act_rng
    npairs = np.zeros(len(idx), int)
    nsit = np.zeros(len(idx), int)
    for j, e in enumerate(idx):
        one.set_state(t(S["qpos"][e][None]), t(S["qvel"][e][None]), t(S["warm"][e][None]), t(S["params"][e][None]))
        d = one.forward_dump(0, t(ctrl[j]))
        npairs[j] = int((d["efc_type"][:d["nefc"]] == 5).sum()) // 2
        nsit[j] = d["noslip_iter"]
    hist = {int(k): int(c) for k, c in zip(*np.unique(npairs, return_counts=True))}
    # the oracle's noslip sweep count on the same (fp32) state, first substep
    onsit = {}
    for j in list(np.where(~ok)[0]) + list(range(0, len(idx), max(1, len(idx) // 64))):
        e = idx[j]
        o.forward1(S["params"][e].astype(np.float64), S["qpos"][e].astype(np.float64),
                   S["qvel"][e].astype(np.float64), S["warm"][e].astype(np.float64), ctrl[j])
        onsit[int(j)] = int(o.get("scalars")[3])
    same = [nsit[j] == onsit[j] for j in onsit if ok[j]]
    rep_ns = dict(sampled_ok_envs=len(same), same_noslip_iters=int(sum(same)),
                  ok_examples=[(int(idx[j]), int(nsit[j]), onsit[j]) for j in onsit if ok[j]][:16])
    miss = [dict(env=int(idx[j]), pairs=int(npairs[j]), noslip_iter=int(nsit[j]), oracle_noslip_iter=onsit[int(j)],
                 dq=float(np.abs(q2[idx[j]] - st["qpos"][j]).max()),
                 dv=float(np.abs(v2[idx[j]] - st["qvel"][j]).max())) for j in np.where(~ok)[0]]
    rep = dict(tag=tag, n=n, checked=len(idx), misses=len(miss), frac=float(ok.mean()),
               pair_hist=hist, noslip_iters=rep_ns, miss_cases=miss)
    for other in ("main",):
        f = os.path.join(OUT, f"diag_ns_{other}.npz")
        if other != tag and os.path.exists(f):
            O = np.load(f)
            dq = np.abs(O["qpos"] - q2).max(axis=1)
            rep[f"vs_{other}"] = dict(max_dq=float(dq.max()), n_dq_gt_1e4=int((dq > 1e-4).sum()),
                                      worst=[(int(e), float(dq[e])) for e in np.argsort(-dq)[:8]])
    print(json.dumps(rep), flush=True)
    with open(os.path.join(OUT, f"diag_ns_{tag}.json"), "w") as fh:
        json.dump(rep, fh, indent=1)


if __name__ == "__main__":
    main()

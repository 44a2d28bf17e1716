"""Replay one (env, step) case of tests/test_gpu_scale.py::test_config3_full_size_16384_envs (GPU box).

    python tools/diag_c3_case.py <env_id> <step> <env> [n_envs]

Re-runs the test's rollout (same seeds: reset seed 7, staggered episode phases, Philox actions
keyed (9, step), auto-reset seed 7) on the GPU alone up to <step>, takes env <env>'s pre-step state,
action and tier flag, and compares the env-step four ways: the big handle's own result, a one-env
handle in automatic tier mode, the same forced through the wide tier (aw_set_tier(1)) and the fp64
oracle; then tools/diag_tf.analyse_case walks the substeps (aw_forward_dump vs the oracle's forward).
Writes gpurun_out/diag_c3_<task>_<step>_<env>.json.
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tools"))
from mj_envs_amd import _native  # noqa: E402
from mj_envs_amd.tasks import attach_task, load_model  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402
from diag_tf import analyse_case, pair_geoms  # noqa: E402


def main(env_id, K, E, n=16384):
    m = attach_task(load_model(env_id), env_id)
    blob = m.to_blob()
    sim = _native.Sim(blob, n)
    obs, rew = sim.empty(n, sim.obs_dim), sim.empty(n)
    done, goal = sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    sim.reset(obs, seed=7)
    sim.set_episode(ep_len=torch.from_numpy((np.arange(n) * 7919 % sim.horizon).astype(np.int32)).cuda())
    sim.clear_status()
    q, v, w, p = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv), sim.empty(n, sim.nparam)
    last = sim.empty(n, dtype=torch.int32)
    act = sim.empty(n, sim.nu)
    for k in range(K + 1):
        if k == K:
            sim.get_state(q, v, w, p)
            torch.cuda.synchronize()
            pre = dict(qpos=q[E].cpu().numpy().astype(np.float64), qvel=v[E].cpu().numpy().astype(np.float64),
                       warm=w[E].cpu().numpy().astype(np.float64), params=p[E].cpu().numpy().astype(np.float64))
        sim.random_actions(act, 9, k)
        sim.step(act, obs, rew, done, goal, autoreset=True, seed=7)
    sim.get_state(q, v)
    sim.status(last)
    torch.cuda.synchronize()
    a = act[E].cpu().numpy().astype(np.float64)
    big = dict(qpos=q[E].cpu().numpy().astype(np.float64), qvel=v[E].cpu().numpy().astype(np.float64),
               status=int(last[E].item()), done=int(done[E].item()))
    o = Oracle(blob)
    st = {kk: vv[None].copy() for kk, vv in pre.items()}
    _, r_ref, _, _, ost = o.step(st, a[None], nthreads=1)
    ref = dict(qpos=st["qpos"][0], qvel=st["qvel"][0], status=int(ost[0]))

    def one_env(tier):
        one = _native.Sim(blob, 1)
        one.set_tier(tier)
        t = lambda x: torch.tensor(np.asarray(x)[None], dtype=torch.float32, device="cuda")
        one.set_state(t(pre["qpos"]), t(pre["qvel"]), t(pre["warm"]), t(pre["params"]))
        ob, rw = one.empty(1, one.obs_dim), one.empty(1)
        dn, gl = one.empty(1, dtype=torch.uint8), one.empty(1, dtype=torch.uint8)
        one.clear_status()
        one.step(t(a), ob, rw, dn, gl)
        qq, vv = one.empty(1, one.nq), one.empty(1, one.nv)
        one.get_state(qq, vv)
        ls = one.empty(1, dtype=torch.int32)
        one.status(ls)
        torch.cuda.synchronize()
        return dict(qpos=qq[0].cpu().numpy().astype(np.float64), qvel=vv[0].cpu().numpy().astype(np.float64),
                    status=int(ls[0].item()))

    res = dict(big=big, auto=one_env(0), wide=one_env(1))
    out = dict(env_id=env_id, step=K, env=E, action=a.tolist(), oracle_status=ref["status"])
    for name, r in res.items():
        out[name] = dict(status=r["status"], wide=bool(r["status"] & _native.ST_WIDE),
                         dqpos=float(np.abs(r["qpos"] - ref["qpos"]).max()),
                         dqvel=float(np.abs(r["qvel"] - ref["qvel"]).max()),
                         vs_big_qpos=float(np.abs(r["qpos"] - big["qpos"]).max()))
        print(name, out[name], flush=True)
    one = _native.Sim(blob, 1)
    rec = analyse_case(m, o, one, sim.frame_skip, pair_geoms(m), K, E, pre, a,
                       out["big"]["dqpos"], out["big"]["dqvel"])
    for sub in rec["substeps"]:
        print(json.dumps({kk: vv for kk, vv in sub.items() if kk != "state"}), flush=True)
    out["case"] = rec
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", f"diag_c3_{env_id.split('-')[0]}_{K}_{E}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0], int(a[1]), int(a[2]), int(a[3]) if len(a) > 3 else 16384)

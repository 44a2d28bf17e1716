"""Attribute teacher-forced parity misses to a substep and a contact (GPU box diagnostic).

    python tools/diag_tf.py <env_id> [dapg|random] [steps] [n_envs] [max_cases] [disableflags] [variation]

Runs the teacher-forced rollout of tests/test_gpu_parity.py (GPU env-steps, each re-run by the
fp64 oracle from the GPU's own pre-step state).  For each (env, step) outside the one-step
tolerance it replays the oracle substep by substep and, at every substep state, compares one
forward pass of the GPU (aw_forward_dump on that fp32 state) with the oracle's: ncon, the
contact list (geom pair names / types, dist), nefc, solver iterations and qacc.  Prints the
first substep where they part, so a miss is attributed to a collider, a margin switch or the
solver.  Writes gpurun_out/diag_<task>.json.
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from mj_envs_amd import _native  # noqa: E402
from mj_envs_amd.policy import GaussianMLP  # noqa: E402
from mj_envs_amd.tasks import attach_task, load_model, sample_params  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402

TYPES = {0: "plane", 2: "sphere", 3: "capsule", 5: "cylinder", 6: "box"}


def pair_geoms(m):
    return list(zip(m.arrays["pair_geom1"].tolist() + m.arrays["cand_geom1"].tolist(),
                    m.arrays["pair_geom2"].tolist() + m.arrays["cand_geom2"].tolist()))


def gname(m, g):
    return f"{m.names['geom'][g] or g}:{TYPES.get(int(m.geom_type[g]), m.geom_type[g])}"


def analyse_case(m, o, one, frame_skip, pg, k, e, pre, a, dq, dv):
    """substep-by-substep GPU (aw_forward_dump) vs oracle comparison of one (env, step) case"""
    t = lambda x: torch.tensor(np.asarray(x), dtype=torch.float32, device="cuda")
    ctrl = m.task_act_mid + np.clip(a, -1, 1) * m.task_act_rng
    qp, qv, wm = pre["qpos"].copy(), pre["qvel"].copy(), pre["warm"].copy()
    rec = dict(step=k, env=e, dqpos=dq, dqvel=dv, substeps=[],
               pre=dict(qpos=pre["qpos"].tolist(), qvel=pre["qvel"].tolist(), warm=pre["warm"].tolist(),
                        params=np.asarray(pre["params"]).tolist(), action=np.asarray(a).tolist()))
    for j in range(frame_skip):
        # both sides start the substep from the same (fp32-representable) state
        qp, qv, wm = (x.astype(np.float32).astype(np.float64) for x in (qp, qv, wm))
        o.forward1(pre["params"], qp, qv, wm, ctrl)
        sc = o.get("scalars")
        oc = o.get("contact").reshape(-1, 23)
        oq = o.get("qacc")
        one.set_state(t(qp[None]), t(qv[None]), t(wm[None]), t(pre["params"][None]))
        d = one.forward_dump(0, t(ctrl))
        gq = d["qacc"]
        rq = float(np.abs(gq - oq).max() / (np.abs(oq).max() + 1e-9))
        ocs = sorted((gname(m, int(c[13])) + "|" + gname(m, int(c[14])), round(float(c[0]), 6)) for c in oc)
        gcs = sorted((gname(m, pg[p][0]) + "|" + gname(m, pg[p][1]), round(float(dd), 6))
                     for p, dd in zip(d["con_pair"], d["con_dist"]))
        sub = dict(j=j, rel_qacc=rq, ncon=(d["ncon"], int(sc[0])), nefc=(d["nefc"], int(sc[1])),
                   newton=(d["solver_iter"], int(sc[2])), newton_exit=d.get("solver_exit"),
                   noslip=(d["noslip_iter"], int(sc[3])),
                   status=d["status"])
        if d["nefc"] != int(sc[1]):
            ot, oi, op = o.get("efc_type").astype(int), o.get("efc_id").astype(int), o.get("efc_pos")
            gt = d["efc_type"].astype(int)
            diff = {}
            for ty in range(6):
                if (ot == ty).sum() != (gt == ty).sum():
                    diff[ty] = dict(gpu=int((gt == ty).sum()), oracle=int((ot == ty).sum()),
                                    oracle_rows=[(int(i), float(pp)) for i, pp in zip(oi[ot == ty], op[ot == ty])])
            sub["row_types_differ"] = diff
        if d["nefc"] == int(sc[1]) and d["nefc"]:
            ost, gst = o.get("efc_state").astype(int), d["efc_state"].astype(int)
            if (ost != gst).any():
                ty, of = o.get("efc_type").astype(int), o.get("efc_force")
                ofl = o.get("efc_frictionloss")
                sub["row_states_differ"] = [dict(row=int(r), type=int(ty[r]), gpu=int(gst[r]), oracle=int(ost[r]),
                                                 force_gpu=float(d["efc_force"][r]), force_oracle=float(of[r]),
                                                 frictionloss=float(ofl[r]))
                                            for r in np.nonzero(ost != gst)[0][:8]]
        if ocs != gcs and (len(ocs) != len(gcs) or any(abs(x[1] - y[1]) > 2e-5 for x, y in zip(ocs, gcs))
                           or any(x[0] != y[0] for x, y in zip(ocs, gcs))):
            sub["contacts_gpu"] = gcs
            sub["contacts_oracle"] = ocs
        if rq > 2e-3 and d["nefc"] == int(sc[1]):
            # same rows: where does the solve part?  per-row D / aref / force, contact frames
            ne = d["nefc"]
            od, oa, of = o.get("efc_D"), o.get("efc_aref"), o.get("efc_force")
            rel = lambda a, b: float(np.abs(a - b).max() / (np.abs(b).max() + 1e-12))
            sub["rows"] = dict(D=rel(d["efc_D"][:ne], od), aref=rel(d["efc_aref"][:ne], oa),
                               force=rel(d["efc_force"][:ne], of),
                               worst_force_rows=[(int(r), int(d["efc_type"][r]), float(d["efc_force"][r]),
                                                  float(of[r])) for r in np.argsort(-np.abs(d["efc_force"][:ne] - of))[:4]])
            sub["state"] = dict(qpos=qp.tolist(), qvel=qv.tolist(), warm=wm.tolist(), ctrl=np.asarray(ctrl).tolist())
            if len(oc):
                sub["contact_pos_err"] = float(np.abs(d["con_pos"] - oc[:, 1:4]).max())
                pe = np.abs(d["con_pos"] - oc[:, 1:4]).max(axis=1)
                sub["pos_err_by_contact"] = [
                    dict(pair=gname(m, int(c[13])) + "|" + gname(m, int(c[14])), idx=int(i), err=round(float(pe[i]), 6),
                         gpu=[round(float(x), 6) for x in d["con_pos"][i]], oracle=[round(float(x), 6) for x in c[1:4]],
                         dist_gpu=float(d["con_dist"][i]), dist_oracle=float(c[0]))
                    for i, c in enumerate(oc)]
                fe = np.abs(d["con_frame"] - oc[:, 4:13]).max(axis=1)
                sub["contact_frame_err"] = float(fe.max())
                sub["frame_err_by_contact"] = [(gname(m, int(c[13])) + "|" + gname(m, int(c[14])), round(float(e), 5),
                                                [round(float(x), 4) for x in c[4:7]])
                                               for c, e in zip(oc, fe) if e > 1e-4]
            sub["qacc_smooth"] = rel(d["qacc_smooth"], o.get("qacc_smooth"))
            sub["qM"] = rel(d["qM"], o.get("qM").reshape(len(oq), len(oq)))
        rec["substeps"].append(sub)
        o.mjstep1(pre["params"], qp, qv, wm, ctrl, 1)
        if rq > 2e-3 or "contacts_gpu" in sub or "row_states_differ" in sub:
            break
    return rec


def main(env_id="hammer-v0", pol_kind="dapg", steps=80, n=64, max_cases=12, dsbl=0, variation=None):
    m = attach_task(load_model(env_id), env_id, variation)
    blob = m.to_blob()
    o = Oracle(blob)
    pg = pair_geoms(m)
    sim = _native.Sim(blob, n)
    one = _native.Sim(blob, 1)
    if dsbl:
        sim.set_option(disableflags=dsbl)
        one.set_option(disableflags=dsbl)
        o.set_option(disableflags=dsbl & 0xFFFF)
    P = sample_params(env_id, m, np.random.default_rng(11), n, variation).astype(np.float32).astype(np.float64)
    obs = sim.empty(n, sim.obs_dim)
    t = lambda a: torch.tensor(np.asarray(a), dtype=torch.float32, device="cuda")
    sim.reset(obs, params=t(P))
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    q, v, w = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv)
    pol = GaussianMLP.from_npz(os.path.join(REPO, "tests", "golden", f"dapg_{env_id.split('-')[0]}.npz")) \
        if pol_kind == "dapg" else None
    rng = np.random.default_rng(13)
    cases = []
    for k in range(steps):
        sim.get_state(q, v, w)
        torch.cuda.synchronize()
        st = dict(qpos=q.cpu().numpy().astype(np.float64), qvel=v.cpu().numpy().astype(np.float64),
                  warm=w.cpu().numpy().astype(np.float64), params=P.copy())
        pre = {kk: vv.copy() for kk, vv in st.items()}
        act = pol.mean_np(obs.cpu().numpy()) if pol is not None else rng.uniform(-1, 1, (n, sim.nu))
        act = np.asarray(act, np.float32).astype(np.float64)      # the GPU's action is the oracle's
        sim.step(t(act), obs, rew, done, goal)
        sim.get_state(q, v)
        torch.cuda.synchronize()
        o.step(st, act, nthreads=8)
        qg, vg = q.cpu().numpy(), v.cpu().numpy()
        okq = (np.abs(qg - st["qpos"]) <= 2e-5 + 1e-5 * np.abs(st["qpos"])).all(axis=1)
        okv = (np.abs(vg - st["qvel"]) <= 5e-3 * (1 + np.abs(st["qvel"]))).all(axis=1)
        for e in np.where(~(okq & okv))[0]:
            cases.append((k, int(e), {kk: vv[e].copy() for kk, vv in pre.items()}, act[e].copy(),
                          float(np.abs(qg[e] - st["qpos"][e]).max()), float(np.abs(vg[e] - st["qvel"][e]).max())))
    print(f"{env_id} {pol_kind}: {len(cases)} of {n * steps} cases outside tolerance", flush=True)
    report = []
    # one case per distinct step first (the misses of one step are often one replicated state),
    # then the remaining ones in order
    seen, pick, rest = set(), [], []
    for c in cases:
        (rest if c[0] in seen else pick).append(c)
        seen.add(c[0])
    hist = {}
    for c in cases:
        hist[c[0]] = hist.get(c[0], 0) + 1
    print("misses per step:", sorted(hist.items(), key=lambda x: -x[1])[:20], flush=True)
    for (k, e, pre, a, dq, dv) in (pick + rest)[:max_cases]:
        rec = analyse_case(m, o, one, sim.frame_skip, pg, k, e, pre, a, dq, dv)
        report.append(rec)
        print(json.dumps(rec), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    tag = f"{env_id.split('-')[0]}_{pol_kind}" + (f"_{variation}" if variation else "") + (f"_{dsbl:#x}" if dsbl else "")
    with open(os.path.join(REPO, "gpurun_out", f"diag_{tag}.json"), "w") as f:
        json.dump(dict(env_id=env_id, policy=pol_kind, n=n, steps=steps, misses=len(cases),
                       misses_per_step={int(k): v for k, v in sorted(hist.items())}, cases=report), f, indent=1)


if __name__ == "__main__":
    a = sys.argv[1:]
    main(a[0] if a else "hammer-v0", a[1] if len(a) > 1 else "dapg", int(a[2]) if len(a) > 2 else 80,
         int(a[3]) if len(a) > 3 else 64, int(a[4]) if len(a) > 4 else 12, int(a[5], 0) if len(a) > 5 else 0,
         a[6] if len(a) > 6 else None)

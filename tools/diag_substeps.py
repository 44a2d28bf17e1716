"""Substep-by-substep replay of one env-step on the GPU and the oracle (GPU box diagnostic).

    python tools/diag_substeps.py <case.json>     (a tools/diag_c3_case.py output)

A one-env handle built with frame_skip 1 makes every aw_step ONE mj_step, so the env-step's five
substeps can be compared two ways: (a) free-running -- GPU and oracle each from their own previous
substep state -- showing where the divergence grows; (b) local -- the GPU's single substep from the
oracle's substep state -- the per-substep error of the whole mj_step (forward + Euler), which
aw_forward_dump's qacc comparison does not cover.  Prints max |dqpos| / |dqvel| (and the dof) per
substep.
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from mj_envs_amd import _native  # noqa: E402
from mj_envs_amd.tasks import attach_task, load_model  # noqa: E402
from oracle.pyoracle import Oracle  # noqa: E402


def main(path):
    d = json.load(open(path))
    env_id, pre = d["env_id"], d["case"]["pre"]
    m = attach_task(load_model(env_id), env_id)
    fs = int(m.dims["task_frame_skip"])
    o = Oracle(m.to_blob())
    m.dims["task_frame_skip"] = 1
    one = _native.Sim(m.to_blob(), 1)
    t = lambda x: torch.tensor(np.asarray(x, np.float64)[None], dtype=torch.float32, device="cuda")
    a = np.asarray(pre["action"], np.float64)
    ctrl = m.task_act_mid + np.clip(a, -1, 1) * m.task_act_rng
    P = np.asarray(pre["params"], np.float64)
    ob, rw = one.empty(1, one.obs_dim), one.empty(1)
    dn, gl = one.empty(1, dtype=torch.uint8), one.empty(1, dtype=torch.uint8)
    qq, vv, ww = one.empty(1, one.nq), one.empty(1, one.nv), one.empty(1, one.nv)

    def gpu_substep(q, v, w):
        one.set_state(t(q), t(v), t(w), t(P))
        one.step(t(a), ob, rw, dn, gl)
        one.get_state(qq, vv, ww)
        torch.cuda.synchronize()
        return (qq[0].cpu().numpy().astype(np.float64), vv[0].cpu().numpy().astype(np.float64),
                ww[0].cpu().numpy().astype(np.float64))

    f32 = lambda x: np.asarray(x, np.float32).astype(np.float64)
    qo, vo, wo = (f32(pre[k]) for k in ("qpos", "qvel", "warm"))
    qg, vg, wg = qo.copy(), vo.copy(), wo.copy()
    out = []
    for j in range(fs):
        # local: one GPU substep from the oracle's (fp32-rounded) state
        lq, lv, lw = gpu_substep(f32(qo), f32(vo), f32(wo))
        q1, v1, w1 = f32(qo), f32(vo), f32(wo)
        o.mjstep1(P, q1, v1, w1, ctrl, 1)
        # free-running: the GPU from its own state, the oracle from its own
        qg, vg, wg = gpu_substep(qg, vg, wg)
        o.mjstep1(P, qo, vo, wo, ctrl, 1)
        rec = dict(j=j,
                   local=dict(dq=float(np.abs(lq - q1).max()), dv=float(np.abs(lv - v1).max()),
                              dof_v=int(np.argmax(np.abs(lv - v1))), dw=float(np.abs(lw - w1).max())),
                   free=dict(dq=float(np.abs(qg - qo).max()), dv=float(np.abs(vg - vo).max()),
                             dof_v=int(np.argmax(np.abs(vg - vo)))),
                   v_oracle_at_dof=float(vo[int(np.argmax(np.abs(vg - vo)))]),
                   max_abs_qacc_oracle=float(np.abs(o.get("qacc")).max()))
        out.append(rec)
        print(json.dumps(rec), flush=True)
    with open(os.path.join(REPO, "gpurun_out", "diag_substeps.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1])

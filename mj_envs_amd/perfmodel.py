"""Frozen algorithmic work model of one env-step: bytes and FLOPs.

The step kernel is neither HBM- nor MFMA-bound: its state stays on chip for all substeps.
Its roofline is the FP32 compute rate (157.3 TFLOP/s on gfx950, shared by VALU and the
f32-input MFMA), priced with the formula below on the average per-substep counts (contacts,
constraint rows, Newton / noslip iterations) logged by the CPU oracle on a hammer-v0 random-
policy trajectory (profiles/work_counts_hammer.json, made by tools/work_counts.py).

One FLOP = one fp32 add or multiply (an FMA counts 2).  The formula counts the arithmetic a
dense-but-tree-aware implementation must do; it is the same for the oracle and the kernel.
"""
from __future__ import annotations

import json
import os

PEAK_FP32_TFLOPS = 157.3      # MI355X dense FP32 (vector == f32-input MFMA), MI355X_MICROARCH.md
PEAK_HBM_GBPS = 8000.0        # MI355X HBM3E spec


def step_bytes(nq: int, nv: int, nu: int, obs_dim: int, nparam: int) -> int:
    """Compulsory HBM bytes per env-step (fp32): state in/out, action in, params in, outputs."""
    state = (nq + 2 * nv) * 4
    return 2 * state + nu * 4 + nparam * 4 + obs_dim * 4 + 4 + 2 + 16   # + reward, done/goal, ep counters


def substep_flops(dims: dict, c: dict) -> float:
    """FLOPs of one mj_step given model dims and average per-substep counts c."""
    nv, nb, njnt = dims["nv"], dims["nbody"], dims["njnt"]
    ng, ns, nt, npair = dims["ngeom_coll"], dims["nsite"], dims["ntendon"], dims["npair_all"]
    sub = dims["avg_subtree"]          # mean bodies per subtree
    anc = dims["avg_ancestors"]        # mean ancestor dofs per dof (M nonzeros per row)
    ncon, nefc, nden = c["ncon"], c["nefc"], c["ndense"]
    it, nsit, lsit = c["newton_iter"], c["noslip_iter"], c["ls_iter"]
    chol = 2.0 * nv ** 3 / 3.0
    solve = 4.0 * nv ** 2
    f = 0.0
    f += nb * 110 + njnt * 120 + ng * 75 + ns * 18             # kinematics, geom/site frames
    f += nb * (sub * 6 + 110) + nv * 20                        # subtree com, cinert, cdof
    f += nb * sub * 10 + nv * (72 + (2 * anc + 1) * 12)        # crb, M rows
    f += nb * 150 + nv * 80                                    # comVel, RNE, passive, actuation
    f += chol + solve                                          # qacc_smooth
    f += npair * 12 + ncon * 400                               # bounding tests + narrowphase
    f += nt * 6 + nefc * (40 + 2 * nv) + ncon * nv * 60        # rows, impedance, contact J
    # Newton: H = M + J'DJ (dense rows), factor, solve, matvecs, line search, gradient
    f += it * (nden * nv * nv * 2 + chol + solve + 4 * nv * nv + lsit * nefc * 12 + nefc * 4 * nv)
    # noslip: inv(M), X = inv(M) J_E', pair constants, sweeps
    if nsit > 0:
        f += 2 * nv ** 3 + nden * nv * 2 * nv + nden * 3 * nv * 2
        f += nsit * (nv * (2 * nv + 10) + nden / 2 * (8 * nv + 30))
    f += chol + solve + 6 * nv                                 # implicit Euler
    return f


def model_dims(model) -> dict:
    import numpy as np
    nb = model.nbody
    par = model.body_parentid
    size = np.ones(nb)
    for b in range(nb - 1, 0, -1):
        size[par[b]] += size[b]
    anc = []
    for j in range(model.nv):
        k, a = model.dof_parentid[j], 0
        while k >= 0:
            a += 1
            k = model.dof_parentid[k]
        anc.append(a)
    coll = [g for g in range(model.ngeom) if model.geom_type[g] != 7 and
            (model.geom_contype[g] or model.geom_conaffinity[g])]
    return dict(nv=model.nv, nbody=nb, njnt=model.njnt, ngeom_coll=len(coll), nsite=model.nsite,
                ntendon=model.ntendon, npair_all=model.npair + model.ncand,
                avg_subtree=float(size[1:].mean()), avg_ancestors=float(np.mean(anc)))


def counts_path(env_id: str) -> str:
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return os.path.join(here, "profiles", f"work_counts_{env_id.split('-')[0]}.json")


def step_flops(env_id: str, model, frame_skip: int) -> tuple[float, dict]:
    with open(counts_path(env_id)) as f:
        c = json.load(f)
    return frame_skip * substep_flops(model_dims(model), c["avg"]), c

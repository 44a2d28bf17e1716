"""Frozen algorithmic work model of one env-step: bytes and FLOPs.

The step kernel is neither HBM- nor MFMA-bound: its state stays on chip for all substeps.
Its roofline is the FP32 compute rate (157.3 TFLOP/s on gfx950, shared by VALU and the
f32-input MFMA), priced with the formula below on the average per-substep counts (contacts,
constraint rows, Newton iterations, line-search evaluations per Newton iteration, noslip sweeps)
logged by the CPU oracle in the regime the bench times: random actions
(profiles/work_counts_<task>.json) or the pretrained DAPG closed loop (work_counts_<task>_dapg.json),
both made by tools/work_counts.py.

One FLOP = one fp32 add or multiply (an FMA counts 2).  The formula counts the arithmetic
MuJoCo 2.1's own algorithms do: the joint-space inertia M is factored and
solved over the dof tree (mj_factorM / mj_solveM: work per dof proportional to its ancestor
count, ``tree_factor_flops`` / ``tree_solve_flops`` below), and only the Newton Hessian
H = M + J'DJ is dense (mj_solNewton's dense path: an nv x nv Cholesky per factorisation).  The
noslip rows' coupling J inv(M) J' is priced as sparse solves of M per row plus the dense products,
as mj_projectConstraint forms it.  Round 3's formula (``dense_m=True``) priced every M factor
and solve as dense and noslip's inv(M) as a dense 2 nv^3 inverse -- ~32 % more FLOPs than either
MuJoCo or this kernel does; it is kept only to compare against the round-3 fractions.
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


def tree_factor_flops(dof_parentid) -> float:
    """mj_factorM (L'DL over the dof tree): for dof k (leaf to root) and each ancestor i of k,
    one divide and an fma per entry of i's ancestor chain incl. i (M[i][j] -= t M[k][j])."""
    anc = _ancestors(dof_parentid)
    return float(sum(sum(1 + 2 * (len(anc[i]) + 1) for i in anc[k]) for k in range(len(anc))))


def tree_solve_flops(dof_parentid) -> float:
    """mj_solveM (x = inv(L'DL) b): an fma per ancestor entry in each of the two triangular
    sweeps, plus the diagonal scaling."""
    anc = _ancestors(dof_parentid)
    return float(4 * sum(len(a) for a in anc) + len(anc))


def _ancestors(dof_parentid):
    out = []
    for j in range(len(dof_parentid)):
        k, a = int(dof_parentid[j]), []
        while k >= 0:
            a.append(k)
            k = int(dof_parentid[k])
        out.append(a)
    return out


def substep_flops(dims: dict, c: dict, dense_m: bool = False) -> float:
    """FLOPs of one mj_step given model dims and average per-substep counts c (``dense_m``: the
    round-3 formula with dense M factors / solves and a dense noslip inverse)."""
    nv, nb, njnt = dims["nv"], dims["nbody"], dims["njnt"]
    ng, ns, nt, npair = dims["ngeom_coll"], dims["nsite"], dims["ntendon"], dims["npair_all"]
    sub = dims["avg_subtree"]          # mean bodies per subtree
    anc = dims["avg_ancestors"]        # mean ancestor dofs per dof (M nonzeros per row)
    ncon, nefc, nden = c["ncon"], c["nefc"], c["ndense"]
    it, nsit, lsit = c["newton_iter"], c["noslip_iter"], c["ls_iter"]
    chol = 2.0 * nv ** 3 / 3.0           # dense Cholesky (Newton Hessian)
    solve = 4.0 * nv ** 2
    factm, solvem = (chol, solve) if dense_m else (dims["factor_m"], dims["solve_m"])
    f = 0.0
    f += nb * 110 + njnt * 120 + ng * 75 + ns * 18             # kinematics, geom/site frames
    f += nb * (sub * 6 + 110) + nv * 20                        # subtree com, cinert, cdof
    f += nb * sub * 10 + nv * (72 + (2 * anc + 1) * 12)        # crb, M rows
    f += nb * 150 + nv * 80                                    # comVel, RNE, passive, actuation
    f += factm + solvem                                        # qacc_smooth (mj_factorM, mj_solveM)
    f += npair * 12 + ncon * 400                               # bounding tests + narrowphase
    f += nt * 6 + nefc * (40 + 2 * nv) + ncon * nv * 60        # rows, impedance, contact J
    # Newton: H = M + J'DJ (dense rows), factor, solve, matvecs, line search, gradient
    f += it * (nden * nv * nv * 2 + chol + solve + 4 * nv * nv + lsit * nefc * 12 + nefc * 4 * nv)
    # noslip: the rows' coupling J inv(M) J' (frictionloss rows J = e_d, opposing friction-edge
    # pairs through their difference rows), pair constants, sweeps
    if nsit > 0:
        if dense_m:
            f += 2 * nv ** 3 + nden * nv * 2 * nv
        else:
            npr = nden / 2
            f += (nv + npr) * solvem + npr * npr * 2 * nv          # inv(M) e_d, inv(M) jd', jd . xd
        f += nden * 3 * nv * 2
        f += nsit * (nv * (2 * nv + 10) + nden / 2 * (8 * nv + 30))
    f += factm + solvem + 6 * nv                               # implicit Euler (M + h D)
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
                avg_subtree=float(size[1:].mean()), avg_ancestors=float(np.mean(anc)),
                factor_m=tree_factor_flops(model.dof_parentid), solve_m=tree_solve_flops(model.dof_parentid))


def counts_path(env_id: str, policy: str = "none") -> str:
    """the oracle's work counts of the regime the bench times: the DAPG closed loop
    (work_counts_<task>_dapg.json) or i.i.d. random actions (work_counts_<task>.json)"""
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    suffix = "_dapg" if policy == "dapg" else ""
    return os.path.join(here, "profiles", f"work_counts_{env_id.split('-')[0]}{suffix}.json")


def step_flops(env_id: str, model, frame_skip: int, dense_m: bool = False, policy: str = "none") -> tuple[float, dict]:
    """FLOPs per env-step priced on the oracle-logged counts of the same regime (policy "dapg":
    the pretrained DAPG closed loop; otherwise the random-action counts)"""
    path = counts_path(env_id, policy)
    with open(path) as f:
        c = json.load(f)
    c["source"] = os.path.relpath(path, os.path.dirname(os.path.dirname(path)))
    return frame_skip * substep_flops(model_dims(model), c["avg"], dense_m=dense_m), c

"""Diagnose unexplained parity misses saved by tests/parity_classify.py (AW_SAVE_UNEXPLAINED=dir).

    python tools/diag_unexplained.py gpurun_out/unexplained/*.npz

For each saved miss the oracle's env-step is replayed substep by substep and, at the first substep
state where the GPU forward (aw_forward_dump) and the oracle's disagree, prints:
  * the contacts of every geom pair whose lists differ (count, depth, point) on both sides, and the
    same pair through the colliders alone (aw_collide_test vs Oracle.collide on the oracle's poses),
    which separates a collider difference from a kinematics difference;
  * the constraint-row type sequences when the row counts differ;
  * for Newton rows in different states: iterations / exit reasons, jar on both sides, and the
    REFERENCE's own Newton objective (fp64) evaluated at both solutions -- the optimality gap of the
    GPU's qacc in the reference's problem.
GPU box only (needs the HIP library)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]


def newton_cost(M, a0, J, aref, D, fl, ty, a):
    """mj_solNewton's objective: Gauss term + per-row piecewise-quadratic costs"""
    d = a - a0
    c = 0.5 * d @ M @ d
    jar = J @ a - aref
    R = 1.0 / D
    for r in range(len(jar)):
        x = jar[r]
        if ty[r] <= 1:
            f = fl[r]
            if x <= -R[r] * f:
                c += -f * x - 0.5 * R[r] * f * f
            elif x >= R[r] * f:
                c += f * x - 0.5 * R[r] * f * f
            else:
                c += 0.5 * D[r] * x * x
        elif x < 0:
            c += 0.5 * D[r] * x * x
    return c


def main(paths):
    from parity_classify import DSBL_NOSLIP, context, _contacts
    for path in paths:
        z = np.load(path, allow_pickle=False)
        env_id = str(z["env_id"])
        ctx = context(env_id)
        o, one, m = ctx.o, ctx.one, ctx.m
        nv = int(m.dims["nv"])
        print(f"=== {os.path.basename(path)}: {len(z['step'])} misses")
        for i in range(len(z["step"])):
            P, q, v, w, act = (z[k][i] for k in ("params", "qpos", "qvel", "warm", "act"))
            ctrl = ctx.ctrl(act)
            print(f"--- step {int(z['step'][i])} env {int(z['env'][i])}")
            gpu_traj = os.environ.get("AW_DIAG_GPU_TRAJ") == "1"   # walk the GPU's own substeps instead
            q0, v0, w0 = q.copy(), v.copy(), w.copy()
            for j in range(ctx.frame_skip):
                d = ctx.gpu_forward(P, q, v, w, ctrl)
                orc = ctx.oracle_forward(P, q, v, w, ctrl)
                oc = orc["contact"].reshape(-1, 23)
                gc, occ = _contacts(ctx, d, oc)
                diff_pairs = []
                for key in dict.fromkeys(list(gc) + list(occ)):
                    gl, ol = gc.get(key, []), occ.get(key, [])
                    same = len(gl) == len(ol) and all(abs(a[0] - b[0]) < 1e-5 and np.abs(a[1] - b[1]).max() < 1e-4
                                                      for a, b in zip(gl, ol))
                    if not same:
                        diff_pairs.append(key)
                gst, ost = d["efc_state"].astype(int), orc["efc_state"].astype(int)
                nefc_o = int(orc["scalars"][1])
                rows_diff = d["nefc"] == nefc_o and (gst != ost).any()
                if not diff_pairs and d["nefc"] == nefc_o and not rows_diff:
                    if gpu_traj:
                        q, v, w = ctx.gpu_substeps(P, q0.astype(np.float32).astype(np.float64), v0.astype(np.float32).astype(np.float64),
                                                   w0.astype(np.float32).astype(np.float64), act, j + 1)
                    else:
                        q, v, w = ctx.oracle_steps(P, q, v, w, ctrl, 1)
                    continue
                print(f"  substep {j}: ncon GPU {d['ncon']} / oracle {int(orc['scalars'][0])}, nefc {d['nefc']} / "
                      f"{nefc_o}, Newton GPU {d['solver_iter']} it ({d['solver_exit']}) / oracle {int(orc['scalars'][2])} it")
                gxp = o.get("geom_xpos").reshape(-1, 3)
                gxm = o.get("geom_xmat").reshape(-1, 9)
                gsz = np.asarray(m.arrays["geom_size"], float).reshape(-1, 3)
                for key in diff_pairs:
                    name = f"{ctx.gname(key[0])}|{ctx.gname(key[1])}"
                    mg = ctx.margin_of[key][0]
                    print(f"    pair {name} (margin {mg}):")
                    for side, lst in (("GPU", gc.get(key, [])), ("oracle", occ.get(key, []))):
                        for dist, pos in lst:
                            print(f"      {side:6s} dist {dist:+.6e} pos {np.array2string(pos, precision=6)}")
                    a, b = key
                    if ctx.gtype[a] > ctx.gtype[b]:
                        a, b = b, a
                    ro = o.collide(ctx.gtype[a], gxp[a], gxm[a], gsz[a], ctx.gtype[b], gxp[b], gxm[b], gsz[b], mg)
                    rg = one.collide_test([[ctx.gtype[a], ctx.gtype[b]]], [[gxp[a], gxp[b]]],
                                          [[gxm[a].reshape(3, 3), gxm[b].reshape(3, 3)]], [[gsz[a], gsz[b]]], [mg])[0]
                    print(f"      colliders alone on the oracle's poses: oracle {len(ro)} contacts "
                          f"{[round(float(x), 7) for x in ro[:, 0]]}, GPU {len(rg)} {[round(float(x), 7) for x in rg[:, 0]]}")
                    for r in ro:
                        print(f"        oracle collide: dist {r[0]:+.6e} pos {np.array2string(r[1:4], precision=6)} n {np.array2string(r[4:7], precision=4)}")
                    for r in rg:
                        print(f"        GPU collide:    dist {r[0]:+.6e} pos {np.array2string(r[1:4], precision=6)} n {np.array2string(r[4:7], precision=4)}")
                if d["nefc"] != nefc_o:
                    print(f"    row types GPU    {d['efc_type'].astype(int).tolist()}")
                    print(f"    row types oracle {orc['efc_type'].astype(int).tolist()}")
                if rows_diff:
                    dn = ctx.gpu_forward(P, q, v, w, ctrl, disableflags=DSBL_NOSLIP)
                    on = ctx.oracle_forward(P, q, v, w, ctrl, disableflags=DSBL_NOSLIP)
                    o.set_option(disableflags=DSBL_NOSLIP)
                    o.forward1(P, q, v, w, ctrl)
                    M = o.get("qM").reshape(nv, nv)
                    a0 = o.get("qacc_smooth")
                    Dv = o.get("efc_D")
                    o.set_option(disableflags=0)
                    J = on["efc_J"].reshape(-1, nv)
                    ty, fl = on["efc_type"].astype(int), on["efc_frictionloss"]
                    co = newton_cost(M, a0, J, on["efc_aref"], Dv, fl, ty, on["qacc"])
                    cg = newton_cost(M, a0, J, on["efc_aref"], Dv, fl, ty, dn["qacc"])
                    c_sm = newton_cost(M, a0, J, on["efc_aref"], Dv, fl, ty, a0)
                    mi = float(m.opt.get("meaninertia", 1.0))
                    print(f"    Newton (noslip off): reference objective at oracle qacc {co:.9e}, at GPU qacc {cg:.9e}, "
                          f"gap {cg - co:+.3e} (relative {(cg - co) / max(abs(c_sm - co), 1e-30):.2e} of the solve's "
                          f"decrease; MuJoCo tolerance x meaninertia x nv = {1e-8 * mi * nv:.2e}); GPU {dn['solver_iter']} it "
                          f"({dn['solver_exit']})")
                    da = np.abs(dn["qacc"] - on["qacc"])
                    top = np.argsort(da)[::-1][:5]
                    print(f"    |dqacc| top dofs {top.tolist()}: {np.round(da[top], 4).tolist()} (max |qacc| {np.abs(on['qacc']).max():.3e})")
                    jo = J @ on["qacc"] - on["efc_aref"]
                    jg = J @ dn["qacc"] - dn["efc_aref"]
                    for r in np.nonzero(gst != ost)[0]:
                        print(f"    row {r} type {ty[r]}: state GPU {gst[r]} oracle {ost[r]}, jar GPU {jg[r]:+.4e} "
                              f"oracle {jo[r]:+.4e}, R floss {fl[r] / Dv[r]:.3e}")
                break


if __name__ == "__main__":
    main(sys.argv[1:])

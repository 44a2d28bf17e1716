"""Classification of teacher-forced parity misses (TEST INFRASTRUCTURE: imported by the -m gpu tests).

A miss is an (env, step) case whose GPU post-step state leaves the one-step tolerance of
tests/test_gpu_parity.py (qpos 2e-5 + 1e-5 |q|, qvel 5e-3 (1 + |v|)) against the fp64 oracle run from
the same pre-step state with the same action (hammer_v0.py:54-90 and the other tasks' step).  In the
contact regimes the step is piecewise smooth, so fp32 and fp64 can land on different sides of a
switch; a miss is accepted only when that is DEMONSTRATED, as one of:

 (a) a switch: replaying the oracle substep by substep and running the GPU forward (aw_forward_dump)
     on each oracle substep state from the identical state, the two forwards differ ONLY by
       - contacts present on one side: matched by geom pair and emission order, every unmatched
         contact within DEC_EPS (2e-6 m, aw_collide.h) of its margin on the side that emitted it, or
         contacts equal but one within MARGIN_TOL of its margin, AND causally: the oracle re-run with
         that pair's margin moved across the contact's distance (Oracle.set_margin_nudge) reproduces
         the GPU's env-step within tolerance, or moves by at least 1 / SPREAD_FACTOR of the GPU's
         deviation (the reference itself cannot resolve the step at that switch);
       - Newton rows in different states (mj_solNewton): every such row's switching quantity
         jar = J qacc - aref lies within JAR_REL of its threshold (frictionloss: +-R floss; contact /
         limit rows: 0) on BOTH sides -- the GPU's jar from the oracle's J and the GPU's Newton qacc
         and aref, the oracle's from its own -- with the two sides on opposite sides of it;
     anything else the two forwards disagree on from an identical state (a contact away from its
     margin, rows that differ without a contact difference, a row state away from its switch) is a
     kernel disagreement: the miss is UNEXPLAINED, whatever the later classes would say;
 (c) an oracle-shadowed trajectory: every GPU substep from the GPU's OWN previous state within
     LOCAL_FRACTION of the one-step tolerance of the oracle's substep from that state, the replay
     ending on the GPU's env-step result; where a substep parts from the oracle's, (a)'s tests run at
     that GPU state (a switch on the GPU's own trajectory, the causal check local to that substep);
 (b) an fp32-sensitive reference: the oracle's own env-step re-run on the fp32-rounded model and from
     the state perturbed by <= 16 fp32 ulps leaves the tolerance, AND the GPU's deviation is within
     SPREAD_FACTOR x that spread.
Every accepted miss records the ratio of the GPU's deviation to the reference spread that excused it
(classes (a)-causal and (b)); the tests gate the maximum (advisor r05).  tests/test_gpu_classifier.py
holds the negative tests: faults injected through aw_set_fault must come out unexplained.
"""
from __future__ import annotations

import numpy as np

from conftest import load_task_model

DEC_EPS = 2e-6            # aw_collide.h: near-margin candidates decided in fp64
MARGIN_TOL = 1e-6         # a contact "at its margin" when the contact sets agree
JAR_REL = 1e-3            # Newton switch: |jar - threshold| within this fraction of the row's terms
SPREAD_FACTOR = 4.0
LOCAL_FRACTION = 0.1
# Per-class caps on the deviation a class may excuse (max |dqpos|, max |dqvel| / (1 + |v|)): ~4x the
# largest each class showed over the whole r06 suite (profiles/r06e_pytest_gpu.txt) -- margin switches
# 5.4e-4 / 4.6e-2 (pen DAPG), oracle-shadowed trajectories 9.9e-4 / 0.19 (pen C3), fp32-sensitive
# references 3.0e-5 / 5.7e-3, collider ties 1.5e-2 / 1.0 (door C3: the thumb capsule 1 cm deep in the
# palm box, parallel to a face, whose contact point the reference itself moves under 16-ulp inputs).
CLASS_CAP = {"contact": (2.5e-3, 0.2), "Newton row switch": (2.5e-3, 0.2), "switch on the GPU's own trajectory": (2.5e-3, 0.2),
             "oracle-shadowed trajectory": (4e-3, 0.8), "fp32-sensitive reference": (2e-4, 0.03),
             "collider tie": (6e-2, 4.0)}


def class_cap(key):
    for k, c in CLASS_CAP.items():
        if key.startswith(k):
            return c
    return None
DSBL_NOSLIP = 1 << 14
_GTYPES = {0: "plane", 2: "sphere", 3: "capsule", 5: "cylinder", 6: "box"}


def f32(a):
    return np.asarray(a, np.float32).astype(np.float64)


def within_tol(q, v, q_ref, v_ref):
    q, v, q_ref, v_ref = (np.asarray(x, float) for x in (q, v, q_ref, v_ref))
    return bool((np.abs(q - q_ref) <= 2e-5 + 1e-5 * np.abs(q_ref)).all()
                and (np.abs(v - v_ref) <= 5e-3 * (1 + np.abs(v_ref))).all())


def deviation(q, v, q_ref, v_ref):
    """(max |dqpos|, max |dqvel| / (1 + |v_ref|))"""
    q, v, q_ref, v_ref = (np.asarray(x, float) for x in (q, v, q_ref, v_ref))
    return float(np.abs(q - q_ref).max()), float((np.abs(v - v_ref) / (1 + np.abs(v_ref))).max())


class Ctx:
    """Per (task, variation): the model, an uncapped fp64 oracle (MuJoCo's nconmax / njmax), a one-env
    GPU handle with frame_skip 1 (forward dumps and single substeps) and the kernel's pair table."""

    def __init__(self, env_id, variation=None):
        import torch
        from mj_envs_amd import _native
        from oracle.pyoracle import Oracle
        self.env_id, self.variation = env_id, variation
        self.m = load_task_model(env_id, variation)
        self.frame_skip = int(self.m.dims["task_frame_skip"])
        self.o = Oracle(self.m.to_blob())
        m1 = load_task_model(env_id, variation)
        m1.dims["task_frame_skip"] = 1
        self.one = _native.Sim(m1.to_blob(), 1)
        self._fs, self.fault = {1: self.one}, (0, 0)   # frame_skip-k handles (gpu_substeps)
        self.torch = torch
        A = self.m.arrays
        g1 = list(np.asarray(A["pair_geom1"], int)) + list(np.asarray(A["cand_geom1"], int))
        g2 = list(np.asarray(A["pair_geom2"], int)) + list(np.asarray(A["cand_geom2"], int))
        gm = np.asarray(A["geom_margin"], float)
        gg = np.asarray(A.get("geom_gap", np.zeros_like(gm)), float)
        npair = len(A["pair_geom1"])
        self.pairs = []
        for p, (a, b) in enumerate(zip(g1, g2)):
            if p < npair:
                mg, gp = float(A["pair_margin"][p]), float(A["pair_gap"][p])
            else:
                mg, gp = max(gm[a], gm[b]), max(gg[a], gg[b])
            self.pairs.append((a, b, mg, gp))
        self.margin_of = {(min(a, b), max(a, b)): (mg, gp) for a, b, mg, gp in self.pairs}
        self.gtype = np.asarray(A["geom_type"], int)

    def gname(self, g):
        n = self.m.names["geom"][g] if g < len(self.m.names["geom"]) else None
        return f"{n or g}:{_GTYPES.get(int(self.gtype[g]), self.gtype[g])}"

    def ctrl(self, act):
        return self.m.task_act_mid + np.clip(act, -1, 1) * self.m.task_act_rng

    def _t(self, a):
        return self.torch.tensor(np.asarray(a), dtype=self.torch.float32, device="cuda")

    # --- one forward on each side from an identical state --------------------------------------
    def gpu_forward(self, params, q, v, w, ctrl, disableflags=0, wide=False):
        if disableflags:
            self.one.set_option(disableflags=disableflags)
        self.one.set_state(self._t(q[None]), self._t(v[None]), self._t(w[None]), self._t(np.asarray(params)[None]))
        d = self.one.forward_dump(0, self._t(ctrl), wide=wide)
        if disableflags:
            self.one.set_option(disableflags=0)
        return d

    def oracle_forward(self, params, q, v, w, ctrl, disableflags=0):
        if disableflags:
            self.o.set_option(disableflags=disableflags)
        self.o.forward1(params, q, v, w, ctrl)
        out = {k: self.o.get(k) for k in ("scalars", "contact", "efc_state", "efc_type", "qacc")}
        if disableflags:
            out.update({k: self.o.get(k) for k in ("efc_J", "efc_aref", "efc_R", "efc_frictionloss")})
            self.o.set_option(disableflags=0)
        return out

    def oracle_steps(self, params, q, v, w, ctrl, nsub, nudge=None):
        q, v, w = q.copy(), v.copy(), w.copy()
        if nudge is not None:
            self.o.set_margin_nudge(*nudge)
        try:
            self.o.mjstep1(params, q, v, w, ctrl, nsub)
        finally:
            if nudge is not None:
                self.o.set_margin_nudge()
        return q, v, w

    def set_fault(self, kind, arg):
        """aw_set_fault on every GPU handle of the context (the classifier inspects the faulty kernel)"""
        self.fault = (kind, arg)
        for h in self._fs.values():
            h.set_fault(kind, arg)

    def _fs_handle(self, k):
        h = self._fs.get(k)
        if h is None:
            from mj_envs_amd import _native
            mk = load_task_model(self.env_id, self.variation)
            mk.dims["task_frame_skip"] = k
            h = self._fs[k] = _native.Sim(mk.to_blob(), 1)
            if self.fault != (0, 0):
                h.set_fault(*self.fault)
        return h

    def gpu_substeps(self, params, q, v, w, act, k):
        """the GPU's state after the first k substeps of the env-step from (q, v, w): the env-step of a
        frame_skip-k handle is exactly those substeps.  (Inside an env-step the kernel carries each
        position as qpos + qlo across substeps, so k separate one-substep env-steps from the rounded
        fp32 states would not reproduce it.)"""
        h, torch = self._fs_handle(k), self.torch
        ob, rw = h.empty(1, h.obs_dim), h.empty(1)
        dn, gl = h.empty(1, dtype=torch.uint8), h.empty(1, dtype=torch.uint8)
        qq, vv, ww = h.empty(1, h.nq), h.empty(1, h.nv), h.empty(1, h.nv)
        h.set_state(self._t(q[None]), self._t(v[None]), self._t(w[None]), self._t(np.asarray(params)[None]))
        h.step(self._t(np.asarray(act)[None]), ob, rw, dn, gl)
        h.get_state(qq, vv, ww)
        torch.cuda.synchronize()
        return tuple(x[0].cpu().numpy().astype(np.float64) for x in (qq, vv, ww))


# ----------------------------------------------------------------------------------------------
def _contacts(ctx, d, oc):
    """per unordered geom pair: the GPU's and the oracle's contacts (dist, pos) in emission order"""
    from collections import OrderedDict
    g, o = OrderedDict(), OrderedDict()
    for p, dist, pos in zip(d["con_pair"], d["con_dist"], d["con_pos"]):
        a, b = ctx.pairs[int(p)][:2]
        g.setdefault((min(a, b), max(a, b)), []).append((float(dist), np.asarray(pos, float)))
    for row in oc:
        a, b = int(row[13]), int(row[14])
        o.setdefault((min(a, b), max(a, b)), []).append((float(row[0]), np.asarray(row[1:4], float)))
    return g, o


def _unmatched(gl, ol):
    """contacts of one pair left over on either side after greedy nearest-position matching"""
    if len(gl) == len(ol):
        return [], []
    G, O = list(range(len(gl))), list(range(len(ol)))
    while G and O:
        best = min(((np.linalg.norm(gl[i][1] - ol[j][1]), i, j) for i in G for j in O))
        G.remove(best[1])
        O.remove(best[2])
    return [gl[i] for i in G], [ol[j] for j in O]


POS_TOL, DIST_TOL = 1e-4, 1e-5   # matched contacts: a point 0.1 mm or a depth 10 um apart is a collider difference
TIE_DRAWS, TIE_ULPS = 8, 16


def perturb_qpos(q, eps, rng):
    """qpos moved by up to eps (TIE_ULPS fp32 ulps) of max(|q|, 1) per joint: the fp32 resolution of
    the kinematic chain, whose rounding is absolute (~ulp of the O(1) frame entries) however small the
    joint angle -- a purely relative perturbation of a joint near 0 rad would be far below it"""
    return q + eps * np.maximum(np.abs(q), 1.0) * rng.uniform(-1, 1, q.shape)


def _pair_contacts_oracle(ctx, key, params, q, v, w, ctrl):
    ctx.o.forward1(params, q, v, w, ctrl)
    oc = ctx.o.get("contact").reshape(-1, 23)
    return [(float(r[0]), np.asarray(r[1:4], float)) for r in oc
            if (min(int(r[13]), int(r[14])), max(int(r[13]), int(r[14]))) == key]


def _lists_differ(a, b):
    if len(a) != len(b):
        return True
    return any(abs(x[0] - y[0]) > DIST_TOL or np.abs(x[1] - y[1]).max() > POS_TOL for x, y in zip(a, b))


def oracle_tie(ctx, key, params, q, v, w, ctrl, seed=0):
    """Is the reference's own collider decision for this pair unstable at fp32 resolution?  True when
    the oracle's contacts of the pair change (count, a point by > POS_TOL or a depth by > DIST_TOL)
    under <= TIE_ULPS-ulp perturbations of qpos (perturb_qpos, TIE_DRAWS draws): a degenerate configuration (a
    capsule parallel to a face, a flat minimum of the segment-box distance, a cylinder's line contact)
    whose tie is broken by rounding."""
    base = _pair_contacts_oracle(ctx, key, params, q, v, w, ctrl)
    rng = np.random.default_rng(seed)
    eps = TIE_ULPS * 2.0 ** -23
    for _ in range(TIE_DRAWS):
        qp = perturb_qpos(q, eps, rng)
        if _lists_differ(_pair_contacts_oracle(ctx, key, params, qp, v, w, ctrl), base):
            return True
    return False


POSE_TOL = 1e-5   # body frames: the GPU's fp32 kinematics against the reference's fp64 (m, quaternion units)


def _quat2mat(qt):
    w, x, y, z = np.asarray(qt, float) / np.linalg.norm(qt)
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def pose_tie(ctx, key, d, gl, params, q, v, w, ctrl):
    """Is the GPU's contact list for this pair the REFERENCE's own collider output on the GPU's body
    frames?  True when the two bodies' GPU frames (fp32 kinematics) agree with the reference's to
    POSE_TOL and the oracle's collider, run on the geom poses composed from those frames, reproduces
    the GPU's contacts: the difference is then the reference's decision flipping under an fp32-sized
    pose change (a capsule parallel to a face, a segment inside a box), not a collider difference."""
    A = ctx.m.arrays
    gb = np.asarray(A["geom_bodyid"], int)
    gp = np.asarray(A["geom_pos"], float).reshape(-1, 3)
    gq = np.asarray(A["geom_quat"], float).reshape(-1, 4)
    gs = np.asarray(A["geom_size"], float).reshape(-1, 3)
    xp = np.asarray(d["xpos"], float).reshape(-1, 3)
    xq = np.asarray(d["xquat"], float).reshape(-1, 4)
    ctx.o.forward1(params, q, v, w, ctrl)
    oxp, oxq = ctx.o.get("xpos").reshape(-1, 3), ctx.o.get("xquat").reshape(-1, 4)
    for g in key:
        b = gb[g]
        if np.abs(xp[b] - oxp[b]).max() > POSE_TOL or np.abs(xq[b] - oxq[b]).max() > POSE_TOL:
            return False
    a, b = key
    if ctx.gtype[a] > ctx.gtype[b]:
        a, b = b, a

    def pose(g):
        R = _quat2mat(xq[gb[g]])
        return xp[gb[g]] + R @ gp[g], (R @ _quat2mat(gq[g])).reshape(9)

    (pa, ma), (pb, mb) = pose(a), pose(b)
    ro = ctx.o.collide(ctx.gtype[a], pa, ma, gs[a], ctx.gtype[b], pb, mb, gs[b], ctx.margin_of[key][0])
    lst = [(float(r[0]), np.asarray(r[1:4], float)) for r in ro]
    return len(lst) == len(gl) and not _lists_differ(sorted(lst, key=lambda t: tuple(t[1])),
                                                    sorted(gl, key=lambda t: tuple(t[1])))


def depth_tie(ctx, key, gl, ol, params, q, v, w, ctrl):
    """Capsule-box with the same contact count and depths: is every GPU contact point an exact minimiser
    of the REFERENCE's own capsule-box distance?  Each GPU point is projected on the capsule axis (the
    reference's frames) and the reference's sphere-box collider at that axis point must give the same
    depth (DIST_TOL): the GPU picked another point of a flat minimum (a capsule parallel to a face, a
    segment inside the box), where the order of equal candidates is decided by rounding."""
    a, b = key
    if sorted((ctx.gtype[a], ctx.gtype[b])) != [3, 6] or len(gl) != len(ol) or not gl:
        return False
    if any(abs(x[0] - y[0]) > DIST_TOL for x, y in zip(sorted(gl, key=lambda t: t[0]), sorted(ol, key=lambda t: t[0]))):
        return False
    c, x = (a, b) if ctx.gtype[a] == 3 else (b, a)
    ctx.o.forward1(params, q, v, w, ctrl)
    gxp, gxm = ctx.o.get("geom_xpos").reshape(-1, 3), ctx.o.get("geom_xmat").reshape(-1, 9)
    gs = np.asarray(ctx.m.arrays["geom_size"], float).reshape(-1, 3)
    axis = gxm[c].reshape(3, 3)[:, 2]
    mg = ctx.margin_of[key][0]
    for dist, pos in gl:
        t = float(np.clip(np.dot(pos - gxp[c], axis), -gs[c][1], gs[c][1]))
        r = ctx.o.collide(2, gxp[c] + t * axis, np.eye(3).reshape(9), np.array([gs[c][0], 0.0, 0.0]),
                          6, gxp[x], gxm[x], gs[x], mg)
        if len(r) == 0 or abs(float(np.min(r[:, 0])) - dist) > DIST_TOL:
            return False
    return True


def forward_diff(ctx, params, q, v, w, ctrl, jar_log=None):
    """Compare the two forwards from the identical fp32 state (q, v, w rounded to fp32 for BOTH sides,
    as the GPU holds it).  Returns
       ("same", None)                            no difference,
       ("switch", [records])                     differences that are all switches (module doc, (a)),
       ("contradiction", reason)                 a difference that is not,
       ("overflow", None)                        the fast tier overflowed (nothing can be compared).
    A record is dict(kind="contact" | "tie" | "row", ...)."""
    from mj_envs_amd import _native
    q, v, w = f32(q), f32(v), f32(w)
    d = ctx.gpu_forward(params, q, v, w, ctrl)
    if int(d["status"]) & _native.ST_OVERFLOW:
        return "overflow", None
    orc = ctx.oracle_forward(params, q, v, w, ctrl)
    oc = orc["contact"].reshape(-1, 23)
    gc, occ = _contacts(ctx, d, oc)
    recs = []
    ties = []
    for key in list(dict.fromkeys(list(gc) + list(occ))):
        mg = ctx.margin_of.get(key, (None, None))[0]
        name = f"{ctx.gname(key[0])}|{ctx.gname(key[1])}"
        gl, ol = gc.get(key, []), occ.get(key, [])
        gu, ou = _unmatched(gl, ol)
        far = [(side, dist) for side, lst in (("gpu", gu), ("oracle", ou)) for dist, _ in lst
               if mg is None or abs(dist - mg) > DEC_EPS]
        geo = len(gl) == len(ol) and _lists_differ(gl, ol)
        if far or geo:
            # the colliders disagree on identical inputs away from any margin: only a tie the
            # reference itself breaks differently at fp32 resolution can excuse that
            why = (f"{far[0][0]}-only contact {name} at {far[0][1] - (mg or 0):+.2e} from its margin" if far else
                   f"contacts of {name} differ in point / depth")
            if oracle_tie(ctx, key, params, q, v, w, ctrl):
                ties.append(dict(kind="tie", pair=key, name=name, why=why, pose=False))
            elif pose_tie(ctx, key, d, gl, params, q, v, w, ctrl):
                ties.append(dict(kind="tie", pair=key, name=name, why=why + " (the reference's collider on the GPU's "
                                 "frames gives the GPU's contacts)", pose=True))
            elif not far and depth_tie(ctx, key, gl, ol, params, q, v, w, ctrl):
                ties.append(dict(kind="tie", pair=key, name=name, why=why + " (every GPU point is an equal-depth "
                                 "minimiser of the reference's distance)", pose=True))
            else:
                return "contradiction", why + (" (the reference's decision is stable under 16-ulp perturbations, its "
                                               "collider on the GPU's frames does not give the GPU's contacts and "
                                               "they are not equal-depth minimisers of its distance)")
            continue
        for side, lst in (("gpu", gu), ("oracle", ou)):
            for dist, pos in lst:
                recs.append(dict(kind="contact", what="unmatched", side=side, pair=key, dist=dist, margin=mg,
                                 name=name))
    if ties:
        return "switch", ties + recs
    sets_equal = not recs
    if sets_equal:
        if d["nefc"] != int(orc["scalars"][1]):
            return "contradiction", f"rows differ ({d['nefc']} vs {int(orc['scalars'][1])}) with equal contacts"
        for key, lst in occ.items():
            mg = ctx.margin_of.get(key, (None, None))[0]
            for dist, pos in lst:
                if mg is not None and abs(dist - mg) < MARGIN_TOL:
                    recs.append(dict(kind="contact", what="at margin", side="both", pair=key, dist=dist, margin=mg,
                                     name=f"{ctx.gname(key[0])}|{ctx.gname(key[1])}"))
    if sets_equal and d["nefc"]:
        # equal contact sets: the rows correspond one to one, so every row in a different Newton state
        # must sit at its switch (a contact at its margin elsewhere does not excuse it)
        gst, ost = d["efc_state"].astype(int), orc["efc_state"].astype(int)
        rows = np.nonzero(gst != ost)[0]
        if rows.size:
            # Newton's own qacc on both sides (noslip off: it runs after Newton and moves qacc)
            dn = ctx.gpu_forward(params, q, v, w, ctrl, disableflags=DSBL_NOSLIP)
            on = ctx.oracle_forward(params, q, v, w, ctrl, disableflags=DSBL_NOSLIP)
            nv = len(on["qacc"])
            J = on["efc_J"].reshape(-1, nv)
            if J.shape[0] != d["nefc"] or not np.array_equal(dn["efc_state"].astype(int), gst):
                return "contradiction", "Newton rows differ between the noslip-on and -off forwards"
            jar_o = J @ on["qacc"] - on["efc_aref"]
            jar_g = J @ dn["qacc"] - dn["efc_aref"]
            R, fl, ty = on["efc_R"], on["efc_frictionloss"], on["efc_type"].astype(int)
            # the precision of an fp32 Newton solution on a row: its terms at the scale of the solve
            # (the fp32 exit stops at the rounding floor of the whole gradient, not of each row)
            scale = np.abs(on["efc_aref"]) + R * fl + np.abs(J).sum(1) * np.abs(on["qacc"]).max()
            if jar_log is not None:
                same = gst == ost
                jar_log.append((np.abs(jar_g - jar_o) / np.maximum(scale, 1e-30))[same])
            for r in rows:
                tol = JAR_REL * scale[r]
                # each side's jar must be within tol of the OTHER side's zone (mj_solNewton's row
                # states: LINEARNEG jar <= -R f, QUADRATIC in between, LINEARPOS jar >= R f for
                # frictionloss rows; QUADRATIC jar < 0, SATISFIED jar >= 0 for contact / limit rows)
                def zone_dist(jar, st):
                    if ty[r] <= 1:
                        lo, hi = -R[r] * fl[r], R[r] * fl[r]
                        return max(0.0, jar - lo) if st == 2 else (max(0.0, hi - jar) if st == 3 else
                                                                    max(0.0, lo - jar, jar - hi))
                    return max(0.0, jar) if st == 1 else max(0.0, -jar)
                dg, do = zone_dist(jar_g[r], int(ost[r])), zone_dist(jar_o[r], int(gst[r]))
                if not (dg <= tol and do <= tol):
                    return "contradiction", (f"Newton row {r} (type {ty[r]}) GPU state {gst[r]} vs oracle {ost[r]}: "
                                             f"jar GPU {jar_g[r]:+.3e} / oracle {jar_o[r]:+.3e} (R floss "
                                             f"{R[r] * fl[r]:.2e}), {max(dg, do):.2e} from the other side's state "
                                             f"(tolerance {tol:.2e})")
                recs.append(dict(kind="row", row=int(r), type=int(ty[r]), jar_gpu=float(jar_g[r]),
                                 jar_oracle=float(jar_o[r]), tol=float(tol), name=f"row {r} (type {ty[r]})"))
    return ("switch", recs) if recs else ("same", None)


def _nudges(rec):
    """margin shifts that move the pair's margin across the contact's distance (and DEC_EPS either way)"""
    x = rec["dist"] - rec["margin"]
    return sorted({x - 1e-9, x + 1e-9, -DEC_EPS, DEC_EPS, -2 * DEC_EPS, 2 * DEC_EPS})


def causal(ctx, params, q, v, w, ctrl, nsub, gpu, recs):
    """Do the contact switches in recs account for the GPU's result (gpu = (qpos, qvel) after nsub
    substeps from (q, v, w))?  Returns (ok, ratio): ok when an oracle run with one switched pair's margin
    moved across its contact reproduces the GPU within tolerance (ratio 0), or when the GPU's deviation
    from the unnudged oracle is within SPREAD_FACTOR x the largest deviation the nudges cause."""
    bq, bv, _ = ctx.oracle_steps(params, q, v, w, ctrl, nsub)
    gq, gv = gpu
    eq, ev = deviation(gq, gv, bq, bv)
    sq = sv = 0.0
    for rec in recs:
        if rec["kind"] != "contact":
            continue
        for dl in _nudges(rec):
            nq, nv_, _ = ctx.oracle_steps(params, q, v, w, ctrl, nsub, nudge=(rec["pair"][0], rec["pair"][1], dl))
            if within_tol(gq, gv, nq, nv_):
                return True, 0.0
            a, b = deviation(nq, nv_, bq, bv)
            sq, sv = max(sq, a), max(sv, b)
    rq = eq / sq if sq > 0 else np.inf
    rv = ev / sv if sv > 0 else np.inf
    okq = (np.abs(gq - bq) <= 2e-5 + 1e-5 * np.abs(bq)).all() or rq <= SPREAD_FACTOR
    okv = (np.abs(gv - bv) <= 5e-3 * (1 + np.abs(bv))).all() or rv <= SPREAD_FACTOR
    ratio = max(rq if not (np.abs(gq - bq) <= 2e-5 + 1e-5 * np.abs(bq)).all() else 0.0,
                rv if not (np.abs(gv - bv) <= 5e-3 * (1 + np.abs(bv))).all() else 0.0)
    return bool(okq and okv), float(ratio)


def tie_causal(ctx, params, q, v, w, ctrl, nsub, gpu, trials=8, ulps=16, seed=0):
    """Does a collider tie account for the GPU's result after nsub substeps from (q, v, w)?  The oracle
    re-run from the state perturbed by <= `ulps` fp32 ulps per component (the resolution at which the
    tie is broken): (ok, ratio) -- ok when a perturbed run reproduces the GPU within tolerance (ratio
    0) or the GPU's deviation from the unperturbed run is within SPREAD_FACTOR x the perturbed runs'."""
    rng = np.random.default_rng(seed)
    bq, bv, _ = ctx.oracle_steps(params, q, v, w, ctrl, nsub)
    gq, gv = gpu
    eq, ev = deviation(gq, gv, bq, bv)
    eps = ulps * 2.0 ** -23
    sq = sv = 0.0
    for _ in range(trials):
        pq = perturb_qpos(q, eps, rng)
        pv, pw = (x * (1 + eps * rng.uniform(-1, 1, x.shape)) for x in (v, w))
        nq, nv_, _ = ctx.oracle_steps(params, pq, pv, pw, ctrl, nsub)
        if within_tol(gq, gv, nq, nv_):
            return True, 0.0
        a, b = deviation(nq, nv_, bq, bv)
        sq, sv = max(sq, a), max(sv, b)
    inq = (np.abs(gq - bq) <= 2e-5 + 1e-5 * np.abs(bq)).all()
    inv = (np.abs(gv - bv) <= 5e-3 * (1 + np.abs(bv))).all()
    rq = 0.0 if inq else (eq / sq if sq > 0 else np.inf)
    rv = 0.0 if inv else (ev / sv if sv > 0 else np.inf)
    ratio = max(rq, rv)
    return bool(ratio <= SPREAD_FACTOR), float(ratio)


def switch_event(ctx, params, q, v, w, act, gpu, jar_log=None):
    """(a): the oracle's env-step replayed substep by substep, the two forwards compared at each substep
    state.  Returns (verdict, label, ratio): verdict True (explained), False (contradiction) or None
    (no switch found on the oracle's trajectory, or one that does not account for the GPU)."""
    ctrl = ctx.ctrl(act)
    q, v, w = q.copy(), v.copy(), w.copy()
    q0, v0, w0 = q.copy(), v.copy(), w.copy()
    contact_recs, tie_recs, row_recs = [], [], []
    for j in range(ctx.frame_skip):
        kind, info = forward_diff(ctx, params, q, v, w, ctrl, jar_log)
        if kind == "contradiction":
            return False, f"substep {j}: {info}", None
        if kind == "overflow":
            return None, None, None
        if kind == "switch":
            for r in info:
                r["substep"] = j
            contact_recs += [r for r in info if r["kind"] == "contact"]
            tie_recs += [r for r in info if r["kind"] == "tie"]
            row_recs += [r for r in info if r["kind"] == "row" and "jar_gpu" in r]
        q, v, w = ctx.oracle_steps(params, q, v, w, ctrl, 1)
    notes = []
    if tie_recs:
        ok, ratio = tie_causal(ctx, params, q0, v0, w0, ctrl, ctx.frame_skip, gpu)
        label = f"collider tie ({tie_recs[0]['name']})"
        if ok:
            return True, label, ratio
        if all(r.get("pose") for r in tie_recs):
            # proven on the GPU's own frames (pose_tie); what it may excuse is bounded by the class cap
            return True, label + " [pose]", None
        notes.append(f"{label}: does not account for the GPU (ratio {ratio:.1f})")
    if contact_recs:
        ok, ratio = causal(ctx, params, q0, v0, w0, ctrl, ctx.frame_skip, gpu, contact_recs)
        r0 = contact_recs[0]
        label = f"contact {r0['what']} ({r0['name']})"
        if ok:
            return True, label, ratio
        notes.append(f"{label}: the switch does not account for the GPU (ratio {ratio:.1f})")
    if row_recs and not notes:
        return True, "Newton row switch", None
    return None, "; ".join(notes) or None, None


def shadowed(ctx, params, qpos, qvel, warm, act, gpu, jar_log=None):
    """(c): "shadowed", "switch" / "tie" (a switch / collider tie on the GPU's own trajectory), False (a contradiction there)
    or None; with the reason"""
    ctrl = ctx.ctrl(act)
    q0, v0, w0 = (f32(x) for x in (qpos, qvel, warm))
    q, v, w = q0, v0, w0
    worst = 0.0
    for j in range(ctx.frame_skip):
        qs, vs, ws = q.copy(), v.copy(), w.copy()
        q, v, w = ctx.gpu_substeps(params, q0, v0, w0, act, j + 1)
        qo, vo, _ = ctx.oracle_steps(params, qs, vs, ws, ctrl, 1)
        eq = np.abs(q - qo) / (2e-5 + 1e-5 * np.abs(qo))
        ev = np.abs(v - vo) / (5e-3 * (1 + np.abs(vo)))
        loc = max(float(eq.max()), float(ev.max()))
        if loc > LOCAL_FRACTION:
            kind, info = forward_diff(ctx, params, qs, vs, ws, ctrl, jar_log)
            why = f"substep {j}: the GPU's substep from its own state is {loc:.2f} of the tolerance from the oracle's"
            if kind == "contradiction":
                return False, f"{why}; at that state: {info}"
            if kind != "switch":
                return None, f"{why}; no switch at that state"
            crec = [r for r in info if r["kind"] == "contact"]
            trec = [r for r in info if r["kind"] == "tie"]
            if trec:
                ok, ratio = tie_causal(ctx, params, qs, vs, ws, ctrl, 1, (q, v))
                if not ok and not all(r.get("pose") for r in trec):
                    return None, f"{why}; the tie ({trec[0]['name']}) does not account for it (ratio {ratio:.1f})"
            elif crec:
                ok, ratio = causal(ctx, params, qs, vs, ws, ctrl, 1, (q, v), crec)
                if not ok:
                    return None, f"{why}; the switch ({crec[0]['name']}) does not account for it (ratio {ratio:.1f})"
            return ("tie" if trec else "switch"), f"{why}; at that state: {info[0]['name']}"
        worst = max(worst, loc)
    same = np.array_equal(q.astype(np.float32), np.asarray(gpu[0], np.float32)) and \
        np.array_equal(v.astype(np.float32), np.asarray(gpu[1], np.float32))
    if same:
        return "shadowed", f"local substep errors <= {worst:.3f} of the tolerance"
    return None, "the substep replay does not end on the env-step result"


def newton_cost(M, a0, J, aref, D, fl, ty, a):
    """mj_solNewton's objective at qacc a, in fp64: the Gauss term 1/2 (a - a0)' M (a - a0) plus each
    row's piecewise-quadratic cost (frictionloss rows: quadratic within +-R floss, linear beyond;
    contact / limit rows: quadratic when jar < 0)"""
    d = np.asarray(a, float) - a0
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


def newton_gap(ctx, params, q, v, w, ctrl, wide=False):
    """The GPU's Newton solution (noslip off) in the REFERENCE's own problem: (objective at the oracle's
    qacc, at the GPU's, at qacc_smooth) from the identical fp32 state, and the two dumps"""
    q, v, w = f32(q), f32(v), f32(w)
    dn = ctx.gpu_forward(params, q, v, w, ctrl, disableflags=DSBL_NOSLIP, wide=wide)
    o = ctx.o
    o.set_option(disableflags=DSBL_NOSLIP)
    o.forward1(params, q, v, w, ctrl)
    nv = len(o.get("qacc"))
    M, a0, qa = o.get("qM").reshape(nv, nv), o.get("qacc_smooth"), o.get("qacc")
    J = o.get("efc_J").reshape(-1, nv)
    aref, D, fl, ty = o.get("efc_aref"), o.get("efc_D"), o.get("efc_frictionloss"), o.get("efc_type").astype(int)
    sc = o.get("scalars")
    o.set_option(disableflags=0)
    args = (M, a0, J, aref, D, fl, ty)
    return dict(c_oracle=newton_cost(*args, qa), c_gpu=newton_cost(*args, dn["qacc"]), c_smooth=newton_cost(*args, a0),
                gpu=dn, oracle_qacc=qa, oracle_qacc_smooth=a0, oracle_ncon=int(sc[0]), oracle_nefc=int(sc[1]),
                oracle_iter=int(sc[2]))


_ORACLE_F32 = {}


def oracle_f32_model(env_id, variation=None):
    key = (env_id, variation)
    if key not in _ORACLE_F32:
        from oracle.pyoracle import Oracle
        m = load_task_model(env_id, variation)
        for k, v in list(m.arrays.items()):
            a = np.asarray(v)
            if a.dtype.kind == "f":
                m.arrays[k] = a.astype(np.float32).astype(np.float64)
        m.opt = {k: (float(np.float32(v)) if isinstance(v, float) else v) for k, v in m.opt.items()}
        _ORACLE_F32[key] = Oracle(m.to_blob())
    return _ORACLE_F32[key]


def fp32_spread(o, params, qpos, qvel, warm, act, env_id=None, variation=None, trials=8, ulps=16, seed=0):
    """the oracle's env-step on the fp32-rounded model and from <= `ulps`-ulp perturbed states: (base
    (qpos, qvel), leaves the tolerance, max |dqpos|, max |dqvel| / (1 + |v|))"""
    rng = np.random.default_rng(seed)
    base = dict(qpos=qpos[None].copy(), qvel=qvel[None].copy(), warm=warm[None].copy(), params=params[None].copy())
    o.step(base, act[None])
    runs = []
    if env_id is not None:
        runs.append((oracle_f32_model(env_id, variation), dict(qpos=qpos[None].copy(), qvel=qvel[None].copy(),
                                                              warm=warm[None].copy(), params=params[None].copy())))
    eps = ulps * 2.0 ** -23
    for _ in range(trials):
        st = dict(params=params[None].copy())
        for k, x in (("qpos", qpos), ("qvel", qvel), ("warm", warm)):
            st[k] = (x * (1 + eps * rng.uniform(-1, 1, x.shape)))[None]
        runs.append((o, st))
    leaves, dq, dv = False, 0.0, 0.0
    for oo, st in runs:
        oo.step(st, act[None])
        leaves |= not within_tol(st["qpos"][0], st["qvel"][0], base["qpos"][0], base["qvel"][0])
        a, b = deviation(st["qpos"][0], st["qvel"][0], base["qpos"][0], base["qvel"][0])
        dq, dv = max(dq, a), max(dv, b)
    return (base["qpos"][0], base["qvel"][0]), leaves, dq, dv


def fp32_sensitive(ctx, params, qpos, qvel, warm, act, gpu):
    """(b): (ok, ratio of the GPU's deviation to the reference's spread)"""
    (bq, bv), leaves, dq, dv = fp32_spread(ctx.o, params, qpos, qvel, warm, act, ctx.env_id, ctx.variation)
    if not leaves:
        return False, None
    gq, gv = np.asarray(gpu[0], float), np.asarray(gpu[1], float)
    eq, ev = deviation(gq, gv, bq, bv)
    inq = (np.abs(gq - bq) <= 2e-5 + 1e-5 * np.abs(bq)).all()
    inv = (np.abs(gv - bv) <= 5e-3 * (1 + np.abs(bv))).all()
    rq = 0.0 if inq else (eq / dq if dq > 0 else np.inf)
    rv = 0.0 if inv else (ev / dv if dv > 0 else np.inf)
    ratio = max(rq, rv)
    return bool(ratio <= SPREAD_FACTOR), float(ratio)


_CTX = {}


def context(env_id, variation=None):
    key = (env_id, variation)
    if key not in _CTX:
        _CTX[key] = Ctx(env_id, variation)
    return _CTX[key]


def classify_miss(env_id, ms, variation=None, jar_log=None):
    """ms = (step, env, params, qpos, qvel, warm, action, gpu_qpos, gpu_qvel) -> (class or None, reason,
    ratio, (dq, dv) of the GPU against the oracle's env-step)"""
    ctx = context(env_id, variation)
    k, e, params, q, v, w, a = ms[:7]
    gpu = (np.asarray(ms[7], float), np.asarray(ms[8], float))
    params, q, v, w, a = (np.asarray(x, np.float64) for x in (params, q, v, w, a))
    bq, bv, _ = ctx.oracle_steps(params, q, v, w, ctx.ctrl(a), ctx.frame_skip)
    dev = deviation(gpu[0], gpu[1], bq, bv)
    verdict, label, ratio = switch_event(ctx, params, q, v, w, a, gpu, jar_log)
    if verdict is False:
        return None, label, None, dev
    if verdict:
        return label, label, ratio, dev
    why_a = label
    sh, why = shadowed(ctx, params, q, v, w, a, gpu, jar_log)
    if sh is False:
        return None, why, None, dev
    if sh == "shadowed":
        return "oracle-shadowed trajectory", why, None, dev
    if sh == "switch":
        return "switch on the GPU's own trajectory", why, None, dev
    if sh == "tie":
        return "collider tie on the GPU's own trajectory", why, None, dev
    ok, ratio = fp32_sensitive(ctx, params, q, v, w, a, gpu)
    if ok:
        return "fp32-sensitive reference", f"ratio {ratio:.2f}", ratio, dev
    return None, "; ".join(x for x in (why_a, why, f"fp32 spread ratio {ratio}" if ratio is not None else None) if x), \
        None, dev


def classify_misses(env_id, misses, variation=None, label=""):
    """Classify every miss; prints the tally of classes with the largest deviation and the largest
    excusing ratio per class.  Returns (unexplained [(step, env, reason)], tally dict)."""
    tally = {}
    out = []
    jar_log = []
    for ms in misses:
        cls, reason, ratio, dev = classify_miss(env_id, ms, variation, jar_log)
        if cls is None:
            print(f"  unexplained step {ms[0]} env {ms[1]}: {reason}", flush=True)
            out.append((ms[0], ms[1], reason))
            cls = "UNEXPLAINED"
        key = cls.split(" (")[0]
        t = tally.setdefault(key, dict(n=0, max_dqpos=0.0, max_dqvel=0.0, max_ratio=0.0))
        t["n"] += 1
        t["max_dqpos"] = max(t["max_dqpos"], dev[0])
        t["max_dqvel"] = max(t["max_dqvel"], dev[1])
        if ratio is not None and np.isfinite(ratio):
            t["max_ratio"] = max(t["max_ratio"], ratio)
    save = __import__("os").environ.get("AW_SAVE_UNEXPLAINED")
    if save and out:
        # the unexplained misses' inputs, for tools/diag_unexplained.py
        import os
        import re
        os.makedirs(save, exist_ok=True)
        keep = [ms for ms in misses if any(ms[0] == k and ms[1] == e for k, e, _ in out)]
        fn = os.path.join(save, re.sub(r"[^A-Za-z0-9_.-]+", "_", f"{env_id}_{label}")[:120] + ".npz")
        np.savez(fn, env_id=env_id, variation=str(variation), step=np.array([ms[0] for ms in keep]),
                 env=np.array([ms[1] for ms in keep]), **{k: np.array([np.asarray(ms[i], float) for ms in keep])
                                                          for i, k in enumerate(("params", "qpos", "qvel", "warm",
                                                                                 "act", "gpu_qpos", "gpu_qvel"), 2)})
    if jar_log:
        x = np.concatenate(jar_log)
        print(f"{label} Newton jar agreement over the compared rows: |jar_gpu - jar_oracle| / scale p50 "
              f"{np.median(x):.1e} p99 {np.percentile(x, 99):.1e} max {x.max():.1e} (JAR_REL {JAR_REL:.0e})")
    if misses:
        print(f"{label} miss classes: " + "; ".join(
            f"{k}: {t['n']} (max |dqpos| {t['max_dqpos']:.1e}, |dqvel|/(1+|v|) {t['max_dqvel']:.1e}"
            + (f", max ratio {t['max_ratio']:.2f}" if t['max_ratio'] else "") + ")" for k, t in tally.items()),
            flush=True)
    return out, tally

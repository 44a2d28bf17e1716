"""One saved miss (AW_SAVE_UNEXPLAINED npz): at the GPU's own substep state, the pair's contacts from
the GPU forward, the reference's collider and the GPU's standalone collider (aw_collide_test) on the
GPU's body frames, and under small rotations of the capsule (GPU box only).

    python tools/diag_pose_tie.py FILE.npz SUBSTEP GEOM_A GEOM_B"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]
from parity_classify import _contacts, _quat2mat, context, f32  # noqa: E402

z = np.load(sys.argv[1], allow_pickle=False)
sub, ga, gb_ = int(sys.argv[2]), sys.argv[3], sys.argv[4]
ctx = context(str(z["env_id"]))
P, q, v, w, act = (np.asarray(z[k][0], float) for k in ("params", "qpos", "qvel", "warm", "act"))
q, v, w = ctx.gpu_substeps(P, f32(q), f32(v), f32(w), act, sub) if sub else (f32(q), f32(v), f32(w))
ctrl = ctx.ctrl(act)
d = ctx.gpu_forward(P, q, v, w, ctrl)
orc = ctx.oracle_forward(P, q, v, w, ctrl)
gc, oc = _contacts(ctx, d, orc["contact"].reshape(-1, 23))
names = {ctx.gname(i): i for i in range(len(ctx.gtype))}
a, b = names[ga], names[gb_]
key = (min(a, b), max(a, b))
print("GPU forward:", gc.get(key), "\noracle forward:", oc.get(key))
A = ctx.m.arrays
gbid = np.asarray(A["geom_bodyid"], int)
gp = np.asarray(A["geom_pos"], float).reshape(-1, 3)
gq = np.asarray(A["geom_quat"], float).reshape(-1, 4)
gs = np.asarray(A["geom_size"], float).reshape(-1, 3)
xp, xq = np.asarray(d["xpos"], float).reshape(-1, 3), np.asarray(d["xquat"], float).reshape(-1, 4)
ctx.o.forward1(P, q, v, w, ctrl)
oxp, oxq = ctx.o.get("xpos").reshape(-1, 3), ctx.o.get("xquat").reshape(-1, 4)
for g in key:
    print(f"body of {ctx.gname(g)}: |dxpos| {np.abs(xp[gbid[g]] - oxp[gbid[g]]).max():.2e} |dxquat| {np.abs(xq[gbid[g]] - oxq[gbid[g]]).max():.2e}")
lo, hi = key if ctx.gtype[key[0]] <= ctx.gtype[key[1]] else key[::-1]


def pose(g, frames, rot=None):
    p_, q_ = frames
    R = _quat2mat(q_[gbid[g]])
    if rot is not None:
        R = rot @ R
    return p_[gbid[g]] + R @ gp[g], (R @ _quat2mat(gq[g]))


mg = ctx.margin_of[key][0]
for label, frames in (("GPU frames", (xp, xq)), ("oracle frames", (oxp, oxq))):
    (pa, ma), (pb, mb) = pose(lo, frames), pose(hi, frames)
    ro = ctx.o.collide(ctx.gtype[lo], pa, ma.reshape(9), gs[lo], ctx.gtype[hi], pb, mb.reshape(9), gs[hi], mg)
    rg = ctx.one.collide_test([[ctx.gtype[lo], ctx.gtype[hi]]], [[pa, pb]], [[ma, mb]], [[gs[lo], gs[hi]]], [mg])[0]
    print(label, "oracle collide:", [(round(float(r[0]), 7), np.round(r[1:4], 6).tolist()) for r in ro])
    print(label, "GPU collide_test:", [(round(float(r[0]), 7), np.round(r[1:4], 6).tolist()) for r in rg])
for ang in (1e-7, -1e-7, 1e-6, -1e-6):
    c, s_ = np.cos(ang), np.sin(ang)
    rot = np.array([[1, 0, 0], [0, c, -s_], [0, s_, c]])
    (pa, ma), (pb, mb) = pose(lo, (xp, xq)), pose(hi, (xp, xq))
    if ctx.gtype[hi] == 3:
        pb, mb = pose(hi, (xp, xq), rot)
    else:
        pa, ma = pose(lo, (xp, xq), rot)
    ro = ctx.o.collide(ctx.gtype[lo], pa, ma.reshape(9), gs[lo], ctx.gtype[hi], pb, mb.reshape(9), gs[hi], mg)
    print(f"capsule rotated {ang:+.0e} rad: oracle", [(round(float(r[0]), 7), np.round(r[1:4], 6).tolist()) for r in ro])

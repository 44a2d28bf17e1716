"""Exact-geometry tests of the narrowphase colliders (MuJoCo 2.1 mjc_* constructions restated in
oracle/collide.cc, fp64, and mj_envs_amd/csrc/aw_collide.h, fp32).

Capsule-box (the most frequent hammer pair class): the capsule is its segment
inflated by the radius, so contacts are sphere-box contacts at chosen segment points:
  * lying flat on a face -> two contacts at the ends of the part of the segment over the face
    (clipped to the face), both at the exact depth;
  * crossing an edge, or touching with one end -> one contact.
Box-box: resting face on face -> the corners of the overlap rectangle at the exact depth;
edge across edge -> one contact.  The same cases run through the GPU colliders
(``aw_collide_test``) at fp32 tolerance.
"""
import numpy as np
import pytest

from conftest import make_oracle

CAP, BOX, SPHERE = 3, 6, 2
I3 = np.eye(3)
BOXSZ = np.array([0.2, 0.1, 0.05])
R, H = 0.01, 0.1


def rot_y(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def rot_z(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


# capsule axis = local z: a capsule lying along world x has rotation rot_y(pi/2)
FLAT = rot_y(np.pi / 2)

CASES = {
    # name: (capsule pos, capsule mat, expected contacts [(dist, x, y, z)] sorted by x)
    "flat_inside_face": (np.array([0.0, 0.0, 0.05 + R - 0.002]), FLAT,
                         [(-0.002, -0.1, 0.0, 0.049), (-0.002, 0.1, 0.0, 0.049)]),
    "flat_overhanging": (np.array([0.15, 0.0, 0.05 + R - 0.002]), FLAT,
                         [(-0.002, 0.05, 0.0, 0.049), (-0.002, 0.2, 0.0, 0.049)]),
    "flat_rotated_overhang": (np.array([0.0, 0.08, 0.05 + R - 0.001]), rot_z(np.pi / 2) @ FLAT,
                              [(-0.001, 0.0, -0.02, 0.0495), (-0.001, 0.0, 0.1, 0.0495)]),
    "tilted_one_end": (np.array([0.0, 0.0, 0.05 + R - 0.001]) + H * np.array([np.cos(np.pi / 4), 0,
                                                                              np.sin(np.pi / 4)]),
                       rot_y(np.pi / 4), [(-0.001, 0.0, 0.0, 0.0495)]),
}


def _capsule_box(env_oracle, pos, mat):
    _, o = env_oracle
    return o.collide(CAP, pos, mat, [R, H, 0], BOX, np.zeros(3), I3, BOXSZ, 5e-4)


@pytest.fixture(scope="module")
def orc():
    return make_oracle("hammer-v0")


def _check(out, expect, atol):
    assert len(out) == len(expect), out
    order = np.lexsort((out[:, 2], out[:, 1]))
    for c, (d, x, y, z) in zip(out[order], sorted(expect, key=lambda e: (e[1], e[2]))):
        assert c[0] == pytest.approx(d, abs=atol)
        np.testing.assert_allclose(c[1:4], [x, y, z], atol=atol)


@pytest.mark.parametrize("name", sorted(CASES))
def test_capsule_box_exact_geometry(orc, name):
    pos, mat, expect = CASES[name]
    out = _capsule_box(orc, pos, mat)
    _check(out, expect, 1e-12)
    for c in out:                        # normal from the capsule (geom1) into the box (geom2)
        assert c[6] == pytest.approx(-1.0)


def test_capsule_across_edge_one_contact(orc):
    # tilted 20 deg about y, passing above the x = +0.2 top edge with 0.002 clearance below the
    # radius (penetration 0.002): the closest box feature is the edge -> one contact
    a = np.radians(20)
    u = np.array([np.cos(a), 0, -np.sin(a)])          # axis, descending toward +x
    edge = np.array([0.2, 0.0, 0.05])
    n = np.array([np.sin(a), 0, np.cos(a)])           # perpendicular to the axis, pointing up
    pos = edge + n * (R - 0.002)
    out = _capsule_box(orc, pos, rot_y(np.pi / 2 + a))
    assert len(out) == 1
    assert out[0, 0] == pytest.approx(-0.002, abs=1e-12)
    np.testing.assert_allclose(out[0, 4:7], -n, atol=1e-12)


def test_capsule_box_separated_beyond_margin(orc):
    out = _capsule_box(orc, np.array([0.0, 0.0, 0.05 + R + 0.01]), FLAT)
    assert len(out) == 0


def test_box_box_face_contact_corners(orc):
    _, o = orc
    # a 0.1 cube resting on the box top face, offset so its base overhangs in x: overlap
    # rectangle x in [0.15, 0.2], y in [-0.05, 0.05]; penetration 0.001
    sz = np.array([0.05, 0.05, 0.05])
    pos = np.array([0.2, 0.0, 0.05 + 0.05 - 0.001])
    out = o.collide(BOX, np.zeros(3), I3, BOXSZ, BOX, pos, I3, sz, 5e-4)
    xs = sorted({round(float(x), 9) for x in out[:, 1]})
    ys = sorted({round(float(y), 9) for y in out[:, 2]})
    assert len(out) == 4 and xs == [0.15, 0.2] and ys == [-0.05, 0.05]
    np.testing.assert_allclose(out[:, 0], -0.001, atol=1e-12)


def test_box_box_edge_edge_one_contact(orc):
    _, o = orc
    # a cube rotated 45 deg about x, then 45 deg about z: its lowest feature is an edge, placed
    # 0.001 below the top face just beyond the box's x = +0.2 edge (edge across edge)
    sz = np.array([0.03, 0.03, 0.03])
    Rm = rot_z(np.pi / 4) @ np.array([[1, 0, 0], [0, np.cos(np.pi / 4), -np.sin(np.pi / 4)],
                                      [0, np.sin(np.pi / 4), np.cos(np.pi / 4)]])
    corners = np.array([[sx, sy, sz_] for sx in (-1, 1) for sy in (-1, 1) for sz_ in (-1, 1)]) * sz
    low = (corners @ Rm.T)[:, 2].min()
    pos = np.array([0.2 + 0.005, 0.0, 0.05 - low - 0.001])
    out = o.collide(BOX, np.zeros(3), I3, BOXSZ, BOX, pos, Rm, sz, 5e-4)
    assert 1 <= len(out) <= 2 and np.all(out[:, 0] < 0)


# --------------------------------------------------------------------------------------------
@pytest.mark.gpu
def test_gpu_colliders_match_exact_geometry():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mj_envs_amd import _native
    from mj_envs_amd.tasks import attach_task, load_model
    m = attach_task(load_model("hammer-v0"), "hammer-v0")
    sim = _native.Sim(m.to_blob(), 1)
    names = sorted(CASES)
    types = [[CAP, BOX]] * len(names)
    pos = [[CASES[k][0], np.zeros(3)] for k in names]
    mat = [[CASES[k][1].ravel(), I3.ravel()] for k in names]
    size = [[[R, H, 0], BOXSZ] for _ in names]
    res = sim.collide_test(types, pos, mat, size, [5e-4] * len(names))
    for k, out in zip(names, res):
        _check(out, CASES[k][2], 2e-6)
    # and every case against the oracle, contact by contact in emission order
    _, o = make_oracle("hammer-v0")
    for k, out in zip(names, res):
        ref = o.collide(CAP, CASES[k][0], CASES[k][1], [R, H, 0], BOX, np.zeros(3), I3, BOXSZ, 5e-4)
        np.testing.assert_allclose(out, ref, atol=2e-6)


CYL = 5
MPR_CASES = {
    # name: (type a, pos a, mat a, size a, type b, pos b, mat b, size b) with a.type <= b.type
    "cylinder_tilted_on_box": (CYL, np.array([0.03, -0.02, 0.05 + 0.02 - 0.003]), rot_y(0.4) @ rot_z(0.3),
                               [0.02, 0.04, 0], BOX, np.zeros(3), I3, BOXSZ),
    "cylinder_edge_into_box": (CYL, np.array([0.19, 0.0, 0.05 + 0.015]), rot_y(1.1), [0.015, 0.03, 0],
                               BOX, np.zeros(3), I3, BOXSZ),
    "capsule_end_on_cylinder": (CAP, np.array([-0.03, 0.0, 0.0603702]), rot_y(np.pi / 2 + 0.25), [0.01, 0.05, 0],
                                CYL, np.zeros(3), rot_z(0.1), [0.02, 0.04, 0]),
    "sphere_on_cylinder_rim": (SPHERE, np.array([0.018, 0.0, 0.04 + 0.009]), I3, [0.01, 0, 0],
                               CYL, np.zeros(3), I3, [0.02, 0.04, 0]),
    # line contacts: MPR's point is ill-conditioned along the line (any point of the overlap is a
    # valid contact point; 1e-7 rad of rotation moves it to the other end)
    "cylinder_lying_on_box": (CYL, np.array([0.05, 0.01, 0.05 + 0.02 - 0.002]), rot_y(np.pi / 2), [0.02, 0.04, 0],
                              BOX, np.zeros(3), I3, BOXSZ),
    "hammer_head_on_table": (CYL, np.array([-0.02, 0.03, 0.05 + 0.0245 - 0.0015]), rot_z(0.7) @ rot_y(np.pi / 2),
                             [0.0245, 0.04, 0], BOX, np.zeros(3), I3, BOXSZ),
    "capsule_across_cylinder_face": (CAP, np.array([0.0, 0.005, 0.04 + 0.01 - 0.001]), rot_y(np.pi / 2),
                                     [0.01, 0.03, 0], CYL, np.zeros(3), I3, [0.02, 0.04, 0]),
}


@pytest.mark.gpu
def test_gpu_mpr_pairs_match_oracle():
    """MPR (cylinder) pairs through the GPU narrowphase hook against the oracle's fp64 MPR, on
    identical inputs (poses and margin rounded to fp32 first: the kernel's inputs), contact by
    contact in emission order, on the kernel's fp64 results before their fp32 rounding.  The
    kernel's MPR follows libccd's operation order as the oracle states it (no contraction, 1 / sqrt
    normalisation, aw_collide.h namespace mpr), so depth, normal AND point agree to 1e-12 -- also on
    the line contacts (a cylinder lying on a box, the hammer head on the table, DAPG_hammer.xml:102;
    a capsule across a cylinder's face), where the point is ill-conditioned along the line and any
    difference in rounding moves it (round 4: 2e-3 apart with a different operation order)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mj_envs_amd import _native
    from mj_envs_amd.tasks import attach_task, load_model
    m = attach_task(load_model("hammer-v0"), "hammer-v0")
    sim = _native.Sim(m.to_blob(), 1)
    names = sorted(MPR_CASES)
    f32 = lambda x: np.asarray(x, np.float32).astype(np.float64)
    cases = [[f32(v) if not isinstance(v, int) else v for v in MPR_CASES[k]] for k in names]
    types = [[c[0], c[4]] for c in cases]
    pos = [[c[1], c[5]] for c in cases]
    mat = [[c[2].ravel(), c[6].ravel()] for c in cases]
    size = [[c[3], c[7]] for c in cases]
    margin = float(np.float32(5e-4))
    res = sim.collide_test(types, pos, mat, size, [margin] * len(names), fp64=True)
    res32 = sim.collide_test(types, pos, mat, size, [margin] * len(names))
    _, o = make_oracle("hammer-v0")
    for k, c, out, out32 in zip(names, cases, res, res32):
        ref = o.collide(c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], margin)
        assert len(ref) >= 1, k                     # every case is a penetrating contact
        assert out.shape == ref.shape, (k, out, ref)
        err = np.abs(out - ref).max()
        print(f"{k}: {len(ref)} contact(s), max |GPU fp64 - oracle| = {err:.2e}")
        np.testing.assert_allclose(out, ref, rtol=0, atol=1e-12, err_msg=k)   # depth, point, normal
        np.testing.assert_allclose(out32, ref, rtol=0, atol=1e-7, err_msg=k)  # the fp32 contact the solver gets


def _rot_x(a):
    c, s = np.cos(a), np.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


# box-box through the GPU (fp32 SAT + face clipping, aw_collide.h c_box_box) vs the oracle's fp64
# statement of the same construction: face on face (overlap corners), the Adroit palm box
# (C_palm0, DAPG_Adroit.xml:11, half-sizes 0.032 0.0111 0.049) resting tilted on the table
# (DAPG_relocate.xml:32), an edge across an edge, a corner into a face.
BOXBOX_CASES = {
    "face_on_face_overhang": (np.zeros(3), I3, BOXSZ, np.array([0.2, 0.0, 0.05 + 0.05 - 0.001]), I3,
                              np.array([0.05, 0.05, 0.05])),
    "palm_tilted_on_table": (np.zeros(3), I3, np.array([0.6, 0.6, 0.025]), None,
                             rot_z(0.3) @ _rot_x(np.pi / 2 + 0.05), np.array([0.032, 0.0111, 0.049])),
    "edge_across_edge": (np.zeros(3), I3, BOXSZ, None, rot_z(np.pi / 4) @ _rot_x(np.pi / 4),
                         np.array([0.03, 0.03, 0.03])),
    "corner_into_face": (np.zeros(3), I3, BOXSZ, None, rot_z(0.4) @ _rot_x(0.6) @ rot_y(0.5),
                         np.array([0.02, 0.03, 0.025])),
}


def _boxbox_case(name):
    p1, m1, s1, p2, m2, s2 = BOXBOX_CASES[name]
    if p2 is None:                       # place the second box's lowest feature 0.001 below the top face
        corners = np.array([[a, b, c] for a in (-1, 1) for b in (-1, 1) for c in (-1, 1)]) * s2
        low = (corners @ m2.T)[:, 2].min()
        x = 0.205 if name == "edge_across_edge" else 0.05
        p2 = np.array([x, 0.01, s1[2] - low - 0.001])
    return p1, m1, s1, p2, m2, s2


@pytest.mark.gpu
def test_gpu_boxbox_match_oracle():
    """Box-box contacts of the GPU collider against the oracle, contact by contact in emission
    order, on identical fp32-rounded inputs: depth, point and normal to 2e-6 (fp32 geometry)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mj_envs_amd import _native
    from mj_envs_amd.tasks import attach_task, load_model
    m = attach_task(load_model("relocate-v0"), "relocate-v0")
    sim = _native.Sim(m.to_blob(), 1)
    names = sorted(BOXBOX_CASES)
    f32 = lambda x: np.asarray(x, np.float32).astype(np.float64)
    cases = [[f32(v) for v in _boxbox_case(k)] for k in names]
    margin = float(np.float32(5e-4))
    res = sim.collide_test([[BOX, BOX]] * len(names), [[c[0], c[3]] for c in cases],
                           [[c[1].ravel(), c[4].ravel()] for c in cases], [[c[2], c[5]] for c in cases],
                           [margin] * len(names))
    _, o = make_oracle("relocate-v0")
    for k, c, out in zip(names, cases, res):
        ref = o.collide(BOX, c[0], c[1], c[2], BOX, c[3], c[4], c[5], margin)
        print(f"{k}: {len(ref)} contact(s) oracle, {len(out)} GPU")
        assert len(ref) >= 1, k
        assert out.shape == ref.shape, (k, out, ref)
        np.testing.assert_allclose(out, ref, rtol=0, atol=2e-6, err_msg=k)


def test_boxbox_cases_have_contacts(orc):
    """the box-box GPU cases are penetrating contacts of the intended kind (oracle)"""
    _, o = orc
    f32 = lambda x: np.asarray(x, np.float32).astype(np.float64)
    for k in BOXBOX_CASES:
        c = [f32(v) for v in _boxbox_case(k)]
        out = o.collide(BOX, c[0], c[1], c[2], BOX, c[3], c[4], c[5], float(np.float32(5e-4)))
        assert len(out) >= 1 and (out[:, 0] < 0).all(), (k, out)
        if k == "face_on_face_overhang":
            assert len(out) == 4

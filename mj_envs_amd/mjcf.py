"""Host-side MJCF compiler: parses the Adroit MJCF once and emits a flat model table.

This restates the subset of the MuJoCo 2.1 compiler (``mjCModel::Compile``) that the four
Adroit ``hand_manipulation_suite`` models exercise:

* ``<include>`` expansion (text-level, as MuJoCo does), ``<default>`` classes with
  inheritance, ``childclass``; all ``<default>`` sections are read before ``<worldbody>``
  (MuJoCo's fixed section order), a nested class copies its parent at creation time.
* bodies / joints (hinge, slide) / geoms (plane, sphere, capsule, cylinder, box, mesh as
  visual-only) / sites / fixed tendons / ``general`` actuators with joint transmission /
  sensors / explicit contact ``<pair>`` and ``<exclude>``.
* inertia from geoms for bodies without ``<inertial>`` (``inertiafromgeom="auto"``).
* ``mj_setConst`` equivalents at ``qpos0``: ``body/dof/tendon_invweight0`` and
  ``stat.meaninertia`` (used for constraint regularisation and solver scaling).
* the static collision candidate list: every geom pair that survives contype/conaffinity,
  same-weld-body, parent-child and ``<exclude>`` filtering (broadphase-independent), followed
  by the explicit ``<pair>`` list with its own parameters.

Reference inputs: ``mj_envs_vision/hand_manipulation_suite/assets/DAPG_*.xml``
(``DAPG_assets.xml:3`` options, ``:12-13`` joint/geom defaults, ``:71-91`` pairs,
``:95-240`` tendons, ``:242-267`` actuators, ``:269-342`` sensors).

The result is a :class:`Model` holding numpy arrays keyed by MuJoCo field names
(``body_pos``, ``jnt_range`` ...).  ``Model.to_blob()`` serialises it into the flat
little-endian table consumed by the C-ABI (``include/adroit_wave.h``).
"""
from __future__ import annotations

import copy
import os
import struct
import xml.etree.ElementTree as ET
from typing import Dict, List, Optional

import numpy as np

# ---------------------------------------------------------------------------------------
# enums (values follow mjtGeom / mjtJoint / mjtSensor numbering of MuJoCo 2.1)
GEOM_PLANE, GEOM_HFIELD, GEOM_SPHERE, GEOM_CAPSULE, GEOM_ELLIPSOID, GEOM_CYLINDER, GEOM_BOX, GEOM_MESH = range(8)
GEOM_TYPES = {"plane": 0, "hfield": 1, "sphere": 2, "capsule": 3, "ellipsoid": 4,
              "cylinder": 5, "box": 6, "mesh": 7}
JNT_FREE, JNT_BALL, JNT_SLIDE, JNT_HINGE = range(4)
JNT_TYPES = {"free": 0, "ball": 1, "slide": 2, "hinge": 3}
SENS_TOUCH, SENS_JOINTPOS, SENS_ACTUATORFRC = 0, 1, 2
SENS_TYPES = {"touch": 0, "jointpos": 1, "actuatorfrc": 2}

MJ_MINVAL = 1e-15
DEFAULT_SOLREF = [0.02, 1.0]
DEFAULT_SOLIMP = [0.9, 0.95, 0.001, 0.5, 2.0]

BLOB_MAGIC = b"AWMB"
BLOB_VERSION = 1


# ---------------------------------------------------------------------------------------
# small fp64 rotation helpers (MuJoCo conventions: quaternions are (w, x, y, z))
def quat_mul(a, b):
    return np.array([
        a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3],
        a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2],
        a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1],
        a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0]])


def quat2mat(q):
    w, x, y, z = q
    return np.array([
        [1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
        [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
        [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])


def axisangle2quat(axis, angle):
    axis = np.asarray(axis, float)
    axis = axis / np.linalg.norm(axis)
    s = np.sin(angle / 2)
    return np.array([np.cos(angle / 2), s * axis[0], s * axis[1], s * axis[2]])


def mat2quat(R):
    """Rotation matrix -> unit quaternion with w >= 0 (Shepperd)."""
    t = np.trace(R)
    if t > 0:
        s = np.sqrt(t + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = np.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = np.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = np.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    q = np.array(q)
    q /= np.linalg.norm(q)
    return q if q[0] >= 0 else -q


def euler2quat_mj(euler, seq="xyz"):
    """MuJoCo compiler euler -> quat; lowercase = intrinsic (post-multiply) rotations."""
    q = np.array([1.0, 0, 0, 0])
    for ang, ax in zip(euler, seq):
        axis = {"x": [1, 0, 0], "y": [0, 1, 0], "z": [0, 0, 1]}[ax.lower()]
        r = axisangle2quat(axis, ang)
        q = quat_mul(q, r) if ax.islower() else quat_mul(r, q)
    return q / np.linalg.norm(q)


def _floats(s):
    return [float(v) for v in s.split()]


# ---------------------------------------------------------------------------------------
# XML loading with include expansion
def _load_xml(path: str) -> ET.Element:
    root = ET.parse(path).getroot()
    _expand_includes(root, os.path.dirname(os.path.abspath(path)))
    return root


def _expand_includes(elem: ET.Element, base: str):
    i = 0
    while i < len(elem):
        child = elem[i]
        if child.tag == "include":
            inc = ET.parse(os.path.join(base, child.get("file"))).getroot()
            _expand_includes(inc, base)
            elem.remove(child)
            for j, sub in enumerate(list(inc)):
                elem.insert(i + j, sub)
            i += len(inc)
        else:
            _expand_includes(child, base)
            i += 1


# ---------------------------------------------------------------------------------------
# defaults
_BUILTIN = {
    "joint": dict(type="hinge", pos="0 0 0", axis="0 0 1", limited="false", range="0 0",
                  stiffness="0", damping="0", armature="0", frictionloss="0", margin="0", ref="0",
                  solreflimit="0.02 1", solimplimit="0.9 0.95 0.001 0.5 2",
                  solreffriction="0.02 1", solimpfriction="0.9 0.95 0.001 0.5 2"),
    "geom": dict(type="sphere", size="0 0 0", pos="0 0 0", contype="1", conaffinity="1",
                 condim="3", group="0", priority="0", friction="1 0.005 0.0001", solmix="1",
                 solref="0.02 1", solimp="0.9 0.95 0.001 0.5 2", margin="0", gap="0",
                 density="1000"),
    "site": dict(type="sphere", size="0.005 0.005 0.005", pos="0 0 0", group="0"),
    "tendon": dict(limited="false", range="0 0", margin="0", solreflimit="0.02 1",
                   solimplimit="0.9 0.95 0.001 0.5 2", frictionloss="0", stiffness="0",
                   damping="0", solreffriction="0.02 1", solimpfriction="0.9 0.95 0.001 0.5 2"),
    "general": dict(ctrllimited="false", ctrlrange="0 0", forcelimited="false",
                    forcerange="0 0", gear="1 0 0 0 0 0", gaintype="fixed", gainprm="1 0 0",
                    biastype="none", biasprm="0 0 0", dyntype="none"),
    "mesh": dict(), "inertial": dict(), "pair": dict(),
}


class _Defaults:
    def __init__(self):
        self.classes: Dict[str, Dict[str, Dict[str, str]]] = {"main": copy.deepcopy(_BUILTIN)}

    def read(self, elem: ET.Element, parent: Optional[str]):
        if parent is None:
            name = "main"
        else:
            name = elem.get("class")
            self.classes[name] = copy.deepcopy(self.classes[parent])
        cls = self.classes[name]
        for child in elem:
            if child.tag == "default":
                continue
            cls.setdefault(child.tag, {}).update(child.attrib)
        for child in elem:
            if child.tag == "default":
                self.read(child, name)

    def attrs(self, tag: str, elem: ET.Element, cls: str) -> Dict[str, str]:
        key = "general" if tag in ("general", "motor", "position") else tag
        out = dict(self.classes[cls].get(key, {}))
        out.update(elem.attrib)
        return out


# ---------------------------------------------------------------------------------------
class Model:
    """Flat compiled model: MuJoCo field name -> numpy array, plus name tables."""

    def __init__(self):
        self.arrays: Dict[str, np.ndarray] = {}
        self.names: Dict[str, List[str]] = {}
        self.dims: Dict[str, int] = {}
        self.opt: Dict[str, float] = {}

    def __getattr__(self, key):
        d = self.__dict__
        if "arrays" in d and key in d["arrays"]:
            return d["arrays"][key]
        if "dims" in d and key in d["dims"]:
            return d["dims"][key]
        raise AttributeError(key)

    def name2id(self, kind: str, name: str) -> int:
        return self.names[kind].index(name)

    # --- serialisation -------------------------------------------------------------
    def to_blob(self) -> bytes:
        """Self-describing table: header, then (name[32], kind, rows, cols, data)."""
        entries = []
        for k, v in sorted(self.dims.items()):
            entries.append(("dim_" + k, np.array([[v]], dtype=np.int32)))
        for k, v in sorted(self.opt.items()):
            entries.append(("opt_" + k, np.array([[v]], dtype=np.float64)))
        for k, v in sorted(self.arrays.items()):
            a = np.asarray(v)
            a = a.reshape(a.shape[0], -1) if a.ndim >= 1 and a.size else a.reshape(0, 1)
            if a.dtype.kind in "iub":
                a = a.astype(np.int32)
            else:
                a = a.astype(np.float64)
            entries.append((k, a))
        out = [BLOB_MAGIC, struct.pack("<ii", BLOB_VERSION, len(entries))]
        for name, a in entries:
            nb = name.encode()
            assert len(nb) < 32, name
            kind = 1 if a.dtype == np.int32 else 0
            rows, cols = (a.shape[0], a.shape[1]) if a.ndim == 2 else (a.shape[0], 1)
            out.append(nb.ljust(32, b"\0"))
            out.append(struct.pack("<iii", kind, rows, cols))
            out.append(np.ascontiguousarray(a).tobytes())
        return b"".join(out)

    def save_npz(self, path: str):
        payload = {"a_" + k: v for k, v in self.arrays.items()}
        payload.update({"d_" + k: np.array(v) for k, v in self.dims.items()})
        payload.update({"o_" + k: np.array(v) for k, v in self.opt.items()})
        payload.update({"n_" + k: np.array(v, dtype="U64") for k, v in self.names.items()})
        np.savez_compressed(path, **payload)

    @classmethod
    def load_npz(cls, path: str) -> "Model":
        m = cls()
        with np.load(path, allow_pickle=False) as z:
            for k in z.files:
                v = z[k]
                if k.startswith("a_"):
                    m.arrays[k[2:]] = v
                elif k.startswith("d_"):
                    m.dims[k[2:]] = int(v)
                elif k.startswith("o_"):
                    m.opt[k[2:]] = float(v)
                elif k.startswith("n_"):
                    m.names[k[2:]] = [str(s) for s in v]
        return m


# ---------------------------------------------------------------------------------------
class _Compiler:
    def __init__(self, path: str):
        self.root = _load_xml(path)
        self.defaults = _Defaults()
        for elem in self.root.findall("default"):
            self.defaults.read(elem, None)
        self.opt = dict(timestep=0.002, gravity=[0, 0, -9.81], iterations=100,
                        tolerance=1e-8, noslip_iterations=0, noslip_tolerance=1e-6,
                        impratio=1.0, mpr_tolerance=1e-6, mpr_iterations=50)
        for o in self.root.findall("option"):
            for k, v in o.attrib.items():
                if k in ("iterations", "noslip_iterations", "mpr_iterations"):
                    self.opt[k] = int(v)
                elif k in ("timestep", "tolerance", "noslip_tolerance", "impratio", "mpr_tolerance"):
                    self.opt[k] = float(v)
                elif k == "gravity":
                    self.opt[k] = _floats(v)
        self.eulerseq = "xyz"
        for c in self.root.findall("compiler"):
            if c.get("angle", "radian") != "radian":
                raise NotImplementedError("only angle='radian' is used by the Adroit models")
            self.eulerseq = c.get("eulerseq", self.eulerseq)

        self.bodies, self.joints, self.geoms, self.sites = [], [], [], []
        world = dict(name="world", parent=-1, pos=np.zeros(3), quat=np.array([1.0, 0, 0, 0]),
                     mass=0.0, ipos=np.zeros(3), iquat=np.array([1.0, 0, 0, 0]),
                     inertia=np.zeros(3), mocap=False, joints=[], geoms=[], sites=[], cameras=[],
                     has_inertial=True, cls="main")
        self.bodies.append(world)
        wb = self.root.find("worldbody")
        self._read_body_contents(wb, 0, "main")
        self._finalise_bodies()

    # --- orientation ----------------------------------------------------------------
    def _orient(self, a: Dict[str, str]):
        if "quat" in a:
            q = np.array(_floats(a["quat"]))
            return q / np.linalg.norm(q)
        if "euler" in a:
            return euler2quat_mj(_floats(a["euler"]), self.eulerseq)
        if "axisangle" in a:
            v = _floats(a["axisangle"])
            return axisangle2quat(v[:3], v[3])
        return np.array([1.0, 0, 0, 0])

    # --- tree walk ------------------------------------------------------------------
    def _read_body_contents(self, elem: ET.Element, bid: int, childclass: str):
        body = self.bodies[bid]
        # MuJoCo orders a body's joints/geoms/sites by document order within the body,
        # and numbers all objects body by body (world first), children after.
        children = []
        for child in elem:
            tag = child.tag
            cls = child.get("class", childclass)
            if tag == "inertial":
                a = child.attrib
                body["mass"] = float(a["mass"])
                body["ipos"] = np.array(_floats(a.get("pos", "0 0 0")))
                body["iquat"] = self._orient(a)
                if "diaginertia" in a:
                    body["inertia"] = np.array(_floats(a["diaginertia"]))
                else:
                    raise NotImplementedError("fullinertia not used by the Adroit models")
                body["has_inertial"] = True
            elif tag == "joint":
                a = self.defaults.attrs("joint", child, cls)
                body["joints"].append(a)
            elif tag == "geom":
                a = self.defaults.attrs("geom", child, cls)
                body["geoms"].append(a)
            elif tag == "site":
                a = self.defaults.attrs("site", child, cls)
                body["sites"].append(a)
            elif tag == "camera":
                # position only: the render camera needs cam_xpos (headless_observer.py:59-66)
                body["cameras"].append(np.array(_floats(child.get("pos", "0 0 0"))))
            elif tag == "body":
                children.append(child)
        for child in children:
            a = child.attrib
            nb = dict(name=a.get("name", ""), parent=bid,
                      pos=np.array(_floats(a.get("pos", "0 0 0"))), quat=self._orient(a),
                      mass=0.0, ipos=np.zeros(3), iquat=np.array([1.0, 0, 0, 0]),
                      inertia=np.zeros(3), mocap=a.get("mocap", "false") == "true",
                      joints=[], geoms=[], sites=[], cameras=[], has_inertial=False,
                      cls=a.get("childclass", childclass))
            self.bodies.append(nb)
            self._read_body_contents(child, len(self.bodies) - 1, nb["cls"])

    def _finalise_bodies(self):
        # inertia from geoms for bodies without <inertial>
        for b in self.bodies[1:]:
            if not b["has_inertial"]:
                self._inertia_from_geoms(b)

    @staticmethod
    def _geom_mass_inertia(a):
        t = GEOM_TYPES[a.get("type", "sphere")]
        s = _floats(a["size"]) + [0, 0, 0]
        rho = float(a.get("density", "1000"))
        if t == GEOM_SPHERE:
            vol = 4 / 3 * np.pi * s[0] ** 3
            m = rho * vol
            I = np.full(3, 0.4 * m * s[0] ** 2)
        elif t == GEOM_CAPSULE:
            r, hl = s[0], s[1]
            h = 2 * hl
            ms = rho * 4 / 3 * np.pi * r ** 3
            mc = rho * np.pi * r * r * h
            m = ms + mc
            ixx = mc * (r * r / 4 + h * h / 12) + ms * (2 * r * r / 5 + h * h / 4 + 3 * h * r / 8)
            I = np.array([ixx, ixx, mc * r * r / 2 + ms * 2 * r * r / 5])
        elif t == GEOM_CYLINDER:
            r, hl = s[0], s[1]
            m = rho * np.pi * r * r * 2 * hl
            ixx = m * (3 * r * r + 4 * hl * hl) / 12
            I = np.array([ixx, ixx, m * r * r / 2])
        elif t == GEOM_BOX:
            m = rho * 8 * s[0] * s[1] * s[2]
            I = np.array([m / 3 * (s[1] ** 2 + s[2] ** 2), m / 3 * (s[0] ** 2 + s[2] ** 2),
                          m / 3 * (s[0] ** 2 + s[1] ** 2)])
        else:
            return 0.0, np.zeros(3)
        if "mass" in a:
            scale = float(a["mass"]) / m if m > 0 else 0
            m, I = m * scale, I * scale
        return m, I

    def _inertia_from_geoms(self, b):
        ms, coms, Is = [], [], []
        for a in b["geoms"]:
            m, I = self._geom_mass_inertia(a)
            if m <= 0:
                continue
            R = quat2mat(self._orient(a))
            ms.append(m)
            coms.append(np.array(_floats(a.get("pos", "0 0 0"))))
            Is.append(R @ np.diag(I) @ R.T)
        if not ms:
            return
        M = sum(ms)
        com = sum(m * c for m, c in zip(ms, coms)) / M
        J = np.zeros((3, 3))
        for m, c, I in zip(ms, coms, Is):
            d = c - com
            J += I + m * (np.dot(d, d) * np.eye(3) - np.outer(d, d))
        w, V = np.linalg.eigh(J)
        order = np.argsort(-w)          # descending, like mju_eig3
        w, V = w[order], V[:, order]
        if np.linalg.det(V) < 0:
            V[:, 2] = -V[:, 2]
        b["mass"], b["ipos"], b["inertia"], b["iquat"] = M, com, w, mat2quat(V)

    # --- compile ----------------------------------------------------------------------
    def compile(self) -> Model:
        m = Model()
        B = self.bodies
        nbody = len(B)
        body_parentid = np.array([b["parent"] for b in B], dtype=np.int32)
        # joints / dofs / geoms / sites (numbered body by body)
        jnt, geoms, sites = [], [], []
        body_jntadr, body_jntnum, body_geomadr, body_geomnum = [], [], [], []
        for bi, b in enumerate(B):
            body_jntadr.append(len(jnt) if b["joints"] else -1)
            body_jntnum.append(len(b["joints"]))
            for a in b["joints"]:
                jnt.append((bi, a))
            body_geomadr.append(len(geoms) if b["geoms"] else -1)
            body_geomnum.append(len(b["geoms"]))
            for a in b["geoms"]:
                geoms.append((bi, a))
            for a in b["sites"]:
                sites.append((bi, a))
        njnt, ngeom, nsite = len(jnt), len(geoms), len(sites)

        weldid = np.zeros(nbody, np.int32)
        rootid = np.zeros(nbody, np.int32)
        for bi in range(1, nbody):
            p = body_parentid[bi]
            weldid[bi] = bi if (body_jntnum[bi] > 0) else weldid[p]
            rootid[bi] = bi if p == 0 else rootid[p]
        # mocap bodies are static children of the world
        for bi, b in enumerate(B):
            if b["mocap"]:
                assert body_jntnum[bi] == 0 and body_parentid[bi] == 0
                weldid[bi] = 0

        jnt_type = np.array([JNT_TYPES[a.get("type", "hinge")] for _, a in jnt], np.int32)
        assert np.all((jnt_type == JNT_HINGE) | (jnt_type == JNT_SLIDE)), "Adroit uses hinge/slide only"
        nv = nq = njnt
        jnt_bodyid = np.array([bi for bi, _ in jnt], np.int32)
        jnt_qposadr = np.arange(njnt, dtype=np.int32)
        jnt_dofadr = np.arange(njnt, dtype=np.int32)
        jnt_pos = np.array([_floats(a["pos"]) for _, a in jnt]).reshape(njnt, 3)
        jnt_axis = np.array([_floats(a["axis"]) for _, a in jnt]).reshape(njnt, 3)
        jnt_axis = jnt_axis / np.linalg.norm(jnt_axis, axis=1, keepdims=True)
        jnt_limited = np.array([a["limited"] == "true" for _, a in jnt], np.int32)
        jnt_range = np.array([_floats(a["range"]) for _, a in jnt]).reshape(njnt, 2)
        jnt_margin = np.array([float(a["margin"]) for _, a in jnt])
        jnt_solref = np.array([_floats(a["solreflimit"]) for _, a in jnt]).reshape(njnt, 2)
        jnt_solimp = np.array([_floats(a["solimplimit"]) for _, a in jnt]).reshape(njnt, 5)
        jnt_stiffness = np.array([float(a["stiffness"]) for _, a in jnt])
        assert not np.any(jnt_stiffness), "joint springs not used by the Adroit models"
        jnt_names = [a.get("name", "") for _, a in jnt]

        dof_bodyid = jnt_bodyid.copy()
        dof_jntid = np.arange(nv, dtype=np.int32)
        dof_parentid = np.full(nv, -1, np.int32)
        body_dofadr = np.array(body_jntadr, np.int32)
        body_dofnum = np.array(body_jntnum, np.int32)
        last_dof = np.full(nbody, -1, np.int32)    # last dof on path root..body
        for bi in range(1, nbody):
            prev = last_dof[body_parentid[bi]]
            for k in range(body_dofnum[bi]):
                j = body_dofadr[bi] + k
                dof_parentid[j] = prev
                prev = j
            last_dof[bi] = prev
        dof_armature = np.array([float(a["armature"]) for _, a in jnt])
        dof_damping = np.array([float(a["damping"]) for _, a in jnt])
        dof_frictionloss = np.array([float(a["frictionloss"]) for _, a in jnt])
        dof_solref = np.array([_floats(a["solreffriction"]) for _, a in jnt]).reshape(nv, 2)
        dof_solimp = np.array([_floats(a["solimpfriction"]) for _, a in jnt]).reshape(nv, 5)

        # geoms
        geom_type = np.array([GEOM_TYPES[a.get("type", "sphere")] for _, a in geoms], np.int32)
        geom_bodyid = np.array([bi for bi, _ in geoms], np.int32)
        geom_size = np.zeros((ngeom, 3))
        for i, (_, a) in enumerate(geoms):
            s = _floats(a["size"])
            geom_size[i, :len(s)] = s[:3]
        geom_pos = np.array([_floats(a["pos"]) for _, a in geoms]).reshape(ngeom, 3)
        geom_quat = np.array([self._orient(a) for _, a in geoms]).reshape(ngeom, 4)
        geom_contype = np.array([int(a["contype"]) for _, a in geoms], np.int32)
        geom_conaffinity = np.array([int(a["conaffinity"]) for _, a in geoms], np.int32)
        # mesh geoms are visual-only (meshes are not shipped with the reference)
        for i in range(ngeom):
            if geom_type[i] == GEOM_MESH:
                assert geom_contype[i] == 0 and geom_conaffinity[i] == 0
        geom_condim = np.array([int(a["condim"]) for _, a in geoms], np.int32)
        geom_priority = np.array([int(a["priority"]) for _, a in geoms], np.int32)
        geom_friction = np.array([(_floats(a["friction"]) + [0.005, 0.0001])[:3] for _, a in geoms])
        geom_solmix = np.array([float(a["solmix"]) for _, a in geoms])
        geom_solref = np.array([_floats(a["solref"]) for _, a in geoms]).reshape(ngeom, 2)
        geom_solimp = np.array([_floats(a["solimp"]) for _, a in geoms]).reshape(ngeom, 5)
        geom_margin = np.array([float(a["margin"]) for _, a in geoms])
        geom_gap = np.array([float(a["gap"]) for _, a in geoms])
        geom_rbound = np.zeros(ngeom)
        for i in range(ngeom):
            s, t = geom_size[i], geom_type[i]
            geom_rbound[i] = {GEOM_SPHERE: s[0], GEOM_CAPSULE: s[0] + s[1],
                              GEOM_CYLINDER: np.hypot(s[0], s[1]),
                              GEOM_BOX: np.linalg.norm(s)}.get(t, 0.0)
        geom_names = [a.get("name", "") for _, a in geoms]

        # sites
        site_type = np.array([GEOM_TYPES[a.get("type", "sphere")] for _, a in sites], np.int32)
        site_bodyid = np.array([bi for bi, _ in sites], np.int32)
        site_size = np.zeros((nsite, 3))
        for i, (_, a) in enumerate(sites):
            s = _floats(a["size"])
            site_size[i, :len(s)] = s[:3]
            if len(s) < 3 and site_type[i] == GEOM_SPHERE:
                site_size[i, 1:] = s[0]
        site_pos = np.array([_floats(a["pos"]) for _, a in sites]).reshape(nsite, 3)
        site_quat = np.array([self._orient(a) for _, a in sites]).reshape(nsite, 4)
        site_names = [a.get("name", "") for _, a in sites]

        # tendons (fixed)
        ten_limited, ten_range, ten_margin, ten_solref, ten_solimp, ten_floss = [], [], [], [], [], []
        ten_adr, ten_num, wrap_jnt, wrap_coef, ten_names = [], [], [], [], []
        for tsec in self.root.findall("tendon"):
            for t in tsec:
                if t.tag != "fixed":
                    raise NotImplementedError("only fixed tendons are used by the Adroit models")
                a = self.defaults.attrs("tendon", t, t.get("class", "main"))
                ten_names.append(a.get("name", ""))
                ten_limited.append(a["limited"] == "true")
                ten_range.append(_floats(a["range"]))
                ten_margin.append(float(a["margin"]))
                ten_solref.append(_floats(a["solreflimit"]))
                ten_solimp.append(_floats(a["solimplimit"]))
                ten_floss.append(float(a["frictionloss"]))
                assert float(a["stiffness"]) == 0 and float(a["damping"]) == 0
                ten_adr.append(len(wrap_jnt))
                for w in t.findall("joint"):
                    wrap_jnt.append(jnt_names.index(w.get("joint")))
                    wrap_coef.append(float(w.get("coef")))
                ten_num.append(len(wrap_jnt) - ten_adr[-1])
        ntendon = len(ten_names)
        ten_J0 = np.zeros((ntendon, nv))
        for t in range(ntendon):
            for w in range(ten_adr[t], ten_adr[t] + ten_num[t]):
                ten_J0[t, jnt_dofadr[wrap_jnt[w]]] += wrap_coef[w]

        # actuators (general, joint transmission)
        act_names, act_trnid, act_gain, act_bias, act_ctrlrange, act_ctrllimited = [], [], [], [], [], []
        act_gear, act_forcelimited, act_forcerange = [], [], []
        for asec in self.root.findall("actuator"):
            for t in asec:
                if t.tag != "general":
                    raise NotImplementedError(t.tag)
                a = self.defaults.attrs("general", t, t.get("class", "main"))
                assert a["gaintype"] == "fixed" and a["dyntype"] == "none"
                act_names.append(a.get("name", ""))
                act_trnid.append(jnt_names.index(a["joint"]))
                g = (_floats(a["gainprm"]) + [0] * 3)[:3]
                bp = (_floats(a["biasprm"]) + [0] * 3)[:3] if a["biastype"] == "affine" else [0, 0, 0]
                act_gain.append(g)
                act_bias.append(bp)
                act_ctrlrange.append(_floats(a["ctrlrange"]))
                act_ctrllimited.append(a["ctrllimited"] == "true")
                act_gear.append(_floats(a["gear"])[0])
                act_forcelimited.append(a["forcelimited"] == "true")
                act_forcerange.append(_floats(a["forcerange"]))
        nu = len(act_names)

        # sensors
        sens_type, sens_objid, sens_names, sens_adr = [], [], [], []
        for ssec in self.root.findall("sensor"):
            for s in ssec:
                t = SENS_TYPES[s.tag]
                sens_type.append(t)
                if t == SENS_TOUCH:
                    sens_objid.append(site_names.index(s.get("site")))
                elif t == SENS_JOINTPOS:
                    sens_objid.append(jnt_names.index(s.get("joint")))
                else:
                    sens_objid.append(act_names.index(s.get("actuator")))
                sens_adr.append(len(sens_names))
                sens_names.append(s.get("name", ""))
        nsensor = len(sens_names)

        # explicit pairs and excludes
        pair_g, pair_condim, pair_friction, pair_solref, pair_solimp, pair_margin, pair_gap = [], [], [], [], [], [], []
        excludes = set()
        body_names = [b["name"] for b in B]
        for csec in self.root.findall("contact"):
            for c in csec:
                if c.tag == "pair":
                    a = dict(c.attrib)
                    g1, g2 = geom_names.index(a["geom1"]), geom_names.index(a["geom2"])
                    if geom_bodyid[g1] > geom_bodyid[g2]:
                        g1, g2 = g2, g1
                    # mj_collideGeoms swaps so that geom1 has the lower type
                    if geom_type[g1] > geom_type[g2]:
                        g1, g2 = g2, g1
                    pair_g.append((g1, g2))
                    pair_condim.append(int(a.get("condim", "3")))
                    pair_friction.append(_floats(a.get("friction", "1 1 0.005 0.0001 0.0001")))
                    pair_solref.append(_floats(a.get("solref", "0.02 1")))
                    pair_solimp.append(_floats(a.get("solimp", "0.9 0.95 0.001 0.5 2")))
                    pair_margin.append(float(a.get("margin", "0")))
                    pair_gap.append(float(a.get("gap", "0")))
                elif c.tag == "exclude":
                    b1, b2 = body_names.index(c.get("body1")), body_names.index(c.get("body2"))
                    excludes.add((min(b1, b2), max(b1, b2)))
        npair = len(pair_g)

        # ---- arrays ------------------------------------------------------------------
        A = m.arrays
        A["body_parentid"] = body_parentid
        A["body_rootid"] = rootid
        A["body_weldid"] = weldid
        A["body_jntnum"] = np.array(body_jntnum, np.int32)
        A["body_jntadr"] = np.array(body_jntadr, np.int32)
        A["body_dofnum"] = body_dofnum
        A["body_dofadr"] = body_dofadr
        A["body_geomnum"] = np.array(body_geomnum, np.int32)
        A["body_geomadr"] = np.array(body_geomadr, np.int32)
        A["body_mocap"] = np.array([b["mocap"] for b in B], np.int32)
        A["body_pos"] = np.array([b["pos"] for b in B])
        A["body_quat"] = np.array([b["quat"] for b in B])
        A["body_ipos"] = np.array([b["ipos"] for b in B])
        A["body_iquat"] = np.array([b["iquat"] for b in B])
        A["body_mass"] = np.array([b["mass"] for b in B])
        A["body_inertia"] = np.array([b["inertia"] for b in B])
        A["jnt_type"] = jnt_type
        A["jnt_bodyid"] = jnt_bodyid
        A["jnt_qposadr"] = jnt_qposadr
        A["jnt_dofadr"] = jnt_dofadr
        A["jnt_pos"] = jnt_pos
        A["jnt_axis"] = jnt_axis
        A["jnt_limited"] = jnt_limited
        A["jnt_range"] = jnt_range
        A["jnt_margin"] = jnt_margin
        A["jnt_solref"] = jnt_solref
        A["jnt_solimp"] = jnt_solimp
        A["dof_bodyid"] = dof_bodyid
        A["dof_jntid"] = dof_jntid
        A["dof_parentid"] = dof_parentid
        A["dof_armature"] = dof_armature
        A["dof_damping"] = dof_damping
        A["dof_frictionloss"] = dof_frictionloss
        A["dof_solref"] = dof_solref
        A["dof_solimp"] = dof_solimp
        A["geom_type"] = geom_type
        A["geom_bodyid"] = geom_bodyid
        A["geom_contype"] = geom_contype
        A["geom_conaffinity"] = geom_conaffinity
        A["geom_condim"] = geom_condim
        A["geom_priority"] = geom_priority
        A["geom_size"] = geom_size
        A["geom_pos"] = geom_pos
        A["geom_quat"] = geom_quat
        A["geom_friction"] = geom_friction
        A["geom_solmix"] = geom_solmix
        A["geom_solref"] = geom_solref
        A["geom_solimp"] = geom_solimp
        A["geom_margin"] = geom_margin
        A["geom_gap"] = geom_gap
        A["geom_rbound"] = geom_rbound
        A["site_type"] = site_type
        A["site_bodyid"] = site_bodyid
        A["site_size"] = site_size
        A["site_pos"] = site_pos
        A["site_quat"] = site_quat
        cams = [(bi, c) for bi, b in enumerate(B) for c in b.get("cameras", [])]
        A["cam_bodyid"] = np.array([bi for bi, _ in cams], np.int32)
        A["cam_pos"] = np.array([c for _, c in cams], np.float64).reshape(len(cams), 3)
        A["tendon_adr"] = np.array(ten_adr, np.int32)
        A["tendon_num"] = np.array(ten_num, np.int32)
        A["tendon_limited"] = np.array(ten_limited, np.int32)
        A["tendon_range"] = np.array(ten_range).reshape(ntendon, 2)
        A["tendon_margin"] = np.array(ten_margin)
        A["tendon_solref"] = np.array(ten_solref).reshape(ntendon, 2)
        A["tendon_solimp"] = np.array(ten_solimp).reshape(ntendon, 5)
        A["tendon_frictionloss"] = np.array(ten_floss)
        A["wrap_jnt"] = np.array(wrap_jnt, np.int32)
        A["wrap_coef"] = np.array(wrap_coef)
        A["actuator_trnid"] = np.array(act_trnid, np.int32)
        A["actuator_gear"] = np.array(act_gear)
        A["actuator_gainprm"] = np.array(act_gain).reshape(nu, 3)
        A["actuator_biasprm"] = np.array(act_bias).reshape(nu, 3)
        A["actuator_ctrlrange"] = np.array(act_ctrlrange).reshape(nu, 2)
        A["actuator_ctrllimited"] = np.array(act_ctrllimited, np.int32)
        A["actuator_forcelimited"] = np.array(act_forcelimited, np.int32)
        A["actuator_forcerange"] = np.array(act_forcerange).reshape(nu, 2)
        A["sensor_type"] = np.array(sens_type, np.int32)
        A["sensor_objid"] = np.array(sens_objid, np.int32)
        A["sensor_adr"] = np.array(sens_adr, np.int32)
        A["pair_geom1"] = np.array([p[0] for p in pair_g], np.int32)
        A["pair_geom2"] = np.array([p[1] for p in pair_g], np.int32)
        A["pair_condim"] = np.array(pair_condim, np.int32)
        A["pair_friction"] = np.array(pair_friction).reshape(npair, 5)
        A["pair_solref"] = np.array(pair_solref).reshape(npair, 2)
        A["pair_solimp"] = np.array(pair_solimp).reshape(npair, 5)
        A["pair_margin"] = np.array(pair_margin)
        A["pair_gap"] = np.array(pair_gap)
        A["qpos0"] = np.zeros(nq)

        m.names = dict(body=body_names, joint=jnt_names, geom=geom_names, site=site_names,
                       tendon=ten_names, actuator=act_names, sensor=sens_names)
        m.dims = dict(nq=nq, nv=nv, nu=nu, nbody=nbody, njnt=njnt, ngeom=ngeom, nsite=nsite,
                      ntendon=ntendon, nwrap=len(wrap_jnt), nsensor=nsensor, nsensordata=nsensor,
                      npair=npair, nexclude=len(excludes))
        m.opt = dict(timestep=self.opt["timestep"], gravity_x=self.opt["gravity"][0],
                     gravity_y=self.opt["gravity"][1], gravity_z=self.opt["gravity"][2],
                     iterations=self.opt["iterations"], tolerance=self.opt["tolerance"],
                     noslip_iterations=self.opt["noslip_iterations"],
                     noslip_tolerance=self.opt["noslip_tolerance"], impratio=self.opt["impratio"],
                     mpr_tolerance=self.opt["mpr_tolerance"], mpr_iterations=self.opt["mpr_iterations"])
        A["exclude_body1"] = np.array([e[0] for e in sorted(excludes)], np.int32)
        A["exclude_body2"] = np.array([e[1] for e in sorted(excludes)], np.int32)

        _set_const(m)
        _collision_candidates(m)
        return m


# ---------------------------------------------------------------------------------------
def _kinematics0(m: Model, body_pos=None, body_quat=None):
    """Body poses at qpos0 (all Adroit joints are hinge/slide with qpos0 = 0)."""
    nb = m.nbody
    bp = m.body_pos if body_pos is None else body_pos
    bq = m.body_quat if body_quat is None else body_quat
    xpos = np.zeros((nb, 3))
    xquat = np.zeros((nb, 4))
    xquat[0] = [1, 0, 0, 0]
    for b in range(1, nb):
        p = m.body_parentid[b]
        xpos[b] = xpos[p] + quat2mat(xquat[p]) @ bp[b]
        q = quat_mul(xquat[p], bq[b])
        xquat[b] = q / np.linalg.norm(q)
    xmat = np.array([quat2mat(q) for q in xquat])
    return xpos, xquat, xmat


def _com_and_mass(m: Model):
    """Restates mj_comPos + mj_crb at qpos0; returns cdof, subtree_com, M (nv x nv)."""
    nb, nv = m.nbody, m.nv
    xpos, xquat, xmat = _kinematics0(m)
    xipos = np.array([xpos[b] + xmat[b] @ m.body_ipos[b] for b in range(nb)])
    ximat = np.array([quat2mat(quat_mul(xquat[b], m.body_iquat[b])) for b in range(nb)])
    mass = m.body_mass
    subtree_mass = mass.copy()
    subtree_mc = mass[:, None] * xipos
    for b in range(nb - 1, 0, -1):
        p = m.body_parentid[b]
        subtree_mass[p] += subtree_mass[b]
        subtree_mc[p] += subtree_mc[b]
    subtree_com = np.where(subtree_mass[:, None] > MJ_MINVAL,
                           subtree_mc / np.maximum(subtree_mass, MJ_MINVAL)[:, None], xipos)
    # spatial inertia (6x6, motion=[w;v]) about the root subtree com
    cinert = np.zeros((nb, 6, 6))
    for b in range(1, nb):
        r = xipos[b] - subtree_com[m.body_rootid[b]]
        Ic = ximat[b] @ np.diag(m.body_inertia[b]) @ ximat[b].T
        rx = np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])
        mb = mass[b]
        cinert[b, :3, :3] = Ic - mb * rx @ rx
        cinert[b, :3, 3:] = mb * rx
        cinert[b, 3:, :3] = -mb * rx
        cinert[b, 3:, 3:] = mb * np.eye(3)
    cdof = np.zeros((nv, 6))
    for j in range(nv):
        b = m.dof_bodyid[j]
        R = xmat[b]
        axis = R @ m.jnt_axis[j]
        anchor = xpos[b] + R @ m.jnt_pos[j]
        if m.jnt_type[j] == JNT_HINGE:
            cdof[j, :3] = axis
            cdof[j, 3:] = np.cross(axis, subtree_com[m.body_rootid[b]] - anchor)
        else:
            cdof[j, 3:] = axis
    crb = cinert.copy()
    for b in range(nb - 1, 0, -1):
        crb[m.body_parentid[b]] += crb[b]
    M = np.zeros((nv, nv))
    for i in range(nv):
        f = crb[m.dof_bodyid[i]] @ cdof[i]
        j = i
        while j >= 0:
            M[i, j] = M[j, i] = cdof[j] @ f
            j = m.dof_parentid[j]
    M[np.diag_indices(nv)] += m.dof_armature
    return dict(xpos=xpos, xmat=xmat, xipos=xipos, subtree_com=subtree_com, cdof=cdof, M=M,
                subtree_mass=subtree_mass)


def _body_ancestor_dofs(m: Model, b: int):
    out = []
    while b > 0:
        for k in range(m.body_dofnum[b] - 1, -1, -1):
            out.append(m.body_dofadr[b] + k)
        b = m.body_parentid[b]
    return out


def _set_const(m: Model):
    """mj_setConst restatement: invweight0 and meaninertia at qpos0."""
    k = _com_and_mass(m)
    M, cdof = k["M"], k["cdof"]
    Minv = np.linalg.inv(M)
    m.arrays["dof_invweight0"] = np.diag(Minv).copy()
    m.arrays["tendon_invweight0"] = np.einsum("ti,ij,tj->t", _tendon_J(m), Minv, _tendon_J(m))
    inv0 = np.zeros((m.nbody, 2))
    for b in range(1, m.nbody):
        if m.body_weldid[b] == 0:
            continue
        jac = np.zeros((6, m.nv))
        off = k["xipos"][b] - k["subtree_com"][m.body_rootid[b]]
        for j in _body_ancestor_dofs(m, b):
            jac[:3, j] = cdof[j, 3:] + np.cross(cdof[j, :3], off)
            jac[3:, j] = cdof[j, :3]
        A = jac @ Minv @ jac.T
        inv0[b] = [np.trace(A[:3, :3]) / 3, np.trace(A[3:, 3:]) / 3]
    m.arrays["body_invweight0"] = inv0
    # compile-time subtree mass; mj_comPos divides by it even after runtime mass edits
    m.arrays["body_subtreemass"] = k["subtree_mass"]
    m.opt["meaninertia"] = float(np.trace(M) / m.nv)


def _tendon_J(m: Model):
    J = np.zeros((m.ntendon, m.nv))
    for t in range(m.ntendon):
        for w in range(m.tendon_adr[t], m.tendon_adr[t] + m.tendon_num[t]):
            J[t, m.jnt_dofadr[m.wrap_jnt[w]]] += m.wrap_coef[w]
    return J


def _collision_candidates(m: Model):
    """Static candidate geom-pair list (mj_collision filters), then explicit pairs.

    Filters (MuJoCo 2.1 ``mj_collision``/``filterBodyPair``): contype/conaffinity
    compatibility, same weld body, parent-child weld bodies (world excluded), ``<exclude>``.
    Pairs that are also listed as explicit ``<pair>`` are left to the explicit list.
    """
    ng = m.ngeom
    excl = set(zip(m.exclude_body1.tolist(), m.exclude_body2.tolist()))
    explicit = set(zip(m.pair_geom1.tolist(), m.pair_geom2.tolist()))
    explicit |= {(b, a) for a, b in explicit}
    g1s, g2s = [], []
    wp = lambda w: m.body_weldid[m.body_parentid[w]] if w > 0 else 0
    for a in range(ng):
        for b in range(a + 1, ng):
            ta, tb = m.geom_type[a], m.geom_type[b]
            if ta == GEOM_MESH or tb == GEOM_MESH:
                continue
            if not ((m.geom_contype[a] & m.geom_conaffinity[b]) or (m.geom_contype[b] & m.geom_conaffinity[a])):
                continue
            ba, bb = m.geom_bodyid[a], m.geom_bodyid[b]
            wa, wb = m.body_weldid[ba], m.body_weldid[bb]
            if wa == wb:
                continue
            if wa != 0 and wb != 0 and (wa == wp(wb) or wb == wp(wa)):
                continue
            if (min(ba, bb), max(ba, bb)) in excl:
                continue
            if (a, b) in explicit:
                continue
            # order so that geom1 has the lower type (collision table is upper-triangular)
            if ta > tb:
                a2, b2 = b, a
            else:
                a2, b2 = a, b
            g1s.append(a2)
            g2s.append(b2)
    m.arrays["cand_geom1"] = np.array(g1s, np.int32)
    m.arrays["cand_geom2"] = np.array(g2s, np.int32)
    m.dims["ncand"] = len(g1s)


def compile_mjcf(path: str) -> Model:
    return _Compiler(path).compile()

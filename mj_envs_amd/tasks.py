"""Task specs for the four Adroit envs: ids, horizons, obs layout, per-env model params.

Mirrors the task layer of the reference:
  * registry ids / horizons          ``mj_envs_vision/__init__.py:4-28``
  * hammer  ``hand_manipulation_suite/hammer_v0.py``  (frame_skip 5 ``:20``, reset ``:106-132``)
  * door    ``hand_manipulation_suite/door_v0.py``    (frame_skip 1 ``:10,22``, reset ``:103-119``)
  * pen     ``hand_manipulation_suite/pen_v0.py``     (frame_skip 5 ``:27``, reset ``:115-132``)
  * relocate ``hand_manipulation_suite/relocate_v0.py`` (frame_skip 5 ``:17``, reset ``:85-103``)

Per-env model parameters: the reference mutates the *shared* ``mjModel`` at reset
(``hammer_v0.py:109`` ``body_pos[nail_board, 2]`` ...).  The batched simulator keeps one
model and a small per-env override vector ``params[N, P]``; each entry names the model
field it overrides (``PARAM_FIELDS``) so the kernel applies it when it stages the model.
Derived constants (``invweight0``, ``rbound``, ``subtreemass``) are *not* recomputed,
exactly as MuJoCo does not recompute them after such writes.
"""
from __future__ import annotations

import dataclasses
import os
from typing import Dict, List, Optional, Tuple

import numpy as np

# model field codes understood by the kernel's override stage
PARAM_FIELDS = {"body_pos": 0, "body_quat": 1, "site_pos": 2, "body_mass": 3,
                "geom_pos": 4, "geom_size": 5}

TASK_IDS = {"hammer-v0": 0, "door-v0": 1, "pen-v0": 2, "relocate-v0": 3}


@dataclasses.dataclass
class TaskSpec:
    env_id: str
    kind: int
    xml: str
    frame_skip: int
    horizon: int
    obs_dim: int
    nu: int
    success_steps: int          # evaluate_success: > this many goal steps
    entry_point: str


TASKS: Dict[str, TaskSpec] = {
    "hammer-v0": TaskSpec("hammer-v0", 0, "DAPG_hammer.xml", 5, 200, 46, 26, 25,
                          "mj_envs_amd.envs:HammerEnvV0"),
    "door-v0": TaskSpec("door-v0", 1, "DAPG_door.xml", 1, 200, 39, 28, 25,
                        "mj_envs_amd.envs:DoorEnvV0"),
    "pen-v0": TaskSpec("pen-v0", 2, "DAPG_pen.xml", 5, 100, 45, 24, 20,
                       "mj_envs_amd.envs:PenEnvV0"),
    "relocate-v0": TaskSpec("relocate-v0", 3, "DAPG_relocate.xml", 5, 200, 39, 30, 25,
                            "mj_envs_amd.envs:RelocateEnvV0"),
}

MODEL_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "models")


def load_model(env_id: str):
    """Compiled model for ``env_id`` (committed ``models/*.npz``, built by tools/compile_assets.py)."""
    from .mjcf import Model
    spec = TASKS[env_id]
    path = os.path.join(MODEL_DIR, spec.xml.replace(".xml", ".npz"))
    if not os.path.exists(path):
        raise FileNotFoundError(f"compiled model {path} missing; run tools/compile_assets.py")
    return Model.load_npz(path)


# ---------------------------------------------------------------------------------------
def param_layout(env_id: str, model, variation_type: Optional[str] = None) -> List[Tuple[str, int, int]]:
    """(field, object id, component) for every per-env parameter, in params[] order."""
    n = model.name2id
    if env_id == "hammer-v0":
        # the whole nail-board position: set_env_state writes all of board_pos (hammer_v0.py:152);
        # reset draws only z (:109)
        board = n("body", "nail_board")
        lay = [("body_pos", board, 0), ("body_pos", board, 1), ("body_pos", board, 2)]
        head, neck = n("geom", "head"), n("geom", "neck")
        if variation_type == "mass":
            lay.append(("body_mass", n("body", "Object"), 0))
        elif variation_type == "pos":
            lay += [("geom_pos", head, 0), ("geom_pos", neck, 0)]
        elif variation_type == "size":
            lay += [("geom_size", head, 0), ("geom_size", head, 1)]
        elif variation_type is not None:
            raise Exception(f"Unsupported variation type {variation_type}")
        return lay
    if env_id == "door-v0":
        b = n("body", "frame")
        return [("body_pos", b, 0), ("body_pos", b, 1), ("body_pos", b, 2)]
    if env_id == "pen-v0":
        b = n("body", "target")
        return [("body_quat", b, k) for k in range(4)]
    if env_id == "relocate-v0":
        # object body_pos (all three: set_env_state writes obj_pos, relocate_v0.py:127) and the
        # target site; reset draws object x / y and target x / y / z (:89-93)
        b, s = n("body", "Object"), n("site", "target")
        return [("body_pos", b, 0), ("body_pos", b, 1), ("body_pos", b, 2),
                ("site_pos", s, 0), ("site_pos", s, 1), ("site_pos", s, 2)]
    raise KeyError(env_id)


# source of each param at a reset: the index of a uniform draw (reset_ranges order), or
# PD_DEFAULT (keeps its current value -- the model value for a fresh env: a field reset_model does
# not write keeps what was last written), PD_NECK (hammer 'pos' variation: neck x = -0.14 - (-0.24 - x),
# hammer_v0.py:122), PD_QUAT (pen: euler2quat of draws 0 / 1, pen_v0.py:119-122)
PD_DEFAULT, PD_NECK, PD_QUAT = -1, -2, -3


def param_draws(env_id: str, variation_type: Optional[str] = None) -> List[int]:
    if env_id == "hammer-v0":
        return [PD_DEFAULT, PD_DEFAULT, 0] + {None: [], "mass": [1], "pos": [1, PD_NECK],
                                              "size": [1, 2]}[variation_type]
    if env_id == "door-v0":
        return [0, 1, 2]
    if env_id == "pen-v0":
        return [PD_QUAT] * 4
    if env_id == "relocate-v0":
        return [0, 1, PD_DEFAULT, 2, 3, 4]
    raise KeyError(env_id)


# reset distributions: (low, high) per uniform draw, in draw order (reference np_random order)
def reset_ranges(env_id: str, variation_type: Optional[str] = None) -> List[Tuple[float, float]]:
    if env_id == "hammer-v0":                       # hammer_v0.py:109-125
        r = [(0.1, 0.25)]
        if variation_type == "mass":
            r.append((0.05, 2.5))
        elif variation_type == "pos":
            r.append((-0.24, -0.10))
        elif variation_type == "size":
            r += [(0.01, 0.04), (0.02, 0.08)]
        return r
    if env_id == "door-v0":                         # door_v0.py:107-109
        return [(-0.3, -0.2), (0.25, 0.35), (0.252, 0.35)]
    if env_id == "pen-v0":                          # pen_v0.py:119-122
        return [(-1.0, 1.0), (-1.0, 1.0)]
    if env_id == "relocate-v0":                     # relocate_v0.py:89-93
        return [(-0.15, 0.15), (-0.15, 0.3), (-0.2, 0.2), (-0.2, 0.2), (0.15, 0.35)]
    raise KeyError(env_id)


def euler2quat(euler):
    """``utils/quatmath.py:60-76`` (reference convention, not the MJCF one)."""
    euler = np.asarray(euler, dtype=np.float64)
    ai, aj, ak = euler[..., 2] / 2, -euler[..., 1] / 2, euler[..., 0] / 2
    si, sj, sk = np.sin(ai), np.sin(aj), np.sin(ak)
    ci, cj, ck = np.cos(ai), np.cos(aj), np.cos(ak)
    cc, cs = ci * ck, ci * sk
    sc, ss = si * ck, si * sk
    quat = np.empty(euler.shape[:-1] + (4,), dtype=np.float64)
    quat[..., 0] = cj * cc + sj * ss
    quat[..., 3] = cj * sc - sj * cs
    quat[..., 2] = -(cj * ss + sj * cc)
    quat[..., 1] = cj * cs - sj * sc
    return quat


def draws_to_params(env_id: str, u: np.ndarray, variation_type: Optional[str] = None,
                    defaults: Optional[np.ndarray] = None) -> np.ndarray:
    """Map uniform draws (already scaled to reset_ranges) to the override vector
    (``param_draws``); ``defaults``: the current params (``default_params`` for a fresh env)."""
    u = np.atleast_2d(np.asarray(u, np.float64))
    if env_id == "pen-v0":
        e = np.zeros((u.shape[0], 3))
        e[:, 0], e[:, 1] = u[:, 0], u[:, 1]
        return euler2quat(e)
    codes = param_draws(env_id, variation_type)
    out = np.zeros((u.shape[0], len(codes)))
    for p, c in enumerate(codes):
        if c >= 0:
            out[:, p] = u[:, c]
        elif c == PD_NECK:
            out[:, p] = -0.14 - (-0.24 - u[:, 1])
        else:
            if defaults is None:
                raise ValueError("draws_to_params: defaults needed for params kept at the model value")
            out[:, p] = defaults[p]
    return out


def default_params(env_id: str, model, variation_type: Optional[str] = None) -> np.ndarray:
    """Current model values of the overridden fields (what an un-reset env sees)."""
    out = []
    for field, obj, comp in param_layout(env_id, model, variation_type):
        arr = getattr(model, field)
        out.append(float(arr[obj] if arr.ndim == 1 else arr[obj, comp]))
    return np.array(out)


def sample_params(env_id: str, model, rng: np.random.Generator, n: int,
                  variation_type: Optional[str] = None) -> np.ndarray:
    """Host-side reset sampler (numpy Generator, as the reference's ``np_random``)."""
    ranges = reset_ranges(env_id, variation_type)
    u = np.empty((n, len(ranges)))
    for i in range(n):
        for k, (lo, hi) in enumerate(ranges):
            u[i, k] = rng.uniform(low=lo, high=hi)
    return draws_to_params(env_id, u, variation_type, default_params(env_id, model, variation_type))


# ---------------------------------------------------------------------------------------
def task_indices(env_id: str, model) -> np.ndarray:
    """Object ids the task layer reads (order fixed per task, see adroit_task.h)."""
    n = model.name2id
    if env_id == "hammer-v0":   # hammer_v0.py:44-48, sensor S_nail (:100)
        return np.array([n("site", "S_grasp"), n("body", "Object"), n("site", "tool"),
                         n("site", "S_target"), n("site", "nail_goal"),
                         model.sensor_adr[n("sensor", "S_nail")]], np.int32)
    if env_id == "door-v0":     # door_v0.py:49-52
        return np.array([n("site", "S_grasp"), n("site", "S_handle"),
                         model.jnt_dofadr[n("joint", "door_hinge")], n("body", "frame")], np.int32)
    if env_id == "pen-v0":      # pen_v0.py:48-55
        return np.array([n("site", "S_grasp"), n("body", "Object"), n("site", "eps_ball"),
                         n("site", "object_top"), n("site", "object_bottom"),
                         n("site", "target_top"), n("site", "target_bottom"),
                         n("body", "target")], np.int32)
    if env_id == "relocate-v0":  # relocate_v0.py:36-38
        return np.array([n("site", "S_grasp"), n("body", "Object"), n("site", "target")], np.int32)
    raise KeyError(env_id)


def pen_lengths(model) -> Tuple[float, float]:
    """``pen_v0.py:57-58``: lengths measured from the initial kinematics (rotation-invariant)."""
    n = model.name2id
    a = model.site_pos[n("site", "object_top")] - model.site_pos[n("site", "object_bottom")]
    b = model.site_pos[n("site", "target_top")] - model.site_pos[n("site", "target_bottom")]
    return float(np.linalg.norm(a)), float(np.linalg.norm(b))


def attach_task(model, env_id: str, variation_type: Optional[str] = None):
    """Add the task block (kind, indices, params layout, frame skip ...) to a model copy."""
    import copy
    spec = TASKS[env_id]
    m = copy.copy(model)
    m.arrays = dict(model.arrays)
    m.dims = dict(model.dims)
    m.opt = dict(model.opt)
    lay = param_layout(env_id, model, variation_type)
    m.arrays["task_idx"] = task_indices(env_id, model)
    m.arrays["task_param_field"] = np.array([PARAM_FIELDS[f] for f, _, _ in lay], np.int32)
    m.arrays["task_param_obj"] = np.array([o for _, o, _ in lay], np.int32)
    m.arrays["task_param_comp"] = np.array([c for _, _, c in lay], np.int32)
    m.arrays["task_param_default"] = default_params(env_id, model, variation_type)
    m.arrays["task_param_draw"] = np.array(param_draws(env_id, variation_type), np.int32)
    rr = reset_ranges(env_id, variation_type)
    m.arrays["task_draw_lo"] = np.array([r[0] for r in rr])
    m.arrays["task_draw_hi"] = np.array([r[1] for r in rr])
    var = {None: 0, "mass": 1, "pos": 2, "size": 3}[variation_type]
    m.dims.update(task_kind=spec.kind, task_frame_skip=spec.frame_skip, task_horizon=spec.horizon,
                  task_obs_dim=spec.obs_dim, task_nparam=len(lay), task_variation=var,
                  task_success_steps=spec.success_steps)
    if env_id == "pen-v0":
        pl, tl = pen_lengths(model)
        m.opt.update(task_pen_length=pl, task_tar_length=tl)
    # act_mid / act_rng (hammer_v0.py:49-50)
    cr = model.actuator_ctrlrange
    m.arrays["task_act_mid"] = np.mean(cr, axis=1)
    m.arrays["task_act_rng"] = 0.5 * (cr[:, 1] - cr[:, 0])
    return m


# ---------------------------------------------------------------------------------------
# get_env_state / set_env_state dicts <-> per-env params (hammer_v0.py:134-153,
# door_v0.py:121-138, pen_v0.py:134-152, relocate_v0.py:105-129)
def env_state_to_params(env_id: str, state: dict, params: np.ndarray) -> np.ndarray:
    """params after ``set_env_state(state)`` of an env whose params were ``params``: the model
    fields the reference writes, whole vectors (variation params are left as they are)."""
    p = np.array(params, np.float64, copy=True)
    if env_id == "hammer-v0":
        p[0:3] = np.asarray(state["board_pos"], np.float64).ravel()[:3]
    elif env_id == "door-v0":
        p[0:3] = np.asarray(state["door_body_pos"], np.float64).ravel()[:3]
    elif env_id == "pen-v0":
        p[0:4] = np.asarray(state["desired_orien"], np.float64).ravel()[:4]
    elif env_id == "relocate-v0":
        # obj_pos is the object's body_xpos (joint displacement included) written into body_pos:
        # the reference's quirk is kept (relocate_v0.py:127)
        p[0:3] = np.asarray(state["obj_pos"], np.float64).ravel()[:3]
        p[3:6] = np.asarray(state["target_pos"], np.float64).ravel()[:3]
    else:
        raise KeyError(env_id)
    return p


def env_state_from(env_id: str, model, qpos, qvel, params, xpos=None, site_xpos=None) -> dict:
    """The reference's get_env_state dict from the state, the params and (hammer target_pos,
    relocate obj / palm / target) the kinematics of the last forward pass."""
    qpos = np.asarray(qpos, np.float64).copy()
    qvel = np.asarray(qvel, np.float64).copy()
    p = np.asarray(params, np.float64)
    idx = task_indices(env_id, model)
    if env_id == "hammer-v0":
        return dict(qpos=qpos, qvel=qvel, board_pos=p[0:3].copy(),
                    target_pos=np.asarray(site_xpos[idx[3]], np.float64).copy())
    if env_id == "door-v0":
        return dict(qpos=qpos, qvel=qvel, door_body_pos=p[0:3].copy())
    if env_id == "pen-v0":
        return dict(qpos=qpos, qvel=qvel, desired_orien=p[0:4].copy())
    if env_id == "relocate-v0":
        return dict(hand_qpos=qpos[:30].copy(), obj_pos=np.asarray(xpos[idx[1]], np.float64).copy(),
                    target_pos=np.asarray(site_xpos[idx[2]], np.float64).copy(),
                    palm_pos=np.asarray(site_xpos[idx[0]], np.float64).copy(), qpos=qpos, qvel=qvel)
    raise KeyError(env_id)

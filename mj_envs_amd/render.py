"""Depth-camera observations (BASELINE config 5).

The reference renders RGB through OpenGL from mujoco-py's offscreen free camera
(``hand_manipulation_suite/headless_observer.py:20-52``):

* ``mj_viewer_headless_setup`` (``:20-31``): free camera, ``azimuth = 90``, ``distance = 4.5``,
  then ``set_view('default')`` (``:59-66``): ``elevation = -45 + deg(arccos(v_x / v_z)) / 2`` with
  ``v = body_xpos[obj_bid] - cam_xpos[-1]`` (the model's last camera);
* the camera's look-at point is mujoco-py's free-camera default: the per-axis median of
  ``geom_xpos`` when the render context is created;
* ``render`` (``:34-52``): a 640x480 frame, flipped upright, centre-cropped to 128x128 ("mimic
  zoom") and, with ``enable_resize``, resized to 64x64.

The build replaces the GL rasteriser with a HIP ray caster (``aw_render_depth``): one
workgroup per env, forward kinematics of the env's qpos on one wave, then each geom's pixel
box (its projected bounding sphere); each wave takes 64 pixels, ballots the geoms whose box
meets those rows and casts its rays against only those.  The output is metric z-depth on the
64x64 grid whose pixels are the 2x2 blocks of that 128x128 crop.  Depth has no reference
counterpart (the reference returns RGB), so this path is parity-unpinned against the
reference; it is checked against an independent numpy ray caster on the fp64 oracle's
kinematics (``oracle/depth.py``, ``tests/test_render.py``).

Reference quirks kept: hammer sets up its observer once, in ``__init__``, while ``obj_bid`` is
still the placeholder ``-1`` (``hammer_v0.py:15,35-38``), so the elevation uses the LAST body.
door and relocate construct their observer with placeholder body 0 (``door_v0.py:16,41``,
``relocate_v0.py:14,32``) and call its setup on EVERY reset (``door_v0.py:114``,
``relocate_v0.py:98``): body 0 is the world, so the camera is the same each time.  pen overrides
``mj_viewer_headless_setup`` (its second definition, ``pen_v0.py:163-177``, wins) and calls it on
every reset (``:127``) with ``target_obj_bid``, the 'target' body, whose position reset never
moves (only its orientation is drawn).  Meshes (the hand's visual geoms) are not available
offline; the primitive collision proxies are rendered in their place.
"""
from __future__ import annotations

import math

import numpy as np

from .mjcf import _kinematics0, quat2mat

CAM_FLOATS = 17
ZFAR = 10.0
FULL_W, FULL_H, CROP = 640, 480, 128
FOVY_DEG = 45.0                    # MuJoCo default visual/global/fovy
OBS_BID = {"hammer-v0": -1, "door-v0": 0, "pen-v0": "target", "relocate-v0": 0}   # body id or name


def _geom_world0(model):
    xpos, xquat, xmat = _kinematics0(model)
    gb = model.geom_bodyid
    gpos = np.array([xpos[b] + xmat[b] @ model.geom_pos[g] for g, b in enumerate(gb)])
    return xpos, gpos


def free_camera(model, env_id: str, width: int = 64, height: int = 64, zfar: float = ZFAR,
                aerial: bool = False) -> np.ndarray:
    """The reference's headless camera as the ``AW_CAM_FLOATS`` record of ``aw_render_depth``
    (``aerial``: ``set_view('aerial')``, elevation -45 - deg(...)/2, ``headless_observer.py:62-63``).

    Layout: position[3], forward[3], up[3], right[3], u0, du, v0, dv, zfar.  A ray through output
    pixel (row i, col j) has direction forward + (u0 + du*j) * right + (v0 - dv*i) * up.
    """
    xpos, gpos = _geom_world0(model)
    lookat = np.median(gpos, axis=0)                        # mujoco-py free-camera default
    cam = model.cam_pos[-1] if len(model.cam_pos) else np.zeros(3)
    cam_b = int(model.cam_bodyid[-1]) if len(model.cam_bodyid) else 0
    xq = _kinematics0(model)[1][cam_b]
    cam_world = xpos[cam_b] + quat2mat(xq) @ cam
    bid = OBS_BID.get(env_id, 0)
    if isinstance(bid, str):
        bid = model.name2id("body", bid)
    v = xpos[bid] - cam_world
    ratio = float(np.clip(v[0] / v[2], -1.0, 1.0)) if v[2] != 0 else 0.0
    elevation = -45.0 + (-1.0 if aerial else 1.0) * math.degrees(math.acos(ratio)) / 2.0
    azimuth, distance = 90.0, 4.5
    az, el = math.radians(azimuth), math.radians(elevation)
    fwd = np.array([math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el)])
    up = np.array([-math.sin(el) * math.cos(az), -math.sin(el) * math.sin(az), math.cos(el)])
    right = np.cross(fwd, up)
    pos = lookat - distance * fwd
    # full-frame image plane at unit distance: x in [-tx, tx], y in [-ty, ty]
    ty = math.tan(math.radians(FOVY_DEG) / 2.0)
    tx = ty * FULL_W / FULL_H
    # output pixel (i, j) = centre of a (CROP/width) x (CROP/height) block of the centred crop
    bx, by = CROP / width, CROP / height
    x0, y0 = (FULL_W - CROP) / 2.0, (FULL_H - CROP) / 2.0
    u0 = (2.0 * (x0 + 0.5 * bx) / FULL_W - 1.0) * tx
    du = 2.0 * bx / FULL_W * tx
    v0 = (1.0 - 2.0 * (y0 + 0.5 * by) / FULL_H) * ty
    dv = 2.0 * by / FULL_H * ty
    rec = np.concatenate([pos, fwd, up, right, [u0, du, v0, dv, zfar]]).astype(np.float32)
    assert rec.size == CAM_FLOATS
    return rec


def pixel_rays(cam: np.ndarray, width: int, height: int) -> np.ndarray:
    """Unit ray directions [height, width, 3] of a camera record (host-side helper)."""
    cam = np.asarray(cam, np.float64)
    fwd, up, right = cam[3:6], cam[6:9], cam[9:12]
    u = cam[12] + cam[13] * np.arange(width)
    v = cam[14] - cam[15] * np.arange(height)
    d = fwd[None, None] + u[None, :, None] * right[None, None] + v[:, None, None] * up[None, None]
    return d / np.linalg.norm(d, axis=-1, keepdims=True)

"""ctypes wrapper of the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It loads oracle/liboracle.so (built by ``make -C oracle``), an fp64 restatement of the
reference hot path (see oracle/oracle.h for what is restated and what is unpinned).
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

_dp = ctypes.POINTER(ctypes.c_double)
_u8p = ctypes.POINTER(ctypes.c_uint8)
_u32p = ctypes.POINTER(ctypes.c_uint32)
_lib = None


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-C", HERE, "-s"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.or_create.restype = ctypes.c_void_p
        L.or_create.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
        L.or_destroy.argtypes = [ctypes.c_void_p]
        L.or_set_option.argtypes = [ctypes.c_void_p] + [ctypes.c_int] * 5
        L.or_dims.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.or_set_margin_nudge.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double]
        L.or_reset.argtypes = [ctypes.c_void_p, ctypes.c_int, _dp, _dp, _dp, _dp, _dp, ctypes.c_int]
        L.or_step.argtypes = [ctypes.c_void_p, ctypes.c_int, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _u8p,
                              _u8p, _u32p, ctypes.c_int]
        L.or_step_stats.argtypes = [ctypes.c_void_p, ctypes.c_int, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _u8p,
                                    _u8p, ctypes.POINTER(ctypes.c_int32), ctypes.c_int]
        L.or_forward1.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp, _dp]
        L.or_mjstep1.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp, _dp, ctypes.c_int]
        L.or_get1.argtypes = [ctypes.c_void_p, ctypes.c_char_p, _dp, ctypes.c_int]
        L.or_quat2euler.argtypes = [_dp, _dp]
        L.or_task_eval.argtypes = [ctypes.c_void_p, _dp, _dp, _dp, _dp, _dp, _dp, _dp, _dp]
        L.or_collide.argtypes = [ctypes.c_void_p, ctypes.c_int, _dp, _dp, _dp, ctypes.c_int, _dp, _dp, _dp,
                                 ctypes.c_double, _dp]
        _lib = L
    return _lib


def _p(a: Optional[np.ndarray], ty=_dp):
    if a is None:
        return ty()
    return a.ctypes.data_as(ty)


def quat2euler(q) -> np.ndarray:
    q = np.ascontiguousarray(q, np.float64)
    e = np.zeros(3)
    lib().or_quat2euler(_p(q), _p(e))
    return e


class Oracle:
    """Batched fp64 CPU env over one compiled model + task block."""

    def __init__(self, blob: bytes):
        self._blob = ctypes.create_string_buffer(blob, len(blob))
        self.h = lib().or_create(self._blob, len(blob))
        if not self.h:
            raise RuntimeError("oracle: bad model blob")
        self._dims()

    def _dims(self):
        out = (ctypes.c_int * 16)()
        lib().or_dims(self.h, out)
        (self.nq, self.nv, self.nu, self.nbody, self.ngeom, self.nsite, self.obs_dim, self.nparam,
         self.frame_skip, self.horizon, self.nsensor, self.ntendon, self.max_con, self.max_efc) = out[:14]

    def set_option(self, disableflags=-1, max_con=-1, max_efc=-1, iterations=-1, noslip_iterations=-1):
        lib().or_set_option(self.h, disableflags, max_con, max_efc, iterations, noslip_iterations)
        self._dims()

    def set_margin_nudge(self, g1: int = -1, g2: int = -1, delta: float = 0.0):
        """shift the margin of the geom pair (g1, g2) (model geom ids) by delta; g1 < 0 clears"""
        lib().or_set_margin_nudge(self.h, int(g1), int(g2), float(delta))

    def __del__(self):
        try:
            if self.h:
                lib().or_destroy(self.h)
        except Exception:
            pass

    def reset(self, params: np.ndarray, nthreads: int = 0):
        params = np.ascontiguousarray(params, np.float64).reshape(-1, max(self.nparam, 1))
        n = params.shape[0]
        qpos = np.zeros((n, self.nq)); qvel = np.zeros((n, self.nv)); warm = np.zeros((n, self.nv))
        obs = np.zeros((n, self.obs_dim))
        lib().or_reset(self.h, n, _p(params), _p(qpos), _p(qvel), _p(warm), _p(obs), nthreads)
        return dict(qpos=qpos, qvel=qvel, warm=warm, params=params), obs

    def step(self, state: dict, action: np.ndarray, nthreads: int = 0):
        n = state["qpos"].shape[0]
        action = np.ascontiguousarray(action, np.float64).reshape(n, self.nu)
        obs = np.zeros((n, self.obs_dim)); rew = np.zeros(n)
        done = np.zeros(n, np.uint8); goal = np.zeros(n, np.uint8); status = np.zeros(n, np.uint32)
        lib().or_step(self.h, n, _p(state["params"]), _p(action), _p(state["qpos"]), _p(state["qvel"]),
                      _p(state["warm"]), _p(obs), _p(rew), _p(done, _u8p), _p(goal, _u8p),
                      _p(status, _u32p), nthreads)
        return obs, rew, done.astype(bool), goal.astype(bool), status

    def step_stats(self, state: dict, action: np.ndarray, nthreads: int = 0):
        """step() plus per-env work counts of the env-step: int32 [n, 12] = max ncon, max nefc, max
        dense rows over the substeps, summed Newton iterations, line-search evaluations, noslip
        sweeps, substeps, status flags, summed ncon, nefc, dense rows, substeps with a box-box contact"""
        n = state["qpos"].shape[0]
        action = np.ascontiguousarray(action, np.float64).reshape(n, self.nu)
        obs = np.zeros((n, self.obs_dim)); rew = np.zeros(n)
        done = np.zeros(n, np.uint8); goal = np.zeros(n, np.uint8); stats = np.zeros((n, 12), np.int32)
        lib().or_step_stats(self.h, n, _p(state["params"]), _p(action), _p(state["qpos"]), _p(state["qvel"]),
                            _p(state["warm"]), _p(obs), _p(rew), _p(done, _u8p), _p(goal, _u8p),
                            stats.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), nthreads)
        return obs, rew, done.astype(bool), goal.astype(bool), stats

    # --- single env ---------------------------------------------------------------------
    def forward1(self, params, qpos, qvel, warm=None, ctrl=None):
        c = lambda a: None if a is None else np.ascontiguousarray(a, np.float64)
        params, qpos, qvel, warm, ctrl = map(c, (params, qpos, qvel, warm, ctrl))
        lib().or_forward1(self.h, _p(params), _p(qpos), _p(qvel), _p(warm), _p(ctrl))

    def mjstep1(self, params, qpos, qvel, warm, ctrl=None, nstep=1):
        """In-place mj_step on (qpos, qvel, warm) float64 arrays; returns status flags."""
        ctrl = None if ctrl is None else np.ascontiguousarray(ctrl, np.float64)
        params = None if params is None else np.ascontiguousarray(params, np.float64)
        return lib().or_mjstep1(self.h, _p(params), _p(qpos), _p(qvel), _p(warm), _p(ctrl), nstep)

    def get(self, name: str) -> np.ndarray:
        n = lib().or_get1(self.h, name.encode(), None, 0)
        if n < 0:
            raise KeyError(name)
        out = np.zeros(max(n, 1))
        lib().or_get1(self.h, name.encode(), _p(out), n)
        return out[:n]

    def collide(self, t1, pos1, mat1, size1, t2, pos2, mat2, size2, margin):
        """narrowphase of two primitives (test hook): [(dist, pos[3], normal[3]), ...]"""
        c = lambda a: np.ascontiguousarray(a, np.float64).ravel()
        out = np.zeros(16 * 7)
        n = lib().or_collide(self.h, int(t1), _p(c(pos1)), _p(c(mat1)), _p(c(size1)), int(t2), _p(c(pos2)),
                             _p(c(mat2)), _p(c(size2)), float(margin), _p(out))
        return out[:7 * n].reshape(n, 7)

    def task_eval(self, qpos, qvel, xpos, xquat, site_xpos, sensordata):
        c = lambda a: np.ascontiguousarray(a, np.float64).ravel()
        obs = np.zeros(self.obs_dim); rdg = np.zeros(3)
        lib().or_task_eval(self.h, _p(c(qpos)), _p(c(qvel)), _p(c(xpos)), _p(c(xquat)), _p(c(site_xpos)),
                           _p(c(sensordata)), _p(obs), _p(rdg))
        return obs, rdg[0], bool(rdg[1]), bool(rdg[2])

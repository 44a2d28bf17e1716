"""ctypes binding of the C-ABI in include/adroit_wave.h (libadroit_hip.so).

The product path: every compute call goes to the HIP library.  There is no CPU fallback:
if the library is missing or cannot be loaded, ``load()`` raises.  Device memory is managed
with torch (``torch.cuda`` tensors are HIP allocations on ROCm); pointers and the current
stream are passed through as plain integers.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# AW_LIB selects a diagnostic build (e.g. libadroit_hip_prof.so with the stage profiler)
LIB_PATH = os.environ.get("AW_LIB") or os.path.join(HERE, "libadroit_hip.so")

AW_NDIMS = 21
# the fast tier's capacities (aw_common.h FAST_*; the aw_forward_dump layout uses them); the
# effective ones are the reference model's nconmax / njmax, held by the wide tier (aw_dims)
MAXCON, MAXEFC, MAXDENSE = 48, 192, 128
NCONMAX, NJMAX = 100, 500
ST_BADQPOS, ST_BADQVEL, ST_BADQACC, ST_CON_OVERFLOW, ST_EFC_OVERFLOW, ST_WIDE = 1, 2, 4, 8, 16, 32
ST_OVERFLOW = ST_CON_OVERFLOW | ST_EFC_OVERFLOW   # constraints dropped at MuJoCo's own caps


def dump_layout(maxcon=MAXCON, maxefc=MAXEFC):
    """float offsets inside the aw_forward_dump output (adroit_wave.hip k_dump, DUMP_*)"""
    c, e = 1768, 1768 + 14 * maxcon
    return dict(xpos=(0, 96), xquat=(96, 128), site_xpos=(224, 96), qacc_smooth=(320, 36),
                qfrc_smooth=(356, 36), qacc=(392, 36), qfrc_constraint=(428, 36), qM=(464, 1296),
                scalars=(1760, 8), con_dist=(c, maxcon), con_pos=(c + maxcon, 3 * maxcon),
                con_frame=(c + 4 * maxcon, 9 * maxcon), con_pair=(c + 13 * maxcon, maxcon),
                efc_force=(e, maxefc), efc_aref=(e + maxefc, maxefc), efc_D=(e + 2 * maxefc, maxefc),
                efc_type=(e + 3 * maxefc, maxefc), efc_state=(e + 4 * maxefc, maxefc))


DUMP_LAYOUT = dump_layout()
WIDE_MAXCON_STORE, WIDE_MAXEFC = 128, 512       # the wide tier's contact storage and row slots
DUMP_LAYOUT_WIDE = dump_layout(WIDE_MAXCON_STORE, WIDE_MAXEFC)
AW_DUMP_SIZE_WIDE = 1768 + 14 * WIDE_MAXCON_STORE + 5 * WIDE_MAXEFC
# why the Newton solve stopped (aw_solver.h NT_EXIT_*)
NT_EXIT = ("max_iterations", "no_descent", "fp32_noise_floor", "improvement", "gradient", "no_constraints")
AW_DUMP_SIZE = 1768 + 14 * MAXCON + 5 * MAXEFC

_lib = None
_vp = ctypes.c_void_p


class NativeError(RuntimeError):
    pass


def load():
    """Load libadroit_hip.so (raises if absent: the HIP path is the only path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise NativeError(f"{LIB_PATH} not built; run `python -c 'import __graft_entry__ as g; g.build()'`")
    L = ctypes.CDLL(LIB_PATH)
    L.aw_last_error.restype = ctypes.c_char_p
    L.aw_create.argtypes = [_vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, ctypes.POINTER(_vp)]
    L.aw_destroy.argtypes = [_vp]
    L.aw_dims.argtypes = [_vp, ctypes.POINTER(ctypes.c_int)]
    L.aw_set_option.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    L.aw_reset.argtypes = [_vp, _vp, _vp, ctypes.c_uint64, _vp, _vp]
    L.aw_step.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _vp, ctypes.c_int, ctypes.c_uint64, _vp]
    L.aw_random_actions.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint64, _vp, _vp]
    L.aw_set_env_offset.argtypes = [_vp, ctypes.c_uint64]
    L.aw_set_tier.argtypes = [_vp, ctypes.c_int]
    if hasattr(L, "aw_forward_dump_wide"):
        L.aw_forward_dump_wide.argtypes = [_vp, ctypes.c_int, _vp, _vp, _vp]
        L.aw_forward_dump_wide.restype = ctypes.c_int
    if hasattr(L, "aw_set_fault"):
        L.aw_set_fault.argtypes = [_vp, ctypes.c_int, ctypes.c_int]
        L.aw_set_fault.restype = ctypes.c_int
    L.aw_clear_status.argtypes = [_vp, _vp]
    L.aw_episode_totals.argtypes = [_vp, _vp, _vp, _vp, _vp]
    L.aw_get_episode.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp]
    L.aw_set_episode.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp]
    L.aw_get_state.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp]
    L.aw_set_state.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp, _vp]
    L.aw_status.argtypes = [_vp, _vp, _vp, _vp]
    L.aw_episode_stats.argtypes = [_vp, _vp, _vp, _vp, _vp, _vp]
    L.aw_task_eval.argtypes = [_vp, ctypes.c_int] + [_vp] * 10 + [_vp]
    L.aw_forward_dump.argtypes = [_vp, ctypes.c_int, _vp, _vp, _vp]
    L.aw_stage_profile.argtypes = [_vp, ctypes.c_int]
    L.aw_collide_test.argtypes = [_vp, ctypes.c_int] + [_vp] * 9
    L.aw_collide_test.restype = ctypes.c_int
    # (diagnostic builds of older revisions, selected with AW_LIB, may lack the newer entry points;
    # calling one of those then raises AttributeError)
    if hasattr(L, "aw_set_episode_totals"):
        L.aw_set_episode_totals.argtypes = [_vp, _vp, _vp, _vp, _vp]
        L.aw_set_episode_totals.restype = ctypes.c_int
    if hasattr(L, "aw_render_depth"):
        L.aw_render_depth.argtypes = [_vp, _vp, ctypes.c_int, ctypes.c_int, _vp, _vp]
        L.aw_render_depth.restype = ctypes.c_int
    if hasattr(L, "aw_policy_mlp"):
        L.aw_policy_mlp.argtypes = [ctypes.c_int] * 4 + [_vp, _vp, _vp, ctypes.c_int, ctypes.c_uint64,
                                                         ctypes.c_uint64, ctypes.c_uint64, _vp]
        L.aw_policy_mlp.restype = ctypes.c_int
    for f in ("aw_create", "aw_destroy", "aw_dims", "aw_set_option", "aw_reset", "aw_step",
              "aw_random_actions", "aw_get_state", "aw_set_state", "aw_status", "aw_episode_stats",
              "aw_task_eval", "aw_forward_dump", "aw_stage_profile", "aw_set_env_offset", "aw_clear_status",
              "aw_episode_totals", "aw_get_episode", "aw_set_episode", "aw_set_tier"):
        getattr(L, f).restype = ctypes.c_int
    _lib = L
    return L


EXPORTS = ("aw_create", "aw_destroy", "aw_dims", "aw_set_option", "aw_set_tier", "aw_set_fault", "aw_reset", "aw_step",
           "aw_random_actions", "aw_set_env_offset", "aw_get_state", "aw_set_state", "aw_status",
           "aw_clear_status", "aw_episode_stats", "aw_episode_totals", "aw_set_episode_totals", "aw_get_episode",
           "aw_set_episode",
           "aw_task_eval", "aw_forward_dump", "aw_forward_dump_wide", "aw_stage_profile", "aw_render_depth", "aw_policy_mlp",
           "aw_collide_test", "aw_last_error")

STAGES = ("pre", "kinematics", "collision", "com_crb", "rne_smooth_solve", "constraints", "newton",
          "noslip", "jt_touch", "euler", "task_obs", "reset", "checks")
SUBSTAGES = ("nt_init", "nt_hess", "nt_chol", "nt_solve", "nt_ls", "nt_upd", "ns_minv", "ns_setup", "ns_iter",
             "co_broad", "co_narrow", "com", "rne", "co_plane", "co_round", "co_roundbox", "co_boxbox",
             "nt_hsparse", "nt_hoffd")
# timed intervals recorded in slots past the counters (stage_profile: v[39..41])
EXTRA_STAGES = ("co_kin64", "cs_sparse", "cs_j")


def stage_profile(reset: bool = True) -> dict:
    """Per-stage shader-clock cycles of k_step (diagnostic build only, see aw_stage_profile)."""
    buf = (ctypes.c_ulonglong * 44)()
    _check(load().aw_stage_profile(buf, int(reset)))
    v = list(buf)
    out = {name: v[i] for i, name in enumerate(STAGES)}
    out["waves"], out["substeps"] = v[13], v[14]
    out["newton_iters"], out["noslip_iters"], out["nefc"], out["ncon"] = v[15], v[16], v[17], v[18]
    for i, name in enumerate(SUBSTAGES):
        out[name] = v[19 + i]
    out["offd_rows"] = v[38]
    out["co_kin64"] = v[39]
    out["cs_sparse"], out["cs_j"] = v[40], v[41]
    out["mpr_pairs"], out["mpr_contacts"] = v[42], v[43]
    return out


def kernel_build_id() -> str:
    """Short hash of the HIP sources, the C-ABI header and the compile flags the product library
    is built from: ties a committed rocprof summary to the kernel revision it measured."""
    import hashlib
    import sys
    root = os.path.dirname(HERE)
    h = hashlib.sha256()
    for d in (os.path.join(HERE, "csrc"), os.path.join(root, "include")):
        for f in sorted(os.listdir(d)):
            with open(os.path.join(d, f), "rb") as fh:
                h.update(f.encode() + b"\0" + fh.read())
    if root not in sys.path:
        sys.path.insert(0, root)
    import __graft_entry__
    h.update(" ".join(__graft_entry__.HIPCC_FLAGS).encode())
    if os.environ.get("AW_LIB"):
        h.update(os.path.basename(os.environ["AW_LIB"]).encode())
    return h.hexdigest()[:12]


def _check(rc: int):
    if rc != 0:
        raise NativeError(f"adroit_wave error {rc}: {load().aw_last_error().decode()}")


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    return t.data_ptr()


def _stream():
    import torch
    return torch.cuda.current_stream().cuda_stream


class Sim:
    """One batch of ``n_envs`` envs of one task on one GPU (owns the device state)."""

    def __init__(self, blob: bytes, n_envs: int, device: int = 0, env_offset: int = 0):
        import torch
        L = load()
        self.device = device
        self.torch_device = torch.device("cuda", device)
        self._blob = ctypes.create_string_buffer(blob, len(blob))
        h = _vp()
        with torch.cuda.device(device):
            _check(L.aw_create(self._blob, len(blob), n_envs, device, ctypes.byref(h)))
        self.h = h
        d = (ctypes.c_int * AW_NDIMS)()
        _check(L.aw_dims(self.h, d))
        (self.nq, self.nv, self.nu, self.obs_dim, self.nparam, self.frame_skip, self.horizon,
         self.task_kind, self.n_envs, self.nbody, self.nsite, self.ngeom, self.npair,
         self.maxcon, self.maxefc, self.maxdense, self.grid, self.fast_maxcon, self.fast_maxefc,
         self.fast_maxdense, self.wide_grid) = list(d)
        self.env_offset = 0
        if env_offset:
            self.set_env_offset(env_offset)

    def set_env_offset(self, env_offset: int):
        """global id of env 0 (shards): Philox streams are keyed by the global env id"""
        _check(load().aw_set_env_offset(self.h, int(env_offset)))
        self.env_offset = int(env_offset)

    def close(self):
        if getattr(self, "h", None):
            load().aw_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # --- buffers ---------------------------------------------------------------------------
    def empty(self, *shape, dtype=None):
        import torch
        return torch.empty(*shape, dtype=dtype or torch.float32, device=self.torch_device)

    def set_option(self, disableflags: int = -1, iterations: int = -1, noslip_iterations: int = -1):
        _check(load().aw_set_option(self.h, disableflags, iterations, noslip_iterations))

    def set_tier(self, mode: int):
        """0: automatic (fast tier, wide tier for overflowing env-steps); 1: wide tier only (tests)"""
        _check(load().aw_set_tier(self.h, int(mode)))

    def set_fault(self, kind: int, arg: int = 0):
        """test hook (include/adroit_wave.h aw_set_fault): 0 none, 1 class-1 margins + arg um,
        2 frictionloss row `arg` held in the stick state"""
        _check(load().aw_set_fault(self.h, int(kind), int(arg)))

    def reset(self, obs, params=None, mask=None, seed: int = 1):
        _check(load().aw_reset(self.h, _ptr(mask), _ptr(params), seed, _ptr(obs), _stream()))

    def step(self, actions, obs, reward, done, goal, terminal_obs=None, autoreset: bool = False,
             seed: int = 1):
        _check(load().aw_step(self.h, _ptr(actions), _ptr(obs), _ptr(reward), _ptr(done), _ptr(goal),
                              _ptr(terminal_obs), int(autoreset), seed, _stream()))

    def random_actions(self, out, seed: int, step: int):
        _check(load().aw_random_actions(self.h, seed, step, _ptr(out), _stream()))

    def get_state(self, qpos=None, qvel=None, warm=None, params=None):
        _check(load().aw_get_state(self.h, _ptr(qpos), _ptr(qvel), _ptr(warm), _ptr(params), _stream()))

    def set_state(self, qpos=None, qvel=None, warm=None, params=None, obs=None):
        _check(load().aw_set_state(self.h, _ptr(qpos), _ptr(qvel), _ptr(warm), _ptr(params), _ptr(obs),
                                   _stream()))

    def status(self, last=None, sticky=None):
        """per-env flags (ST_*): of the last step (last) / OR since create or clear_status (sticky)"""
        _check(load().aw_status(self.h, _ptr(last), _ptr(sticky), _stream()))

    def clear_status(self):
        _check(load().aw_clear_status(self.h, _stream()))

    def episode_totals(self, episodes=None, sum_return=None, successes=None):
        _check(load().aw_episode_totals(self.h, _ptr(episodes), _ptr(sum_return), _ptr(successes), _stream()))

    def set_episode_totals(self, episodes=None, sum_return=None, successes=None):
        """restore the running totals (checkpoint); see include/adroit_wave.h aw_set_episode_totals"""
        _check(load().aw_set_episode_totals(self.h, _ptr(episodes), _ptr(sum_return), _ptr(successes), _stream()))

    def get_episode(self, ep_len=None, ep_ret=None, ep_goal=None, episodes=None):
        _check(load().aw_get_episode(self.h, _ptr(ep_len), _ptr(ep_ret), _ptr(ep_goal), _ptr(episodes),
                                     _stream()))

    def set_episode(self, ep_len=None, ep_ret=None, ep_goal=None, episodes=None):
        _check(load().aw_set_episode(self.h, _ptr(ep_len), _ptr(ep_ret), _ptr(ep_goal), _ptr(episodes),
                                     _stream()))

    def episode_stats(self, last_return=None, last_goal=None, last_len=None, episodes=None):
        _check(load().aw_episode_stats(self.h, _ptr(last_return), _ptr(last_goal), _ptr(last_len),
                                       _ptr(episodes), _stream()))

    def task_eval(self, n, qpos, qvel, xpos, xquat, site_xpos, touch, obs, reward, done, goal):
        _check(load().aw_task_eval(self.h, n, _ptr(qpos), _ptr(qvel), _ptr(xpos), _ptr(xquat),
                                   _ptr(site_xpos), _ptr(touch), _ptr(obs), _ptr(reward), _ptr(done),
                                   _ptr(goal), _stream()))

    def render_depth(self, out, cam: np.ndarray):
        """Depth frames of every env's current state into out [N, H, W] (device, fp32);
        cam: the host camera record of mj_envs_amd.render.free_camera."""
        n, h, w = out.shape
        assert n == self.n_envs and out.is_contiguous(), "render_depth: out must be [n_envs, H, W]"
        c = np.ascontiguousarray(cam, np.float32)
        assert c.size == 17, "render_depth: camera record has 17 floats"
        _check(load().aw_render_depth(self.h, c.ctypes.data, w, h, _ptr(out), _stream()))

    def collide_test(self, types, pos, mat, size, margin, fp64: bool = False):
        """narrowphase of n primitive pairs (test hook): list of arrays [(dist, pos[3], normal[3]), ...]
        (fp64: the MPR pairs' fp64 results instead of the fp32 contacts)"""
        import torch
        n = len(types)
        dev = self.torch_device
        t = lambda a, dt=torch.float32: torch.tensor(np.asarray(a), dtype=dt, device=dev).contiguous()
        out = torch.zeros(n, 8, 7, device=dev)
        cnt = torch.zeros(n, dtype=torch.int32, device=dev)
        out64 = torch.zeros(n, 8, 7, dtype=torch.float64, device=dev) if fp64 else None
        args = [t(types, torch.int32), t(pos), t(mat), t(size), t(margin)]   # alive until the kernel ran
        _check(load().aw_collide_test(self.h, n, *[_ptr(a) for a in args], _ptr(out), _ptr(cnt), _ptr(out64),
                                      _stream()))
        o = (out64 if fp64 else out).cpu().numpy().astype(np.float64)
        c = cnt.cpu().numpy()
        return [o[i, :c[i]] for i in range(n)]

    def forward_dump(self, env: int, ctrl=None, wide: bool = False) -> dict:
        """one forward of env `env` (ctrl: raw controls or None = 0) and its internals; wide=True runs it
        through the wide-capacity tier (aw_forward_dump_wide: MuJoCo's nconmax / njmax)"""
        out = self.empty(AW_DUMP_SIZE_WIDE if wide else AW_DUMP_SIZE)
        fn = load().aw_forward_dump_wide if wide else load().aw_forward_dump
        _check(fn(self.h, env, _ptr(ctrl), _ptr(out), _stream()))
        o = out.cpu().numpy().astype(np.float64)
        res = {k: o[a:a + n] for k, (a, n) in (DUMP_LAYOUT_WIDE if wide else DUMP_LAYOUT).items()}
        nv, nb, ns = self.nv, self.nbody, self.nsite
        res["xpos"] = res["xpos"][:3 * nb].reshape(nb, 3)
        res["xquat"] = res["xquat"][:4 * nb].reshape(nb, 4)
        res["site_xpos"] = res["site_xpos"][:3 * ns].reshape(ns, 3)
        for k in ("qacc_smooth", "qfrc_smooth", "qacc", "qfrc_constraint"):
            res[k] = res[k][:nv]
        res["qM"] = res["qM"][:nv * nv].reshape(nv, nv)
        sc = res["scalars"]
        ncon, nefc = int(sc[0]), int(sc[1])
        res.update(ncon=ncon, nefc=nefc, nsparse=int(sc[2]), ndense=int(sc[3]), touch=sc[4], status=int(sc[5]),
                   solver_iter=int(sc[6]) % 1000, solver_exit=NT_EXIT[int(sc[6]) // 1000], noslip_iter=int(sc[7]))
        res["con_dist"] = res["con_dist"][:ncon]
        res["con_pos"] = res["con_pos"][:3 * ncon].reshape(ncon, 3)
        res["con_frame"] = res["con_frame"][:9 * ncon].reshape(ncon, 9)
        res["con_pair"] = res["con_pair"][:ncon].astype(int)
        for k in ("efc_force", "efc_aref", "efc_D", "efc_type", "efc_state"):
            res[k] = res[k][:nefc]
        return res

"""Gym-style facades over the batched HIP simulator.

Two ways in, both backed by the same C-ABI (``include/adroit_wave.h``) and nothing else:

* ``HammerEnvV0`` / ``DoorEnvV0`` / ``PenEnvV0`` / ``RelocateEnvV0`` -- one env per object with
  the reference's per-env API (``hand_manipulation_suite/*_v0.py``): ``step(a) -> (obs, reward,
  done, {'goal_achieved'})``, ``reset() -> (obs, {})``, ``get_obs``, ``get_env_state`` /
  ``set_env_state`` (same dict keys), ``evaluate_success(paths)``, ``act_mid`` / ``act_rng``,
  ``frame_skip``, ``action_space`` / ``observation_space``.  numpy in, numpy out.
* ``AdroitVecEnv`` -- N envs of one task on one GPU, torch device tensors in and out, in-kernel
  auto-reset, 5-tuple ``(obs, reward, terminated, truncated, info)`` like the reference's
  ``CustomPixelObservationWrapper`` (``wrappers.py:32-76``) hands to its trainers.

Model-parameter resets (nail-board height, door frame position, pen target orientation,
relocate object / target) are per-env override vectors (``tasks.param_layout``), so envs in one
batch never share mutated model state.
"""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from . import _native
from .tasks import TASKS, attach_task, env_state_from, env_state_to_params, load_model, param_layout


class Box:
    """Minimal stand-in for ``gym.spaces.Box`` (gym is not a dependency of the hot path)."""

    def __init__(self, low, high, shape, dtype=np.float32):
        self.shape = tuple(shape)
        self.dtype = np.dtype(dtype)
        self.low = np.full(self.shape, low, self.dtype)
        self.high = np.full(self.shape, high, self.dtype)

    def sample(self, rng: Optional[np.random.Generator] = None):
        rng = rng or np.random.default_rng()
        return rng.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))


def _evaluate_success(env_id: str, paths: List[dict]) -> float:
    """``hammer_v0.py:167-175`` (and door/pen/relocate): % of paths with > k goal steps."""
    k = TASKS[env_id].success_steps
    if not paths:
        return 0.0
    n = sum(1 for p in paths if np.sum(p["env_infos"]["goal_achieved"]) > k)
    return n * 100.0 / len(paths)


class AdroitVecEnv:
    """``num_envs`` envs of ``env_id`` on GPU ``device``; every buffer stays in HBM."""

    def __init__(self, env_id: str, num_envs: int, device: int = 0, variation_type: Optional[str] = None,
                 seed: int = 1, autoreset: bool = True):
        import torch
        self.env_id = env_id
        self.spec = TASKS[env_id]
        self.model = attach_task(load_model(env_id), env_id, variation_type)
        self.variation_type = variation_type
        self.sim = _native.Sim(self.model.to_blob(), num_envs, device)
        self.num_envs = num_envs
        self.seed = int(seed)
        self.autoreset = autoreset
        s = self.sim
        self.nq, self.nv, self.nu, self.obs_dim, self.nparam = s.nq, s.nv, s.nu, s.obs_dim, s.nparam
        self.frame_skip, self.horizon = s.frame_skip, s.horizon
        self.act_mid = self.model.arrays["task_act_mid"].astype(np.float32)
        self.act_rng = self.model.arrays["task_act_rng"].astype(np.float32)
        self.action_space = Box(-1.0, 1.0, (self.nu,))
        self.observation_space = Box(-np.inf, np.inf, (self.obs_dim,))
        self.obs = s.empty(num_envs, self.obs_dim)
        self.reward = s.empty(num_envs)
        self.done = s.empty(num_envs, dtype=torch.uint8)
        self.goal = s.empty(num_envs, dtype=torch.uint8)
        self.terminal_obs = s.empty(num_envs, self.obs_dim)
        self._status = s.empty(num_envs, dtype=torch.int32)
        self._resets = 0

    # --- episode control -------------------------------------------------------------------
    def reset(self, mask=None, params=None, seed: Optional[int] = None):
        """Reset all envs (or those with ``mask[i] != 0``); params [N, nparam] or sampled."""
        if seed is None:
            seed = self.seed + 7919 * self._resets
        self._resets += 1
        self.sim.reset(self.obs, params=params, mask=mask, seed=seed)
        return self.obs

    def step(self, actions):
        """actions: device tensor [N, nu] in [-1, 1] (clipped and scaled in the kernel)."""
        self.sim.step(actions, self.obs, self.reward, self.done, self.goal,
                      terminal_obs=self.terminal_obs if self.autoreset else None,
                      autoreset=self.autoreset, seed=self.seed)
        terminated = (self.done & 1).bool()
        truncated = (self.done & 2).bool()
        self.sim.status(last=self._status)
        info = {"goal_achieved": self.goal.bool(), "terminal_obs": self.terminal_obs,
                "status": self._status}    # AW_ST_* flags of this step (NaN reset, overflow)
        return self.obs, self.reward, terminated, truncated, info

    def random_actions(self, out, step: int, seed: int = 0):
        self.sim.random_actions(out, seed, step)
        return out

    def mj_viewer_headless_setup(self, width: Optional[int] = None, height: Optional[int] = None,
                                 aerial: Optional[bool] = None):
        """``headless_observer.py:20-31`` (+ ``set_view``, ``:59-66``): the offscreen free camera
        (azimuth 90, distance 4.5, elevation from the observed body; ``aerial`` flips the
        elevation's sign as ``set_view('aerial')`` / pen's ``use_aerial_view`` do).  Here it builds
        the camera record every env of the batch is rendered from (``render.free_camera``) and
        returns it; ``render_depth`` uses it from then on.  ``aerial`` None: the single-env facade
        this batch belongs to decides (pen_v0.py:174-177 reads its ``use_aerial_view``), so the
        reference's ``gym_env.env.mj_viewer_headless_setup()`` through a wrapper keeps the flag."""
        from .render import free_camera
        if aerial is None:
            fac = getattr(self, "_facade", None)
            aerial = bool(fac is not None and self.env_id == "pen-v0" and getattr(fac, "use_aerial_view", False))
        w, h = (width or self._cam_key[0], height or self._cam_key[1]) if getattr(self, "_cam_key", None) \
            else (width or 64, height or 64)
        self._aerial = bool(aerial)
        self._cam, self._cam_key = free_camera(self.model, self.env_id, w, h, aerial=self._aerial), (w, h)
        return self._cam

    def render_depth(self, width: int = 64, height: int = 64, out=None):
        """Depth frames [N, height, width] (metres, device) of every env's current state from
        the reference's headless camera (headless_observer.py; mj_envs_amd/render.py)."""
        if getattr(self, "_cam_key", None) != (width, height):
            self.mj_viewer_headless_setup(width, height, aerial=getattr(self, "_aerial", False))
        if out is None:
            out = self.sim.empty(self.num_envs, height, width)
        self.sim.render_depth(out, self._cam)
        return out

    # --- state -----------------------------------------------------------------------------
    def get_state(self) -> Dict[str, "object"]:
        s = self.sim
        st = dict(qpos=s.empty(self.num_envs, self.nq), qvel=s.empty(self.num_envs, self.nv),
                  qacc_warmstart=s.empty(self.num_envs, self.nv), params=s.empty(self.num_envs, self.nparam))
        s.get_state(st["qpos"], st["qvel"], st["qacc_warmstart"], st["params"])
        return st

    def set_state(self, qpos=None, qvel=None, qacc_warmstart=None, params=None):
        self.sim.set_state(qpos, qvel, qacc_warmstart, params, obs=self.obs)
        return self.obs

    def episode_stats(self):
        import torch
        s = self.sim
        out = dict(last_return=s.empty(self.num_envs), last_goal_steps=s.empty(self.num_envs, dtype=torch.int32),
                   last_len=s.empty(self.num_envs, dtype=torch.int32),
                   episodes=s.empty(self.num_envs, dtype=torch.int32))
        s.episode_stats(out["last_return"], out["last_goal_steps"], out["last_len"], out["episodes"])
        return out

    def status(self, sticky: bool = False):
        """AW_ST_* flags per env: of the last step, or (sticky) OR'ed since creation"""
        import torch
        out = self.sim.empty(self.num_envs, dtype=torch.int32)
        self.sim.status(**({"sticky": out} if sticky else {"last": out}))
        return out

    def episode_totals(self):
        """every finished episode counted once: episodes, sum of returns, successes per env"""
        import torch
        s = self.sim
        out = dict(episodes=s.empty(self.num_envs, dtype=torch.int32), sum_return=s.empty(self.num_envs),
                   successes=s.empty(self.num_envs, dtype=torch.int32))
        s.episode_totals(out["episodes"], out["sum_return"], out["successes"])
        return out

    def evaluate_success(self, paths: List[dict]) -> float:
        return _evaluate_success(self.env_id, paths)

    def close(self):
        self.sim.close()


def _reference_base():
    """mjrl's ``MujocoEnv`` when it is importable, else ``object``.  The reference's driver reports
    an episode's success only for instances of it (``utils/helpers.py:53``:
    ``isinstance(env.unwrapped, mjrl.envs.mujoco_env.MujocoEnv)``), so with mjrl installed the
    facades pass that check unchanged.  Its ``__init__`` (mujoco-py) is never called: every
    method the reference's env layer uses is defined below."""
    try:
        from mjrl.envs.mujoco_env import MujocoEnv
        return MujocoEnv
    except Exception:
        return object


class _AdroitEnv(_reference_base()):
    """Single-env facade with the reference's method set (one ``AdroitVecEnv`` of size 1)."""

    env_id: str = ""

    def __init__(self, render_mode=None, width: int = 64, height: int = 64, is_headless: bool = True,
                 variation_type: Optional[str] = None, device: int = 0, seed: Optional[int] = None):
        import torch
        self.render_mode, self.width, self.height = render_mode, width, height
        self.is_headless = is_headless
        self.variation_type = variation_type
        self.observer = None            # the camera record once mj_viewer_headless_setup() ran
        self.vec = AdroitVecEnv(self.env_id, 1, device=device, variation_type=variation_type,
                                seed=1, autoreset=False)
        self.vec._facade = self         # camera flags (pen's use_aerial_view) of this facade
        self.model = self.vec.model
        self.frame_skip = self.vec.frame_skip
        self.act_mid = self.vec.act_mid.astype(np.float64)
        self.act_rng = self.vec.act_rng.astype(np.float64)
        self.action_space = self.vec.action_space
        self.observation_space = self.vec.observation_space
        self._dev = self.vec.sim.torch_device
        self._act = torch.zeros(1, self.vec.nu, device=self._dev)
        self.np_random = np.random.default_rng(seed)
        self._layout = param_layout(self.env_id, self.model, variation_type)
        self._obs = np.zeros(self.vec.obs_dim, np.float32)
        self.reset()

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)
        return [seed]

    @property
    def unwrapped(self):
        return self

    # --- reference API ---------------------------------------------------------------------
    def step(self, a):
        import torch
        a = np.asarray(a, np.float32).reshape(1, -1)
        self._act.copy_(torch.from_numpy(a))
        obs, rew, term, _trunc, info = self.vec.step(self._act)
        self._obs = obs[0].cpu().numpy().copy()
        return self._obs, float(rew[0]), bool(term[0]), {"goal_achieved": bool(info["goal_achieved"][0])}

    def reset(self, seed=None):
        if seed is not None:
            self.seed(seed)
        s = int(self.np_random.integers(1, 2 ** 63 - 1))
        self.vec.reset(seed=s)
        self._obs = self.vec.obs[0].cpu().numpy().copy()
        return self._obs, {}

    def reset_model(self):
        return self.reset()

    def get_obs(self):
        return self._obs.copy()

    def _params(self) -> np.ndarray:
        return self.vec.get_state()["params"][0].cpu().numpy().astype(np.float64)

    def get_env_state(self):
        """``get_env_state`` of the reference task (hammer_v0.py:134-143, door_v0.py:121-128,
        pen_v0.py:134-141, relocate_v0.py:105-116): same keys, fp64 copies."""
        qp, qv = self._qpos_qvel()
        xpos = site_xpos = None
        if self.env_id == "hammer-v0":
            site_xpos = {int(self.model.arrays["task_idx"][3]): self._obs[42:45]}   # last forward's S_target
        elif self.env_id == "relocate-v0":
            d = self.vec.sim.forward_dump(0)
            xpos, site_xpos = d["xpos"], d["site_xpos"]
        return env_state_from(self.env_id, self.model, qp, qv, self._params(), xpos=xpos, site_xpos=site_xpos)

    def set_env_state(self, state_dict):
        """``set_env_state``: qpos / qvel, then the whole model-field vectors the reference writes
        (hammer board_pos, door frame body_pos, pen target quat, relocate obj / target pos)."""
        p = env_state_to_params(self.env_id, state_dict, self._params())
        self._set(state_dict["qpos"], state_dict["qvel"], p)

    def _set(self, qpos, qvel, params):
        import torch
        t = lambda x: torch.as_tensor(np.asarray(x, np.float32).reshape(1, -1), device=self._dev)
        self.vec.set_state(qpos=t(qpos), qvel=t(qvel), params=t(params))
        self._obs = self.vec.obs[0].cpu().numpy().copy()

    def _qpos_qvel(self):
        st = self.vec.get_state()
        return (st["qpos"][0].cpu().numpy().astype(np.float64), st["qvel"][0].cpu().numpy().astype(np.float64))

    def evaluate_success(self, paths: List[dict]) -> float:
        return _evaluate_success(self.env_id, paths)

    def render(self, *args, **kwargs):
        """Depth frame [height, width] (float64, metres) of the current state.  The reference
        returns an RGB frame from OpenGL (headless_observer.py:34-52); RGB is not rendered here,
        the HIP ray caster produces metric depth from the same camera (mj_envs_amd/render.py)."""
        return self.vec.render_depth(self.width, self.height)[0].cpu().numpy().astype(np.float64)

    # pen's flag (pen_v0.py:23, read by its mj_viewer_headless_setup, :174-177)
    use_aerial_view = False

    def mj_viewer_headless_setup(self):
        """The reference's offscreen camera setup, called by ``record_policy``
        (``utils/visualize_env.py:115``) and by door / pen / relocate on every reset
        (``hammer_v0.py:161-165``, ``door_v0.py:146``, ``pen_v0.py:160-177``, ``relocate_v0.py:138``):
        builds the free camera of ``render.free_camera`` for this env's frame size (pen: from its
        'target' body, with ``use_aerial_view`` flipping the elevation).  Returns the camera record."""
        self.observer = self.vec.mj_viewer_headless_setup(
            self.width, self.height, aerial=self.env_id == "pen-v0" and bool(self.use_aerial_view))
        return self.observer

    # --- mjrl MujocoEnv members (inherited when mjrl is importable; mujoco-py is never created) ---
    @property
    def dt(self) -> float:
        """mjrl ``MujocoEnv.dt``: model timestep x frame_skip."""
        return float(self.model.opt["timestep"]) * self.frame_skip

    def state_vector(self):
        """mjrl ``MujocoEnv.state_vector``: concatenated qpos, qvel (fp64)."""
        qp, qv = self._qpos_qvel()
        return np.concatenate([qp, qv])

    def set_state(self, qpos, qvel):
        """mjrl ``MujocoEnv.set_state``: qpos / qvel with the current model parameters, then a
        forward pass (the next ``get_obs`` reflects the new state)."""
        self._set(qpos, qvel, self._params())

    def do_simulation(self, ctrl, n_frames):
        raise NotImplementedError(
            "do_simulation: the HIP step kernel runs frame_skip substeps of the task's own action "
            "scaling inside step(a); raw-ctrl stepping through mujoco-py is not part of the drop-in")

    def mj_viewer_setup(self):
        raise NotImplementedError("mj_viewer_setup: on-screen (GLFW) viewing is out of scope; use "
                                  "mj_viewer_headless_setup() + render()")

    def viewer_setup(self):
        raise NotImplementedError("viewer_setup: on-screen viewing is out of scope")

    def mj_render(self):
        raise NotImplementedError("mj_render: on-screen viewing is out of scope; use render()")

    def close(self):
        self.vec.close()


class HammerEnvV0(_AdroitEnv):
    """``hand_manipulation_suite/hammer_v0.py`` (obs 46, frame_skip 5, horizon 200)."""
    env_id = "hammer-v0"


class DoorEnvV0(_AdroitEnv):
    """``hand_manipulation_suite/door_v0.py`` (obs 39, frame_skip 1, horizon 200)."""
    env_id = "door-v0"


class PenEnvV0(_AdroitEnv):
    """``hand_manipulation_suite/pen_v0.py`` (obs 45, frame_skip 5, horizon 100, done on drop)."""
    env_id = "pen-v0"


class RelocateEnvV0(_AdroitEnv):
    """``hand_manipulation_suite/relocate_v0.py`` (obs 39, frame_skip 5, horizon 200).

    ``get_env_state`` takes object / palm / target positions from a fresh forward pass of the
    current state (the reference reads the previous forward's values, and returns live views of
    them; after ``reset`` or ``set_env_state`` they coincide).  ``set_env_state`` writes all of
    ``obj_pos`` -- the object's body_xpos, joint displacement included -- into the object's
    body_pos, and ``target_pos`` into the target site, as ``relocate_v0.py:118-129`` does.
    """
    env_id = "relocate-v0"

"""Batched counterparts of the reference's env plumbing.

* ``PixelObservationVecEnv`` -- ``utils/wrappers.py:32-76`` ``CustomPixelObservationWrapper``
  over N envs: ``obs_key`` selects ``"pixels"`` or ``"state"`` (``wrappers.py:9-10``), both kept
  (``pixels_only=False``, ``:35``) and readable with ``get_pixels`` / ``get_state``
  (``:72-76``); torch tensors out (``:55,70``); 5-tuple ``(obs, reward, terminated, truncated,
  info)`` (gym 0.26 ``StepAPICompatibility``, ``:34``); an ``action_repeat`` loop with the
  wrapper's ``timer`` and ``max_episode_length`` 200 (``:38-40,57-68``).
  Pixels: the reference renders a 64x64 RGB frame through OpenGL every step; here a pixel
  observation is the HIP ray caster's 64x64 metric depth frame ``[N, 1, H, W]`` from the same
  camera (``mj_envs_amd/render.py``), rendered only when pixels are asked for.
* ``SB3VecEnv`` -- the stable-baselines3 ``VecEnv`` method surface (``reset``, ``step_async`` /
  ``step_wait``, ``step``, ``get_attr`` / ``set_attr`` / ``env_method``, ``env_is_wrapped``,
  ``seed``, ``close``, ``num_envs``, spaces) without importing SB3; numpy out as SB3 expects
  (the reference's PPO baseline, ``algos/baselines.py:106-183``, wraps its one env in SB3's).
* ``make_env`` / ``step`` / ``reset`` -- ``utils/helpers.py:41-78``: ``state_type``
  ``"observation"`` -> pixels, ``"vector"`` -> state; ``step`` returns ``(obs, reward, done,
  success)`` with ``success = info['goal_achieved']``.

Documented differences from the reference wrapper:
  * ``action_repeat > 1`` raises TypeError in the reference (``items[1] += ...`` on a tuple,
    ``wrappers.py:68``).  Here it runs the intended loop per env: an extra repeat's reward is
    added unless the episode ended in the first step or in that repeat, or the timer passed
    ``max_episode_length`` (``:64``), after which the env's later repeats count for nothing.
    The batch keeps stepping, so an env that ended mid-loop was auto-reset by the kernel: its
    terminated / truncated flag is reported (the reference returns the first step's flags).
"""
from __future__ import annotations

from typing import Any, List, Optional, Sequence

import numpy as np

from .envs import AdroitVecEnv, Box

PIXELS_KEY = "pixels"
STATE_KEY = "state"


class PixelObservationVecEnv:
    """``CustomPixelObservationWrapper`` over an ``AdroitVecEnv`` (device tensors), or over a
    single-env facade (``HammerEnvV0`` ...; its batch of one is wrapped).  ``host_tensors=True``
    returns CPU float tensors and takes numpy / CPU actions, as the reference wrapper does
    (``wrappers.py:55,70-76``), so the reference's drivers -- ``record_policy``
    (``utils/visualize_env.py:108-128``): ``gym_env.env.mj_viewer_headless_setup()``,
    ``reset``, ``get_pixels().numpy()``, ``step(gym_env, a)`` -- run unchanged."""

    def __init__(self, env: AdroitVecEnv, obs_key: str = PIXELS_KEY, render_kwargs: Optional[dict] = None,
                 action_repeat: int = 1, host_tensors: bool = False):
        if obs_key not in (PIXELS_KEY, STATE_KEY):
            raise KeyError(obs_key)
        self._facade = None
        if not isinstance(env, AdroitVecEnv) and isinstance(getattr(env, "vec", None), AdroitVecEnv):
            self._facade = env                # its flags (pen's use_aerial_view) stay reachable
            env = env.vec                     # a single-env facade: wrap its batch of one
        self.host_tensors = bool(host_tensors)
        rk = render_kwargs or {}
        self.env = env
        self.num_envs = env.num_envs
        self.obs_key = obs_key
        self.width, self.height = int(rk.get("width", 64)), int(rk.get("height", 64))
        self.action_repeat = int(action_repeat)
        self.max_episode_length = 200          # wrappers.py:39 (hard-coded there too)
        import torch
        self.timer = torch.zeros(env.num_envs, dtype=torch.int32, device=env.sim.torch_device)
        self._pixels = None
        self._pixels_fresh = False
        self.action_space = env.action_space
        self.state_space = env.observation_space
        self.pixel_space = Box(0.0, np.inf, (1, self.height, self.width))
        self.observation_space = self.pixel_space if obs_key == PIXELS_KEY else self.state_space

    # --- observations --------------------------------------------------------------------
    def _out(self, t):
        return t.cpu().clone() if self.host_tensors else t

    def get_state(self):
        return self._out(self.env.obs)

    def get_pixels(self):
        if not self._pixels_fresh:
            if self._pixels is None:
                self._pixels = self.env.sim.empty(self.num_envs, 1, self.height, self.width)
            self.env.render_depth(self.width, self.height, out=self._pixels.view(self.num_envs, self.height,
                                                                                 self.width))
            self._pixels_fresh = True
        return self._out(self._pixels)

    def _obs(self):
        return self.get_pixels() if self.obs_key == PIXELS_KEY else self.get_state()

    def mj_viewer_headless_setup(self):
        """forwarded to the env, as gym's wrapper attribute lookup does for the reference; a wrapped
        single-env facade keeps its own flags (pen_v0.py:174-177 reads use_aerial_view)"""
        return self.env.mj_viewer_headless_setup(self.width, self.height)

    def _actions(self, actions):
        import torch
        if isinstance(actions, torch.Tensor) and actions.device == self.env.sim.torch_device:
            return actions
        a = torch.as_tensor(np.asarray(actions, np.float32) if not isinstance(actions, torch.Tensor)
                            else actions.float())
        return a.reshape(self.num_envs, -1).to(self.env.sim.torch_device)

    # --- episode control -----------------------------------------------------------------
    def reset(self, **kw):
        self.timer.zero_()
        self.env.reset(**kw)
        self._pixels_fresh = False
        return self._obs(), {}

    def step(self, actions):
        actions = self._actions(actions)
        obs, rew, term, trunc, info = self.env.step(actions)
        self._pixels_fresh = False
        reward = rew.clone()
        term, trunc = term.clone(), trunc.clone()
        info = dict(info)
        self.timer += 1
        if self.action_repeat > 1:
            # wrappers.py:62-68 per env: after each extra step, stop counting once the first
            # step or this one terminated or the timer passed max_episode_length
            live = ~(term | trunc)
            for _ in range(self.action_repeat - 1):
                _, r2, t2, u2, _ = self.env.step(actions)
                ended_now = (t2 | u2) & live     # the kernel auto-reset it: report the end
                term |= t2 & live
                trunc |= u2 & live
                live &= ~t2 & ~u2 & (self.timer <= self.max_episode_length)
                reward += r2 * live
                self.timer += live.int()
                live &= ~ended_now
            info["goal_achieved"] = self.env.goal.bool()
        ended = term | trunc
        self.timer.masked_fill_(ended, 0)       # the kernel auto-reset these envs
        if self.host_tensors:
            reward, term, trunc = reward.cpu(), term.cpu(), trunc.cpu()
            info = {k: (v.cpu() if hasattr(v, "cpu") else v) for k, v in info.items()}
        return self._obs(), reward, term, trunc, info

    def close(self):
        self.env.close()


class SB3VecEnv:
    """stable-baselines3 ``VecEnv`` surface over an ``AdroitVecEnv`` (numpy in / out)."""

    def __init__(self, env: AdroitVecEnv):
        self.env = env
        self.num_envs = env.num_envs
        self.observation_space = env.observation_space
        self.action_space = env.action_space
        self._actions = None
        import torch
        self._act = torch.zeros(env.num_envs, env.nu, device=env.sim.torch_device)

    def reset(self):
        return self.env.reset().cpu().numpy().copy()

    def step_async(self, actions):
        self._actions = np.asarray(actions, np.float32).reshape(self.num_envs, -1)

    def step_wait(self):
        import torch
        self._act.copy_(torch.from_numpy(self._actions))
        obs, rew, term, trunc, info = self.env.step(self._act)
        o = obs.cpu().numpy().copy()
        r = rew.cpu().numpy().copy()
        t, u = term.cpu().numpy(), trunc.cpu().numpy()
        g = info["goal_achieved"].cpu().numpy()
        ended = t | u
        tobs = info["terminal_obs"].cpu().numpy() if ended.any() else None
        infos: List[dict] = []
        for e in range(self.num_envs):
            d = {"goal_achieved": bool(g[e])}
            if ended[e]:
                d["terminal_observation"] = tobs[e].copy()
                d["TimeLimit.truncated"] = bool(u[e] and not t[e])
            infos.append(d)
        return o, r, ended, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def _idx(self, indices) -> Sequence[int]:
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return list(indices)

    def get_attr(self, attr_name: str, indices=None) -> List[Any]:
        v = getattr(self.env, attr_name)
        return [v for _ in self._idx(indices)]

    def set_attr(self, attr_name: str, value: Any, indices=None) -> None:
        setattr(self.env, attr_name, value)

    def env_method(self, method_name: str, *args, indices=None, **kwargs) -> List[Any]:
        fn = getattr(self.env, method_name)
        return [fn(*args, **kwargs) for _ in self._idx(indices)]

    def env_is_wrapped(self, wrapper_class, indices=None) -> List[bool]:
        return [False for _ in self._idx(indices)]

    def seed(self, seed: Optional[int] = None) -> List[Optional[int]]:
        if seed is not None:
            self.env.seed = int(seed)
        return [seed for _ in range(self.num_envs)]

    def close(self):
        self.env.close()


# ---------------------------------------------------------------------------------------
def make_env(config, num_envs: int = 1, device: int = 0):
    """``utils/helpers.py:56-78`` make_env for the Adroit suite, batched: ``config.env_name``,
    ``config.variation_type``, ``config.state_type`` ('observation' -> pixels, 'vector' ->
    state), ``config.nogui`` (False: the GUI wrapper, state tensors, no pixels)."""
    env = AdroitVecEnv(config.env_name, num_envs, device=device,
                       variation_type=getattr(config, "variation_type", None),
                       seed=int(getattr(config, "seed", 1) or 1))
    rk = dict(width=64, height=64)
    if not getattr(config, "nogui", True):
        return PixelObservationVecEnv(env, obs_key=STATE_KEY, render_kwargs=rk)
    st = getattr(config, "state_type", "vector")
    if st == "observation":
        return PixelObservationVecEnv(env, obs_key=PIXELS_KEY, render_kwargs=rk)
    if st == "vector":
        return PixelObservationVecEnv(env, obs_key=STATE_KEY, render_kwargs=rk)
    raise Exception(f"Unsupported state type '{st}'")


def reset(env):
    return env.reset()


def step(env, action):
    """``utils/helpers.py:44-54``: ``(obs, reward, done, success)``, success = goal_achieved."""
    obs, reward, term, trunc, info = env.step(action)
    return obs, reward, term, info["goal_achieved"]

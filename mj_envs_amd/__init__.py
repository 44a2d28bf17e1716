"""mj_envs_amd -- MI355X-native batched simulator for the Adroit hand_manipulation_suite.

Drop-in for the hot path of mj_envs_vision (env.step / reset / get_obs of hammer-v0,
door-v0, pen-v0, relocate-v0).  Registry mirrors mj_envs_vision/__init__.py:4-28.
"""
from .tasks import TASKS  # noqa: F401

__all__ = ["make", "register", "registry", "TASKS"]

registry = {}


def register(id: str, entry_point: str, max_episode_steps: int):
    registry[id] = dict(entry_point=entry_point, max_episode_steps=max_episode_steps)


# mj_envs_vision/__init__.py:4-28
register(id="door-v0", entry_point="mj_envs_amd.envs:DoorEnvV0", max_episode_steps=200)
register(id="hammer-v0", entry_point="mj_envs_amd.envs:HammerEnvV0", max_episode_steps=200)
register(id="pen-v0", entry_point="mj_envs_amd.envs:PenEnvV0", max_episode_steps=100)
register(id="relocate-v0", entry_point="mj_envs_amd.envs:RelocateEnvV0", max_episode_steps=200)


def make(id: str, **kwargs):
    import importlib
    spec = registry[id]
    mod, cls = spec["entry_point"].split(":")
    return getattr(importlib.import_module(mod), cls)(**kwargs)

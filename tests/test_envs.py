"""Gym-style facades (mj_envs_amd/envs.py): reference method set and semantics."""
import numpy as np
import pytest
import torch

from mj_envs_amd import make, registry
from mj_envs_amd.envs import Box, _evaluate_success
from mj_envs_amd.tasks import TASKS


def test_registry_matches_reference():
    # mj_envs_vision/__init__.py:4-28
    assert {k: v["max_episode_steps"] for k, v in registry.items()} == {
        "door-v0": 200, "hammer-v0": 200, "pen-v0": 100, "relocate-v0": 200}


def test_evaluate_success_thresholds():
    # hammer_v0.py:167-175 (> 25 goal steps), pen_v0.py:180-188 (> 20)
    p = lambda k: {"env_infos": {"goal_achieved": np.array([1] * k + [0] * (100 - k))}}
    assert _evaluate_success("hammer-v0", [p(25), p(26)]) == 50.0
    assert _evaluate_success("pen-v0", [p(21), p(20), p(0), p(99)]) == 50.0
    assert _evaluate_success("door-v0", []) == 0.0


def test_box():
    b = Box(-1.0, 1.0, (26,))
    x = b.sample(np.random.default_rng(0))
    assert x.shape == (26,) and x.dtype == np.float32 and b.contains(x)
    assert not b.contains(np.full(26, 2.0, np.float32))


@pytest.mark.gpu
@pytest.mark.parametrize("env_id", list(TASKS))
def test_single_env_api(env_id):
    env = make(env_id)
    spec = TASKS[env_id]
    obs, info = env.reset()
    assert obs.shape == (spec.obs_dim,) and obs.dtype == np.float32 and info == {}
    assert env.frame_skip == spec.frame_skip
    assert env.action_space.shape == (spec.nu,)
    rng = np.random.default_rng(0)
    for _ in range(3):
        o, r, d, inf = env.step(rng.uniform(-1, 1, spec.nu))
        assert o.shape == (spec.obs_dim,) and np.isfinite(o).all()
        assert isinstance(r, float) and isinstance(d, bool) and set(inf) == {"goal_achieved"}
    np.testing.assert_array_equal(env.get_obs(), o)
    assert env.unwrapped is env
    env.close()


@pytest.mark.gpu
@pytest.mark.parametrize("env_id", list(TASKS))
def test_env_state_roundtrip(env_id):
    env = make(env_id)
    env.reset(seed=3)
    rng = np.random.default_rng(1)
    for _ in range(5):
        env.step(rng.uniform(-1, 1, env.action_space.shape[0]))
    st = env.get_env_state()
    acts = rng.uniform(-1, 1, (3, env.action_space.shape[0]))
    ref = [env.step(a)[0] for a in acts]
    env.reset(seed=9)                      # different model params
    env.set_env_state(st)
    again = [env.step(a)[0] for a in acts]
    # warm start is not part of the reference's env state, so the Newton solve restarts
    # from a different point: same solution to solver tolerance
    for a, b in zip(ref, again):
        np.testing.assert_allclose(a, b, rtol=2e-3, atol=2e-3)
    st2 = env.get_env_state()
    assert set(st2) == set(st)
    env.close()


@pytest.mark.gpu
def test_vec_env_autoreset_and_stats():
    from mj_envs_amd.envs import AdroitVecEnv
    n = 256
    venv = AdroitVecEnv("pen-v0", n, seed=5)
    obs = venv.reset()
    assert obs.shape == (n, 45)
    act = torch.empty(n, venv.nu, device=obs.device)
    any_trunc = False
    for k in range(venv.horizon):
        venv.random_actions(act, k)
        obs, rew, term, trunc, info = venv.step(act)
        any_trunc |= bool(trunc.any())
        assert torch.isfinite(obs).all() and torch.isfinite(rew).all()
        assert torch.isfinite(info["terminal_obs"][term | trunc]).all()
    assert any_trunc                      # horizon 100 reached inside the loop
    st = venv.episode_stats()
    assert int(st["episodes"].min()) >= 1
    assert int(st["last_len"].max()) <= venv.horizon
    venv.close()

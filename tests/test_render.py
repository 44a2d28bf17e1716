"""Depth-camera observations: camera construction, the numpy checker on
analytic scenes (CPU), and the HIP ray caster against the checker on the fp64 oracle's
kinematics (GPU).

Parity is unpinned against the reference (it renders RGB through OpenGL,
headless_observer.py:34-52); the GPU kernel is held to the geometry: >= 99.5 % of pixels
within 2e-3 m of the fp64 checker (the rest are silhouette pixels whose ray grazes a geom edge
and may flip between two surfaces in fp32).
"""
import numpy as np
import pytest

from conftest import ENVS, make_oracle


def test_camera_record():
    from mj_envs_amd.render import CAM_FLOATS, free_camera
    from mj_envs_amd.tasks import load_model
    for env_id in ENVS:
        c = free_camera(load_model(env_id), env_id).astype(np.float64)
        assert c.shape == (CAM_FLOATS,)
        fwd, up, right = c[3:6], c[6:9], c[9:12]
        for v in (fwd, up, right):
            assert abs(np.linalg.norm(v) - 1) < 1e-6
        assert abs(fwd @ up) < 1e-6 and abs(fwd @ right) < 1e-6
        # headless_observer.py:27-28: azimuth 90 -> the camera looks along +y from distance 4.5
        assert abs(fwd[0]) < 1e-6
        # the 64x64 grid spans the centred 128x128 crop of a 640x480, fovy-45 frame
        ty = np.tan(np.radians(22.5))
        assert np.isclose(c[13] * 64, 2 * 128 / 480 * ty, rtol=1e-5)    # du (square pixels)
        assert np.isclose(c[12] + c[13] * 31.5, 0.0, atol=1e-6)          # centred
        assert np.isclose(c[14] - c[15] * 31.5, 0.0, atol=1e-6)


def test_camera_aerial_view():
    """set_view('aerial') (headless_observer.py:62-63; pen's use_aerial_view, pen_v0.py:174-175):
    elevation -45 - d/2 instead of -45 + d/2, same azimuth, distance and look-at point."""
    from mj_envs_amd.render import free_camera
    from mj_envs_amd.tasks import load_model
    m = load_model("pen-v0")
    c0 = free_camera(m, "pen-v0").astype(np.float64)
    c1 = free_camera(m, "pen-v0", aerial=True).astype(np.float64)
    el0, el1 = np.degrees(np.arcsin(c0[5])), np.degrees(np.arcsin(c1[5]))
    assert np.isclose(el0 + el1, -90.0, atol=1e-3) and not np.isclose(el0, el1)
    look0, look1 = c0[:3] + 4.5 * c0[3:6], c1[:3] + 4.5 * c1[3:6]
    assert np.allclose(look0, look1, atol=1e-5)


def test_checker_analytic():
    """numpy checker on shapes with closed-form depth"""
    from oracle.depth import render_depth
    cam = np.array([0, -5, 0, 0, 1, 0, 0, 0, 1, 1, 0, 0, -0.1, 0.2 / 9, 0.1, 0.2 / 9, 10.0])
    eye = np.eye(3)
    # sphere radius 0.5 at the origin: centre pixel depth 4.5
    d = render_depth(cam, 10, 10, [(2, [0.5, 0, 0], np.zeros(3), eye)])
    assert abs(d[4:6, 4:6].min() - 4.5) < 0.02
    # box half-size 0.3 at the origin: front face at y = -0.3 -> depth 4.7 everywhere it is hit
    d = render_depth(cam, 10, 10, [(6, [0.3, 0.3, 0.3], np.zeros(3), eye)])
    hit = d < 10
    assert hit.any() and np.allclose(d[hit], 4.7)
    # capsule along z (r 0.2, half-length 0.5): z-depth of the lateral surface near the axis
    d = render_depth(cam, 10, 10, [(3, [0.2, 0.5, 0], np.zeros(3), eye)])
    assert abs(d.min() - 4.8) < 0.01
    # cylinder seen end-on from above: cap at z = 0.4 for a camera looking down -z
    cam2 = np.array([0, 0, 5, 0, 0, -1, 0, 1, 0, -1, 0, 0, -0.1, 0.2 / 9, 0.1, 0.2 / 9, 10.0])
    d = render_depth(cam2, 10, 10, [(5, [0.3, 0.4, 0], np.zeros(3), eye)])
    assert np.allclose(d[4:6, 4:6], 4.6)
    # finite plane: misses outside its half-size
    d = render_depth(cam2, 10, 10, [(0, [0.05, 0.05, 0], np.zeros(3), eye)])
    assert (d < 10).sum() < 10 and np.allclose(d[d < 10], 5.0)
    # nearest of two geoms wins
    d = render_depth(cam, 10, 10, [(6, [0.3, 0.3, 0.3], np.zeros(3), eye),
                                   (2, [0.1, 0, 0], np.array([0, -1.0, 0]), eye)])
    assert abs(d.min() - 3.9) < 0.05 and d.min() < 4.7


@pytest.mark.gpu
@pytest.mark.parametrize("env_id", ENVS)
def test_gpu_depth_vs_checker(env_id):
    """BASELINE config 5's depth path on every task: 16 envs after 6 random steps (pen's camera
    elevation comes from its 'target' body, pen_v0.py:163-177; door / relocate from body 0)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mj_envs_amd import _native
    from mj_envs_amd.render import free_camera
    from mj_envs_amd.tasks import attach_task, load_model
    from oracle.depth import oracle_geoms, render_depth
    m, orc = make_oracle(env_id)
    n, W, H = 16, 64, 64
    sim = _native.Sim(m.to_blob(), n)
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, seed=3)
    act = sim.empty(n, sim.nu)
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    for k in range(6):                      # move away from the rest pose
        sim.random_actions(act, 7, k)
        sim.step(act, obs, rew, done, goal)
    cam = free_camera(m, env_id, W, H)
    depth = sim.empty(n, H, W)
    sim.render_depth(depth, cam)
    qpos, qvel = sim.empty(n, sim.nq), sim.empty(n, sim.nv)
    params = sim.empty(n, max(sim.nparam, 1))
    sim.get_state(qpos, qvel, None, params if sim.nparam else None)
    torch.cuda.synchronize()
    D = depth.cpu().numpy()
    assert np.isfinite(D).all()
    for e in range(n):
        p = params[e].cpu().numpy().astype(np.float64)[: sim.nparam]
        orc.forward1(p, qpos[e].cpu().numpy().astype(np.float64), qvel[e].cpu().numpy().astype(np.float64))
        R = render_depth(cam, W, H, oracle_geoms(orc, m))
        ok = np.abs(D[e] - R) <= 2e-3
        assert ok.mean() >= 0.995, (env_id, e, ok.mean(), np.abs(D[e] - R).max())
        assert (D[e] < cam[16]).mean() > 0.5      # the scene fills the frame


@pytest.mark.gpu
def test_gpu_depth_config5_size():
    """BASELINE config 5 at its own size (hammer-v0 + 64x64 depth, 8 192 envs): a 60-step random
    rollout with auto-reset from staggered episode phases (the bench's regime), then the depth frames
    of 64 envs sampled evenly across the whole batch against the fp64 checker."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mj_envs_amd import _native
    from mj_envs_amd.render import free_camera
    from oracle.depth import oracle_geoms, render_depth
    env_id, n, W, H, steps = "hammer-v0", 8192, 64, 64, 60
    m, orc = make_oracle(env_id)
    sim = _native.Sim(m.to_blob(), n)
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, seed=11)
    sim.set_episode(ep_len=torch.from_numpy((np.arange(n) * 7919 % sim.horizon).astype(np.int32)).cuda())
    act = sim.empty(n, sim.nu)
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    cam = free_camera(m, env_id, W, H)
    depth = sim.empty(n, H, W)
    for k in range(steps):
        sim.random_actions(act, 13, k)
        sim.step(act, obs, rew, done, goal, autoreset=True, seed=11)
        sim.render_depth(depth, cam)          # every env-step, as bench.py --depth times it
    qpos, qvel = sim.empty(n, sim.nq), sim.empty(n, sim.nv)
    params = sim.empty(n, sim.nparam)
    sim.get_state(qpos, qvel, None, params)
    torch.cuda.synchronize()
    idx = np.unique(np.linspace(0, n - 1, 64).round().astype(int))
    D = depth.cpu().numpy()[idx]
    assert np.isfinite(D).all()
    Q, V, Pm = (x.cpu().numpy().astype(np.float64)[idx] for x in (qpos, qvel, params))
    fr = []
    for j in range(len(idx)):
        orc.forward1(Pm[j], Q[j], V[j])
        R = render_depth(cam, W, H, oracle_geoms(orc, m))
        ok = np.abs(D[j] - R) <= 2e-3
        fr.append(ok.mean())
        assert ok.mean() >= 0.995, (int(idx[j]), ok.mean(), np.abs(D[j] - R).max())
        assert (D[j] < cam[16]).mean() > 0.5
    print(f"config 5 depth: {len(idx)} envs of {n}, pixels within 2e-3 m: min {min(fr):.4f}, mean {np.mean(fr):.4f}")

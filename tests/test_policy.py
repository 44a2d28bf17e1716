"""On-device Gaussian MLP policy against a numpy restatement of mjrl's
FCNetwork forward pass.  Tolerance (fp32 kernel vs fp64 numpy): |err| <= 1e-5 + 1e-5|ref|.
Exploration noise: exp(log_std) * N(0, 1), checked by its sample moments."""
import numpy as np
import pytest


def np_forward(pol, obs):
    x = (np.asarray(obs, np.float64) - pol.in_shift) / (pol.in_scale + 1e-8)
    (W0, b0), (W1, b1), (W2, b2) = pol.weights
    h = np.tanh(x @ W0.T + b0)
    h = np.tanh(h @ W1.T + b1)
    return (h @ W2.T + b2) * pol.out_scale + pol.out_shift


def test_init_semantics(monkeypatch):
    from mj_envs_amd.policy import GaussianMLP
    monkeypatch.setattr(GaussianMLP, "upload", lambda self: None)
    a = GaussianMLP(46, 26, (32, 32), init_log_std=-1.0, seed=3)
    b = GaussianMLP(46, 26, (32, 32), init_log_std=-1.0, seed=3)
    for (wa, ba), (wb, bb) in zip(a.weights, b.weights):
        assert np.array_equal(wa, wb) and np.array_equal(ba, bb)      # seeded like mjrl
    W2, b2 = a.weights[-1]
    W0, _ = a.weights[0]
    assert np.abs(W2).max() <= 1e-2 / np.sqrt(32) + 1e-9              # last layer scaled by 1e-2
    assert np.abs(W0).max() <= 1 / np.sqrt(46) + 1e-9                 # nn.Linear default init bound
    assert np.all(a.log_std == -1.0)
    flat = a.flat_params()
    assert flat.size == 2 * 46 + 32 * 46 + 32 + 32 * 32 + 32 + 26 * 32 + 4 * 26
    with pytest.raises(ValueError):
        GaussianMLP(46, 26, (32, 16))


@pytest.mark.gpu
def test_gpu_mlp_mean_and_noise():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mj_envs_amd.policy import GaussianMLP
    for (od, ad, hid) in [(46, 26, 32), (39, 28, 32), (45, 24, 64)]:
        pol = GaussianMLP(od, ad, (hid, hid), init_log_std=-1.0, seed=1)
        # non-trivial transforms
        rng = np.random.default_rng(0)
        pol.in_shift = rng.normal(size=od)
        pol.in_scale = rng.uniform(0.5, 2, size=od)
        pol.out_shift = rng.normal(size=ad) * 0.1
        pol.out_scale = rng.uniform(0.5, 2, size=ad)
        pol.weights[-1] = (pol.weights[-1][0] * 100, pol.weights[-1][1] * 100)   # O(1) outputs
        pol.upload()
        obs = rng.normal(size=(2000, od)).astype(np.float32)
        ot = torch.tensor(obs, device="cuda")
        mean = pol.act(ot).cpu().numpy()
        ref = np_forward(pol, obs)
        np.testing.assert_allclose(mean, ref, rtol=1e-5, atol=1e-5)
        s1 = pol.act(ot, sample=True, seed=5, step=9).cpu().numpy()
        s2 = pol.act(ot, sample=True, seed=5, step=9).cpu().numpy()
        s3 = pol.act(ot, sample=True, seed=5, step=10).cpu().numpy()
        assert np.array_equal(s1, s2) and not np.array_equal(s1, s3)
        z = (s1 - mean) / np.exp(pol.log_std)
        assert abs(z.mean()) < 0.02 and abs(z.std() - 1) < 0.02


@pytest.mark.gpu
def test_gpu_closed_loop_hammer():
    """policy -> step on device for a full episode: finite, no faults, auto-reset bookkeeping"""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from mj_envs_amd import _native
    from mj_envs_amd.policy import GaussianMLP
    from mj_envs_amd.tasks import attach_task, load_model
    m = attach_task(load_model("hammer-v0"), "hammer-v0")
    n = 256
    sim = _native.Sim(m.to_blob(), n)
    pol = GaussianMLP(sim.obs_dim, sim.nu, (32, 32), init_log_std=-1.0, seed=0)
    obs = sim.empty(n, sim.obs_dim)
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    act = sim.empty(n, sim.nu)
    sim.reset(obs, seed=2)
    for k in range(sim.horizon):
        pol.act(obs, out=act, sample=True, seed=1, step=k)
        sim.step(act, obs, rew, done, goal, autoreset=True, seed=2)
    flags = sim.empty(n, dtype=torch.int32)
    sim.status(sticky=flags)
    eps = sim.empty(n, dtype=torch.int32)
    sim.episode_stats(episodes=eps)
    torch.cuda.synchronize()
    assert torch.isfinite(obs).all()
    assert (flags.cpu().numpy() == 0).all()        # no bad state, no capacity overflow
    assert (eps.cpu().numpy() == 1).all()          # every env finished exactly one episode

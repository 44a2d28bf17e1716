"""Closed-loop, shard and fault-path tests of the HIP simulator (GPU box).

* DAPG behavioural pin: the reference's pretrained DAPG policies
  (``algos/dapg_pretrained/*.pickle`` -> ``tests/golden/dapg_*.npz``, extracted without
  unpickling by ``tests/golden/make_dapg.py``; queried as ``algos/baselines.py:82-86`` does,
  the mean action) drive 1 024 envs per task for one horizon through ``k_mlp`` + ``k_step``.
  The same first 64 (params, policy) episodes run on the fp64 oracle at MuJoCo's capacities
  (nconmax 100 / njmax 500).  GPU and oracle success rates (``evaluate_success``) must agree
  within a binomial bound, hammer / pen / relocate must succeed (DAPG's published regime), and
  no env may raise a contact / constraint overflow.  door-v0 fails in both: the reference runs it
  at frame_skip 1 (``door_v0.py:10``), 5x finer than the policy was trained at.
* Shards: one batch of N envs vs two shards of N/2 with global env
  offsets, bit for bit over 250 steps with auto-reset.
* Fault path: a NaN qvel injected through ``aw_set_state`` raises AW_ST_BADQVEL
  and resets the env as MuJoCo's mj_checkVel does, matching the oracle.
"""
import os

import numpy as np
import pytest

from conftest import ENVS, GOLDEN, make_oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _t(a, dtype=None):
    return torch.tensor(np.asarray(a), dtype=dtype or torch.float32, device="cuda")


def _sim(env_id, n, variation=None, env_offset=0):
    from mj_envs_amd import _native
    from mj_envs_amd.tasks import attach_task, load_model
    m = attach_task(load_model(env_id), env_id, variation)
    return m, _native.Sim(m.to_blob(), n, env_offset=env_offset)


def _bufs(sim, n):
    return (sim.empty(n, sim.obs_dim), sim.empty(n), sim.empty(n, dtype=torch.uint8),
            sim.empty(n, dtype=torch.uint8))


def _sticky(sim, n):
    st = sim.empty(n, dtype=torch.int32)
    sim.status(sticky=st)
    torch.cuda.synchronize()
    return st.cpu().numpy()


# --------------------------------------------------------------------------------------------
# expected success (%) of the pretrained policies in this physics (oracle, 32 envs,
# profiles/dapg_oracle_*.json): the band the GPU rate must also fall in
DAPG_MIN_SUCCESS = {"hammer-v0": 90.0, "pen-v0": 80.0, "relocate-v0": 90.0}


@pytest.mark.parametrize("env_id", ENVS)
def test_dapg_closed_loop_success(env_id):
    from mj_envs_amd import _native
    from mj_envs_amd.policy import GaussianMLP
    from mj_envs_amd.tasks import TASKS
    spec = TASKS[env_id]
    n, n_orc = 1024, 64
    m, sim = _sim(env_id, n)
    pol = GaussianMLP.from_npz(os.path.join(GOLDEN, f"dapg_{env_id.split('-')[0]}.npz"))
    obs, rew, done, goal = _bufs(sim, n)
    act = sim.empty(n, sim.nu)
    sim.reset(obs, seed=123)
    params = sim.empty(n, sim.nparam)
    sim.get_state(params=params)
    # k_mlp mean vs the fp64 host forward on the reset observations
    pol.act(obs, out=act)
    torch.cuda.synchronize()
    np.testing.assert_allclose(act.cpu().numpy(), pol.mean_np(obs.cpu().numpy()), rtol=1e-4, atol=1e-4)
    goals = torch.zeros(n, dtype=torch.int32, device="cuda")
    alive = torch.ones(n, dtype=torch.bool, device="cuda")
    for _ in range(spec.horizon):
        pol.act(obs, out=act)
        sim.step(act, obs, rew, done, goal)
        goals += (goal.bool() & alive).int()
        alive &= (done & 1) == 0           # pen: the episode ends at done (wrappers / trainers)
    g = goals.cpu().numpy()
    succ_gpu = 100.0 * np.mean(g > spec.success_steps)
    st = _sticky(sim, n)
    assert not (st & _native.ST_OVERFLOW).any(), f"{int(((st & _native.ST_OVERFLOW) != 0).sum())} envs overflowed"
    # the oracle on the first n_orc episodes (same params, same policy, fp64, MuJoCo's caps)
    _, o = make_oracle(env_id)
    P = params.cpu().numpy()[:n_orc].astype(np.float64)
    ost, oobs = o.reset(P)
    og = np.zeros(n_orc, int)
    oalive = np.ones(n_orc, bool)
    ostatus = np.zeros(n_orc, np.uint32)
    for _ in range(spec.horizon):
        oobs, _, od, ogl, ostt = o.step(ost, pol.mean_np(oobs), nthreads=8)
        ostatus |= ostt
        og += ogl & oalive
        oalive &= ~od
    succ_orc = 100.0 * np.mean(og > spec.success_steps)
    assert not (ostatus & 24).any()
    same = np.mean((g[:n_orc] > spec.success_steps) == (og > spec.success_steps))
    print(f"DAPG {env_id}: success GPU {succ_gpu:.1f} % ({n} envs), oracle {succ_orc:.1f} % ({n_orc} envs), "
          f"same outcome on {100 * same:.1f} % of the shared episodes, mean goal steps GPU {g.mean():.1f} "
          f"oracle {og.mean():.1f}")
    p = max(min((succ_gpu + succ_orc) / 200.0, 1 - 1e-3), 1e-3)
    bound = 100.0 * (3.0 * np.sqrt(p * (1 - p) * (1.0 / n + 1.0 / n_orc)) + 0.03)
    assert abs(succ_gpu - succ_orc) <= bound, (succ_gpu, succ_orc, bound)
    if env_id in DAPG_MIN_SUCCESS:
        assert succ_gpu >= DAPG_MIN_SUCCESS[env_id] and succ_orc >= DAPG_MIN_SUCCESS[env_id]
    else:   # door-v0 at the reference's frame_skip 1
        assert succ_gpu <= 10.0 and succ_orc <= 10.0


# --------------------------------------------------------------------------------------------
@pytest.mark.parametrize("env_id", ["hammer-v0", "pen-v0"])
def test_shards_bitwise_equal_to_one_batch(env_id):
    """shards keyed by the global env id reproduce one batch bit for bit."""
    n, steps, seed = 256, 250, 77
    _, full = _sim(env_id, n)
    _, s0 = _sim(env_id, n // 2, env_offset=0)
    _, s1 = _sim(env_id, n // 2, env_offset=n // 2)
    outs = []
    for sims in ([full], [s0, s1]):
        bufs = [(s, *_bufs(s, s.n_envs), s.empty(s.n_envs, s.nu)) for s in sims]
        for s, obs, *_ in bufs:
            s.reset(obs, seed=seed)
        acc = []
        for k in range(steps):
            for s, obs, rew, done, goal, act in bufs:
                s.random_actions(act, 5, k)
                s.step(act, obs, rew, done, goal, autoreset=True, seed=seed)
            acc.append(torch.cat([b[2] for b in bufs]).clone())
        obs = torch.cat([b[1] for b in bufs])
        ep = [s.empty(s.n_envs, dtype=torch.int32) for s in sims]
        ret = [s.empty(s.n_envs) for s in sims]
        for s, e, r in zip(sims, ep, ret):
            s.episode_totals(episodes=e, sum_return=r)
        torch.cuda.synchronize()
        outs.append((obs, torch.stack(acc), torch.cat(ep), torch.cat(ret)))
    (o1, r1, e1, t1), (o2, r2, e2, t2) = outs
    assert int(e1.min()) >= 1                   # every env finished at least one episode
    assert torch.equal(o1, o2) and torch.equal(r1, r2) and torch.equal(e1, e2) and torch.equal(t1, t2)


@pytest.mark.parametrize("n", [2049, 6149, 16387])
def test_persistent_claims_cover_every_env_once(n):
    """k_step's persistent grid hands envs out in XCD-contiguous ranges with per-class counters
    and stealing (adroit_wave.hip claim_env): with env counts that split unevenly over the eight
    classes, every env is stepped exactly once per launch (ep_len) and the states equal, bit for
    bit, a launch with one workgroup per env (AW_STEP_GRID=0) and one with an odd grid of 1 001
    workgroups on the single-counter path."""
    steps, seed = 3, 11
    res = []
    for grid in (None, "0", "1001"):
        old = os.environ.pop("AW_STEP_GRID", None)
        if grid is not None:
            os.environ["AW_STEP_GRID"] = grid
        try:
            _, s = _sim("hammer-v0", n)
        finally:
            os.environ.pop("AW_STEP_GRID", None)
            if old is not None:
                os.environ["AW_STEP_GRID"] = old
        obs, rew, done, goal = _bufs(s, n)
        act = s.empty(n, s.nu)
        s.reset(obs, seed=seed)
        for k in range(steps):
            s.random_actions(act, 9, k)
            s.step(act, obs, rew, done, goal, autoreset=False, seed=seed)
        ep_len = s.empty(n, dtype=torch.int32)
        s.get_episode(ep_len=ep_len)
        qpos = s.empty(n, s.nq)
        s.get_state(qpos=qpos)
        torch.cuda.synchronize()
        assert torch.all(ep_len == steps), f"grid {grid}: env step counts {torch.unique(ep_len).tolist()}"
        res.append((obs.clone(), qpos.clone(), rew.clone()))
    for o, q, r in res[1:]:
        assert torch.equal(o, res[0][0]) and torch.equal(q, res[0][1]) and torch.equal(r, res[0][2])


def test_global_offset_changes_streams():
    """Envs at different global ids draw different resets / actions (the offset is live)."""
    _, a = _sim("relocate-v0", 64, env_offset=0)
    _, b = _sim("relocate-v0", 64, env_offset=64)
    pa, pb = a.empty(64, a.nparam), b.empty(64, b.nparam)
    for s, p in ((a, pa), (b, pb)):
        o = s.empty(64, s.obs_dim)
        s.reset(o, seed=3)
        s.get_state(params=p)
    xa, xb = a.empty(64, a.nu), b.empty(64, b.nu)
    a.random_actions(xa, 1, 0)
    b.random_actions(xb, 1, 0)
    torch.cuda.synchronize()
    assert not torch.equal(pa, pb) and not torch.equal(xa, xb)


def test_checkpoint_resume_bitwise():
    """The checkpoint contract of include/adroit_wave.h: aw_get_state + aw_get_episode +
    aw_episode_totals saved mid-run and restored into a NEW handle (aw_set_state, aw_set_episode,
    aw_set_episode_totals) continue the run bit for bit -- auto-resets (Philox keyed by the
    finished-episode count) and the running totals (count, summed return, successes) included."""
    env_id, n, seed = "pen-v0", 128, 31
    _, a = _sim(env_id, n)
    _, b = _sim(env_id, n)
    act = a.empty(n, a.nu)
    bufs_a, bufs_b = _bufs(a, n), _bufs(b, n)
    a.reset(bufs_a[0], seed=seed)

    def run(s, bufs, k0, k1):
        for k in range(k0, k1):
            s.random_actions(act, 9, k)
            s.step(act, *bufs, autoreset=True, seed=seed)

    def totals(s):
        e, r, c = s.empty(n, dtype=torch.int32), s.empty(n), s.empty(n, dtype=torch.int32)
        s.episode_totals(e, r, c)
        return e, r, c

    run(a, bufs_a, 0, 150)                       # pen horizon 100: every env has reset once
    q, v, w, p = a.empty(n, a.nq), a.empty(n, a.nv), a.empty(n, a.nv), a.empty(n, a.nparam)
    a.get_state(q, v, w, p)
    el, er, eg = a.empty(n, dtype=torch.int32), a.empty(n), a.empty(n, dtype=torch.int32)
    a.get_episode(el, er, eg)
    te, tr, ts = totals(a)
    b.set_state(q, v, w, p, obs=bufs_b[0])
    b.set_episode(el, er, eg)
    b.set_episode_totals(te, tr, ts)
    run(a, bufs_a, 150, 320)
    run(b, bufs_b, 150, 320)
    ta, tb = totals(a), totals(b)
    torch.cuda.synchronize()
    assert int(te.min()) >= 1 and int(ta[0].min()) >= 3
    assert torch.equal(bufs_a[0], bufs_b[0])
    for x, y in zip(ta, tb):
        assert torch.equal(x, y)


# --------------------------------------------------------------------------------------------
@pytest.mark.parametrize("field", ["qvel", "qpos"])
def test_nan_state_flags_and_resets_like_oracle(field):
    """mj_checkPos / mj_checkVel: a bad state raises the flag, the env restarts from
    qpos0 with zero velocity and zero ctrl for the rest of the env-step -- as the oracle."""
    from mj_envs_amd import _native
    from mj_envs_amd.tasks import sample_params
    env_id, n = "hammer-v0", 8
    m, o = make_oracle(env_id)
    P = sample_params(env_id, m, np.random.default_rng(2), n).astype(np.float32).astype(np.float64)
    st, _ = o.reset(P)
    rng = np.random.default_rng(3)
    for _ in range(5):
        o.step(st, rng.uniform(-1, 1, (n, o.nu)), nthreads=8)
    for k in ("qpos", "qvel", "warm"):   # the GPU's fp32 state, for both sides
        st[k] = st[k].astype(np.float32).astype(np.float64)
    bad = [1, 5]
    for e in bad:
        st[field][e, 3] = np.nan
    _, sim = _sim(env_id, n)
    sim.set_state(_t(st["qpos"]), _t(st["qvel"]), _t(st["warm"]), _t(P))
    sim.clear_status()
    act = rng.uniform(-1, 1, (n, sim.nu))
    obs, rew, done, goal = _bufs(sim, n)
    sim.step(_t(act), obs, rew, done, goal)
    last = sim.empty(n, dtype=torch.int32)
    sim.status(last=last)
    q, v = sim.empty(n, sim.nq), sim.empty(n, sim.nv)
    sim.get_state(q, v)
    torch.cuda.synchronize()
    o_ref, r_ref, _, _, ost = o.step(st, act, nthreads=8)
    flag = _native.ST_BADQVEL if field == "qvel" else _native.ST_BADQPOS
    fl = last.cpu().numpy()
    for e in range(n):
        assert bool(fl[e] & flag) == (e in bad) == bool(ost[e] & flag), (e, fl[e], ost[e])
    q, v = q.cpu().numpy(), v.cpu().numpy()
    assert np.isfinite(q).all() and np.isfinite(v).all()
    okq = np.abs(q - st["qpos"]) <= 2e-5 + 1e-5 * np.abs(st["qpos"])
    okv = np.abs(v - st["qvel"]) <= 5e-3 * (1 + np.abs(st["qvel"]))
    assert okq[bad].all() and okv[bad].all()
    np.testing.assert_allclose(rew.cpu().numpy()[bad], r_ref[bad], rtol=1e-3, atol=1e-3)


# --------------------------------------------------------------------------------------------
# steps of the config-4 run at which sampled envs are teacher-forced against the oracle
C4_CHECK = (0, 50, 100, 150, 205)


def test_config4_262144_envs_one_gpu_properties():
    """BASELINE config 4 (hammer, 262 144 envs; 8 x 32 768 per GPU) on one GPU over 210 env-steps,
    across the horizon-200 auto-reset: the rank-3 shard (offset 98 304) agrees bit for bit with the
    262 144-env handle on its envs at EVERY step (obs, reward, done); all outputs finite; no env drops
    a constraint MuJoCo keeps; and at five steps 64 envs sampled across the whole batch are
    teacher-forced against the oracle (one-step tolerance, misses classified)."""
    from mj_envs_amd import _native
    from test_gpu_parity import ONE_STEP_MIN, _classify_misses, _hard_cap, _state_err
    env_id, n, per, steps = "hammer-v0", 262144, 32768, 210
    _, o = make_oracle(env_id)
    _, full = _sim(env_id, n)
    _, shard = _sim(env_id, per, env_offset=3 * per)
    bf, bs = _bufs(full, n), _bufs(shard, per)
    af, ash = full.empty(n, full.nu), shard.empty(per, shard.nu)
    full.reset(bf[0], seed=4)
    shard.reset(bs[0], seed=4)
    full.clear_status()
    idx = np.unique(np.linspace(0, n - 1, 64).round().astype(int))
    ti = torch.from_numpy(idx).cuda()
    q, v, w, p = full.empty(n, full.nq), full.empty(n, full.nv), full.empty(n, full.nv), full.empty(n, full.nparam)
    oks, eqs, evs, misses, n_done = [], [], [], [], 0
    for k in range(steps):
        if k in C4_CHECK:
            full.get_state(q, v, w, p)
            pre = dict(qpos=q[ti].cpu().numpy().astype(np.float64), qvel=v[ti].cpu().numpy().astype(np.float64),
                       warm=w[ti].cpu().numpy().astype(np.float64), params=p[ti].cpu().numpy().astype(np.float64))
        full.random_actions(af, 9, k)
        shard.random_actions(ash, 9, k)
        full.step(af, *bf, autoreset=True, seed=4)
        shard.step(ash, *bs, autoreset=True, seed=4)
        for a, b in zip(bf[:3], bs[:3]):
            assert torch.equal(a[3 * per:4 * per], b), f"shard differs from the full batch at step {k}"
        n_done += int((bf[2] != 0).sum())   # done = terminated | truncated << 1
        if k in C4_CHECK:
            full.get_state(q, v)
            dn = bf[2][ti].cpu().numpy()
            sel = np.nonzero(dn == 0)[0]   # an env whose episode ended holds the new episode's state
            a = af[ti].cpu().numpy().astype(np.float64)[sel]
            st = {key: val[sel].copy() for key, val in pre.items()}
            _, _, _, _, ost = o.step(st, a, nthreads=8)
            assert not (np.bitwise_or.reduce(ost) & 24), "oracle dropped constraints at MuJoCo's caps"
            qg, vg = q[ti].cpu().numpy()[sel], v[ti].cpu().numpy()[sel]
            eq, ev, okk = _state_err(qg, vg, st["qpos"], st["qvel"])
            oks.append(okk)
            eqs.append(eq)
            evs.append(ev)
            misses += [(k, int(idx[sel[j]]), st["params"][j], st["qpos"][j], st["qvel"][j], st["warm"][j], a[j],
                        qg[j].astype(np.float64), vg[j].astype(np.float64)) for j in np.where(~okk)[0]]
    torch.cuda.synchronize()
    assert bool(torch.isfinite(bf[0]).all()) and bool(torch.isfinite(bf[1]).all())
    assert n_done >= n, f"the run crossed no horizon boundary ({n_done} episode ends)"
    sticky = _sticky(full, n)
    n_over = int(((sticky & _native.ST_OVERFLOW) != 0).sum())
    ok = np.concatenate(oks)
    label = f"config 4 {env_id} ({n} envs, {steps} steps, {len(C4_CHECK)} checked steps)"
    print(f"{label}: {ok.mean():.4f} of {ok.size} teacher-forced cases within tolerance; {n_done} episode ends; "
          f"envs dropping constraints: {n_over}")
    _hard_cap(np.concatenate(eqs), np.concatenate(evs), label)
    unexplained = _classify_misses(env_id, misses, label=label)
    assert n_over == 0, n_over
    assert ok.mean() >= ONE_STEP_MIN, ok.mean()
    assert not unexplained, unexplained

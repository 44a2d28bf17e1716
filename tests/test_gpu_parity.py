"""GPU (HIP, fp32) vs CPU oracle (fp64) parity through the C-ABI.  Runs on the MI355X box.

Tolerances (stated per the north star's "fp32 tolerance"):
  * task layer on golden vectors: obs |err| <= 2e-5 + 2e-5|ref|, reward |err| <= 1e-4 + 1e-5|ref|;
    done/goal exact except references within 1e-5 of a bonus threshold.
  * forward internals from identical states: relative (max-norm) error <= 1e-4 for kinematics,
    M, qacc_smooth; qacc / constraint force <= 2e-3 (Newton on the soft problem in fp32).
  * one env-step (frame_skip mj_steps) from identical states: qpos |err| <= 2e-5 + 1e-5|q|,
    qvel |err| <= 5e-3 (1 + |v|) in >= 99.5 % of envs / (env, step) cases; the rest may differ
    only where a contact switches on/off at the margin in one precision and not the other.
"""
import numpy as np
import pytest

from conftest import ENVS, golden, load_task_model, make_oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


def _t(a, dtype=None):
    return torch.tensor(np.asarray(a), dtype=dtype or torch.float32, device="cuda")


def _sim(env_id, n, variation=None):
    from mj_envs_amd import _native
    m = load_task_model(env_id, variation)
    return m, _native.Sim(m.to_blob(), n)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


# --------------------------------------------------------------------------------------------
@pytest.mark.parametrize("env_id", ENVS)
def test_task_layer_golden(env_id):
    g = golden(f"task_{env_id.split('-')[0]}.npz")
    m, sim = _sim(env_id, 1)
    n = g["qpos"].shape[0]
    touch = np.zeros(n)
    if env_id == "hammer-v0":
        touch = g["sensordata"][:, m.sensor_adr[m.name2id("sensor", "S_nail")]]
    obs = sim.empty(n, sim.obs_dim)
    rew = sim.empty(n)
    done = sim.empty(n, dtype=torch.uint8)
    goal = sim.empty(n, dtype=torch.uint8)
    sim.task_eval(n, _t(g["qpos"]), _t(g["qvel"]), _t(g["xpos"]), _t(g["xquat"]), _t(g["site_xpos"]),
                  _t(touch), obs, rew, done, goal)
    torch.cuda.synchronize()
    o = obs.cpu().numpy()
    np.testing.assert_allclose(o, g["obs"], rtol=2e-5, atol=2e-5)
    np.testing.assert_allclose(rew.cpu().numpy(), g["reward"], rtol=1e-5, atol=1e-4)
    assert (done.cpu().numpy().astype(bool) == g["done"]).all()
    assert (goal.cpu().numpy().astype(bool) == g["goal"]).all()


# --------------------------------------------------------------------------------------------
def f32(a):
    """the fp32 value the GPU holds (its state and per-env params are fp32), as fp64 for the oracle"""
    return np.asarray(a, np.float32).astype(np.float64)


def contact_states(env_id, n, steps, seed=0):
    """Oracle rollouts with random actions -> (params, qpos, qvel, warm) with contacts, rounded to
    fp32 so that GPU and oracle start from the same state."""
    from mj_envs_amd.tasks import sample_params
    m, o = make_oracle(env_id)           # MuJoCo's capacities: nconmax 100 / njmax 500
    rng = np.random.default_rng(seed)
    P = f32(sample_params(env_id, m, rng, n))
    st, _ = o.reset(P)
    for _ in range(steps):
        o.step(st, rng.uniform(-1, 1, (n, o.nu)), nthreads=8)
    for k in ("qpos", "qvel", "warm"):
        st[k] = f32(st[k])
    return m, o, P, st


def rel(a, b):
    a, b = np.asarray(a, float), np.asarray(b, float)
    return np.abs(a - b).max() / (np.abs(b).max() + 1e-9)


# Pass fractions (per env or per (env, step) case) of the one-step state tolerance.  The
# remainder are discrete events: a contact within fp32 rounding of the margin, or a bonus
# threshold, switching in one precision and not the other.
ONE_STEP_MIN = 0.995
VARIATION_MIN = 0.995   # 'pos' measured 0.94 in round 2 (the hammer rests on its moved cylinder
                        # head: the MPR line contact), 1.0 with MPR on fp64 geometry; every miss
                        # must still be classified (tests/parity_classify.py)
REWARD_MIN = 0.995

# Grasp regime (DAPG policies; hammer: fingers closed on the handle, head striking the nail):
# the same one-step tolerance, on every (env, step) of 80-step policy rollouts.  Resting
# contacts sit AT their margin by construction (MuJoCo's contact reference acceleration drives
# dist -> margin), so fp32 geometry (~1e-7 m) can switch one on or off where fp64 does not:
# those are the discrete events the thresholds leave room for.


def _no_overflow(sim, n):
    """the kernel's capacities held: no env raised a contact / constraint overflow (sticky flags)"""
    from mj_envs_amd import _native
    st = sim.empty(n, dtype=torch.int32)
    sim.status(sticky=st)
    torch.cuda.synchronize()
    st = st.cpu().numpy()
    assert not (st & _native.ST_OVERFLOW).any(), f"{int(((st & _native.ST_OVERFLOW) != 0).sum())} envs overflowed"


def _state_err(qg, vg, q_ref, v_ref):
    """per-env max |dqpos|, max |dqvel| / (1 + |v|) and the one-step tolerance verdict"""
    dq = np.abs(qg - q_ref)
    dv = np.abs(vg - v_ref)
    okq = (dq <= 2e-5 + 1e-5 * np.abs(q_ref)).all(axis=1)
    okv = (dv <= 5e-3 * (1 + np.abs(v_ref))).all(axis=1)
    return dq.max(axis=1), (dv / (1 + np.abs(v_ref))).max(axis=1), okq & okv


def _err_report(label, eq, ev, ok):
    """p50 / p99 / max of the per-case errors over the cases within tolerance (the misses are
    classified separately): printed, and returned for the distribution gates below."""
    eq, ev = np.asarray(eq)[ok], np.asarray(ev)[ok]
    r = dict(qpos=np.percentile(eq, [50, 99, 100]) if eq.size else np.zeros(3),
             qvel=np.percentile(ev, [50, 99, 100]) if ev.size else np.zeros(3))
    print(f"{label}: |dqpos| p50 {r['qpos'][0]:.2e} p99 {r['qpos'][1]:.2e} max {r['qpos'][2]:.2e}; "
          f"|dqvel|/(1+|v|) p50 {r['qvel'][0]:.2e} p99 {r['qvel'][1]:.2e} max {r['qvel'][2]:.2e}")
    return r


# Error-distribution gates (the per-case tolerance sits orders of magnitude
# above the achieved error, so a 10x regression could pass it).  Over the (env, step) cases within
# tolerance, the p50 / p99 of max |dqpos| and max |dqvel| / (1 + |v|) must stay below these bounds,
# set at ~4x the r04 measurements of the worst task / regime (profiles/r04z8_pytest_gpu.txt: p50
# qpos 2.0e-7, qvel 1.8e-5; p99 qpos 1.95e-6 (relocate C3), qvel 1.2e-4), so a 10x regression of
# the median or of the tail fails even when every case stays inside the per-case tolerance.
ERR_P50 = dict(qpos=8e-7, qvel=8e-5)
ERR_P99 = dict(qpos=8e-6, qvel=5e-4)


def _err_gate(r):
    for k in ("qpos", "qvel"):
        assert r[k][0] <= ERR_P50[k], (k, "p50", r[k][0])
        assert r[k][1] <= ERR_P99[k], (k, "p99", r[k][1])


# Hard cap on every (env, step) case, misses included (NaN fails): the physical ceiling (a contact
# switching under the hand moves a free object by at most a few cm / tens of mrad in one env-step).
# Each class that excuses a miss has its own, tighter cap (tests/parity_classify.py CLASS_CAP: ~4x the
# largest deviation that class showed over the r06 suite).
HARD_CAP = dict(qpos=5e-2, qvel=2.0)


def _hard_cap(eq, ev, label):
    eq, ev = np.asarray(eq, float), np.asarray(ev, float)
    mq, mv = float(np.max(eq)) if eq.size else 0.0, float(np.max(ev)) if ev.size else 0.0
    print(f"{label}: max over all cases |dqpos| {mq:.2e}, |dqvel|/(1+|v|) {mv:.2e} "
          f"(hard cap {HARD_CAP['qpos']:.0e} / {HARD_CAP['qvel']:.0e})")
    assert mq <= HARD_CAP["qpos"] and mv <= HARD_CAP["qvel"], (label, mq, mv)


def _classify_misses(env_id, misses, frame_skip=None, variation=None, label=""):
    """every miss through tests/parity_classify.py (a switch demonstrated structurally and causally,
    an oracle-shadowed trajectory, or a bounded fp32-sensitive reference); returns the unexplained
    (step, env) cases, after printing the class tallies"""
    from parity_classify import SPREAD_FACTOR, class_cap, classify_misses
    out, tally = classify_misses(env_id, misses, variation, label=label or env_id)
    for k, t in tally.items():
        assert t["max_ratio"] <= SPREAD_FACTOR, (k, t)
        cap = class_cap(k)
        if cap is not None:     # what a class may excuse is bounded (parity_classify.CLASS_CAP)
            assert t["max_dqpos"] <= cap[0] and t["max_dqvel"] <= cap[1], (k, t, cap)
    return [(k, e) for k, e, _ in out]


def _rewards_close(r, r_ref, check=True):
    """per-env reward agreement: |r - r_ref| <= 1e-3 + 1e-3 |r_ref|.  With check, at least
    REWARD_MIN (99.5 %) of the envs must agree -- the remainder is room for a bonus threshold of
    the task (2, 8, 10, 20, 25, 50, 75) that an fp32 state crosses and the fp64 one does not."""
    d = np.abs(np.asarray(r, float) - np.asarray(r_ref, float))
    tol = 1e-3 + 1e-3 * np.abs(r_ref)
    ok = d <= tol
    if check:
        frac = ok.mean()
        assert frac >= REWARD_MIN, (frac, np.where(~ok)[0], d[~ok])
    return ok


@pytest.mark.parametrize("env_id", ENVS)
def test_forward_internals_match_oracle(env_id):
    n = 8
    m, o, P, st = contact_states(env_id, n, 40)
    _, sim = _sim(env_id, n)
    sim.set_state(_t(st["qpos"]), _t(st["qvel"]), _t(st["warm"]), _t(P))
    ncon_total = 0
    for e in range(n):
        d = sim.forward_dump(e)
        o.forward1(P[e], st["qpos"][e], st["qvel"][e], st["warm"][e])
        sc = o.get("scalars")
        assert rel(d["xpos"], o.get("xpos").reshape(-1, 3)) < 1e-5
        assert rel(d["qM"], o.get("qM").reshape(sim.nv, sim.nv)) < 1e-4
        assert rel(d["qacc_smooth"], o.get("qacc_smooth")) < 1e-3
        if d["ncon"] == int(sc[0]):
            ncon_total += d["ncon"]
            c = o.get("contact").reshape(-1, 23)
            if d["ncon"]:
                np.testing.assert_allclose(d["con_dist"], c[:, 0], atol=2e-5)
                np.testing.assert_allclose(d["con_pos"], c[:, 1:4], atol=2e-4)
            assert d["nefc"] == int(sc[1])
            assert rel(d["qacc"], o.get("qacc")) < 2e-3, (env_id, e)
    assert ncon_total > 0 or env_id == "door-v0"


def test_forward_dump_rows_in_grasp_regime():
    """aw_forward_dump's constraint rows (efc_D, aref, type) on DAPG grasp states with the most
    dense rows: noslip parks its pair rows in dead LDS, and the dump kernel keeps efc_D out of
    that parking, so the reported rows are the solver's (tools/diag_tf.py compares them)."""
    import os
    from conftest import GOLDEN
    from mj_envs_amd.policy import GaussianMLP
    env_id, n = "hammer-v0", 64
    m, o = make_oracle(env_id)
    _, sim = _sim(env_id, n)
    pol = GaussianMLP.from_npz(os.path.join(GOLDEN, "dapg_hammer.npz"))
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, seed=21)
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    for _ in range(120):
        sim.step(_t(pol.mean_np(obs.cpu().numpy())), obs, rew, done, goal)
    q, v, w, p = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv), sim.empty(n, sim.nparam)
    sim.get_state(q, v, w, p)
    torch.cuda.synchronize()
    dumps = [sim.forward_dump(e) for e in range(n)]
    order = np.argsort([-d["ndense"] for d in dumps])[:8]
    assert dumps[order[0]]["ndense"] > 40, dumps[order[0]]["ndense"]
    checked = 0
    for e in order:
        d = dumps[e]
        o.forward1(p[e].cpu().numpy().astype(np.float64), q[e].cpu().numpy().astype(np.float64),
                   v[e].cpu().numpy().astype(np.float64), w[e].cpu().numpy().astype(np.float64))
        if d["nefc"] != int(o.get("scalars")[1]):
            continue                          # a contact decided by fp32 rounding: rows differ
        np.testing.assert_array_equal(d["efc_type"], o.get("efc_type"))
        np.testing.assert_allclose(d["efc_D"], o.get("efc_D"), rtol=2e-3)
        np.testing.assert_allclose(d["efc_aref"], o.get("efc_aref"), rtol=2e-3, atol=2e-3)
        checked += 1
    print(f"forward_dump rows: {checked} grasp states, max dense rows {dumps[order[0]]['ndense']}")
    assert checked >= 4


@pytest.mark.parametrize("env_id", ENVS)
def test_one_env_step_from_identical_states(env_id):
    n = 64
    m, o, P, st = contact_states(env_id, n, 50, seed=2)
    _, sim = _sim(env_id, n)
    sim.set_state(_t(st["qpos"]), _t(st["qvel"]), _t(st["warm"]), _t(P))
    rng = np.random.default_rng(5)
    act = f32(rng.uniform(-1, 1, (n, sim.nu)))
    obs, rew = sim.empty(n, sim.obs_dim), sim.empty(n)
    done, goal = sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    sim.step(_t(act), obs, rew, done, goal)
    q, v = sim.empty(n, sim.nq), sim.empty(n, sim.nv)
    sim.get_state(q, v)
    torch.cuda.synchronize()
    o_ref, r_ref, d_ref, g_ref, _ = o.step(st, act, nthreads=8)
    q, v = q.cpu().numpy(), v.cpu().numpy()
    okq = (np.abs(q - st["qpos"]) <= 2e-5 + 1e-5 * np.abs(st["qpos"])).all(axis=1)
    okv = (np.abs(v - st["qvel"]) <= 5e-3 * (1 + np.abs(st["qvel"]))).all(axis=1)
    ok = okq & okv
    print(f"one-step {env_id}: {ok.mean():.4f} of {n} envs within tolerance")
    assert ok.mean() >= ONE_STEP_MIN, (env_id, np.where(~ok)[0])
    _no_overflow(sim, n)
    _rewards_close(rew.cpu().numpy(), r_ref)


def test_smooth_dynamics_tight():
    """Constraints off: the smooth path (FK, CRB, RNE, LL' solve, implicit Euler) in fp32."""
    from mj_envs_amd.tasks import sample_params
    env_id, n = "hammer-v0", 32
    m, o = make_oracle(env_id)
    o.set_option(disableflags=1)
    _, sim = _sim(env_id, n)
    sim.set_option(disableflags=1)
    P = f32(sample_params(env_id, m, np.random.default_rng(0), n))
    st, _ = o.reset(P)
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, params=_t(P))
    rng = np.random.default_rng(1)
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    for _ in range(10):
        a = rng.uniform(-1, 1, (n, sim.nu))
        sim.step(_t(a), obs, rew, done, goal)
        o_ref, _, _, _, _ = o.step(st, a, nthreads=8)
    torch.cuda.synchronize()
    assert rel(obs.cpu().numpy(), o_ref) < 1e-4


# --------------------------------------------------------------------------------------------
def test_random_actions_and_reset_sampling():
    from mj_envs_amd.tasks import reset_ranges
    n = 4096
    m, sim = _sim("relocate-v0", n)
    a1, a2 = sim.empty(n, sim.nu), sim.empty(n, sim.nu)
    sim.random_actions(a1, 0, 7)
    sim.random_actions(a2, 0, 7)
    torch.cuda.synchronize()
    assert torch.equal(a1, a2)
    x = a1.cpu().numpy()
    assert x.min() >= -1 and x.max() < 1 and abs(x.mean()) < 0.01
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, seed=3)
    p = sim.empty(n, sim.nparam)
    sim.get_state(params=p)
    torch.cuda.synchronize()
    p = p.cpu().numpy()
    from mj_envs_amd.tasks import param_draws
    rr = reset_ranges("relocate-v0")
    for k, c in enumerate(param_draws("relocate-v0")):
        if c < 0:                         # not drawn at reset: keeps the model value
            assert p[:, k].std() == 0
            continue
        lo, hi = rr[c]
        assert p[:, k].min() >= lo and p[:, k].max() <= hi
        assert p[:, k].std() > 0.2 * (hi - lo)


def test_reset_obs_matches_oracle_all_tasks():
    from mj_envs_amd.tasks import sample_params
    for env_id in ENVS:
        n = 16
        m, o = make_oracle(env_id)
        _, sim = _sim(env_id, n)
        P = f32(sample_params(env_id, m, np.random.default_rng(4), n))
        _, obs_ref = o.reset(P)
        obs = sim.empty(n, sim.obs_dim)
        sim.reset(obs, params=_t(P))
        torch.cuda.synchronize()
        np.testing.assert_allclose(obs.cpu().numpy(), obs_ref, rtol=1e-5, atol=2e-5)


def test_state_roundtrip_and_autoreset():
    n = 128
    m, sim = _sim("pen-v0", n)
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, seed=9)
    act = sim.empty(n, sim.nu)
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    tobs = sim.empty(n, sim.obs_dim)
    ended = 0
    for k in range(sim.horizon):
        sim.random_actions(act, 11, k)
        sim.step(act, obs, rew, done, goal, terminal_obs=tobs, autoreset=True, seed=9)
        ended += int((done != 0).sum())
    torch.cuda.synchronize()
    assert ended >= n                        # every env truncated at the horizon (or dropped)
    lr, lg, ll, ep = sim.empty(n), sim.empty(n, dtype=torch.int32), sim.empty(n, dtype=torch.int32), \
        sim.empty(n, dtype=torch.int32)
    sim.episode_stats(lr, lg, ll, ep)
    torch.cuda.synchronize()
    assert (ep.cpu().numpy() >= 1).all()
    assert (ll.cpu().numpy() <= sim.horizon).all() and (ll.cpu().numpy() >= 1).all()
    # get/set state round trip reproduces the observation
    q, v, w, p = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv), sim.empty(n, sim.nparam)
    sim.get_state(q, v, w, p)
    o1 = sim.empty(n, sim.obs_dim)
    sim.set_state(q, v, w, p, obs=o1)
    o2 = sim.empty(n, sim.obs_dim)
    sim.set_state(q, v, w, p, obs=o2)
    torch.cuda.synchronize()
    assert torch.equal(o1, o2)
    st = sim.empty(n, dtype=torch.int32)
    sim.status(st)
    torch.cuda.synchronize()
    assert (st.cpu().numpy() & 7 == 0).all()


def test_determinism():
    n = 256
    outs = []
    for _ in range(2):
        m, sim = _sim("hammer-v0", n)
        obs = sim.empty(n, sim.obs_dim)
        sim.reset(obs, seed=5)
        act = sim.empty(n, sim.nu)
        rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
        for k in range(20):
            sim.random_actions(act, 1, k)
            sim.step(act, obs, rew, done, goal)
        torch.cuda.synchronize()
        outs.append(obs.clone())
    assert torch.equal(outs[0], outs[1])


# Minimum fraction of (env, step) cases within the one-step tolerance, for every task and regime
# (random actions, DAPG grasping, C3 at full size, the 4 096-env headline configuration).  The
# remainder are discrete events: a contact or row within fp32 rounding of its activation margin.
TEACHER_FORCED_MIN = {"hammer-v0": 0.995, "door-v0": 0.995, "relocate-v0": 0.995, "pen-v0": 0.995}
# hammer: 0.9955 in r04, 0.9990 since the fp64 near-margin contact decision (r05f); VERDICT r04's
# target for it is 0.998
GRASP_MIN = {"hammer-v0": 0.998, "door-v0": 0.995, "pen-v0": 0.995, "relocate-v0": 0.995}
# C3 at full size.  Round 2 measured hammer-v0 at 0.9939: tools/diag_tf.py attributed 38 of 40
# misses (profiles/r03a_diag_c3_hammer.json) to one contact -- the hammer's cylinder head lying
# on the table, a line contact whose MPR point jumps between the ends of the line under 1e-7 rad
# of rotation (fp32 kinematics) while the fp64 oracle is stable under input rounding.  MPR now
# runs on fp64 geometry (aw_dynamics.h stage_kin64): 0.9999 (r03d, 7 of 51 200).
C3_MIN = {"hammer-v0": 0.995, "door-v0": 0.995, "pen-v0": 0.995, "relocate-v0": 0.995}


@pytest.mark.parametrize("env_id", ENVS)
def test_teacher_forced_trajectory(env_id):
    frac = _teacher_forced(env_id, 0)
    assert frac >= TEACHER_FORCED_MIN[env_id], (env_id, frac)


@pytest.mark.parametrize("env_id", ENVS)
def test_teacher_forced_dapg_grasp(env_id):
    """Teacher forcing along DAPG-policy rollouts (grasp / manipulation regime: up to ~20
    contacts and ~100 dense rows per substep), oracle at MuJoCo's capacities, no overflow."""
    frac = _teacher_forced(env_id, 0, policy=True, steps=80)
    assert frac >= GRASP_MIN[env_id], (env_id, frac)


@pytest.mark.parametrize("env_id", ENVS)
def test_c3_correctness_run_256x200(env_id):
    """SURVEY §8d C3 at its stated size: 256 envs x 200 env-steps (one full hammer / door /
    relocate horizon, two pen horizons' worth of steps), random actions, teacher-forced."""
    frac = _teacher_forced(env_id, 0, steps=200, n=256)
    assert frac >= C3_MIN[env_id], (env_id, frac)


def _teacher_forced(env_id, disableflags, policy=False, steps=40, n=64):
    """SURVEY §8d C3 (multi-task correctness vs the CPU path): along a 40-step GPU rollout of
    64 envs, every env-step is re-run by the fp64 oracle from the GPU's own pre-step state
    (qpos, qvel, warmstart, params) with the same action; the GPU's post-step state must match
    within the one-step tolerance in the 2 560 (env, step) cases.  Teacher forcing
    keeps the comparison per-step: free-running fp32 vs fp64 contact trajectories diverge
    (chaos), which says nothing about either.  Thresholds: TEACHER_FORCED_MIN."""
    from mj_envs_amd.tasks import sample_params
    m, o = make_oracle(env_id)
    _, sim = _sim(env_id, n)
    sim.set_option(disableflags=disableflags)
    P = f32(sample_params(env_id, m, np.random.default_rng(11), n))
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, params=_t(P))
    rew = sim.empty(n)
    done, goal = sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    q, v, w = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv)
    rng = np.random.default_rng(13)
    pol = None
    if policy:
        import os
        from conftest import GOLDEN
        from mj_envs_amd.policy import GaussianMLP
        pol = GaussianMLP.from_npz(os.path.join(GOLDEN, f"dapg_{env_id.split('-')[0]}.npz"))
    oks, rok, eqs, evs, misses = [], [], [], [], []
    ostatus = 0
    for k in range(steps):
        sim.get_state(q, v, w)
        torch.cuda.synchronize()
        st = dict(qpos=q.cpu().numpy().astype(np.float64), qvel=v.cpu().numpy().astype(np.float64),
                  warm=w.cpu().numpy().astype(np.float64), params=np.asarray(P, np.float64))
        pre = {key: val.copy() for key, val in st.items()}
        # the action the GPU receives (fp32) is the oracle's action too
        act = f32(pol.mean_np(obs.cpu().numpy()) if pol is not None else rng.uniform(-1, 1, (n, sim.nu)))
        sim.step(_t(act), obs, rew, done, goal)
        sim.get_state(q, v)
        torch.cuda.synchronize()
        _, r_ref, _, _, ost = o.step(st, act, nthreads=8)
        ostatus |= int(np.bitwise_or.reduce(ost))
        qg, vg = q.cpu().numpy(), v.cpu().numpy()
        eq, ev, ok = _state_err(qg, vg, st["qpos"], st["qvel"])
        oks.append(ok)
        eqs.append(eq)
        evs.append(ev)
        misses += [(k, e, pre["params"][e], pre["qpos"][e], pre["qvel"][e], pre["warm"][e], np.asarray(act[e], np.float64),
                    qg[e].astype(np.float64), vg[e].astype(np.float64)) for e in np.where(~ok)[0]]
        rok.append(_rewards_close(rew.cpu().numpy(), r_ref, check=False))
    frac = np.concatenate(oks).mean()
    rfrac = np.concatenate(rok).mean()
    miss_steps = np.array([int((~ok).sum()) for ok in oks])
    if miss_steps.sum():
        top = np.argsort(miss_steps)[::-1][:3]
        print(f"misses per step (top 3): " + ", ".join(f"step {k}: {miss_steps[k]}" for k in top))
    label = f"teacher-forced {env_id} (disableflags {disableflags:#x}{', DAPG policy' if policy else ''})"
    print(f"{label}: {frac:.4f} of {n * steps} (env, step) cases within the state tolerance, rewards {rfrac:.4f}")
    err = _err_report(label, np.concatenate(eqs), np.concatenate(evs), np.concatenate(oks))
    _hard_cap(np.concatenate(eqs), np.concatenate(evs), label)
    unexplained = _classify_misses(env_id, misses, label=label)
    print(f"{label}: {len(misses)} misses, unexplained: {unexplained}")
    assert not (ostatus & 24), "oracle overflowed MuJoCo's capacities"
    _no_overflow(sim, n)
    assert rfrac >= REWARD_MIN, (env_id, rfrac)
    assert not unexplained, (env_id, unexplained)
    _err_gate(err)
    return frac


def test_teacher_forced_headline_config_4096_envs():
    """BASELINE configs[1] (hammer-v0, 4 096 envs, random policy; hammer_v0.py:54-90) through the
    kernel configuration of the headline number: 4 096 envs are more than the resident slots
    (aw_dims GRID, CUs x occupancy = 2 048 on MI355X), so every persistent workgroup steps two envs
    per launch, claiming the second from the launch's counter, and reuses its slot-indexed dense-J
    spill / M-factor blocks.  256 envs sampled evenly over the batch (half of them >= 2 048, the
    claimed ones) are teacher-forced against the fp64 oracle for 60 env-steps: every sampled
    post-step state within the one-step tolerance in >= 99.5 % of the (env, step) cases."""
    from mj_envs_amd.tasks import sample_params
    env_id, n, steps = "hammer-v0", 4096, 60
    m, o = make_oracle(env_id)
    _, sim = _sim(env_id, n)
    assert sim.grid < n, f"grid {sim.grid} covers all {n} envs: the persistent claim path is not exercised"
    idx = np.unique(np.linspace(0, n - 1, 256).round().astype(int))
    assert (idx >= sim.grid).sum() >= 100
    P = f32(sample_params(env_id, m, np.random.default_rng(17), n))
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, params=_t(P))
    rew = sim.empty(n)
    done, goal = sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    q, v, w = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv)
    rng = np.random.default_rng(19)
    oks, roks, eqs, evs, misses = [], [], [], [], []
    for k in range(steps):
        sim.get_state(q, v, w)
        torch.cuda.synchronize()
        st = dict(qpos=q.cpu().numpy()[idx].astype(np.float64), qvel=v.cpu().numpy()[idx].astype(np.float64),
                  warm=w.cpu().numpy()[idx].astype(np.float64), params=np.asarray(P, np.float64)[idx])
        pre = {key: val.copy() for key, val in st.items()}
        act = f32(rng.uniform(-1, 1, (n, sim.nu)))
        sim.step(_t(act), obs, rew, done, goal)
        sim.get_state(q, v)
        torch.cuda.synchronize()
        _, r_ref, _, _, _ = o.step(st, act[idx], nthreads=8)
        qg, vg = q.cpu().numpy()[idx], v.cpu().numpy()[idx]
        eq, ev, okk = _state_err(qg, vg, st["qpos"], st["qvel"])
        oks.append(okk)
        eqs.append(eq)
        evs.append(ev)
        misses += [(k, int(idx[j]), pre["params"][j], pre["qpos"][j], pre["qvel"][j], pre["warm"][j],
                    np.asarray(act[idx[j]], np.float64), qg[j].astype(np.float64), vg[j].astype(np.float64))
                   for j in np.where(~okk)[0]]
        roks.append(_rewards_close(rew.cpu().numpy()[idx], r_ref, check=False))
    ok = np.array(oks)
    frac, rfrac = ok.mean(), np.concatenate(roks).mean()
    hi = ok[:, idx >= sim.grid].mean()
    label = f"headline config (hammer-v0, {n} envs, grid {sim.grid})"
    print(f"{label}: {frac:.4f} of {ok.size} sampled (env, step) "
          f"cases within tolerance ({hi:.4f} for the claimed envs >= {sim.grid}), rewards {rfrac:.4f}")
    err = _err_report(label, np.concatenate(eqs), np.concatenate(evs), ok.reshape(-1))
    _hard_cap(np.concatenate(eqs), np.concatenate(evs), label)
    unexplained = _classify_misses(env_id, misses, label=label)
    print(f"{label}: {len(misses)} misses, unexplained: {unexplained}")
    _no_overflow(sim, n)
    assert frac >= ONE_STEP_MIN and hi >= ONE_STEP_MIN, (frac, hi)
    assert rfrac >= REWARD_MIN, rfrac
    assert not unexplained, unexplained
    _err_gate(err)


@pytest.mark.parametrize("variation", ["mass", "pos", "size"])
def test_hammer_variations_one_step(variation):
    """hammer_v0.py:110-129 variation types: per-env body mass / head+neck position / head size
    overrides reach the kinematics (apply_ovr), the subtree masses and the colliders exactly as
    in the oracle.  Same one-step contract as test_one_env_step_from_identical_states."""
    from mj_envs_amd.tasks import sample_params
    env_id, n = "hammer-v0", 64
    m, o = make_oracle(env_id, variation)
    rng = np.random.default_rng(21)
    P = f32(sample_params(env_id, m, rng, n, variation))
    st, obs_ref = o.reset(P)
    for _ in range(30):
        o.step(st, rng.uniform(-1, 1, (n, o.nu)), nthreads=8)
    for k in ("qpos", "qvel", "warm"):
        st[k] = f32(st[k])
    _, sim = _sim(env_id, n, variation)
    assert sim.nparam == P.shape[1] > 1
    pre = {k: np.array(v, copy=True) for k, v in st.items()}
    obs = sim.empty(n, sim.obs_dim)
    sim.set_state(_t(st["qpos"]), _t(st["qvel"]), _t(st["warm"]), _t(P), obs=obs)
    act = f32(rng.uniform(-1, 1, (n, sim.nu)))
    rew = sim.empty(n)
    done, goal = sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    sim.step(_t(act), obs, rew, done, goal)
    q, v = sim.empty(n, sim.nq), sim.empty(n, sim.nv)
    sim.get_state(q, v)
    torch.cuda.synchronize()
    o_ref, r_ref, _, _, _ = o.step(st, act, nthreads=8)
    q, v = q.cpu().numpy(), v.cpu().numpy()
    okq = (np.abs(q - st["qpos"]) <= 2e-5 + 1e-5 * np.abs(st["qpos"])).all(axis=1)
    okv = (np.abs(v - st["qvel"]) <= 5e-3 * (1 + np.abs(st["qvel"]))).all(axis=1)
    ok = okq & okv
    # every miss classified like the teacher-forced ones (tests/parity_classify.py)
    misses = [(0, int(e), P[e], pre["qpos"][e], pre["qvel"][e], pre["warm"][e], act[e], q[e].astype(np.float64),
               v[e].astype(np.float64)) for e in np.where(~ok)[0]]
    unexplained = _classify_misses(env_id, misses, variation=variation, label=f"variation {variation}")
    print(f"variation {variation}: {ok.mean():.4f} of {n} envs within tolerance; misses not explained by a "
          f"discrete event: {unexplained}")
    assert ok.mean() >= VARIATION_MIN and not unexplained, (variation, np.where(~ok)[0], unexplained)
    _no_overflow(sim, n)
    np.testing.assert_allclose(obs.cpu().numpy()[ok], o_ref[ok], rtol=1e-3, atol=2e-3)
    _rewards_close(rew.cpu().numpy(), r_ref)

"""Negative tests of the parity-miss classifier (tests/parity_classify.py): a kernel error must come
out UNEXPLAINED.  Two faults are injected into the kernel through the test hook aw_set_fault
(include/adroit_wave.h) and the faulty kernel is teacher-forced against the fp64 oracle exactly as
the parity tests do; every miss it produces is handed to the classifier with the faulty kernel as
the one the classifier inspects (its forward dumps and substeps come from a handle with the same
fault):

  (i)  margin fault: the margin of every sphere / capsule pair (collider class 1 -- the finger
       capsules on the hammer handle) moved by 1e-4 m, in the DAPG grasp (hammer_v0.py:54-90 with the
       reference's pretrained policy, algos/baselines.py:82-86): contacts appear up to 1e-4 m past
       the reference's margin (DAPG_assets.xml:3,12-13) and every resting contact's reference
       acceleration shifts;
  (ii) row-state fault: the frictionloss row of FFJ0 (the index finger's distal joint) held in the
       stick state under random actions: mj_solNewton's row never slides where the reference's does.

Each fault must produce misses and the classifier must explain none of them.  The unfaulted
kernel's misses in the same regimes are the parity tests' (all classified).
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, make_oracle

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

MAX_CLASSIFIED = 40     # misses handed to the classifier per fault (it replays each one substep by substep)


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _t(a):
    return torch.tensor(np.asarray(a), dtype=torch.float32, device="cuda")


def _faulty_run(env_id, kind, arg, n, warm_steps, steps, policy):
    """teacher-forced rollout of the faulty kernel: the misses against the oracle (the same tuple
    layout as the parity tests)"""
    from mj_envs_amd import _native
    from mj_envs_amd.policy import GaussianMLP
    from mj_envs_amd.tasks import sample_params
    from parity_classify import f32
    m, o = make_oracle(env_id)
    sim = _native.Sim(m.to_blob(), n)
    P = f32(sample_params(env_id, m, np.random.default_rng(41), n))
    obs = sim.empty(n, sim.obs_dim)
    sim.reset(obs, params=_t(P))
    rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
    pol = GaussianMLP.from_npz(os.path.join(GOLDEN, f"dapg_{env_id.split('-')[0]}.npz")) if policy else None
    rng = np.random.default_rng(43)

    def action():
        return f32(pol.mean_np(obs.cpu().numpy()) if pol is not None else rng.uniform(-1, 1, (n, sim.nu)))

    for _ in range(warm_steps):           # the regime is reached by the correct kernel
        sim.step(_t(action()), obs, rew, done, goal)
    sim.set_fault(kind, arg)
    q, v, w = sim.empty(n, sim.nq), sim.empty(n, sim.nv), sim.empty(n, sim.nv)
    misses = []
    for k in range(steps):
        sim.get_state(q, v, w)
        torch.cuda.synchronize()
        st = dict(qpos=q.cpu().numpy().astype(np.float64), qvel=v.cpu().numpy().astype(np.float64),
                  warm=w.cpu().numpy().astype(np.float64), params=P.copy())
        pre = {key: val.copy() for key, val in st.items()}
        a = action()
        sim.step(_t(a), obs, rew, done, goal)
        sim.get_state(q, v)
        torch.cuda.synchronize()
        o.step(st, a, nthreads=8)
        qg, vg = q.cpu().numpy().astype(np.float64), v.cpu().numpy().astype(np.float64)
        ok = (np.abs(qg - st["qpos"]) <= 2e-5 + 1e-5 * np.abs(st["qpos"])).all(1) & \
             (np.abs(vg - st["qvel"]) <= 5e-3 * (1 + np.abs(st["qvel"]))).all(1)
        misses += [(warm_steps + k, int(e), P[e], pre["qpos"][e], pre["qvel"][e], pre["warm"][e], a[e], qg[e], vg[e])
                   for e in np.nonzero(~ok)[0]]
    sim.close()
    return misses


def _classify_with_fault(env_id, misses, kind, arg):
    from parity_classify import classify_misses, context
    ctx = context(env_id)
    ctx.set_fault(kind, arg)        # the classifier inspects the faulty kernel
    try:
        sample = [misses[i] for i in np.unique(np.linspace(0, len(misses) - 1, MAX_CLASSIFIED).round().astype(int))]
        unexplained, tally = classify_misses(env_id, sample, label=f"fault {kind}/{arg}")
    finally:
        ctx.set_fault(0, 0)
    return sample, unexplained, tally


def test_margin_fault_is_unexplained():
    """(i): class-1 margins + 1e-4 m in the hammer grasp"""
    env_id = "hammer-v0"
    misses = _faulty_run(env_id, 1, 100, n=64, warm_steps=90, steps=12, policy=True)
    print(f"margin fault: {len(misses)} misses of {64 * 12} teacher-forced cases")
    assert len(misses) >= 10, "the fault must be visible in the state"
    sample, unexplained, tally = _classify_with_fault(env_id, misses, 1, 100)
    print(f"margin fault: {len(unexplained)} of {len(sample)} classified misses unexplained; classes {tally}")
    assert len(unexplained) == len(sample), [k for k in tally if k != "UNEXPLAINED"]


def test_stuck_frictionloss_row_is_unexplained():
    """(ii): FFJ0's frictionloss row held in the stick state under random actions"""
    from conftest import load_task_model
    env_id = "hammer-v0"
    m = load_task_model(env_id)
    fl = np.nonzero(np.asarray(m.arrays["dof_frictionloss"]) > 0)[0]
    dof = m.names["joint"].index("FFJ0")          # hinge joints: joint index = dof index
    row = int(np.nonzero(fl == dof)[0][0])       # rows 0..nfl-1 are the frictionloss dofs in order
    misses = _faulty_run(env_id, 2, row, n=64, warm_steps=10, steps=12, policy=False)
    print(f"stuck row {row} (FFJ0): {len(misses)} misses of {64 * 12} teacher-forced cases")
    assert len(misses) >= 10, "the fault must be visible in the state"
    sample, unexplained, tally = _classify_with_fault(env_id, misses, 2, row)
    print(f"stuck row: {len(unexplained)} of {len(sample)} classified misses unexplained; classes {tally}")
    assert len(unexplained) == len(sample), [k for k in tally if k != "UNEXPLAINED"]


def test_fault_hook_restores_the_table():
    """aw_set_fault(0) restores the model table bit for bit: the same rollout as a never-faulted handle"""
    from mj_envs_amd import _native
    env_id, n = "hammer-v0", 128
    m, _ = make_oracle(env_id)
    outs = []
    for cycle in (False, True):
        sim = _native.Sim(m.to_blob(), n)
        if cycle:
            sim.set_fault(1, 100)
            sim.set_fault(2, 3)
            sim.set_fault(0, 0)
        obs = sim.empty(n, sim.obs_dim)
        sim.reset(obs, seed=5)
        act = sim.empty(n, sim.nu)
        rew, done, goal = sim.empty(n), sim.empty(n, dtype=torch.uint8), sim.empty(n, dtype=torch.uint8)
        for k in range(15):
            sim.random_actions(act, 3, k)
            sim.step(act, obs, rew, done, goal)
        torch.cuda.synchronize()
        outs.append(obs.clone())
        sim.close()
    assert torch.equal(outs[0], outs[1])

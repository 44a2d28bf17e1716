"""CPU checks of the parity classifier's building blocks (tests/parity_classify.py): the oracle's
margin-nudge hook that the causal check of a margin switch relies on, and the contact matching."""
import numpy as np

from conftest import make_oracle


def test_oracle_margin_nudge_switches_one_pair():
    """Oracle.set_margin_nudge moves one geom pair's margin (either order) and nothing else: moving it
    below a contact's distance removes exactly that pair's contacts; clearing restores them"""
    m, o = make_oracle("hammer-v0")
    st, _ = o.reset(np.asarray(m.arrays["task_param_default"], float)[None])
    rng = np.random.default_rng(0)
    for _ in range(40):                 # into contact (hand on the table / the hammer)
        o.step(st, rng.uniform(-1, 1, (1, o.nu)))
    q, v, w = st["qpos"][0], st["qvel"][0], st["warm"][0]
    P = st["params"][0]
    o.forward1(P, q, v, w)
    c = o.get("contact").reshape(-1, 23)
    assert len(c) > 0, "contacts after 40 random steps"
    g1, g2, dist = int(c[0, 13]), int(c[0, 14]), float(c[0, 0])
    mg = float(c[0, 17])            # includemargin (gap 0 in these models)
    keys = [(int(r[13]), int(r[14])) for r in c]
    o.set_margin_nudge(g2, g1, dist - mg - 1e-6)       # reversed order on purpose
    o.forward1(P, q, v, w)
    c2 = o.get("contact").reshape(-1, 23)
    keys2 = [(int(r[13]), int(r[14])) for r in c2]
    assert (g1, g2) not in keys2
    assert keys2 == [k for k in keys if k != (g1, g2)]
    o.set_margin_nudge()
    o.forward1(P, q, v, w)
    np.testing.assert_array_equal(o.get("contact").reshape(-1, 23), c)


def test_unmatched_contacts_by_position():
    from parity_classify import _lists_differ, _unmatched
    a = [(0.0, np.array([0.0, 0, 0])), (0.1, np.array([1.0, 0, 0]))]
    b = [(0.1, np.array([1.0, 0, 0]))]
    gu, ou = _unmatched(a, b)
    assert len(gu) == 1 and np.allclose(gu[0][1], [0, 0, 0]) and not ou
    assert _unmatched(a, a) == ([], [])
    assert not _lists_differ(a, [(x + 1e-7, p + 1e-6) for x, p in a])
    assert _lists_differ(a, [(x, p + 1e-3) for x, p in a])

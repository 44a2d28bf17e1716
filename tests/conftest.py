import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

ENVS = ["hammer-v0", "door-v0", "pen-v0", "relocate-v0"]
GOLDEN = os.path.join(REPO, "tests", "golden")
REFERENCE = "/root/reference"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


def load_task_model(env_id, variation_type=None):
    """The task model as the tests build it: the reference's variation types, plus the test-only
    pseudo-variation "margin=X" (every geom margin set to X: far more contacts and rows than the
    reference's regimes, to drive the wide capacity tier)"""
    from mj_envs_amd.tasks import attach_task, load_model
    if variation_type and str(variation_type).startswith("margin="):
        m = attach_task(load_model(env_id), env_id, None)
        m.arrays["geom_margin"] = np.full_like(m.arrays["geom_margin"], float(variation_type.split("=")[1]))
        return m
    return attach_task(load_model(env_id), env_id, variation_type)


def make_oracle(env_id, variation_type=None):
    from oracle.pyoracle import Oracle
    m = load_task_model(env_id, variation_type)
    return m, Oracle(m.to_blob())


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)

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


def make_oracle(env_id, variation_type=None):
    from mj_envs_amd.tasks import attach_task, load_model
    from oracle.pyoracle import Oracle
    m = attach_task(load_model(env_id), env_id, variation_type)
    return m, Oracle(m.to_blob())


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)

import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lmsf-slam_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblmsf_hip.so)")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    oracle.set_threads(1)
    return oracle


@pytest.fixture(scope="session")
def small_workload():
    """C2-shaped (16 x 4096 VLP-16) scans against a reduced 300k-point map: seconds on the oracle."""
    from lmsf import synth
    return synth.make_workload("C2", n_scans=3, map_points=300_000)


@pytest.fixture(scope="session")
def c2_workload():
    """Full C2 workload (64k-point scans, 1M-point map)."""
    from lmsf import synth
    return synth.make_workload("C2", n_scans=2, map_points=1_000_000)


def pose_err(a, b):
    from lmsf import synth
    return synth.pose_delta(a, b)

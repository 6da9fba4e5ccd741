import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    import json

    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def hd_obs_oracle():
    import oracle as O

    return O.obs_from_file(os.path.join(GOLDEN, "HD155358.vels"), Npoints=100)


# HD155358 (BASELINE config 3): the solution mcmc_benchmark_*.py starts from (a, h, k, m, l per planet)
HD_SOL = [6.57730330e-01, -9.72263877e-02, -7.82798396e-02, 8.84031737e-04, 4.42804990e+00,
          1.04404207e+00, -2.05622789e-02, -1.08797961e-01, 8.30379710e-04, 1.49919861e+00]


def hd_planets():
    return [{"m": HD_SOL[3], "a": HD_SOL[0], "h": HD_SOL[1], "k": HD_SOL[2], "l": HD_SOL[4]},
            {"m": HD_SOL[8], "a": HD_SOL[5], "h": HD_SOL[6], "k": HD_SOL[7], "l": HD_SOL[9]}]


S2_PLANETS = [{"m": 1.2e-3, "a": 0.88, "h": 0.218, "k": 0.015, "l": 0.3},
              {"m": 2.1e-3, "a": 1.44 + 0.11, "h": 0.16, "k": 0.02, "l": 2.2}]  # mcmc_benchmark_mh.py:32
S2_SCALES = {"m": 1.5e-3, "a": 0.3, "h": 0.1, "k": 0.1, "l": 3.141592653589793 / 2.}  # mcmc_benchmark_emcee.py:51


def s2_obs_oracle(seed=2017, Npoints=100):
    """BASELINE.md synthetic config: np.random.seed(2017); FakeObservation(Npoints=100, error=1.5e-4,
    errorVar=2.5e-5, tmax=120) on the mcmc_benchmark_mh.py:32 state."""
    import numpy as np
    import oracle as O

    np.random.seed(seed)
    return O.fake_obs(S2_PLANETS, Npoints=Npoints, error=1.5e-4, errorVar=2.5e-5, tmax=120.)

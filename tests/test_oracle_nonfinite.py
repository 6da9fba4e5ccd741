"""The oracle's rule for a halving pass that blows up (oracle/rvoracle.c dir_halve, round 5): the
walker ends NONFINITE after that pass -- it is not refined on to resolve_max -- and the rest of the
rule is unchanged.  CPU only; the GPU side is tests/test_gpu_contract.py."""
import time

import numpy as np

import oracle as O
from conftest import S2_PLANETS, s2_obs_oracle
from test_gpu_contract import NONFINITE_WALKERS


def test_nonfinite_halving_pass_ends_the_walker_on_the_oracle():
    from rvmcmc import engine

    obs = s2_obs_oracle()
    cfg = engine.IntegratorConfig()
    dt, mult, _ = cfg.plan_args(S2_PLANETS)
    tol = cfg.resolve(S2_PLANETS)[0]
    P = np.zeros((2, 2, 7))
    P[:, :, :5] = NONFINITE_WALKERS
    t0 = time.perf_counter()
    for rmax in (2, 12):
        lp, st, rf, _, _ = O.logl_whx_adapt_batch(P, 2, obs, dt, mult, tol, rmax, 0.0)
        np.testing.assert_array_equal(st, [3, 3])
        assert np.all(np.isneginf(lp))
        # walker 1 blows up in the forward direction's first halving pass (stage 2: the extension,
        # then one halving), walker 0 in both directions' second
        assert rf[1].tolist() == [2, 1] and rf[0].tolist() == [3, 3], rf
    assert time.perf_counter() - t0 < 30.0  # (refining on to 2^12 x the steps would take minutes)

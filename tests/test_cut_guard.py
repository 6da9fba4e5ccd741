"""The certain-reject cut's eccentricity guard (round 6; oracle/rvoracle.c CUT_ECC_FACTOR, the kernel's
DevPlan::e2_cut).  No GPU: the oracle restates the kernel's rule.

At HD155358's steady state with 2048 walkers three stretch proposals in 24576 were rejected by the
cut right after the extension although IAS15 accepts them (scripts/probe/decision_mismatch_probe.py):
their outer planets have e = 0.79-0.84, the plan's levels and the extension are far from resolving
their pericentre passages, and the extension's change (a third of the error) was taken as the bound.
Past the cut guard the bound after the extension is chi2 - min(10 d, 100 est) (CUT_GUARD_K), not
chi2 - min(d, 100 est), so those walkers refine to the tolerance and take the reference's decision."""
import json
import os

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN, HD_SOL, hd_planets

pytestmark = pytest.mark.filterwarnings("ignore::RuntimeWarning")


def _plan():
    from rvmcmc import engine

    planets = hd_planets()
    cfg = engine.IntegratorConfig()
    dt, mult, _ = cfg.plan_args(planets)
    tol, rmax, guard, _ = cfg.resolve(planets)
    return dt, mult, tol, rmax, guard


def test_guard_values():
    dt, mult, tol, rmax, guard = _plan()
    assert 0.17 < guard < 0.19  # HD155358's reference planets: e 0.125 -> the verify guard 0.179
    assert abs((1.0 - (1.0 - guard) * 0.6712) - 0.449) < 0.001  # the cut guard: e 0.449
    assert len(HD_SOL) == 10


def test_formerly_cut_walkers_take_the_reference_decision():
    obs = O.obs_from_file(os.path.join(GOLDEN, "HD155358.vels"), Npoints=100)
    dt, mult, tol, rmax, guard = _plan()
    with open(os.path.join(GOLDEN, "cut_guard_walkers.json")) as f:
        rows = json.load(f)["walkers"]
    assert len(rows) == 3
    for r in rows:
        P = np.array([r["params"]])
        ctx = dict(mode=np.ones(1, dtype=np.int32), dim=10, z=np.array([r["z"]]), u=np.array([r["u"]]),
                   lnp0=np.array([r["lnp0"]]))
        logl, status, stage, _, _, cut = O.logl_whx_adapt_batch(P, 2, obs, dt, mult, tol, rmax, 1.0,
                                                                   ecc_guard=guard, ctx=ctx)
        assert status[0] == 0 and not cut[0].any(), (status, stage, cut)
        assert abs(logl[0] - r["ias15_logl"]) <= 1e-6
        # the reference's decision (emcee 2.2.1 stretch: (dim - 1) log z + lnp' - lnp > log u): accept
        assert 9.0 * np.log(r["z"]) + logl[0] - r["lnp0"] > np.log(r["u"])

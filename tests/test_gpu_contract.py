"""The C ABI's launch conventions (include/rvmcmc.h "Conventions"), held by every entry point of an
adaptive plan -- including a plain launch of 32..512 walkers, which runs the eager halving pass on
the plan's side stream (rvm_refine.hip eager_kernel):

  * stream-ordered: the launch is complete -- eager blocks included -- once the caller's stream is,
    so the caller may reuse or free `params` right after synchronising that stream;
  * capturable: the launch sequence (fork, likelihood kernel, refinement kernel, join) captures into
    a hipGraph, and every replay gives the plain launch's bits (the launch generation that tags the
    kernels' hand-off flags lives on the device, so a replay never sees a previous replay's flags);
  * a halving pass that blows up ends its walker NONFINITE at once (oracle/rvoracle.c dir_halve,
    ADVICE r4 medium) instead of refining on to resolve_max (2^12 x the base steps).

The reference's counterpart is the synchronous emcee callback (mcmc.py:28-35): it returns a finished
logp before the caller touches the walker again.
"""
import os

import numpy as np
import pytest

import oracle as O
from conftest import S2_PLANETS, s2_obs_oracle
from test_gpu_resolve import RMAX, TOL, _oracle_P, _plan, wide_walkers

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _torch():
    import torch

    assert torch.cuda.is_available()
    return torch


def _rows(X):
    torch = _torch()
    return torch.as_tensor(np.ascontiguousarray(X.T), device="cuda")


@pytest.mark.parametrize("W", [256, 6144])
def test_adaptive_launch_captures_into_a_graph(W):
    """rvm_logl_batch on an adaptive plan captured into a hipGraph (torch.cuda.graph) and replayed:
    256 walkers (eager pass on the side stream, forked and joined inside the capture) and 6144 (the
    level-split launch with team refinement: split exchanges tagged by the launch generation).  Each
    replay over new walkers gives the bits and statuses of a plain launch over them, and the plan's
    counters add up the same."""
    torch = _torch()
    obs = s2_obs_oracle()
    plan, _, _ = _plan(obs, W)
    ref_plan, _, _ = _plan(obs, W)
    sets = [wide_walkers(W, ball=0.3, seed=s) for s in (5, 6, 7)]
    K = _rows(sets[0])
    lp = torch.empty(W, dtype=torch.float64, device="cuda")
    st = torch.empty(W, dtype=torch.int32, device="cuda")
    plan.logl(K, out=lp, status=st)  # (a plain launch first: lazily created state is in place)
    torch.cuda.synchronize()
    plan.faults(reset=True)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            plan.logl(K, out=lp, status=st)
    torch.cuda.synchronize()
    plan.faults(reset=True)  # (capture enqueues nothing; counters start clean)
    for rep in range(2):
        for X in sets:
            K.copy_(_rows(X))
            g.replay()
            torch.cuda.synchronize()
            got, gst = lp.cpu().numpy().copy(), st.cpu().numpy().copy()
            want, wst, _ = ref_plan.logl(_rows(X))
            torch.cuda.synchronize()
            np.testing.assert_array_equal(gst, wst.cpu().numpy())
            np.testing.assert_array_equal(got, want.cpu().numpy())
    f, fr = plan.faults(reset=True), ref_plan.faults(reset=True)
    assert f == fr, (f, fr)
    assert f["refined"] > 0 and f["handoff_timeouts"] == 0 and f["nonfinite"] == 0


def test_eager_launch_is_complete_when_the_stream_is():
    """An eager launch (256 walkers) on a side stream of the caller's: right after that stream is
    synchronised the caller overwrites `params` with NaN and launches again on new walkers in the
    same buffer; every launch's results equal those of a plan without the eager pass (RVM_EAGER=0).
    Before the join, eager blocks could still read `params` after the caller's stream completed."""
    torch = _torch()
    obs = s2_obs_oracle()
    W = 256
    old = os.environ.get("RVM_EAGER")
    os.environ["RVM_EAGER"] = "0"
    try:
        ref_plan, _, _ = _plan(obs, W)
    finally:
        if old is None:
            os.environ.pop("RVM_EAGER", None)
        else:
            os.environ["RVM_EAGER"] = old
    plan, _, _ = _plan(obs, W)
    cs = torch.cuda.Stream()
    K = torch.empty((10, W), dtype=torch.float64, device="cuda")
    for seed in range(4):
        X = wide_walkers(W, ball=0.3, seed=20 + seed)
        with torch.cuda.stream(cs):
            K.copy_(_rows(X))
            lp, st, _ = plan.logl(K, stream=cs)
        cs.synchronize()
        got, gst = lp.cpu().numpy().copy(), st.cpu().numpy().copy()
        with torch.cuda.stream(cs):
            K.fill_(float("nan"))  # (the caller is done with these walkers)
        want, wst, _ = ref_plan.logl(_rows(X))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(gst, wst.cpu().numpy())
        np.testing.assert_array_equal(got, want.cpu().numpy())
    f, fr = plan.faults(reset=True), ref_plan.faults(reset=True)
    assert f == fr, (f, fr)
    assert f["refined"] > 0


# two prior-passing walkers of the S2 observation set (hill_factor 0: no encounter exit) whose
# halving passes blow up: [1] in pass 1 of its forward direction, [0] in pass 2 of both directions
# (found on the oracle by scripts/probe/find_nonfinite_pass.py; rows m, a, h, k, l per planet)
NONFINITE_WALKERS = np.array([
    [[0.02256103, 0.41693664, -0.97022551, -0.02642071, 0.3], [0.00259106, 0.65391134, -0.90235793, 0.40896047, 2.2]],
    [[0.00505582, 1.19118678, -0.39903947, 0.34994554, 0.3], [0.00316488, 1.01076266, -0.72163793, 0.31746809, 2.2]],
])


@pytest.mark.parametrize("W", [2, 64])
def test_nonfinite_halving_pass_ends_the_walker(W):
    """A walker whose halving pass is non-finite ends NONFINITE after that pass, on the device as in
    the oracle (statuses equal; the plan counts it), beside ordinary wide-ball walkers whose results
    stay T1.  Before round 5 the kernel refined such a walker on to resolve_max = 12 (the last pass
    at 4096 x the base steps) where the oracle had stopped."""
    from rvmcmc import engine

    torch = _torch()
    obs = s2_obs_oracle()
    dt, mult, hint = engine.IntegratorConfig().plan_args(S2_PLANETS)
    t, rv, er = engine.obs_arrays(obs)
    rmax = 12
    plan = engine.LoglPlan(t, rv, er, obs.Npoints, 2, dt, mult, max(W, 2), period_hint=hint, resolve=(TOL, rmax))
    X = np.concatenate([NONFINITE_WALKERS.reshape(2, 10), wide_walkers(64, ball=0.02, seed=9)[:W - 2]])
    lp, st, _ = plan.logl(_rows(X), hill_factor=0.0)
    torch.cuda.synchronize()
    got, gst = lp.cpu().numpy(), st.cpu().numpy()
    ref, st_ref, rf, _, _ = O.logl_whx_adapt_batch(_oracle_P(X), 2, obs, dt, mult, TOL, rmax, 0.0)
    assert st_ref[0] == 3 and st_ref[1] == 3, (st_ref[:2], rf[:2])
    np.testing.assert_array_equal(gst[:2], [3, 3])
    assert np.all(np.isneginf(got[:2]))
    f = plan.faults(reset=True)
    assert f["nonfinite"] == int((gst == 3).sum()) and f["handoff_timeouts"] == 0, f
    ok = (gst == 0) & (st_ref == 0)
    np.testing.assert_array_equal(gst[2:], st_ref[2:])
    if ok.any():
        err = np.abs(got[ok] - ref[ok]) / np.maximum(1.0, np.abs(ref[ok]))
        assert err.max() <= 1e-11 * 35.0, err.max()
    assert RMAX <= rmax

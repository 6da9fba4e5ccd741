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


def test_one_planet_long_schedule_fits_the_lds_coupled_layout():
    """the LDS-coupled layouts' ring of the levels' star velocities took 16 epochs x
    (levels + 1) x 64 walkers x 8 B = 40 KB per one-planet group (80 KB per two-group block), so a
    one-planet fused launch fit only ~1150 epochs per direction -- and a plan between that and the
    refinement kernel's limit was created but failed every launch.  The ring is now sized per plan
    within 24 KB per group (DevPlan::lc_ring; 9 epochs here), rvm_plan_create refuses a schedule the
    worst-case launch cannot stage, and a 1500-epoch-per-direction one-planet plan runs its two-group
    launch: every copy of a walker gets the same bits, and the values are the oracle's (T1)."""
    torch = _torch()
    from rvmcmc import _lib, engine

    one = [{"m": 1.2e-3, "a": 0.88, "h": 0.05, "k": 0.02, "l": 0.3}]
    np.random.seed(7)
    obs = O.fake_obs(one, Npoints=3000, error=1.5e-4, errorVar=2.5e-5, tmax=400.)  # 1501 + 1500 epochs
    dt, mult, hint = engine.IntegratorConfig().plan_args(one)
    t, rv, er = engine.obs_arrays(obs)
    W = 12288  # 192 groups of 64 walkers: two groups per block
    plan = engine.LoglPlan(t, rv, er, obs.Npoints, 1, dt, mult, W, period_hint=hint, resolve=(TOL, RMAX))
    rng = np.random.default_rng(1)
    base = np.array([one[0][k] for k in "mahkl"])
    X16 = base * (1 + 1e-4 * rng.standard_normal((16, 5)))
    X = np.tile(X16, (W // 16, 1))
    lp, st, _ = plan.logl(_rows(X))
    torch.cuda.synchronize()
    lp, st = lp.cpu().numpy().reshape(-1, 16), st.cpu().numpy().reshape(-1, 16)
    assert (st == 0).all()
    assert (lp == lp[0]).all()  # (every copy the same bits)
    P = np.zeros((16, 1, 7))
    P[:, 0, :5] = X16
    ref, sref = O.logl_whx_adapt_batch(P, 1, obs, dt, mult, TOL, RMAX)[:2]
    assert (sref == 0).all()
    err = np.max(np.abs(lp[0] - ref) / np.maximum(1.0, np.abs(ref)))
    assert err < 1e-11 * float(np.abs(O.richardson_weights_seq(mult)).sum()), err
    # a schedule no launch could stage is refused when the plan is created, not at launch
    np.random.seed(7)
    big = O.fake_obs(one, Npoints=12000, error=1.5e-4, errorVar=2.5e-5, tmax=400.)
    t2, rv2, er2 = engine.obs_arrays(big)
    with pytest.raises(_lib.RvmError, match="LDS"):
        engine.LoglPlan(t2, rv2, er2, big.Npoints, 1, dt, mult, W, period_hint=hint, resolve=(TOL, RMAX))


def test_skipped_variants_are_exactly_the_ruled_out_ones():
    """a speculative iteration's half-1 slot is one of two variants of its partner j's
    outcome; when j was not handed to the refinement kernel its decision is final, and the
    refinement kernel skips (RVM_STATUS_SKIPPED) the variant that decision rules out instead of
    refining it.  At the bench chain's steady state, over three iterations: SKIPPED appears only on
    ruled-out variants ((kind 2) != (dec[j] == 1)), never on half 0 or on a chosen variant, and the
    chosen variants' logL and status, the positions and the lnprob are bit-identical to a plan with
    skipping disabled (RVM_SKIP_VARIANTS=0), which skips nothing."""
    torch = _torch()
    from philox_ref import stretch_uniforms
    from rvmcmc import _lib
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.observations import FakeObservation
    from rvmcmc.state import State

    X0 = np.load(os.path.join(HERE, "..", "scripts", "probe", "ens_it2000.npy"))

    def run(skip):
        old = os.environ.get("RVM_SKIP_VARIANTS")
        os.environ["RVM_SKIP_VARIANTS"] = "1" if skip else "0"
        try:
            s = State(planets=[dict(p) for p in S2_PLANETS])
            np.random.seed(2017)
            obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)  # (its own plan)
            ens = EnsembleSampler(len(X0), s, obs, seed=2017)
            ens.set_positions(X0)
            ens.compute_lnprob()
            assert ens.speculating()
            out = []
            for _ in range(3):
                it = ens.iteration
                ens.step()
                torch.cuda.synchronize()
                out.append((it, ens._st_spec.cpu().numpy().copy(), ens._lnp_spec.cpu().numpy().copy(),
                            ens._dec.cpu().numpy().copy()))
            return ens, out
        finally:
            if old is None:
                os.environ.pop("RVM_SKIP_VARIANTS", None)
            else:
                os.environ["RVM_SKIP_VARIANTS"] = old

    ea, oa = run(True)
    eb, ob = run(False)
    n = ea.nloc
    skipped = 0
    for (it, sa_, la, da), (_, sb, lb, db) in zip(oa, ob):
        np.testing.assert_array_equal(da, db)
        _, u2, _ = stretch_uniforms(ea.seed, ea.global_begin(1), n, it, 1)
        j = np.clip(np.floor(u2 * ea.halfk).astype(int), 0, ea.halfk - 1)
        accepted = da[j] == 1
        chosen = np.concatenate([np.arange(n), n + np.arange(n) + np.where(accepted, n, 0)])
        ruled_out = n + np.arange(n) + np.where(accepted, 0, n)
        sk = np.nonzero(sa_ == _lib.RVM_STATUS_SKIPPED)[0]
        assert set(sk.tolist()) <= set(ruled_out.tolist())
        assert not (sb == _lib.RVM_STATUS_SKIPPED).any()
        np.testing.assert_array_equal(sa_[chosen], sb[chosen])
        np.testing.assert_array_equal(la[chosen], lb[chosen])
        skipped += len(sk)
    assert skipped > 0  # (~16 per steady-state iteration)
    for h in (0, 1):
        np.testing.assert_array_equal(ea.pos[h].cpu().numpy(), eb.pos[h].cpu().numpy())
        np.testing.assert_array_equal(ea.lnp[h].cpu().numpy(), eb.lnp[h].cpu().numpy())

"""GPU parity of the likelihood kernel (rvm_logl_batch through the C ABI).

Tiers:
  T1  kernel vs oracle/rvoracle.c's restatement of the SAME algorithm (Richardson-extrapolated
      Wisdom-Holman, identical schedule):  |dlogL| / max(1, |logL|) <= 3x the oracle's own
      roundoff sensitivity over the batch (its response to 1e-15 relative input nudges,
      t1_tol_sens; measured kernel error 0.2-2.2x that sensitivity), model RV within 1e-14 sum|w|
      absolute, identical status codes.  Chaotic walkers (wide ball) are compared within their
      own per-walker sensitivity.
  T2  kernel vs the IAS15 restatement of the reference (reference-equivalent physics):
      |dlogL| <= 5e-8 absolute at the default integrator settings (SURVEY.md §8c allows 1e-6;
      measured 1.4e-9 S2, 1.9e-9 HD155358, 1.2e-8 on the short inclined set below); golden G2/G3.
"""
import os

import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN, S2_PLANETS, s2_obs_oracle

pytestmark = pytest.mark.gpu

# T1: roundoff floor.  ~1e-15 relative differences in the per-level model RV (FMA contraction on
# the GPU, a different Stumpff evaluation) are amplified by the Richardson weights (sum_k |w_k|:
# 6.2 at 4 levels, 26 at 6) and by the likelihood's conditioning (dlogL/drv ~ 2 sum|r|/(N sigma^2)
# ~ 1e4).  Tolerance: 1e-11 * sum|w| * max(1, |logL|)  (measured max 4e-11 at 4 levels).
T1_REL_PER_W = 1e-11
# T1 as used by the batch comparisons below: 3x the oracle's own roundoff sensitivity over the
# batch (t1_tol_sens).  SURVEY.md §8c's 1e-12 is below that sensitivity for these walkers (the
# oracle itself moves by up to 7.5e-11 when an input changes by 1e-15 relative), so it cannot be
# met by any second implementation; t1_tol (the Sigma|w| form above) remains for the sampler and
# derivative tests that compare single values.
T1_SENS_FACTOR = 3.0
T2_ABS = 5e-8
# default integrator (rvmcmc.engine.IntegratorConfig): level multipliers and base steps per orbit
LEVELS = (4, 5, 6, 7)
SPO = 8.0
# model RV: per-level differences of ~1e-14 absolute (roundoff accumulated over thousands of
# steps) times the weights' sum|w| (6.2 harmonic 4 levels, 35 for 4..7)
T1_RV_ABS = 1e-14 * float(np.abs(O.richardson_weights(LEVELS)).sum())


def t1_tol(nl=LEVELS):
    return T1_REL_PER_W * float(np.abs(O.richardson_weights(nl)).sum())


T1_REL = t1_tol(LEVELS)


def _torch():
    import torch

    assert torch.cuda.is_available(), "GPU tests need a HIP device"
    return torch


def _plan(obs, planets, n_levels=LEVELS, steps=SPO, max_walkers=4096, inclined=False):
    from rvmcmc import engine

    pmin = engine.min_period(planets)
    dt = pmin / steps
    t, rv, er = engine.obs_arrays(obs)
    return engine.LoglPlan(t, rv, er, obs.Npoints, len(planets), dt, n_levels, max_walkers,
                           period_hint=pmin, inclined=inclined), dt


def _ball(planets, W, rel=1e-3, seed=0):
    rng = np.random.default_rng(seed)
    base = O.pal_params(planets)
    P = np.repeat(base[None], W, 0)
    P[:, :, :5] *= 1 + rel * rng.standard_normal((W, len(planets), 5))
    return P  # [W][np][7]


def _kernel_params(P, rows=5):
    W, n, _ = P.shape
    return np.ascontiguousarray(np.concatenate([P[:, p, :rows].T for p in range(n)], 0))


def _run(plan, P, hill=1.0, want_rv=False):
    torch = _torch()
    K = torch.as_tensor(_kernel_params(P, 7 if plan.inclined else 5), device="cuda")
    lp, st, rv = plan.logl(K, hill_factor=hill, want_rv=want_rv)
    torch.cuda.synchronize()
    return lp.cpu().numpy(), st.cpu().numpy(), (rv.cpu().numpy() if rv is not None else None)


def _t1_report(err, tol, nl, sens=None):
    """Append the measured T1 maximum of one comparison to $RVM_T1_REPORT (JSON lines)."""
    path = os.environ.get("RVM_T1_REPORT")
    if path:
        import json

        d = {"test": os.environ.get("PYTEST_CURRENT_TEST", "").split(" ")[0],
             "max_rel_err": float(err.max(initial=0.0)), "tol": float(tol),
             "levels": list(np.atleast_1d(nl).tolist()), "sum_abs_w": float(np.abs(O.richardson_weights(nl)).sum())}
        if sens is not None and len(err):
            r = err / np.maximum(sens, 1e-300)
            d.update(max_sens=float(sens.max()), min_sens=float(sens.min()), max_err_over_sens=float(r.max()),
                     p99_err_over_sens=float(np.percentile(r, 99)), max_err_where_sens_zero=float(err[sens == 0].max(initial=0)),
                     max_err_over_max_sens_1e12=float((err / np.maximum(sens, 1e-12)).max()))
        with open(path, "a") as f:
            f.write(json.dumps(d) + "\n")


NUDGES = [(0, 4, 1), (-1, 4, -1), (0, 1, 1), (-1, 1, -1), (0, 2, 1), (-1, 0, 1)]


def oracle_sensitivity(P, n_planets, obs, dt, nl, hill=1.0, has_inc=0):
    """Per-walker roundoff sensitivity of the oracle's logL: the largest relative response to a
    1e-15 relative nudge of one input (l, a, h, m of the first / last planet).  The kernel and the
    oracle round differently (FMA contraction, rcp/rsq Newton math, Stumpff evaluation), so their
    difference is a roundoff path of the same size."""
    ref, st_ref = O.logl_whx_batch(P, n_planets, obs, dt, nl, hill, 1, has_inc)
    sens = np.zeros(len(P))
    for pl, par, sgn in NUDGES:
        P2 = P.copy()
        P2[:, pl, par] *= 1 + sgn * 1e-15
        r2, s2 = O.logl_whx_batch(P2, n_planets, obs, dt, nl, hill, 1, has_inc)
        both = (st_ref == 0) & (s2 == 0)
        sens[both] = np.maximum(sens[both], np.abs(r2[both] - ref[both]) / np.maximum(1.0, np.abs(ref[both])))
    return sens


def t1_tol_sens(sens):
    """T1 from the batch's own roundoff conditioning: T1_SENS_FACTOR x the oracle's largest
    response to a 1-ulp-scale input nudge, floored at SURVEY.md §8c's 1e-12 (a few-walker batch
    samples the sensitivity poorly).  Measured (round 2, every T1 batch of this file): max kernel
    error / max(sensitivity, 1e-12) = 0.2 ... 2.2."""
    return T1_SENS_FACTOR * max(float(np.max(sens, initial=0.0)), 1e-12)


def _assert_t1(got, st, ref, st_ref, nl=LEVELS, sens=None):
    np.testing.assert_array_equal(st, st_ref)
    ok = st == 0
    err = np.abs(got[ok] - ref[ok]) / np.maximum(1.0, np.abs(ref[ok]))
    tol = t1_tol(nl) if sens is None else t1_tol_sens(sens[ok])
    _t1_report(err, tol, nl, None if sens is None else sens[ok])
    assert err.max(initial=0.0) <= tol, (err.max(), tol)
    assert np.all(np.isneginf(got[~ok]))


@pytest.mark.parametrize("W", [1, 63, 64, 65, 256])
def test_t1_s2_tight_ball(W):
    obs = s2_obs_oracle()
    plan, dt = _plan(obs, S2_PLANETS)
    P = _ball(S2_PLANETS, W, seed=W)
    got, st, _ = _run(plan, P)
    ref, st_ref = O.logl_whx_batch(P, 2, obs, dt, LEVELS)
    _assert_t1(got, st, ref, st_ref, sens=oracle_sensitivity(P, 2, obs, dt, LEVELS))


def test_t1_wide_ball_statuses():
    """Wide ball: prior rejections (a, m, e >= 1) and encounters must match the oracle exactly."""
    obs = s2_obs_oracle()
    plan, dt = _plan(obs, S2_PLANETS)
    P = _ball(S2_PLANETS, 256, rel=0.6, seed=3)
    P[0, 0, 1] = 0.02           # a <= 0.02
    P[1, 1, 0] = 5e-6           # m <= 5e-6
    P[2, 0, 2], P[2, 0, 3] = 0.8, 0.6   # h^2 + k^2 = 1
    P[3, 1, 1] = P[3, 0, 1] * 1.01      # near-coorbital -> encounter
    got, st, _ = _run(plan, P)
    ref, st_ref = O.logl_whx_batch(P, 2, obs, dt, LEVELS)
    assert (st == 1).sum() >= 3 and (st == 2).sum() >= 1
    # roundoff sensitivity of each walker: the oracle's own response to a 1e-15 relative nudge.
    # Chaotic walkers (close approaches) may flip a borderline encounter or move logL far beyond
    # the T1 floor; they are compared within their own sensitivity.
    sens = np.zeros(len(P))
    flips = np.zeros(len(P), dtype=bool)
    for k, (pl, par, sgn) in enumerate([(0, 4, 1), (1, 4, -1), (0, 1, 1), (1, 1, -1), (0, 2, 1)]):
        P2 = P.copy()
        P2[:, pl, par] *= 1 + sgn * 1e-15
        ref2, st2 = O.logl_whx_batch(P2, 2, obs, dt, LEVELS)
        flips |= st2 != st_ref
        both = (st_ref == 0) & (st2 == 0)
        sens[both] = np.maximum(sens[both], np.abs(ref2[both] - ref[both]) / np.maximum(1.0, np.abs(ref[both])))
    # borderline encounters: the oracle's closest approach within 1e-6 of the exit distance
    ratio = np.array([O.min_distance_ratio(P[i:i + 1], 2, obs, dt, LEVELS) for i in range(len(P))])
    sensitive = flips | (sens > 1e-9) | (np.abs(ratio - 1.0) < 1e-6)
    mism = st != st_ref
    assert np.all(~mism | sensitive), np.nonzero(mism & ~sensitive)
    assert mism.sum() <= max(1, len(P) // 50)
    np.testing.assert_array_equal(st[st_ref == 1], 1)   # prior rejections are exact
    ok = (st == 0) & (st_ref == 0)
    scale = np.maximum(1.0, np.abs(ref[ok]))
    err = np.abs(got[ok] - ref[ok]) / scale
    assert np.all(err <= np.maximum(T1_REL, 1e3 * sens[ok])), np.max(err / np.maximum(T1_REL, 1e3 * sens[ok]))
    assert np.mean(err <= T1_REL) > 0.9
    assert np.all(np.isneginf(got[st != 0]))


@pytest.mark.parametrize("nl,spo", [(1, 24.0), (2, 24.0), (3, 24.0), (4, 24.0), (5, 24.0), (6, 24.0),
                                    ((2, 3, 4, 5), 16.0), ((3, 4, 5, 6), 12.0), ((4, 5, 6, 7), 8.0),
                                    ((4, 5, 6, 7, 8, 9), 6.0), ((1, 3, 5), 12.0)])
def test_t1_levels(nl, spo):
    """Harmonic levels 1..6 and general multiplier sequences, each against the oracle."""
    obs = s2_obs_oracle()
    plan, dt = _plan(obs, S2_PLANETS, n_levels=nl, steps=spo)
    P = _ball(S2_PLANETS, 96, seed=int(np.sum(nl)))
    got, st, _ = _run(plan, P)
    ref, st_ref = O.logl_whx_batch(P, 2, obs, dt, nl)
    _assert_t1(got, st, ref, st_ref, nl, sens=oracle_sensitivity(P, 2, obs, dt, nl))


EXTRA_PLANETS = [{"m": 1e-3, "a": 2.6, "h": 0.05, "k": 0.0, "l": 1.0},
                 {"m": 5e-4, "a": 4.1, "h": -0.03, "k": 0.02, "l": 4.0}]


@pytest.mark.parametrize("n_planets", [1, 3, 4])
def test_t1_planet_counts(n_planets):
    planets = (S2_PLANETS + EXTRA_PLANETS)[:n_planets]
    np.random.seed(11)
    obs = O.fake_obs(planets, Npoints=40, error=1.5e-4, errorVar=2.5e-5, tmax=60.)
    plan, dt = _plan(obs, planets)
    P = _ball(planets, 70, seed=n_planets)
    got, st, _ = _run(plan, P)
    ref, st_ref = O.logl_whx_batch(P, n_planets, obs, dt, LEVELS)
    _assert_t1(got, st, ref, st_ref, sens=oracle_sensitivity(P, n_planets, obs, dt, LEVELS))


@pytest.mark.parametrize("n_planets,hill", [(3, 4.0), (4, 3.0)])
def test_t1_planet_counts_close_encounters(n_planets, hill):
    """3- and 4-planet closed-form kick (kickN): exit-distance statuses on a wide ball with a
    large Hill factor must match the oracle walker for walker, logL within T1 elsewhere."""
    planets = (S2_PLANETS + EXTRA_PLANETS)[:n_planets]
    np.random.seed(12)
    obs = O.fake_obs(planets, Npoints=30, error=1.5e-4, errorVar=2.5e-5, tmax=40.)
    plan, dt = _plan(obs, planets)
    P = _ball(planets, 128, rel=0.05, seed=30 + n_planets)
    got, st, _ = _run(plan, P, hill=hill)
    ref, st_ref = O.logl_whx_batch(P, n_planets, obs, dt, LEVELS, hill_factor=hill)
    assert 0 < np.count_nonzero(st_ref == 2) < len(P)  # some walkers exit, not all
    _assert_t1(got, st, ref, st_ref, sens=oracle_sensitivity(P, n_planets, obs, dt, LEVELS, hill))


def test_t2_s2_vs_ias15():
    obs = s2_obs_oracle()
    plan, _ = _plan(obs, S2_PLANETS)
    P = _ball(S2_PLANETS, 32, seed=5)
    got, st, _ = _run(plan, P)
    ref, st_ref = O.logl_ias15_batch(P, 2, obs, hill_factor=1.0)
    assert (st == st_ref).all()
    assert np.abs(got - ref).max() < T2_ABS


def test_g2_through_kernel(golden, hd_obs_oracle):
    g = golden["G2"]
    sol = g["sol"]
    planets = [{"m": sol[3], "a": sol[0], "h": sol[1], "k": sol[2], "l": sol[4]},
               {"m": sol[8], "a": sol[5], "h": sol[6], "k": sol[7], "l": sol[9]}]
    plan, _ = _plan(hd_obs_oracle, planets)
    got, st, _ = _run(plan, O.pal_params(planets)[None], hill=g["hillRadiusFactor"])
    ref, _ = O.logl_ias15(planets, hd_obs_oracle, hill_factor=2.0)
    assert st[0] == 0
    assert abs(got[0] - ref) < T2_ABS
    assert abs(got[0] - g["logp_print12"]) < T2_ABS


def test_g3_rv_out(golden):
    g = golden["G3"]
    d = np.load(os.path.join(GOLDEN, g["file"]))
    obs = O.obs_from_file(os.path.join(GOLDEN, g["obs"]), Npoints=100)
    times = np.linspace(obs.tb[0], obs.tf[-1], 1000)
    o = O.OracleObs(tf=times, tb=np.zeros(0), rvf=np.zeros(1000), rvb=np.zeros(0), errorf=np.ones(1000),
                    errorb=np.zeros(0), Npoints=1)
    plan, dt = _plan(o, g["planets"])
    _, st, rv = _run(plan, O.pal_params(g["planets"])[None], hill=0.0, want_rv=True)
    assert st[0] == 0
    rv_whx, _ = O.whx_rv(g["planets"], times, dt, LEVELS)
    np.testing.assert_allclose(rv[:, 0], rv_whx, rtol=0, atol=T1_RV_ABS)   # T1
    np.testing.assert_allclose(rv[:, 0], d["rv"], rtol=0, atol=1e-12)      # T2 vs the stored curve


def test_epoch_edge_cases():
    """t = 0 epochs, duplicate epochs, an empty backward direction, unsorted input."""
    planets = S2_PLANETS
    t = np.array([3.0, 0.0, 0.0, 1.5, 3.0, 12.25, 7.0])
    o = O.OracleObs(tf=t, tb=np.zeros(0), rvf=np.full(len(t), 1e-4), rvb=np.zeros(0),
                    errorf=np.full(len(t), 2e-4), errorb=np.zeros(0), Npoints=7)
    plan, dt = _plan(o, planets)
    info = plan.info()
    assert info["epochs_fwd"] == 7 and info["epochs_bwd"] == 0
    P = _ball(planets, 5, seed=9)
    got, st, rv = _run(plan, P, want_rv=True)
    ref, st_ref = O.logl_whx_batch(P, 2, o, dt, LEVELS)
    _assert_t1(got, st, ref, st_ref, sens=oracle_sensitivity(P, 2, o, dt, LEVELS))
    assert np.all(rv[1] == rv[2]) and np.all(rv[0] == rv[4])


def test_state_api_matches_oracle(golden, hd_obs_oracle):
    from rvmcmc import observations, state

    sol = golden["G2"]["sol"]
    s = state.State(planets=[{"m": sol[3], "a": sol[0], "h": sol[1], "k": sol[2], "l": sol[4]},
                             {"m": sol[8], "a": sol[5], "h": sol[6], "k": sol[7], "l": sol[9]}])
    s.hillRadiusFactor = 2.0
    obs = observations.Observation_FromFile(os.path.join(GOLDEN, "HD155358.vels"), Npoints=100)
    lp = s.get_logp(obs)
    assert abs(lp - golden["G2"]["logp_print12"]) < T2_ABS
    s2 = s.deepcopy()
    assert s2.hillRadiusFactor == 1.0  # state.py:212-213 quirk reproduced
    s2.planets[0]["a"] = 0.01
    assert s2.get_logp(obs) == -np.inf


def test_fake_observation_matches_oracle():
    from rvmcmc import observations, state

    s = state.State(planets=[dict(p) for p in S2_PLANETS])
    np.random.seed(2017)
    o = observations.FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    from rvmcmc import engine

    dt = engine.min_period(S2_PLANETS) / SPO
    np.random.seed(2017)
    r = O.fake_obs(S2_PLANETS, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.,
                   rv_fn=lambda pl, t: O.whx_rv(pl, t, dt, LEVELS)[0])
    np.testing.assert_array_equal(o.tf, r.tf)
    np.testing.assert_array_equal(o.tb, r.tb)
    np.testing.assert_array_equal(o.errorf, r.errorf)
    np.testing.assert_array_equal(o.errorb, r.errorb)
    np.testing.assert_allclose(o.rvf, r.rvf, rtol=0, atol=T1_RV_ABS)   # T1
    np.testing.assert_allclose(o.rvb, r.rvb, rtol=0, atol=T1_RV_ABS)
    r2 = s2_obs_oracle()                                               # IAS15 data (T2)
    np.testing.assert_allclose(o.rvf, r2.rvf, rtol=0, atol=1e-10)
    np.testing.assert_allclose(o.rvb, r2.rvb, rtol=0, atol=1e-10)


@pytest.mark.parametrize("W", [4096, 4128, 6000, 6400, 8192])
def test_large_batch_size_independent_results(W):
    """A walker's logL does not depend on the batch it is launched in (W vs 1).  4096 runs one
    walker group per block; 4128 and 8192 exceed one block per CU and run two groups per block
    with mirrored level order (4128: the last block's second group is partly empty); 6000 and
    6400 run the level-split layout (level 1 in type-B blocks meeting the unit's combiner through
    HBM, level 0 split into a head and a tail; type-B blocks of 6 units with split pairs at 6000,
    of 8 whole units at 6400, where 6-unit blocks would not fit the CUs; the last type-B block
    partly empty) and must give the same bits as the LDS-coupled single launches."""
    obs = s2_obs_oracle()
    plan, _ = _plan(obs, S2_PLANETS, max_walkers=W)
    P = _ball(S2_PLANETS, W, seed=21)
    big, st_big, rv_big = _run(plan, P, want_rv=True)
    for i in (0, 32, 1000, 4095, W - 1):  # 0 and 32: walkers whose bits once depended on the layout
        one, st1, rv1 = _run(plan, P[i:i + 1], want_rv=True)
        assert one[0] == big[i] and st1[0] == st_big[i]
        np.testing.assert_array_equal(rv1[:, 0], rv_big[:, i])
    assert np.isfinite(big).all()


@pytest.mark.parametrize("W", [2048, 6000])
def test_wide_ball_redos_keep_bits(W):
    """Wide ball (relative 0.1): the speculative levels redo segments gated and back off
    (rvm_logl.hip spec_off / spec_bo: 2933 level-2 redos per 6144-slot launch at this width,
    profiles/r02h_prof_clock_ball.jsonl), and a wave's redo and back-off history depends on its
    wave-mates -- different in the full batch than for a walker launched alone.  A walker's bits
    (logL, status, model RVs) must not; 2048 runs the LDS-coupled layout, 6000 the level-split one."""
    obs = s2_obs_oracle()
    plan, _ = _plan(obs, S2_PLANETS, max_walkers=W)
    P = _ball(S2_PLANETS, W, rel=0.1, seed=41)
    big, st_big, rv_big = _run(plan, P, want_rv=True)
    rng = np.random.default_rng(3)
    for i in np.r_[0, 1, 63, W - 1, rng.choice(W, 12, replace=False)]:
        one, st1, rv1 = _run(plan, P[i:i + 1], want_rv=True)
        assert st1[0] == st_big[i]
        np.testing.assert_array_equal(one[0], big[i])
        np.testing.assert_array_equal(rv1[:, 0], rv_big[:, i])
    # (statuses of a wide ball: some walkers meet the exit distance, most integrate to the end)
    assert (st_big == 0).mean() > 0.5


@pytest.mark.parametrize("one_sided,npoints", [(False, 300), (True, 300), (True, 100)])
def test_level_split_ring_wrap_and_empty_direction(one_sided, npoints):
    """Level-split hand-off (rvm_logl.hip): levels 3, 2, 0 pass their per-epoch RVs to the unit's
    combiner through an LDS ring of RVM_LS_RING = 64 epochs and wait when a whole ring ahead;
    level 1 through HBM granules.  301 epochs (151 forward) wrap the ring and exercise that wait;
    the one-sided sets (all epochs at t >= 0) leave the backward units with no epoch at all (with
    51 forward epochs the ring holds a whole direction, so level 0 runs split into a head that
    then combines and a tail: the empty direction's head hands over at once).  Every walker gives
    the bits (logL, status, model RVs) of its LDS-coupled single launch, and T1 against the
    oracle on a subset."""
    np.random.seed(13)
    obs = O.fake_obs(S2_PLANETS, Npoints=npoints, error=1.5e-4, errorVar=2.5e-5, tmax=150. * npoints / 300)
    if one_sided:
        e = np.zeros(0)
        obs = O.OracleObs(tf=obs.tf, rvf=obs.rvf, errorf=obs.errorf, tb=e, rvb=e, errorb=e, Npoints=obs.Npoints)
    W = 6000  # 376 (group, direction) units: the level-split layout
    plan, dt = _plan(obs, S2_PLANETS, max_walkers=W)
    P = _ball(S2_PLANETS, W, seed=31)
    big, st_big, rv_big = _run(plan, P, want_rv=True)
    assert np.isfinite(big).all()
    for i in (0, 31, 2999, W - 1):
        one, st1, rv1 = _run(plan, P[i:i + 1], want_rv=True)
        assert one[0] == big[i] and st1[0] == st_big[i]
        np.testing.assert_array_equal(rv1[:, 0], rv_big[:, i])
    idx = np.r_[0:12, W - 12:W]
    ref, st_ref = O.logl_whx_batch(P[idx], 2, obs, dt, LEVELS)
    _assert_t1(big[idx], st_big[idx], ref, st_ref, sens=oracle_sensitivity(P[idx], 2, obs, dt, LEVELS))
    # a second launch finds every hand-off slot empty again (the combiners restore the sentinel)
    again, st2, _ = _run(plan, P)
    np.testing.assert_array_equal(again, big)
    np.testing.assert_array_equal(st2, st_big)


@pytest.mark.parametrize("W", [4160, 2900])
def test_two_group_blocks_vs_oracle_three_planets(W):
    """3 planets: 16 walkers per wave; 4160 walkers run two mirrored groups per block, 2900 the
    level-split layout.  T1 on a subset against the oracle, and the full batch against single
    launches (bit-identical)."""
    planets = (S2_PLANETS + EXTRA_PLANETS)[:3]
    np.random.seed(11)
    obs = O.fake_obs(planets, Npoints=40, error=1.5e-4, errorVar=2.5e-5, tmax=60.)
    plan, dt = _plan(obs, planets, max_walkers=W)
    P = _ball(planets, W, seed=5)
    got, st, _ = _run(plan, P)
    idx = np.r_[0:24, 2000:2024, W - 24:W]
    ref, st_ref = O.logl_whx_batch(P[idx], 3, obs, dt, LEVELS)
    _assert_t1(got[idx], st[idx], ref, st_ref, sens=oracle_sensitivity(P[idx], 3, obs, dt, LEVELS))
    for i in (15, 16, W - 1):
        one, st1, _ = _run(plan, P[i:i + 1])
        assert one[0] == got[i] and st1[0] == st[i]


# ---- inclined systems (REBOUND Pal ix, iy; 3-D integration) ---------------------------------------
# No stored reference output has an inclined system (the reference only checks ix^2 + iy^2 < 4 in
# priorHard, state.py:311-313): the 3-D Pal rotation is the oracle's restatement of REBOUND's
# (pinned in the plane by G1), so these tiers are pinned to the oracle only.
S2_INCLINED = [dict(S2_PLANETS[0], ix=0.12, iy=-0.05), dict(S2_PLANETS[1], ix=0.04, iy=0.18)]


def _inclined_ball(W, seed, rel=1e-3):
    P = _ball(S2_INCLINED, W, rel=rel, seed=seed)
    rng = np.random.default_rng(seed + 100)
    P[:, :, 5:7] += 1e-3 * rng.standard_normal((W, 2, 2))
    return P


def test_t1_inclined_vs_oracle():
    np.random.seed(7)
    obs = O.fake_obs(S2_INCLINED, Npoints=60, error=1.5e-4, errorVar=2.5e-5, tmax=80.)
    plan, dt = _plan(obs, S2_INCLINED, inclined=True)
    P = _inclined_ball(96, seed=8)
    P[0, 1, 5], P[0, 1, 6] = 1.5, 1.4      # ix^2 + iy^2 >= 4 -> prior (state.py:311-313)
    got, st, _ = _run(plan, P)
    ref, st_ref = O.logl_whx_batch(P, 2, obs, dt, LEVELS, has_inc=1)
    assert st[0] == 1
    _assert_t1(got, st, ref, st_ref, sens=oracle_sensitivity(P, 2, obs, dt, LEVELS, has_inc=1))


def test_t2_inclined_vs_ias15():
    np.random.seed(7)
    obs = O.fake_obs(S2_INCLINED, Npoints=60, error=1.5e-4, errorVar=2.5e-5, tmax=80.)
    plan, _ = _plan(obs, S2_INCLINED, inclined=True)
    P = _inclined_ball(16, seed=9)
    got, st, _ = _run(plan, P)
    ref, st_ref = O.logl_ias15_batch(P, 2, obs, hill_factor=1.0, has_inc=1)
    assert (st == st_ref).all()
    assert np.abs(got - ref).max() < T2_ABS


def test_inclined_kernel_with_zero_inclination_equals_planar():
    """ix = iy = 0 through the 3-D kernel is bit-identical to the planar kernel."""
    obs = s2_obs_oracle()
    plan2, _ = _plan(obs, S2_PLANETS)
    plan3, _ = _plan(obs, S2_PLANETS, inclined=True)
    P = _ball(S2_PLANETS, 64, seed=10)
    a, sa, _ = _run(plan2, P)
    b, sb, _ = _run(plan3, P)
    np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(sa, sb)


def test_state_api_inclined_free_parameters():
    """A State whose planets carry ix/iy (free) maps onto an inclined plan (7 rows per planet)."""
    torch = _torch()
    from rvmcmc import state

    s = state.State(planets=[dict(p) for p in S2_INCLINED])
    assert s.Nvars == 14
    pm = s.param_map()
    assert pm.inclined and pm.identity
    np.random.seed(7)
    obs = O.fake_obs(S2_INCLINED, Npoints=60, error=1.5e-4, errorVar=2.5e-5, tmax=80.)
    X = torch.as_tensor(np.repeat(s.get_params()[:, None], 3, 1), device="cuda")
    lp, st, _ = s.get_logp_batch(obs, X, hill_factor=1.0)
    ref, _ = O.logl_ias15_batch(O.pal_params(S2_INCLINED)[None], 2, obs, hill_factor=1.0, has_inc=1)
    assert (st.cpu().numpy() == 0).all()
    assert np.abs(lp.cpu().numpy() - ref[0]).max() < T2_ABS


@pytest.mark.parametrize("n_planets", [3, 4])
def test_t1_inclined_planet_counts(n_planets):
    """3-D closed-form kick for 3 and 4 planets against the oracle."""
    planets = [dict(p, ix=0.03 * (i + 1), iy=-0.02 * i) for i, p in enumerate((S2_PLANETS + EXTRA_PLANETS)[:n_planets])]
    np.random.seed(13)
    obs = O.fake_obs(planets, Npoints=40, error=1.5e-4, errorVar=2.5e-5, tmax=50.)
    plan, dt = _plan(obs, planets, inclined=True)
    P = _ball(planets, 64, seed=40 + n_planets)
    rng = np.random.default_rng(50 + n_planets)
    P[:, :, 5:7] += 1e-3 * rng.standard_normal((64, n_planets, 2))
    got, st, _ = _run(plan, P)
    ref, st_ref = O.logl_whx_batch(P, n_planets, obs, dt, LEVELS, has_inc=1)
    _assert_t1(got, st, ref, st_ref, sens=oracle_sensitivity(P, n_planets, obs, dt, LEVELS, has_inc=1))


def test_empty_observation_set_and_odd_batch_sizes():
    """No epochs at all: chi2 = 0, logl = -0 for valid walkers; the prior still applies
    (state.py:104) but no encounter can be raised -- get_rv of an empty epoch list integrates
    nothing (state.py:61-73), so REBOUND never checks exit_min_distance; batch sizes that do not
    fill a wave (1, 33)."""
    o = O.OracleObs(tf=np.zeros(0), tb=np.zeros(0), rvf=np.zeros(0), rvb=np.zeros(0), errorf=np.zeros(0),
                    errorb=np.zeros(0), Npoints=100)
    plan, dt = _plan(o, S2_PLANETS)
    for W in (1, 33):
        P = _ball(S2_PLANETS, W, seed=W)
        if W > 1:
            P[1, 0, 1] = 0.01                      # prior
            P[2, 1, :5] = P[2, 0, :5]              # planets on top of each other: would be an encounter
            P[2, 1, 1] += 0.01                     # at t = 0, but nothing is integrated
        got, st, _ = _run(plan, P)
        ref, st_ref = O.logl_whx_batch(P, 2, o, dt, LEVELS)
        assert list(st) == list(st_ref)
        ok = st == 0
        assert np.all(got[ok] == 0.0) and np.all(np.isneginf(got[~ok]))
        if W > 1:
            assert st[1] == 1 and st[2] == 0


def test_maximum_epochs_per_direction():
    """RVM_MAX_EPOCHS_PER_DIRECTION epochs in each direction (the LDS-staged schedule at its
    limit) against the oracle; one more is an argument error (tests/test_abi_load.py)."""
    from rvmcmc import _lib

    n = 1700
    rng = np.random.default_rng(5)
    tf = np.sort(rng.uniform(0.0, 60.0, n))
    tb = -np.sort(rng.uniform(0.0, 60.0, n))
    o = O.OracleObs(tf=tf, tb=tb, rvf=1e-4 * np.sin(tf), rvb=1e-4 * np.cos(tb), errorf=np.full(n, 1.5e-4),
                    errorb=np.full(n, 1.5e-4), Npoints=2 * n)
    plan, dt = _plan(o, S2_PLANETS, max_walkers=64)
    info = plan.info()
    assert info["epochs_fwd"] == n and info["epochs_bwd"] == n
    P = _ball(S2_PLANETS, 3, seed=2)
    got, st, _ = _run(plan, P)
    ref, st_ref = O.logl_whx_batch(P, 2, o, dt, LEVELS)
    _assert_t1(got, st, ref, st_ref, sens=oracle_sensitivity(P, 2, o, dt, LEVELS))

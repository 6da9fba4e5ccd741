"""Adaptive resolution and the plan's fault counters (include/rvmcmc.h).

The reference integrates every proposal with adaptive IAS15 (state.py:36-73), so its accuracy does
not depend on where a walker is; a plan's Wisdom-Holman step is fixed from the sampler's initial
state.  With rvm_config.resolve_tol a direction whose extrapolation-error estimate (the chi2
change when the coarsest Richardson level is dropped) exceeds resolve_tol / 2 first gets the
extension level joined to its stored levels, and if that does not settle it is integrated again
with every step halved, up to resolve_max times.  Checked here:

  * T1 of the adaptive kernel against the oracle's restatement of the same rule
    (oracle.logl_whx_adapt_batch), both launch layouts, on a wide ball that refines heavily;
  * the bench's tight ball never refines, and gives the bits of a plan without the rule;
  * resolve_max = 0 flags (UNRESOLVED) exactly the walkers the oracle flags;
  * a level-split hand-off that gives up is counted (rvm_plan_faults), its walkers are NONFINITE,
    the plan stays poisoned until reset, and after the reset the next launch is bit-identical to a
    fresh plan's.
Reference-physics (IAS15) accuracy of the rule over the proposals a sampler makes is in
tests/test_gpu_ias15_decisions.py.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle as O
from conftest import S2_PLANETS, S2_SCALES, s2_obs_oracle

pytestmark = pytest.mark.gpu

TOL, RMAX = 5e-7, 4
T1_REL = 1e-11 * 35.0  # tests/test_gpu_logl.py: 1e-11 sum|w| (levels 4..7)


def _torch():
    import torch

    assert torch.cuda.is_available()
    return torch


def _plan(obs, W, resolve=(TOL, RMAX)):
    from rvmcmc import engine

    dt, mult, hint = engine.IntegratorConfig().plan_args(S2_PLANETS)
    t, rv, er = engine.obs_arrays(obs)
    return engine.LoglPlan(t, rv, er, obs.Npoints, 2, dt, mult, W, period_hint=hint, resolve=resolve), dt, mult


def _x0():
    return np.array([p[k] for p in S2_PLANETS for k in "mahkl"]), np.array([S2_SCALES[k] for _ in S2_PLANETS
                                                                             for k in "mahkl"])


def wide_walkers(W, ball=0.6, seed=3):
    """Half a sampler-like ball (x0 + ball * scales * N(0,1), mcmc.py:45-51), half stretch
    proposals between its members (q = c - z (c - x), z in [1/2, 2]): [W][10] kernel rows."""
    x0, sc = _x0()
    rng = np.random.default_rng(seed)
    n = W // 2
    X = x0 + ball * sc * rng.standard_normal((n, 10))
    j = rng.integers(0, n, W - n)
    z = (rng.random(W - n) + 1.0) ** 2 / 2.0
    Q = X[j] - z[:, None] * (X[j] - X[:W - n])
    return np.concatenate([X, Q])


def _oracle_P(X):
    P = np.zeros((len(X), 2, 7))
    P[:, :, :5] = X.reshape(-1, 2, 5)
    return P


def _run(plan, X):
    torch = _torch()
    K = torch.as_tensor(np.ascontiguousarray(X.T), device="cuda")
    lp, st, _ = plan.logl(K)
    torch.cuda.synchronize()
    return lp.cpu().numpy(), st.cpu().numpy()


def _par(fn, P, nt=16):
    idx = np.array_split(np.arange(len(P)), nt)
    with ThreadPoolExecutor(nt) as ex:
        parts = list(ex.map(lambda ix: fn(P[ix]), idx))
    return [np.concatenate([p[k] for p in parts]) for k in range(len(parts[0]))]


def _par_ix(fn, P, nt=16):
    """_par for fn(P_chunk, index_chunk)."""
    idx = np.array_split(np.arange(len(P)), nt)
    with ThreadPoolExecutor(nt) as ex:
        parts = list(ex.map(lambda ix: fn(P[ix], ix), idx))
    return [np.concatenate([p[k] for p in parts]) for k in range(len(parts[0]))]


def _adapt_oracle(P, obs, dt, mult, tol=TOL, rmax=RMAX):
    return _par(lambda p: O.logl_whx_adapt_batch(p, 2, obs, dt, mult, tol, rmax), P)


def assert_t1_adaptive(got, st, P, n_planets, obs, dt, mult, tol=TOL, rmax=RMAX, has_inc=0, ctx=None, ecc_guard=0.0):
    """T1 of an adaptive-resolution launch against the oracle's restatement of the same rule
    (oracle.logl_whx_adapt_batch): statuses and logL, up to sensitivity.  Chaotic walkers (close
    approaches) and decisions at roundoff distance from their bound may legitimately go the other
    way in a second implementation: the oracle's own response to 1e-15 relative input nudges (of
    logL, of the status, of the stage reached and of the final estimate -- a difference of two
    extrapolations, which near a close approach moves by up to tens of percent under such a nudge),
    and its closest approach to any decision's bound.  ctx: the sampler's accept inputs (the
    certain-reject cut; oracle.logl_whx_adapt_batch).  Returns (stages [W][2], sensitive [W]) and,
    with ctx, the oracle's cut [W][2]."""
    W = len(got)

    def fn(p, ix=None):
        c = None if ctx is None else dict(ctx, **{k: np.asarray(ctx[k])[ix] for k in ("mode", "z", "u", "lnp0")})
        r = O.logl_whx_adapt_batch(p, n_planets, obs, dt, mult, tol, rmax, has_inc=has_inc, ctx=c, ecc_guard=ecc_guard)
        return r if ctx is not None else r + (np.zeros((len(p), 2), dtype=np.int32),)

    ref, st_ref, rf, est, margin, cut = _par_ix(fn, P)
    sens = np.zeros(W)
    flips = np.zeros(W, dtype=bool)
    for pl, par, sgn in [(0, 4, 1), (-1, 4, -1), (0, 1, 1)]:
        P2 = P.copy()
        P2[:, pl, par] *= 1 + sgn * 1e-15
        r2, s2, rf2, est2, _, cut2 = _par_ix(fn, P2)
        flips |= (s2 != st_ref) | np.any(rf2 != rf, axis=1) | np.any(cut2 != cut, axis=1)
        with np.errstate(invalid="ignore"):  # (an estimate whose roundoff response is not small
            # against its distance from the bound)
            flips |= np.any(np.abs(est2 - est) > 0.02 * np.abs(est - 0.5 * tol), axis=1)
        both = (st_ref == 0) & (s2 == 0)
        sens[both] = np.maximum(sens[both], np.abs(r2[both] - ref[both]) / np.maximum(1.0, np.abs(ref[both])))
    sensitive = flips | (sens > 1e-9) | (margin.min(axis=1) < 1e-6)
    mism = st != st_ref
    assert np.all(~mism | sensitive), np.nonzero(mism & ~sensitive)
    assert mism.sum() <= max(2, W // 100)
    ok = (st == 0) & (st_ref == 0)
    err = np.abs(got[ok] - ref[ok]) / np.maximum(1.0, np.abs(ref[ok]))
    bound = np.maximum(T1_REL, 1e3 * sens[ok])
    bad = (err > bound) & ~sensitive[ok]
    assert not bad.any(), (np.nonzero(ok)[0][bad][:10], err[bad][:10])
    assert np.mean(err <= T1_REL) > 0.9
    # walkers the oracle leaves UNRESOLVED are UNRESOLVED on the device too (up to sensitivity)
    assert np.all(((st == 4) == (st_ref == 4)) | sensitive)
    if ctx is not None:
        return rf, sensitive, cut
    return rf, sensitive


# a few walkers: the extension after the main pass (RVM_CX_MIN_WALKERS); 512: its concurrent wave in the
# LDS-coupled layout; 6144: the level-split layout with the extension as a fifth level (bench shape)
@pytest.mark.parametrize("W", [24, 512, 6144])
def test_t1_adaptive_wide_ball(W):
    obs = s2_obs_oracle()
    plan, dt, mult = _plan(obs, W)
    assert plan.ext_mult == O.ext_multiplier(mult, RMAX) == max(mult) + 1
    X = wide_walkers(W)
    got, st = _run(plan, X)
    f = plan.faults(reset=True)
    rf, sensitive = assert_t1_adaptive(got, st, _oracle_P(X), 2, obs, dt, mult)
    print(f"W={W}: oracle walker-directions at the extension {int((rf == 1).sum())}, halved {int((rf >= 2).sum())}; "
          f"kernel counters {f}, statuses {np.bincount(st, minlength=5).tolist()}, sensitive {int(sensitive.sum())}")
    assert (rf == 1).sum() >= max(1, W // 20) and (rf >= 2).sum() >= max(1, W // 20), \
        "the wide ball must exercise both stages"
    assert f["refined"] > 0 and f["handoff_timeouts"] == 0
    assert f["unresolved"] == int((st == 4).sum())


def test_tight_ball_never_refines_and_keeps_the_bits():
    """The bench config (6144 walker slots of the tight S2 ball): no walker crosses the bound, so
    the rule costs nothing and changes no bit."""
    obs = s2_obs_oracle()
    W = 6144
    x0, sc = _x0()
    X = x0 + 1e-3 * sc * np.random.default_rng(7).standard_normal((W, 10))
    plan, _, _ = _plan(obs, W)
    plan_off, _, _ = _plan(obs, W, resolve=(0.0, 0))
    got, st = _run(plan, X)
    got0, st0 = _run(plan_off, X)
    f = plan.faults()
    np.testing.assert_array_equal(st, st0)
    np.testing.assert_array_equal(got, got0)
    assert f == dict(handoff_timeouts=0, nonfinite=0, unresolved=0, refined=0, truncated=0, floor_settled=0, skipped=0), f


def test_flag_only_matches_oracle():
    """resolve_max = 0: walkers above the bound are reported UNRESOLVED (logl -inf), not refined."""
    obs = s2_obs_oracle()
    W = 256
    X = wide_walkers(W, ball=0.3, seed=11)
    plan, dt, mult = _plan(obs, W, resolve=(TOL, 0))
    got, st = _run(plan, X)
    ref, st_ref, rf, est, margin = _adapt_oracle(_oracle_P(X), obs, dt, mult, TOL, 0)
    near = margin.min(axis=1) < 1e-6
    assert (st_ref == 4).sum() > 10
    assert np.all((st == st_ref) | near)
    assert np.all(np.isneginf(got[st == 4]))
    f = plan.faults()
    assert f["unresolved"] == int((st == 4).sum()) and f["refined"] == 0


@pytest.mark.parametrize("resolve", [(0.0, 0), (TOL, RMAX)], ids=["fixed-split", "adaptive-lsx"])
def test_handoff_timeout_is_reported_and_reset(resolve):
    """A level-split hand-off that gives up (forced by a 10 ns timeout) is counted, its walkers
    are NONFINITE, later launches on the poisoned plan report NONFINITE rather than stale values,
    check_faults raises, and after the reset the next launch gives a fresh plan's bits.
    The adaptive plan runs the extension as a fifth level of the split layout (lsx), whose
    combiners start once their own level is integrated: they may find every value already there
    and never wait, so there a timeout that did not fire must change nothing."""
    from rvmcmc import _lib

    obs = s2_obs_oracle()
    W = 6144
    x0, sc = _x0()
    X = x0 + 1e-3 * sc * np.random.default_rng(5).standard_normal((W, 10))
    fresh, _, _ = _plan(obs, W, resolve)
    want, st_want = _run(fresh, X)
    plan, _, _ = _plan(obs, W, resolve)
    plan.set_handoff_timeout(1e-8)
    got0, st = _run(plan, X)
    f = plan.faults()
    if resolve[1] > 0 and f["handoff_timeouts"] == 0:
        assert f["nonfinite"] == 0, f
        np.testing.assert_array_equal(st, st_want)
        np.testing.assert_array_equal(got0, want)
        return
    assert f["handoff_timeouts"] > 0 and f["nonfinite"] > 0, f
    assert (st == _lib.RVM_STATUS_NONFINITE).sum() == f["nonfinite"]
    plan.set_handoff_timeout(2.0)
    _, st2 = _run(plan, X)  # poisoned workspace: nothing stale passes as a value
    assert np.all(st2 == _lib.RVM_STATUS_NONFINITE)
    with pytest.raises(_lib.RvmError, match="hand-off timeout"):
        plan.check_faults("test")  # (reads and resets)
    got, st3 = _run(plan, X)
    np.testing.assert_array_equal(st3, st_want)
    np.testing.assert_array_equal(got, want)
    assert plan.faults()["handoff_timeouts"] == 0


def test_level_split_encounter_on_the_last_lower_lane_stays_local():
    """Regression (found by the wide-ball T1 test above): the level-split head -> tail hand-off
    rebuilt the 64-bit encounter mask from two 32-bit readfirstlane values and the lower one
    sign-extended, so an encounter of the walker on lanes 30/31 (slot 15 of a 32-walker group) marked
    all 16 walkers of the group's upper half ENCOUNTER.  Walkers with planet 2 beside planet 1 on
    slot 15 of every other group of a tight ball: every other walker must stay OK, as the oracle says."""
    obs = s2_obs_oracle()
    W = 6144
    x0, sc = _x0()
    X = x0 + 1e-3 * sc * np.random.default_rng(9).standard_normal((W, 10))
    hit = np.arange(15, W, 64)
    X[hit, 6] = X[hit, 1] * 1.01  # planet 2 next to planet 1: an encounter from t = 0
    X[hit, 9] = X[hit, 4] + 0.01
    plan, dt, mult = _plan(obs, W)
    got, st = _run(plan, X)
    ref, st_ref, _, _, _ = _adapt_oracle(_oracle_P(X), obs, dt, mult)
    assert np.all(st_ref[hit] == 2) and np.all(np.delete(st_ref, hit) == 0)
    np.testing.assert_array_equal(st, st_ref)


@pytest.mark.parametrize("W", [4096, 12288])  # halves of 2048 (LDS-coupled) / 6144 (level-split) walkers
def test_certain_reject_cut_matches_oracle(W):
    """A fused stretch half-step (the sampler's own launch) on a wide ensemble: refinements whose
    proposal is rejected whatever further passes give stop early (rvm_plan_faults `truncated`);
    every proposal's logL and status follow the oracle's restatement of the rule with the same
    accept inputs (Philox draws restated, tests/philox_ref.py), and the decisions are the sampler's
    emcee test on those values.  An accepted proposal is never cut: its value is fully resolved."""
    torch = _torch()
    import ias15_parity as IP
    from philox_ref import stretch_uniforms
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.state import State

    s = State(planets=[dict(p) for p in S2_PLANETS])
    obs = s2_obs_oracle()
    X0 = wide_walkers(W, ball=0.6, seed=13)
    ens = EnsembleSampler(W, s, obs, seed=5)
    ens.set_positions(X0)
    ens.compute_lnprob()
    n, it = ens.nloc, ens.iteration
    before = ens.pos[0].t().cpu().numpy().copy()
    c = ens.pos[1].t().cpu().numpy().copy()
    lnp0 = ens.lnp[0].cpu().numpy().copy()
    ens.plan.faults(reset=True)
    ens.half_step(ens.pos[0], ens.lnp[0], ens.pos[1], 0)
    torch.cuda.synchronize()
    f = ens.plan.faults(reset=True)
    got, st = ens._lnp_new.cpu().numpy(), ens._status.cpu().numpy()
    after = ens.pos[0].t().cpu().numpy()
    u1, u2, u3 = stretch_uniforms(ens.seed, ens.global_begin(0), n, it, 0)
    q, z = IP.stretch_proposal(before, c, u1, u2, ens.a)
    plan = ens.plan
    ctx = dict(mode=np.ones(n, dtype=np.int32), dim=s.Nvars, z=z, u=u3, lnp0=lnp0)
    assert plan.ecc_guard > 0.0  # (the sampler's plan carries the eccentricity guard)
    rf, sensitive, cut = assert_t1_adaptive(got, st, IP.to_oracle(s.param_map(), q), 2, obs, plan.dt, plan.mult,
                                            plan.resolve_tol, plan.resolve_max, ctx=ctx, ecc_guard=plan.ecc_guard)
    ncut = int(cut.sum())
    print(f"W={W}: directions extended {int((rf == 1).sum())}, halved {int((rf >= 2).sum())}, cut {ncut} "
          f"(oracle); kernel {f}")
    assert ncut > 10 and abs(f["truncated"] - ncut) <= int(sensitive.sum())
    with np.errstate(invalid="ignore"):
        acc = (s.Nvars - 1.0) * np.log(z) + got - lnp0 > np.log(u3)
    np.testing.assert_array_equal(np.any(after != before, axis=1), acc)
    assert not np.any(acc & np.any(cut == 1, axis=1) & ~sensitive)


def test_near_parabolic_pericentre_reports_the_encounter(hd_obs_oracle):
    """Regression (found when the samplers began raising on NONFINITE, HD155358 posterior run):
    two affine proposals whose outer planet has e = 0.98 / 0.93 (pericentre inside the inner
    planet's orbit, within exit_min_distance of the star) came out NONFINITE: a Halley step from a
    guess far outside the Stumpff series' range gave a NaN correction, which the acceptance test
    let through.  The oracle's solver, and IAS15, report the encounter; so must the kernel, with the
    adaptive resolution off and on."""
    from rvmcmc import engine

    obs = hd_obs_oracle
    # free parameters a, h, k, m, l per planet ((Ex)HD155358.ipynb order)
    Q = np.array([[0.6657403462735857, -0.03598508261780334, -0.22616251032911833, 0.001067427963625652,
                   4.809278256084164, 1.0225890089859921, 0.5008569502269338, 0.839486028623608,
                   0.000508558297134821, 1.813555010417457],
                  [0.6674899135343648, -0.09193415567815766, 0.3058258300122595, 0.000628834189154814,
                   5.562596065758877, 1.0267865106849083, -0.8167984417091974, 0.45176536412785595,
                   0.0008402837623474788, 1.4987361800115173]])
    P = np.zeros((len(Q), 2, 7))
    for p in range(2):
        a, h, k, m, l = Q[:, 5 * p:5 * p + 5].T
        P[:, p, :5] = np.stack([m, a, h, k, l], 1)
    sol = [{"m": 8.84031737e-04, "a": 6.57730330e-01, "h": -9.72263877e-02, "k": -7.82798396e-02, "l": 4.42804990},
           {"m": 8.30379710e-04, "a": 1.04404207, "h": -2.05622789e-02, "k": -1.08797961e-01, "l": 1.49919861}]
    dt, mult, hint = engine.IntegratorConfig().plan_args(sol)
    t, rv, er = engine.obs_arrays(obs)
    _, st_ref = O.logl_whx_batch(P, 2, obs, dt, mult)
    _, st_ias = O.logl_ias15_batch(P, 2, obs)
    assert st_ref.tolist() == [2, 2] and st_ias.tolist() == [2, 2]
    K = np.concatenate([P[:, p, :5].T for p in range(2)], 0)
    for res in [(0.0, 0), engine.IntegratorConfig().resolve()]:
        plan = engine.LoglPlan(t, rv, er, obs.Npoints, 2, dt, mult, 64, period_hint=hint, resolve=res)
        _, st = _run(plan, K.T)
        assert st.tolist() == [2, 2], (res, st)
        assert plan.faults()["nonfinite"] == 0


@pytest.mark.parametrize("W", [512, 6144])
def test_t1_eccentricity_guard(W):
    """rvm_plan_set_verify_eccentricity: walkers with a planet above the guard get the extension
    whatever their estimate (IntegratorConfig.verify_speedup; the sampler plans carry it).  Both
    layouts against the oracle's restatement of the same rule; the guard must add extensions."""
    from rvmcmc import engine

    obs = s2_obs_oracle()
    guard = engine.IntegratorConfig().ecc_guard(S2_PLANETS)
    assert 0.26 < guard < 0.27
    dt, mult, hint = engine.IntegratorConfig().plan_args(S2_PLANETS)
    t, rv, er = engine.obs_arrays(obs)
    plan = engine.LoglPlan(t, rv, er, obs.Npoints, 2, dt, mult, W, period_hint=hint, resolve=(TOL, RMAX, guard))
    assert plan.ecc_guard == guard
    X = wide_walkers(W, ball=0.3, seed=21)
    got, st = _run(plan, X)
    rf, _ = assert_t1_adaptive(got, st, _oracle_P(X), 2, obs, dt, mult, ecc_guard=guard)
    rf0 = O.logl_whx_adapt_batch(_oracle_P(X), 2, obs, dt, mult, TOL, RMAX)[2]
    print(f"W={W}: directions extended {int((rf == 1).sum())} with the guard, {int((rf0 == 1).sum())} without")
    assert (rf >= 1).sum() > (rf0 >= 1).sum()


@pytest.mark.parametrize("system", ["s2", "hd155358"])
def test_refinement_layouts_bit_identical(system):
    """The refinement kernel's layouts -- teams (passes 1, 2, 3 at once, the default; 2 and 4 teams),
    one team with each direction on its own workgroup (RVM_REFINE_TEAMS=0), both directions in one
    workgroup (RVM_REFINE_SPLIT=0) -- take the same decisions with the same bits: speculative
    iterations of the sampler at a steady state (extensions, halving passes, certain rejects,
    two-pass walkers; HD155358's launches climb to passes 3 and 4), positions, log-probabilities and
    plan counters compared."""
    import os

    from conftest import ROOT, hd_planets
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.state import State

    torch = _torch()
    if system == "s2":
        planets, obs = S2_PLANETS, s2_obs_oracle
        X0 = np.load(os.path.join(ROOT, "scripts", "probe", "ens_it2000.npy"))
        iters = 4
    else:
        planets = hd_planets()
        obs = lambda: O.obs_from_file(os.path.join(ROOT, "tests", "golden", "HD155358.vels"), Npoints=100)  # noqa: E731
        X0 = np.load(os.path.join(ROOT, "scripts", "probe", "ens_hd155358_it1000.npy"))
        iters = 6
    runs = []
    for env in ({}, {"RVM_REFINE_TEAMS": "2"}, {"RVM_REFINE_TEAMS": "4"}, {"RVM_REFINE_TEAMS": "0"},
                {"RVM_REFINE_SPLIT": "0"}):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            s = State(planets=[dict(p) for p in planets])
            ens = EnsembleSampler(len(X0), s, obs(), seed=2017)  # (a fresh observation set: fresh plans)
            ens.set_positions(X0)
            ens.compute_lnprob()
            ens.plan.faults(reset=True)
            for _ in range(iters):
                ens.step()
            torch.cuda.synchronize()
            runs.append((ens.gather_positions(), np.concatenate([l.cpu().numpy() for l in ens.lnp]),
                         ens.plan.faults(reset=True)))
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    assert runs[0][2]["refined"] > 0 and runs[0][2]["truncated"] > 0
    assert runs[0][2]["handoff_timeouts"] == 0
    for X, lp, f in runs[1:]:
        np.testing.assert_array_equal(X, runs[0][0])
        np.testing.assert_array_equal(lp, runs[0][1])
        assert f == runs[0][2], (f, runs[0][2])


def test_certain_reject_can_be_switched_off():
    """IntegratorConfig.certain_reject = False (rvm_plan_set_certain_reject): no refinement is cut
    short -- every open walker refines to the bound -- and the sampler still runs at the steady
    state."""
    import dataclasses
    import os

    from conftest import ROOT
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.state import State

    torch = _torch()
    X0 = np.load(os.path.join(ROOT, "scripts", "probe", "ens_it2000.npy"))
    s = State(planets=[dict(p) for p in S2_PLANETS])
    s.integrator = dataclasses.replace(s.integrator, certain_reject=False)
    ens = EnsembleSampler(len(X0), s, s2_obs_oracle(), seed=2017)
    assert not ens.plan.certain_reject
    ens.set_positions(X0)
    ens.compute_lnprob()
    for _ in range(2):
        ens.step()
    torch.cuda.synchronize()
    f = ens.plan.faults(reset=True)
    assert f["refined"] > 0 and f["truncated"] == 0 and f["unresolved"] == 0, f


@pytest.mark.parametrize("W,passes", [(32, "1"), (256, "1"), (512, "1"), (32, "2"), (256, "2")])
def test_eager_halving_passes_bit_identical(W, passes):
    """Plain launches of few walkers run the first halving pass (RVM_EAGER_PASSES=2: the first two)
    of every walker beside the likelihood kernel (rvm_refine.hip eager_kernel) and the refinement
    kernel replays them: the same logL, status bits and plan counters as the refinement kernel
    integrating them after the likelihood kernel (RVM_EAGER=0), on wide-ball walkers (extensions,
    one- and two-pass walkers, deeper ones, encounters, prior rejections)."""
    import os

    obs = s2_obs_oracle()
    X = wide_walkers(W, ball=0.3, seed=5)
    res = []
    for env in ("1", "0"):
        old = {k: os.environ.get(k) for k in ("RVM_EAGER", "RVM_EAGER_PASSES")}
        os.environ["RVM_EAGER"] = env
        os.environ["RVM_EAGER_PASSES"] = passes
        try:
            plan, _, _ = _plan(obs, W)
            got, st = _run(plan, X)
            res.append((got, st, plan.faults(reset=True)))
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
    np.testing.assert_array_equal(res[0][1], res[1][1])
    np.testing.assert_array_equal(res[0][0], res[1][0])
    assert res[0][2] == res[1][2], (res[0][2], res[1][2])
    assert res[0][2]["refined"] > 0

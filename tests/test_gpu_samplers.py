"""Device samplers vs numpy restatements of the reference samplers with injected random numbers.

* emcee 2.2.1 stretch move (EnsembleSampler.sample/_propose_stretch):
  decisions must be identical to a numpy restatement fed the same (u1, u2, u3) draws, except
  walkers with |lnpdiff - ln u3| < 1e-9 (counted; none expected at these sizes).
* Metropolis-Hastings (mcmc.py:89-121) with injected N(0,1) and U(0,1).
"""
import numpy as np
import pytest

import oracle as O
from conftest import S2_PLANETS, S2_SCALES, s2_obs_oracle

pytestmark = pytest.mark.gpu


def _torch():
    import torch

    assert torch.cuda.is_available()
    return torch


def _state_and_obs():
    from rvmcmc import state

    s = state.State(planets=[dict(p) for p in S2_PLANETS])
    return s, s2_obs_oracle()


def _oracle_logl(X, s, obs, dt):
    """X [W][dim] in the State's free-parameter order -> oracle logL with the kernel algorithm
    (the State's integrator level sequence)."""
    pm = s.param_map()
    P = np.stack([O.kernel_params_to_oracle(pm.vector_to_kernel_np(x)[:, None], 2)[0] for x in X])
    return O.logl_whx_batch(P, 2, obs, dt, s.integrator.mult)[0]


def numpy_stretch_half(p_s0, lnp_s0, c, u1, u2, u3, lnprob_fn, a=2.0):
    """emcee 2.2.1 _propose_stretch + in-place update, restated (rows = walkers)."""
    Ns, dim = p_s0.shape
    Nc = len(c)
    zz = ((a - 1.) * u1 + 1) ** 2. / a
    rint = np.floor(u2 * Nc).astype(int)
    q = c[rint] - zz[:, None] * (c[rint] - p_s0)
    newlnp = lnprob_fn(q)
    lnpdiff = (dim - 1.) * np.log(zz) + newlnp - lnp_s0
    acc = lnpdiff > np.log(u3)
    p = p_s0.copy()
    l = lnp_s0.copy()
    p[acc] = q[acc]
    l[acc] = newlnp[acc]
    return p, l, acc, np.abs(lnpdiff - np.log(u3))


def test_stretch_decisions_match_numpy_emcee():
    torch = _torch()
    from rvmcmc.ensemble import EnsembleSampler

    s, obs = _state_and_obs()
    W, dim = 128, s.Nvars
    rng = np.random.default_rng(0)
    scales = np.array([S2_SCALES[k] for k in s.get_rawkeys()])
    X0 = s.get_params()[None] + 1e-3 * scales * rng.standard_normal((W, dim))
    ens = EnsembleSampler(W, s, obs, seed=1)
    ens.set_positions(X0)
    ens.compute_lnprob()
    dt = ens.plan.dt
    lnp0 = np.concatenate([l.cpu().numpy() for l in ens.lnp])
    ref_lnp0 = _oracle_logl(X0, s, obs, dt)
    t1 = 1e-11 * float(np.abs(O.richardson_weights(s.integrator.mult)).sum())
    np.testing.assert_allclose(lnp0, ref_lnp0, rtol=t1, atol=0)  # T1 tier (tests/test_gpu_logl.py)
    n = W // 2
    pos = [X0[:n].copy(), X0[n:].copy()]
    lnp = [lnp0[:n].copy(), lnp0[n:].copy()]
    near = 0
    for it in range(3):
        for half in (0, 1):
            u1, u2, u3 = rng.random(n), rng.random(n), rng.random(n)
            dp = torch.as_tensor(np.concatenate([u1, u2]), device="cuda")
            da = torch.as_tensor(u3, device="cuda")
            A, B = ens.pos[half], ens.pos[1 - half]
            ens.half_step(A, ens.lnp[half], B, half, draws_propose=dp, draws_accept=da)
            p_new, l_new, acc, margin = numpy_stretch_half(pos[half], lnp[half], pos[1 - half], u1, u2, u3,
                                                           lambda q: _oracle_logl(q, s, obs, dt))
            near += int((margin < 1e-9).sum())
            pos[half], lnp[half] = p_new, l_new
            got = ens.pos[half].t().cpu().numpy()
            same = np.all(got == p_new, axis=1) | (margin < 1e-9)
            assert same.all(), f"iteration {it} half {half}: {np.nonzero(~same)[0]}"
            # keep both sides bit-identical for the next half-step
            pos[half] = got
            lnp[half] = ens.lnp[half].cpu().numpy()
        ens.iteration += 1
    assert near == 0


def test_mh_chains_match_numpy():
    torch = _torch()
    from rvmcmc.mcmc import MhChains

    s, obs = _state_and_obs()
    C, dim = 64, s.Nvars
    scales = {"m": 1.e-3, "a": 0.3, "h": 0.5, "k": 0.5, "l": np.pi / 2.}  # mcmc_benchmark_mh.py:52
    mh = MhChains(s, obs, scales, 1e-3, C, seed=3)
    dt = mh.plan.dt
    sc = np.array([scales[k] for k in s.get_rawkeys()])
    X = np.tile(s.get_params()[:, None], (1, C))
    lnp = _oracle_logl(X.T, s, obs, dt)
    rng = np.random.default_rng(5)
    for it in range(3):
        g = rng.standard_normal((dim, C))
        u = rng.random(C)
        mh.step(draws_propose=torch.as_tensor(g, device="cuda"), draws_accept=torch.as_tensor(u, device="cuda"))
        Q = X + (1e-3 * sc)[:, None] * g
        lq = _oracle_logl(Q.T, s, obs, dt)
        acc = np.exp(lq - lnp) > u
        X = np.where(acc[None], Q, X)
        lnp = np.where(acc, lq, lnp)
        got = mh.X.cpu().numpy()
        np.testing.assert_array_equal(got, X)


def test_ensemble_reproducible_and_moves():
    from rvmcmc.ensemble import EnsembleSampler

    s, obs = _state_and_obs()
    W = 256
    rng = np.random.default_rng(1)
    scales = np.array([S2_SCALES[k] for k in s.get_rawkeys()])
    X0 = s.get_params()[None] + 1e-3 * scales * rng.standard_normal((W, s.Nvars))
    runs = []
    for _ in range(2):
        e = EnsembleSampler(W, s, obs, seed=42)
        e.set_positions(X0)
        for _ in range(5):
            e.step()
        runs.append((e.gather_positions(), e.gather_lnprob(), e.acceptance_fraction().cpu().numpy()))
    np.testing.assert_array_equal(runs[0][0], runs[1][0])
    assert 0.05 < runs[0][2].mean() < 0.95
    assert np.isfinite(runs[0][1]).all()


@pytest.mark.parametrize("case", ["s2", "s2_fixed_params", "s2_wide", "s2_two_groups", "three_planets"])
def test_fused_half_step_matches_three_launch_path(case):
    """rvm_stretch_half_step (propose + logL + accept in one launch) against the separate
    propose / logl / accept launches with the same Philox draws: positions, lnp and accept counts
    bit-identical after several iterations.  Covers fixed (non-free) kernel rows, prior /
    encounter proposals (wide ball), two walker groups per block (large halves) and 3 planets."""
    torch = _torch()
    from rvmcmc import state
    from rvmcmc.ensemble import EnsembleSampler

    planets = [dict(p) for p in S2_PLANETS]
    kw = {}
    W, rel, iters = 256, 1e-3, 4
    if case == "s2_fixed_params":
        kw = dict(ignore_params=[["h"], ["k", "l"]])
    elif case == "s2_wide":
        rel = 0.1
    elif case == "s2_two_groups":
        W, iters = 2 * 8256, 2
    elif case == "three_planets":
        planets.append({"m": 1e-3, "a": 2.6, "h": 0.05, "k": 0.0, "l": 1.0})
    s = state.State(planets=planets, **kw)
    obs = s2_obs_oracle()
    rng = np.random.default_rng(3)
    scales = np.array([S2_SCALES[k] for k in s.get_rawkeys()])
    X0 = s.get_params()[None] + rel * scales * rng.standard_normal((W, s.Nvars))
    runs = []
    for fused in (True, False):
        e = EnsembleSampler(W, s, obs, seed=77)
        assert e.fused
        e.fused = fused
        e.speculative = False  # one launch per half-step (the speculative iteration: next test)
        e.set_positions(X0)
        for _ in range(iters):
            e.step()
        torch.cuda.synchronize()
        runs.append((e.gather_positions(), e.gather_lnprob(), e.naccepted.cpu().numpy()))
    np.testing.assert_array_equal(runs[0][0], runs[1][0])
    np.testing.assert_array_equal(runs[0][1], runs[1][1])
    np.testing.assert_array_equal(runs[0][2], runs[1][2])
    acc = runs[0][2].sum() / (W * iters)
    assert 0.0 < acc < 1.0
    if case == "s2_wide":
        assert not np.isfinite(runs[0][1]).all() or acc < 0.5  # prior / encounter proposals exercised


@pytest.mark.parametrize("case", ["s2", "s2_fixed_params", "s2_wide", "one_planet", "three_planets", "inclined",
                                  "s2_large", "s2_config2", "s2_bench_shape", "s2_bench_shape_wide"])
def test_speculative_iteration_matches_half_steps(case):
    """rvm_stretch_iteration_begin / _end (both half-steps from one launch of 3 n walker slots,
    half 1 evaluated against both possible positions of its partner) against two fused half-step
    launches: positions, lnp, accept counts and the mirrors bit-identical after several
    iterations.  Covers fixed kernel rows, prior / encounter proposals, 1 / 2 / 3 planets (1, 2 and
    4 lanes per walker), inclined orbits and a batch whose 3 n slots need two-group blocks."""
    torch = _torch()
    from rvmcmc import state
    from rvmcmc.ensemble import EnsembleSampler

    planets = [dict(p) for p in S2_PLANETS]
    kw = {}
    W, rel, iters = 256, 1e-3, 5
    if case == "s2_fixed_params":
        kw = dict(ignore_params=[["h"], ["k", "l"]])
    elif case == "s2_wide":
        rel = 0.1
    elif case == "one_planet":
        planets = planets[:1]
    elif case == "three_planets":
        planets.append({"m": 1e-3, "a": 2.6, "h": 0.05, "k": 0.0, "l": 1.0})
    elif case == "inclined":
        planets[0].update(ix=0.05, iy=-0.02)
        planets[1].update(ix=0.01, iy=0.03)
    elif case == "s2_large":
        W, iters = 2 * 8256, 2
    elif case == "s2_config2":  # BASELINE config 2: 1024 walkers, 2-planet S2 (512 per half, 1536 slots)
        W, iters = 1024, 4
    elif case == "s2_bench_shape":  # bench.py's shape: the 6144-slot launch runs the level-split layout
        W, iters = 4096, 3
    elif case == "s2_bench_shape_wide":  # the same under uneven load: redone segments, prior / encounter exits
        W, iters, rel = 4096, 3, 0.1
    s = state.State(planets=planets, **kw)
    obs = s2_obs_oracle()
    rng = np.random.default_rng(5)
    scales = np.array([S2_SCALES.get(k, 0.05) for k in s.get_rawkeys()])
    X0 = s.get_params()[None] + rel * scales * rng.standard_normal((W, s.Nvars))
    runs = []
    for spec in (True, False):
        e = EnsembleSampler(W, s, obs, seed=91)
        e.speculative = spec
        e.set_positions(X0)
        for _ in range(iters):
            e.step()
        torch.cuda.synchronize()
        assert e.speculating() == spec
        mirrors = [m.cpu().numpy() for m in e.pos_aos]
        for h in (0, 1):
            np.testing.assert_array_equal(mirrors[h], e.pos[h].t().cpu().numpy())  # mirrors in step
        runs.append((e.gather_positions(), e.gather_lnprob(), e.naccepted.cpu().numpy(), e.nevals))
    np.testing.assert_array_equal(runs[0][0], runs[1][0])
    np.testing.assert_array_equal(runs[0][1], runs[1][1])
    np.testing.assert_array_equal(runs[0][2], runs[1][2])
    assert runs[0][3] == runs[1][3] == W * iters + W  # useful evaluations only (+ the initial lnprob)
    acc = runs[0][2].sum() / (W * iters)
    assert 0.0 < acc < 1.0


def test_speculation_is_chosen_by_launch_shape():
    """The bench workload (4096 walkers, 2 planets: 2048 per half) speculates -- 6144 slots in one
    launch of two-group blocks beat two launches of 2048 -- while 3 planets at 8192 walkers per GPU
    (config 5: one half already needs two-group blocks) keep one launch per half-step."""
    from rvmcmc import state
    from rvmcmc.ensemble import EnsembleSampler

    obs = s2_obs_oracle()
    s2 = state.State(planets=[dict(p) for p in S2_PLANETS])
    assert EnsembleSampler(4096, s2, obs, seed=1).speculating()
    assert EnsembleSampler(1024, s2, obs, seed=1).speculating()
    s3 = state.State(planets=[dict(p) for p in S2_PLANETS] + [{"m": 1e-3, "a": 2.6, "h": 0.05, "k": 0.0, "l": 1.0}])
    assert not EnsembleSampler(8192, s3, obs, seed=1).speculating()


def test_speculative_mh_is_bit_identical_to_sequential():
    """Mh(speculate=8): proposals drawn ahead and evaluated in one launch, consumed with the
    reference's test -- same chain, same logp values and the same global RNG stream as the
    sequential reference Mh (mcmc.py:107-121), including prior rejections (no uniform drawn)."""
    from rvmcmc import mcmc

    s, obs = _state_and_obs()
    runs = []
    for spec in (1, 8):
        np.random.seed(11)
        mh = mcmc.Mh(s, obs, speculate=spec)
        mh.set_scales({"m": 1.e-3, "a": 0.3, "h": 0.5, "k": 0.5, "l": np.pi / 2.})
        mh.step_size = 4e-2  # large enough for prior rejections (h, k scales 0.5)
        out = []
        for _ in range(60):
            out.append((mh.step(), mh.state.logp, tuple(mh.state.get_params())))
        mh.flush()  # proposals drawn ahead are dropped, the RNG rewound to the sequential chain's
        runs.append((out, np.random.uniform()))
    assert runs[0] == runs[1]
    moves = sum(o[0] for o in runs[0][0])
    assert 0 < moves < 60


@pytest.mark.parametrize("kind", ["mh", "smala", "smala_exact"])
def test_chain_samplers_checkpoint_resume_bit_identical(kind, tmp_path):
    """MhChains / SmalaChains: checkpoint after 2 steps, restore into a fresh sampler, 2 more
    steps == 4 uninterrupted steps (SURVEY.md §5 checkpoint / resume)."""
    from rvmcmc.mcmc import MhChains
    from rvmcmc.smala import SmalaChains

    s, obs = _state_and_obs()

    def make():
        if kind == "mh":
            return MhChains(s, obs, S2_SCALES, 1e-3, 32, seed=3)
        return SmalaChains(s, obs, eps=0.5, alpha=1e3, n_chains=16, seed=3,
                           hessian="exact" if kind == "smala_exact" else "gauss-newton")

    a = make()
    for _ in range(4):
        a.step()
    b = make()
    for _ in range(2):
        b.step()
    b.checkpoint(tmp_path / "c.npz")
    c = make()
    c.restore(tmp_path / "c.npz")
    for _ in range(2):
        c.step()
    np.testing.assert_array_equal(c.X.cpu().numpy(), a.X.cpu().numpy())
    np.testing.assert_array_equal(c.accepted.cpu().numpy(), a.accepted.cpu().numpy())


def test_reference_api_ensemble_and_mh_step():
    from rvmcmc import mcmc

    s, obs = _state_and_obs()
    np.random.seed(0)
    ens = mcmc.Ensemble(s, obs, scales=S2_SCALES, nwalkers=32)
    moved = ens.step()
    assert isinstance(moved, bool) and len(ens.states) == 32 and len(ens.lnprob) == 32
    mh = mcmc.Mh(s, obs)
    mh.set_scales({"m": 1.e-3, "a": 0.3, "h": 0.5, "k": 0.5, "l": np.pi / 2.})
    mh.step_size = 1e-4
    tries = mh.step_force()
    assert tries >= 1 and np.isfinite(mh.state.logp)


def test_reference_lnprob_shim():
    """mcmc.lnprob (mcmc.py:28-35), the emcee callback: the State's logp for a valid vector,
    -inf through priorHard (state.py:299-315), and -inf when get_logp raises -- here the
    Encounter of a near-coorbital pair (rebound.Encounter in the reference, any exception there)."""
    from rvmcmc import mcmc

    s, obs = _state_and_obs()
    e = mcmc.Mcmc(s, obs)
    x = e.state.get_params().copy()
    lp = mcmc.lnprob(x, e)
    ref = s.deepcopy()
    ref.set_params(x)
    assert np.isfinite(lp) and lp == ref.get_logp(obs)
    keys = e.state.get_rawkeys()
    a_idx = [i for i, k in enumerate(keys) if k == "a"]
    bad = x.copy()
    bad[a_idx[0]] = 0.01  # a <= 0.02
    assert mcmc.lnprob(bad, e) == -np.inf
    enc = x.copy()
    for k in ("h", "k", "l"):  # planet 2 on planet 1's orbit, 1 % wider: inside the exit distance at t = 0
        ki = [i for i, kk in enumerate(keys) if kk == k]
        enc[ki[1]] = enc[ki[0]]
    enc[a_idx[1]] = enc[a_idx[0]] * 1.01
    assert mcmc.lnprob(enc, e) == -np.inf
    with pytest.raises(Exception):
        e.state.get_logp(obs)  # (the State itself raises; the shim maps it to -inf)
    assert mcmc.lnprob(x, e) == lp  # and recovers


def test_smala_chains_run():
    from rvmcmc.smala import SmalaChains

    s, obs = _state_and_obs()
    sm = SmalaChains(s, obs, eps=0.5, alpha=1e3, n_chains=16, seed=0)
    for _ in range(5):
        sm.step()
    assert sm.iteration == 5
    assert np.isfinite(sm.cache["lp"].cpu().numpy()).all()
    assert int(sm.accepted.sum()) > 0


def _smala_numpy(lp, g, H, x, alpha, eps):
    """mcmc.py:135-150 restated in numpy for one chain: SoftAbs metric, G^-1, chol, drift."""
    lam, Q = np.linalg.eigh(-0.5 * (H + H.T))
    with np.errstate(divide="ignore", invalid="ignore"):
        lt = np.where(np.abs(alpha * lam) < 1e-8, 1.0 / alpha, lam / np.tanh(alpha * lam))
    G = Q @ np.diag(lt) @ Q.T
    Ginv = Q @ np.diag(1.0 / lt) @ Q.T
    L = np.linalg.cholesky(Ginv)
    mu = x + eps ** 2 * Ginv @ g / 2.0
    return dict(G=G, Ginv=Ginv, L=L, mu=mu, logdet=float(np.sum(np.log(1.0 / lt))))


def test_smala_derive_matches_numpy_softabs():
    """rvm_smala_derive (Jacobi eigen-solver, SoftAbs, Cholesky, drift on device) vs numpy on the
    gradient/Hessian of the same stencil launch (smala.fd_logp_grad_metric, torch)."""
    torch = _torch()
    from rvmcmc.smala import SmalaChains, fd_logp_grad_metric

    s, obs = _state_and_obs()
    C_, dim = 24, s.Nvars
    rng = np.random.default_rng(4)
    scales = np.array([S2_SCALES[k] for k in s.get_rawkeys()])
    X0 = (s.get_params()[None] + 1e-3 * scales * rng.standard_normal((C_, dim))).T.copy()
    sm = SmalaChains(s, obs, eps=0.5, alpha=1e3, n_chains=C_, X0=X0, seed=3)
    X = torch.as_tensor(X0, device="cuda")
    lp, g, H, st = fd_logp_grad_metric(sm.state, obs, X, sm.rel_step, sm.pmap, hill_factor=1.0)
    lp, g, H = lp.cpu().numpy(), g.cpu().numpy(), H.cpu().numpy()
    c = {k: v.cpu().numpy() for k, v in sm.cache.items() if k != "_c"}
    np.testing.assert_array_equal(c["lp"], lp)
    np.testing.assert_array_equal(c["grad"], g)
    assert (c["ok"] == 1).all()
    for i in range(C_):
        ref = _smala_numpy(lp[i], g[:, i], H[:, :, i], X0[:, i], 1e3, 0.5)
        G = c["G"][:, i].reshape(dim, dim)
        L = c["L"][:, i].reshape(dim, dim)
        np.testing.assert_allclose(G, ref["G"], rtol=1e-9, atol=1e-9 * np.abs(ref["G"]).max())
        np.testing.assert_allclose(L @ L.T, ref["Ginv"], rtol=1e-9, atol=1e-9 * np.abs(ref["Ginv"]).max())
        np.testing.assert_allclose(np.tril(L), L)
        np.testing.assert_allclose(c["mu"][:, i], ref["mu"], rtol=1e-10, atol=1e-14)
        assert abs(c["logdet"][i] - ref["logdet"]) < 1e-9 * max(1.0, abs(ref["logdet"]))


def test_smala_exact_metric_matches_numpy_softabs():
    """SmalaChains(hessian="exact"): rvm_logl_derivs + rvm_smala_metric (the reference's exact
    Hessian, state.py:253-294) vs numpy SoftAbs on the same exact derivatives; then a few steps."""
    torch = _torch()
    from rvmcmc.smala import SmalaChains

    s, obs = _state_and_obs()
    C_, dim = 12, s.Nvars
    rng = np.random.default_rng(8)
    scales = np.array([S2_SCALES[k] for k in s.get_rawkeys()])
    X0 = (s.get_params()[None] + 1e-3 * scales * rng.standard_normal((C_, dim))).T.copy()
    sm = SmalaChains(s, obs, eps=0.5, alpha=1e3, n_chains=C_, X0=X0, seed=3, hessian="exact")
    lp, g, H, st = sm.state.get_logp_d_dd_batch(obs, torch.as_tensor(X0, device="cuda"), hill_factor=1.0)
    lp, g, H = lp.cpu().numpy(), g.cpu().numpy(), H.cpu().numpy()
    c = {k: v.cpu().numpy() for k, v in sm.cache.items() if k != "_c"}
    # the chains' logp is the likelihood launch's (adaptive resolution: T2), the derivatives the
    # hyper-dual kernel's (the same discrete likelihood to T1)
    lp_ad = sm.state.get_logp_batch(obs, torch.as_tensor(X0, device="cuda"), hill_factor=1.0)[0].cpu().numpy()
    np.testing.assert_array_equal(c["lp"], lp_ad)
    np.testing.assert_allclose(c["lp"], lp, rtol=1e-9)
    np.testing.assert_array_equal(c["grad"], g)
    assert (c["ok"] == 1).all()
    for i in range(C_):
        ref = _smala_numpy(lp_ad[i], g[:, i], H[:, :, i], X0[:, i], 1e3, 0.5)
        G = c["G"][:, i].reshape(dim, dim)
        L = c["L"][:, i].reshape(dim, dim)
        np.testing.assert_allclose(G, ref["G"], rtol=1e-9, atol=1e-9 * np.abs(ref["G"]).max())
        np.testing.assert_allclose(L @ L.T, ref["Ginv"], rtol=1e-9, atol=1e-9 * np.abs(ref["Ginv"]).max())
        np.testing.assert_allclose(c["mu"][:, i], ref["mu"], rtol=1e-10, atol=1e-14)
        assert abs(c["logdet"][i] - ref["logdet"]) < 1e-9 * max(1.0, abs(ref["logdet"]))
    for _ in range(3):
        sm.step()
    assert np.isfinite(sm.cache["lp"].cpu().numpy()).all() and int(sm.accepted.sum()) > 0


def test_reference_api_smala_step_with_exact_derivatives():
    """mcmc.Smala (mcmc.py:126-187, host control flow) on State.get_logp_d_dd's exact derivatives."""
    from rvmcmc.smala import Smala

    s, obs = _state_and_obs()
    np.random.seed(3)
    sm = Smala(s, obs, eps=0.3, alp=1e3)
    acc = sum(bool(sm.step()) for _ in range(4))
    lp, g, H = sm.state.get_logp_d_dd(obs)
    assert np.isfinite(lp) and np.isfinite(g).all() and np.allclose(H, H.T) and acc >= 1


def test_alsmala_and_run_alsmala():
    """mcmc.Alsmala (mcmc.py:191-230) and driver.run_alsmala (driver.py:171-202): the cheap step
    carries the current derivatives to the proposal; both step kinds run and move the chain."""
    from rvmcmc import driver, mcmc

    s, obs = _state_and_obs()
    np.random.seed(5)
    al = mcmc.Alsmala(s, obs, 0.3, 1e3)
    assert al.step_mala() in (True, False)
    lp, g, H = al.state.get_logp_d_dd(obs)
    prop = al.generate_proposal_mala()
    assert prop.logp_d is g and prop.logp_dd is H  # derivatives inherited, not recomputed
    bundle, h = driver.run_alsmala("t", 12, s, obs, 0.3, 1e3, 2.0, 0.0)
    assert bundle.mcmc_chain.shape == (13, s.Nvars) and np.isfinite(bundle.mcmc_chainlogp).all()
    assert len({tuple(r) for r in bundle.mcmc_chain}) > 1


def test_smala_step_matches_numpy_with_injected_draws():
    """One device SMALA step with injected z and u == mcmc.py:167-187 restated in numpy on the
    device's cached derivatives (proposal bit-close, decisions identical away from ties)."""
    torch = _torch()
    from rvmcmc.smala import SmalaChains

    s, obs = _state_and_obs()
    C_, dim, eps = 32, s.Nvars, 0.5
    sm = SmalaChains(s, obs, eps=eps, alpha=1e3, n_chains=C_, seed=5)
    for _ in range(2):
        sm.step()
    rng = np.random.default_rng(6)
    z = rng.standard_normal((C_, dim))
    u = rng.random(C_)
    x0 = sm.X.cpu().numpy().copy()
    c0 = {k: v.cpu().numpy().copy() for k, v in sm.cache.items() if k != "_c"}
    acc0 = sm.accepted.cpu().numpy().copy()
    sm.step(z=torch.as_tensor(z, device="cuda"), u=torch.as_tensor(u, device="cuda"))
    xs = sm.Xs.cpu().numpy()
    p = {k: v.cpu().numpy() for k, v in sm.prop.items() if k != "_c"}
    near = 0
    for i in range(C_):
        L0 = c0["L"][:, i].reshape(dim, dim)
        want = c0["mu"][:, i] + eps * L0 @ z[i] if c0["ok"][i] else x0[:, i]
        np.testing.assert_allclose(xs[:, i], want, rtol=1e-13, atol=1e-16)

        def logq(y, mu, G, logdet):
            d = y - mu
            return -0.5 * (d @ G @ d / eps ** 2 + dim * np.log(eps ** 2) + logdet + dim * np.log(2 * np.pi))

        G0 = c0["G"][:, i].reshape(dim, dim)
        Gp = p["G"][:, i].reshape(dim, dim)
        lr = (p["lp"][i] - c0["lp"][i] + logq(x0[:, i], p["mu"][:, i], Gp, p["logdet"][i])
              - logq(xs[:, i], c0["mu"][:, i], G0, c0["logdet"][i]))
        acc = bool(np.exp(lr) > u[i]) and c0["ok"][i] == 1 and p["ok"][i] == 1 and np.isfinite(p["lp"][i])
        if abs(lr - np.log(u[i])) < 1e-9:
            near += 1
            continue
        got = sm.accepted.cpu().numpy()[i] - acc0[i] == 1
        assert got == acc, (i, lr, np.log(u[i]))
        np.testing.assert_array_equal(sm.X.cpu().numpy()[:, i], xs[:, i] if acc else x0[:, i])
    assert near <= 1


def test_device_philox_matches_restatement():
    """rvm_stretch_propose with the built-in Philox draws == tests/philox_ref.py restatement."""
    torch = _torch()
    from philox_ref import stretch_uniforms
    from rvmcmc import _lib

    lib = _lib.load()
    dim, n0, n1, seed, it, half, begin = 10, 96, 96, 987654321987, 5, 1, 1000
    rng = np.random.default_rng(2)
    x = torch.as_tensor(rng.standard_normal((dim, n0)), device="cuda")
    c = torch.as_tensor(rng.standard_normal((dim, n1)), device="cuda")
    q = torch.empty_like(x)
    z = torch.empty(n0, dtype=torch.float64, device="cuda")
    _lib.check(lib.rvm_stretch_propose(dim, n0, begin, x.data_ptr(), n1, c.data_ptr(), 2.0, seed, it, half, 0,
                                       q.data_ptr(), z.data_ptr(), _lib.stream_handle()), "propose")
    torch.cuda.synchronize()
    u1, u2, _ = stretch_uniforms(seed, begin, n0, it, half)
    zz = ((2.0 - 1.0) * u1 + 1.0) * ((2.0 - 1.0) * u1 + 1.0) / 2.0
    j = np.floor(u2 * n1).astype(int)
    C, X = c.cpu().numpy(), x.cpu().numpy()
    np.testing.assert_array_equal(z.cpu().numpy(), zz)
    np.testing.assert_array_equal(q.cpu().numpy(), C[:, j] - zz[None] * (C[:, j] - X))

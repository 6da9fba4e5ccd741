"""GPU parity of the exact-derivative kernel (rvm_logl_derivs through the C ABI).

The reference's get_chi2_d_dd / get_logp_d_dd (state.py:218-294) integrate REBOUND's order-1 and
order-2 variational equations; rvm_logl_derivs returns the exact derivatives of the plan's own
discrete integrator (hyper-dual forward mode).  No stored reference output holds
derivatives, so the checks are:

  * D1 (same algorithm): central finite differences of the oracle's restatement of the kernel's
    integrator (oracle/rvoracle.c rvo_whx_*, the T1 reference of tests/test_gpu_logl.py), on a
    stencil of steps delta_i and 2 delta_i, Richardson-extrapolated (truncation O(delta^4)), with
    delta_i = SIG_STEP / sqrt|H_ii| a fixed fraction of the posterior width along p_i (fixed
    relative steps are truncation-limited for a and noise-limited for h, k at the same time).  Errors are measured in the posterior's own
    units: gradient |dg_i| / sqrt|H_ii|, Hessian |dH_ij| / sqrt|H_ii H_jj| (a correlation-scale
    error), so every parameter counts alike whatever its units.  FD truncation and roundoff set the
    floor: D1 tolerance 1e-6 for the gradient.  The Hessian is checked against central differences
    of the kernel's own exact gradient (noise eps/delta, tolerance 1e-6; together with the gradient
    check this pins the order-2 variations) and, loosely (1e-3: noise eps/delta^2 in directions the
    data barely constrain), against second differences of the oracle's logp.
  * D2 (reference physics): the same against finite differences of the IAS15 restatement (the
    reference's integrator), whose adaptive steps make its finite differences noisier: 1e-4.
  * logp equals rvm_logl_batch's (T1 tier), the Hessian is symmetric, a sub-set of directions
    gives the sub-block, and non-OK walkers carry the likelihood kernel's status with NaN derivatives.
"""
import numpy as np
import pytest

import oracle as O
from conftest import GOLDEN, S2_PLANETS, s2_obs_oracle
from test_gpu_logl import LEVELS, SPO, T1_REL, _ball, _kernel_params, _plan, _torch

pytestmark = pytest.mark.gpu

FLOOR = {0: 1e-4, 1: 1e-2, 2: 1e-2, 3: 1e-2, 4: 1.0, 5: 1e-2, 6: 1e-2}  # m a h k l ix iy (smala.FD_FLOOR)
D1_GRAD, D1_HESS, D1_HESS_2ND = 1e-6, 1e-6, 1e-3
SIG_STEP = 0.05


def sigma_steps(H, x=None, rows=5, cap=2e-2):
    """FD steps: SIG_STEP posterior widths along each parameter, capped at cap * max(|x_i|, floor_i)
    (directions the data barely constrain, e.g. the inclinations of a coplanar-looking fit, have a
    tiny or positive H_ii and a non-quadratic logp there)."""
    d = SIG_STEP / np.sqrt(np.abs(np.diag(H)))
    if x is not None:
        d = np.minimum(d, cap * np.array([max(abs(x[r]), FLOOR[r % rows]) for r in range(len(x))]))
    return d
D2_GRAD, D2_HESS = 1e-4, 1e-4


def _rows(np_, inclined):
    return 7 if inclined else 5


def _flat_to_oracle(v, np_, rows):
    """kernel-row vectors [N][rows*np] -> oracle params [N][np][7]"""
    N = v.shape[0]
    out = np.zeros((N, np_, 7))
    for p in range(np_):
        out[:, p, :rows] = v[:, rows * p:rows * (p + 1)]
    return out


def _fd_once(f, x, d, R):
    f0 = f[0]
    g = np.zeros(R)
    H = np.zeros((R, R))
    for i in range(R):
        fp, fm = f[1 + 2 * i], f[2 + 2 * i]
        g[i] = (fp - fm) / (2 * d[i])
        H[i, i] = (fp - 2 * f0 + fm) / (d[i] * d[i])
    k = 1 + 2 * R
    for i in range(R):
        for j in range(i):
            fpp, fpm, fmp, fmm = f[k:k + 4]
            k += 4
            H[i, j] = H[j, i] = (fpp - fpm - fmp + fmm) / (4 * d[i] * d[j])
    return f0, g, H


def _stencil(x, d):
    R = len(x)
    pts = [x.copy()]
    for i in range(R):
        for s in (1, -1):
            y = x.copy()
            y[i] += s * d[i]
            pts.append(y)
    for i in range(R):
        for j in range(i):
            for si, sj in ((1, 1), (1, -1), (-1, 1), (-1, -1)):
                y = x.copy()
                y[i] += si * d[i]
                y[j] += sj * d[j]
                pts.append(y)
    return pts


def fd_derivs(logl_fn, x, np_, rows, rel=1e-3, d=None):
    """Central differences of logl_fn ([N][np][7] -> logl[N]) at the kernel-row vector x [R],
    Richardson-extrapolated in the step (steps d and 2d, truncation O(d^4)):
    (logl, grad [R], hess [R][R]); d_i = rel * max(|x_i|, floor_i) unless given."""
    R = len(x)
    if d is None:
        d = np.array([rel * max(abs(x[r]), FLOOR[r % rows]) for r in range(R)])
    pts = _stencil(x, d) + _stencil(x, 2 * d)
    f = logl_fn(_flat_to_oracle(np.array(pts), np_, rows))
    n = len(pts) // 2
    f0, g1, H1 = _fd_once(f[:n], x, d, R)
    _, g2, H2 = _fd_once(f[n:], x, 2 * d, R)
    return f0, (4 * g1 - g2) / 3, (4 * H1 - H2) / 3


def scaled_errors(g, H, g_ref, H_ref):
    s = np.sqrt(np.abs(np.diag(H_ref)))
    eg = np.abs(g - g_ref) / s
    eH = np.abs(H - H_ref) / np.outer(s, s)
    return float(eg.max()), float(eH.max())


def _gpu_derivs(plan, Pw, rows_dir=None):
    torch = _torch()
    rows = _rows(plan.n_planets, plan.inclined)
    K = torch.as_tensor(_kernel_params(Pw, rows), device="cuda")
    dirs = list(range(K.shape[0])) if rows_dir is None else rows_dir
    lp, g, H, st = plan.derivs(K, dirs)
    torch.cuda.synchronize()
    return lp.cpu().numpy(), g.cpu().numpy(), H.cpu().numpy(), st.cpu().numpy()


def _case(planets, obs, W=2, seed=3, inclined=False, steps=SPO):
    plan, dt = _plan(obs, planets, LEVELS, steps, max_walkers=64, inclined=inclined)
    Pw = _ball(planets, W, seed=seed)
    if inclined:
        Pw[:, :, 5] = 0.05 + 0.01 * np.arange(len(planets))[None, :]
        Pw[:, :, 6] = -0.03
    return plan, dt, Pw


def fd_of_gradient(plan, x, d, rows_dir=None):
    """Hessian from central differences of the kernel's own exact gradient (Richardson over d, 2d):
    H_ij ~ (g_i(x + d_j e_j) - g_i(x - d_j e_j)) / 2 d_j.  A first difference of an exact gradient
    has noise ~ eps/d instead of eps/d^2, so this checks the order-2 variations against the order-1
    variations far more tightly than second differences of logp can."""
    torch = _torch()
    R = len(x)
    pts = []
    for sc in (1.0, 2.0):
        for j in range(R):
            for sg in (1, -1):
                y = x.copy()
                y[j] += sg * sc * d[j]
                pts.append(y)
    K = torch.as_tensor(np.array(pts).T.copy(), device="cuda")
    _, g, _, st = plan.derivs(K, list(range(R)) if rows_dir is None else rows_dir)
    g = g.cpu().numpy()
    assert (st.cpu().numpy() == 0).all()
    H = np.zeros((2, R, R))
    for k, sc in enumerate((1.0, 2.0)):
        for j in range(R):
            c = k * 2 * R + 2 * j
            H[k, :, j] = (g[:, c] - g[:, c + 1]) / (2 * sc * d[j])
    Hr = (4 * H[0] - H[1]) / 3
    return 0.5 * (Hr + Hr.T)


@pytest.mark.parametrize("name", ["S2", "S2_inclined", "1planet", "3planet", "4planet"])
def test_derivs_match_fd_of_the_kernel_algorithm(name):
    if name in ("1planet", "3planet", "4planet"):
        extra = [{"m": 1e-3, "a": 2.6, "h": 0.05, "k": 0.0, "l": 1.0}, {"m": 5e-4, "a": 3.9, "h": 0.0, "k": 0.03, "l": 4.0}]
        planets = {"1planet": S2_PLANETS[:1], "3planet": S2_PLANETS + extra[:1], "4planet": S2_PLANETS + extra}[name]
        np.random.seed(5)
        obs = O.fake_obs(planets, Npoints=30, error=1.5e-4, errorVar=2.5e-5, tmax=40.)
    else:
        planets = S2_PLANETS
        obs = s2_obs_oracle(Npoints=40) if name == "S2_inclined" else s2_obs_oracle()
    inclined = name == "S2_inclined"
    plan, dt, Pw = _case(planets, obs, W=2, inclined=inclined)
    rows = _rows(len(planets), inclined)
    lp, g, H, st = _gpu_derivs(plan, Pw)
    assert (st == 0).all()
    for w in range(Pw.shape[0]):
        assert np.allclose(H[:, :, w], H[:, :, w].T, rtol=0, atol=0)  # written symmetric
        x = _kernel_params(Pw[w:w + 1], rows)[:, 0]
        # 4 planets: the outer one (m 5e-4, a 3.9, 30 points over 40 time units) is weakly
        # constrained and logp is far from quadratic over one posterior width, so the FD step
        # shrinks to 0.4 widths (measured: grad err 1.9e-6 -> 4.9e-8, FD(grad) hess err
        # 1.4e-5 -> 3.4e-7 as the step goes 1 -> 0.4 widths: FD truncation, not the kernel)
        d = (0.4 if name == "4planet" else 1.0) * sigma_steps(H[:, :, w], x, rows)
        f0, g_fd, H_fd = fd_derivs(lambda P: O.logl_whx_batch(P, len(planets), obs, dt, LEVELS, has_inc=int(inclined))[0],
                                   x, len(planets), rows, d=d)
        eg, eH2 = scaled_errors(g[:, w], H[:, :, w], g_fd, H_fd)
        _, eH = scaled_errors(g[:, w], H[:, :, w], g[:, w], fd_of_gradient(plan, x, d))
        print(f"{name} walker {w}: logl {lp[w]:.6f} vs oracle {f0:.6f}; scaled grad err {eg:.2e}, "
              f"hess err {eH:.2e} (vs FD of the exact gradient), {eH2:.2e} (vs 2nd differences of the oracle)")
        assert abs(lp[w] - f0) <= T1_REL * max(1.0, abs(f0))
        assert eg < D1_GRAD and eH < D1_HESS and eH2 < D1_HESS_2ND, (eg, eH, eH2)


def test_derivs_match_fd_of_the_reference_integrator():
    """D2: the reference's own physics (IAS15 restatement) differentiated by central differences."""
    obs = s2_obs_oracle()
    plan, dt, Pw = _case(S2_PLANETS, obs, W=1, seed=11)
    lp, g, H, st = _gpu_derivs(plan, Pw)
    x = _kernel_params(Pw, 5)[:, 0]
    f0, g_fd, H_fd = fd_derivs(lambda P: O.logl_ias15_batch(P, 2, obs, 1.0)[0], x, 2, 5, d=2 * sigma_steps(H[:, :, 0], x, 5))
    eg, eH = scaled_errors(g[:, 0], H[:, :, 0], g_fd, H_fd)
    print(f"IAS15 FD: scaled grad err {eg:.2e}, hess err {eH:.2e}")
    assert eg < D2_GRAD and eH < D2_HESS, (eg, eH)


def test_derivs_logp_matches_likelihood_kernel_and_subset_block():
    torch = _torch()
    obs = s2_obs_oracle()
    plan, dt, Pw = _case(S2_PLANETS, obs, W=16, seed=4)
    K = torch.as_tensor(_kernel_params(Pw, 5), device="cuda")
    lp_l, st_l, _ = plan.logl(K)
    lp, g, H, st = plan.derivs(K, list(range(10)))
    sub = [9, 1, 6]  # l2, a1, a2 in a scrambled order
    lp_s, g_s, H_s, st_s = plan.derivs(K, sub)
    torch.cuda.synchronize()
    lp_l, lp, g, H = lp_l.cpu().numpy(), lp.cpu().numpy(), g.cpu().numpy(), H.cpu().numpy()
    assert (st.cpu().numpy() == st_l.cpu().numpy()).all()
    assert np.all(np.abs(lp - lp_l) <= T1_REL * np.maximum(1.0, np.abs(lp_l)))
    # the pair integrations of a sub-block are the same hyper-dual runs (the primal and the
    # diagonal pairs bit-identical; an off-diagonal pair may have its two directions swapped,
    # which reorders the order-2 sums)
    assert np.array_equal(lp_s.cpu().numpy(), lp)
    assert np.array_equal(g_s.cpu().numpy(), g[sub])
    assert np.allclose(H_s.cpu().numpy(), H[np.ix_(sub, sub)], rtol=1e-9, atol=0)


def test_derivs_status_of_prior_and_encounter_walkers():
    torch = _torch()
    obs = s2_obs_oracle()
    plan, dt, Pw = _case(S2_PLANETS, obs, W=4, seed=6)
    Pw[1, 0, 1] = 0.01          # a <= 0.02: prior
    Pw[2, 1, :5] = Pw[2, 0, :5]  # planet 2 next to planet 1 (same orbit phase): encounter at t = 0
    Pw[2, 1, 1] += 0.01
    K = torch.as_tensor(_kernel_params(Pw, 5), device="cuda")
    lp_l, st_l, _ = plan.logl(K)
    lp, g, H, st = plan.derivs(K, list(range(10)))
    torch.cuda.synchronize()
    st, st_l = st.cpu().numpy(), st_l.cpu().numpy()
    assert list(st) == list(st_l) and st[1] == 1 and st[2] == 2
    g, H = g.cpu().numpy(), H.cpu().numpy()
    for w in (1, 2):
        assert np.isneginf(lp[w].item()) and np.isnan(g[:, w]).all() and np.isnan(H[:, :, w]).all()
    for w in (0, 3):
        assert np.isfinite(g[:, w]).all() and np.isfinite(H[:, :, w]).all()


def test_state_get_logp_d_dd_is_exact_and_cached(golden):
    """Reference API: State.get_logp_d_dd (state.py:290-294) on HD155358's best fit (sol), with the
    Python-2 key order of the reference's notebook (a, h, k, m, l), checked against central
    differences of the State's own batched likelihood (so the free-parameter -> kernel-row mapping
    is exercised)."""
    import os

    torch = _torch()
    from rvmcmc.observations import Observation_FromFile
    from rvmcmc.state import State

    sol = golden["G2"]["sol"]
    s = State(planets=[{"a": sol[0], "h": sol[1], "k": sol[2], "m": sol[3], "l": sol[4]},
                       {"a": sol[5], "h": sol[6], "k": sol[7], "m": sol[8], "l": sol[9]}])
    s.hillRadiusFactor = golden["G2"]["hillRadiusFactor"]
    obs = Observation_FromFile(filename=os.path.join(GOLDEN, "HD155358.vels"), Npoints=100)
    lp, g, H = s.get_logp_d_dd(obs)
    assert g.shape == (10,) and H.shape == (10, 10)
    assert abs(lp - golden["G2"]["logp_print12"]) < 5e-8  # T2 (tests/test_gpu_logl.py)
    assert np.allclose(H, H.T, rtol=0, atol=0)
    lp2, g2, H2 = s.get_logp_d_dd(obs)
    assert lp2 == lp and g2 is g and H2 is H  # cached until set_params
    s.set_params(s.get_params())
    chi, chi_d, chi_dd = s.get_chi2_d_dd(obs)
    assert chi == -lp and np.array_equal(chi_d, -g) and np.array_equal(chi_dd, -H)
    # central differences of the same likelihood through get_logp_batch (steps of a fixed fraction
    # of the posterior width, Richardson-extrapolated over d and 2d)
    x = np.asarray(s.get_params())
    P = len(x)
    d = sigma_steps(H)
    pts = [x]
    for sc in (1.0, 2.0):
        for i in range(P):
            for sg in (1, -1):
                y = x.copy()
                y[i] += sg * sc * d[i]
                pts.append(y)
    X = torch.as_tensor(np.array(pts).T.copy(), device="cuda")
    f, st, _ = s.get_logp_batch(obs, X)
    f = f.cpu().numpy()

    def fd(k, sc):
        o = 1 + k * 2 * P
        g_ = np.array([(f[o + 2 * i] - f[o + 2 * i + 1]) / (2 * sc * d[i]) for i in range(P)])
        h_ = np.array([(f[o + 2 * i] - 2 * f[0] + f[o + 2 * i + 1]) / (sc * d[i]) ** 2 for i in range(P)])
        return g_, h_

    (g1, h1), (g2, h2) = fd(0, 1.0), fd(1, 2.0)
    g_fd, H_fd_diag = (4 * g1 - g2) / 3, (4 * h1 - h2) / 3
    sc = np.sqrt(np.abs(np.diag(H)))
    # GPU-logp second differences: noise ~ eps/d^2, so these only pin the parameter mapping
    assert np.max(np.abs(g - g_fd) / sc) < 1e-4
    assert np.max(np.abs(np.diag(H) - H_fd_diag) / sc ** 2) < 1e-3

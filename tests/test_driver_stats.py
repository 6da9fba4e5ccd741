"""Chain statistics of rvmcmc.driver (driver.py:37-43 auto_correlation, :343-382 AC times,
:412-414 efficacy) and the integrated-time / ESS estimator bench.py reports.  CPU only."""
import datetime

import numpy as np

from rvmcmc import driver


def _ar1(rho, n, walkers, seed=0):
    rng = np.random.default_rng(seed)
    x = np.zeros((n, walkers))
    e = rng.standard_normal((n, walkers)) * np.sqrt(1 - rho * rho)
    for i in range(1, n):
        x[i] = rho * x[i - 1] + e[i]
    return x


def test_auto_correlation_matches_reference_definition():
    x = np.random.default_rng(1).standard_normal(257)
    r = driver.auto_correlation(x)
    y = x - x.mean()
    full = np.array([np.dot(y[: len(y) - k], y[k:]) for k in range(len(y))])  # np.correlate, lags >= 0
    np.testing.assert_allclose(r, full / full[0], rtol=1e-12, atol=1e-15)
    assert r[0] == 1.0


def test_ac_time_is_first_lag_below_half():
    rho = 0.9
    x = _ar1(rho, 20000, 1, seed=2)[:, 0]
    # theory: rho^k < 0.5  ->  k = ceil(ln 0.5 / ln rho) = 7
    assert abs(driver.ac_time(x) - np.ceil(np.log(0.5) / np.log(rho))) <= 1


def test_integrated_time_and_ess_on_ar1():
    rho = 0.8
    x = _ar1(rho, 4000, 64, seed=3)
    tau = driver.integrated_time(x)
    assert abs(tau - (1 + rho) / (1 - rho)) < 0.5          # tau_int = (1 + rho) / (1 - rho) = 9
    ess, taus = driver.ess(np.stack([x, _ar1(0.5, 4000, 64, seed=4)], axis=2))
    assert abs(taus[1] - 3.0) < 0.3 and ess[1] > ess[0]


def test_efficacy_reference_formula():
    t0 = datetime.datetime(2017, 1, 1)
    clock = [t0, t0 + datetime.timedelta(seconds=1), t0 + datetime.timedelta(seconds=11)]
    # driver.py:412-414: Niter / ((clock[-1] - clock[1]) * max(AC))
    assert driver.efficacy(100, [2.0, 5.0], clock) == 100 / (10.0 * 5.0)


def test_log_data_and_aux_files(tmp_path, monkeypatch):
    """writing_to_log / save_data / load_data / save_aux_* (driver.py:45-53, 429-448): same file
    names and line formats as the reference."""
    from rvmcmc.state import State

    monkeypatch.chdir(tmp_path)
    s = State(planets=[{"m": 1.2e-3, "a": 0.88, "h": 0.2, "k": 0.0, "l": 0.3}])
    h = driver._hash(s, "run")
    driver.writing_to_log([1.5, 2.0], "_t", True)
    driver.writing_to_log("START", "_t", True)
    driver.writing_to_log([9.0], "_t", False)
    assert open(tmp_path / "log_t").read().splitlines() == ["1.5 2.0 ", "START "]
    driver.save_data(np.arange(4.0), "chain", h)
    np.testing.assert_array_equal(driver.load_data("chain", h), np.arange(4.0))
    driver.save_aux_mh(h, s, "run", 100, {"a": 0.3}, 0.01)
    txt = open(tmp_path / f"aux_{h.hexdigest()}").read().splitlines()
    assert txt[0].startswith("initial = [{'m': 0.0012") and txt[1] == "label, Niter, Scale, Stepsize = 'run', 100, {'a': 0.3}, 0.01"


def test_trimmed_results_burn_in_and_thinning():
    """return_trimmed_results (driver.py:265-333) without the plot: per-walker burn-in for emcee
    bundles (chain = Niter/Nwalkers iterations of walker 0, then walker 1, ...)."""
    from rvmcmc.state import State

    s = State(planets=[{"m": 1.2e-3, "a": 0.88, "h": 0.2, "k": 0.0, "l": 0.3}])

    class _M:
        state = s

    Niter, Nw = 40, 4
    chain = np.tile(s.get_params(), (Niter, 1)) + np.arange(Niter)[:, None] * 1e-6
    b = driver.McmcBundle(_M(), chain, -np.arange(Niter, dtype=float), [], None, Niter, s, is_emcee=True, Nwalkers=Nw)
    states, lp, avg = driver.trimmed_results(b, 0.5, take_every_n=1)
    idx = [c for w in range(Nw) for c in range(w * 10 + 5, (w + 1) * 10)]
    np.testing.assert_array_equal(lp, -np.array(idx, dtype=float))
    np.testing.assert_allclose(avg.get_params(), chain[idx].mean(0))
    b2 = driver.McmcBundle(_M(), chain, -np.arange(Niter, dtype=float), [], None, Niter, s)
    states, lp, _ = driver.trimmed_results(b2, 0.25, take_every_n=2)
    assert list(-lp) == list(range(10, 40, 2)) and len(states) == 15


def test_state_bookkeeping_helpers():
    """State.lnprior (state.py:115-119) and var_pindex_vname (state.py:218-225)."""
    from rvmcmc.state import State

    s = State(planets=[{"m": 1e-3, "a": 0.9, "h": 0.1, "k": 0.0, "l": 0.3},
                       {"m": 2e-3, "a": 1.5, "h": 0.1, "k": 0.0, "l": 2.0}], ignore_vars=["h"])
    assert [s.var_pindex_vname(i) for i in range(s.Nvars)] == [(1, "m"), (1, "a"), (1, "k"), (1, "l"),
                                                               (2, "m"), (2, "a"), (2, "k"), (2, "l")]
    assert s.var_pindex_vname(s.Nvars) is None
    assert State.lnprior([1e-3, 0.9, 0.1, 0.0, 0.3]) == 0.0
    assert State.lnprior([1e-3, 0.009, 0.1, 0.0, 0.3]) == -np.inf
    assert State.lnprior([1e-3, 0.9, 0.8, 0.8, 0.3]) == -np.inf


def test_notebook_era_driver_aliases():
    """The older driver names the reference notebooks call map onto the kept
    functions."""
    assert driver.createEns is driver.run_emcee and driver.createMH is driver.run_mh
    assert driver.createSMALA is driver.run_smala and driver.createALSMALA is driver.run_alsmala
    assert driver.createObs is driver.create_obs and driver.CreateObs is driver.create_obs
    assert driver.ReadObs is driver.read_obs and driver.saveData is driver.save_data
    assert driver.saveAuxSmala is driver.save_aux_smala and driver.saveAuxMH is driver.save_aux_mh

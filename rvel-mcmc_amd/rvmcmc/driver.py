"""Run orchestration and chain diagnostics (mirror of the non-plotting parts of /root/reference/driver.py).

Kept: McmcBundle (driver.py:20-33), auto_correlation (:37-43), run_mh / run_emcee / run_smala
(:57-147), create_obs / read_obs / save_obs (:207-222), efficacy (:412-414), calc_kstatistic
(:423-425), the per-parameter "AC time" of plot_ACTimes / inLinePlotEmceeAcTimes (:343-410).
Plotting (matplotlib, corner) is out of scope.  Bugs listed as "do not reproduce" in SURVEY.md
App. C are fixed: save_obs writes the error column, chains are preallocated instead of
np.append-grown, and run_emcee's acceptance rate counts walkers, not coordinates.
Added: integrated autocorrelation time and ESS (Sokal window), used for the ESS/s metric.
"""
from __future__ import annotations

import hashlib
from datetime import datetime

import numpy as np

from . import mcmc, observations


class McmcBundle(object):
    def __init__(self, mcmc, chain, chainlogp, clocktimes, obs, Niter, initial_state, trimmedchain=None,
                 trimmedchainlogp=None, actimes=None, is_emcee=False, Nwalkers=32):
        self.mcmc = mcmc
        self.mcmc_is_emcee = is_emcee
        self.mcmc_Nwalkers = Nwalkers
        self.mcmc_chain = chain
        self.mcmc_chainlogp = chainlogp
        self.mcmc_clocktimes = clocktimes
        self.mcmc_obs = obs
        self.mcmc_Niter = Niter
        self.mcmc_initial_state = initial_state
        self.mcmc_trimmedchain = trimmedchain
        self.mcmc_trimmedchainlogp = trimmedchainlogp
        self.mcmc_actimes = actimes


def auto_correlation(x):  # driver.py:37-43
    x = np.asarray(x, dtype=np.float64)
    y = x - x.mean()
    result = np.correlate(y, y, mode='full')
    result = result[len(result) // 2:]
    result /= result[0]
    return result


def ac_time(x):
    """The reference's "AC time": first lag at which the normalised autocorrelation drops below 0.5."""
    r = auto_correlation(x)
    below = np.nonzero(r < 0.5)[0]
    return float(below[0]) if len(below) else float(len(r))


def _hash(true_state, label):
    h = hashlib.md5()
    h.update(str(true_state.planets).encode())
    h.update(str(label).encode())
    return h


def run_mh(label, Niter, true_state, obs, scal, step, printing_every=400):  # driver.py:57-84
    mh = mcmc.Mh(true_state, obs)
    mh.set_scales(scal)
    mh.step_size = step
    chain = np.zeros((Niter + 1, mh.state.Nvars))
    chainlogp = np.zeros(Niter + 1)
    tries = 0
    clocktimes = [datetime.utcnow()]
    chainlogp[0] = true_state.get_logp(obs)
    chain[0] = true_state.get_params()
    for i in range(Niter):
        if mh.step():
            tries += 1
        chainlogp[i + 1] = mh.state.get_logp(obs)
        chain[i + 1] = mh.state.get_params()
        if i % printing_every == 1:
            print("Progress: {p:.5}%, {n} accepted steps have been made, time: {t}".format(
                p=100. * (float(i) / Niter), t=datetime.utcnow(), n=tries))
            clocktimes.append(datetime.utcnow())
    clocktimes.append(datetime.utcnow())
    print("Acceptance rate: %.3f%%" % ((tries / float(Niter)) * 100))
    h = _hash(true_state, label)
    return McmcBundle(mh, chain, chainlogp, clocktimes, obs, Niter, true_state), h


def run_emcee(label, Niter, true_state, obs, Nwalkers, scal, printing_every=400):  # driver.py:86-120
    ens = mcmc.Ensemble(true_state, obs, scales=scal, nwalkers=Nwalkers)
    n_it = int(Niter / Nwalkers)
    listchain = np.zeros((Nwalkers, ens.state.Nvars, n_it))
    listchainlogp = np.zeros((Nwalkers, n_it))
    clocktimes = [datetime.utcnow()]
    for i in range(n_it):
        ens.step()
        listchainlogp[:, i] = ens.lnprob
        listchain[:, :, i] = np.asarray(ens.states)
        if i % printing_every == 1:
            print("Progress: {p:.5}%, time: {t}".format(p=100. * (float(i) / n_it), t=datetime.utcnow()))
            clocktimes.append(datetime.utcnow())
    clocktimes.append(datetime.utcnow())
    acc = ens.sampler.acceptance_fraction().mean().item()
    print("Error(s): {e}".format(e=ens.totalErrorCount))
    print("Acceptance rate: %.3f%%" % (acc * 100))
    h = _hash(true_state, label)
    chain = np.concatenate([listchain[w] for w in range(Nwalkers)], axis=1)
    chainlogp = np.concatenate([listchainlogp[w] for w in range(Nwalkers)])
    bundle = McmcBundle(ens, np.transpose(chain), chainlogp, clocktimes, obs, Niter, true_state, is_emcee=True,
                        Nwalkers=Nwalkers)
    return bundle, h


def run_smala(label, Niter, true_state, obs, eps, alpha, printing_every=40):  # driver.py:122-147
    smala = mcmc.Smala(true_state, obs, eps, alpha)
    chain = np.zeros((Niter + 1, smala.state.Nvars))
    chainlogp = np.zeros(Niter + 1)
    tries = 0
    clocktimes = [datetime.utcnow()]
    chainlogp[0] = true_state.get_logp(obs)
    chain[0] = true_state.get_params()
    for i in range(Niter):
        if smala.step():
            tries += 1
        chainlogp[i + 1] = smala.state.get_logp(obs)
        chain[i + 1] = smala.state.get_params()
        if i % printing_every == 1:
            clocktimes.append(datetime.utcnow())
    clocktimes.append(datetime.utcnow())
    print("Acceptance rate: %.2f%%" % ((tries / float(Niter)) * 100))
    return McmcBundle(smala, chain, chainlogp, clocktimes, obs, Niter, true_state), _hash(true_state, label)


def create_obs(state, npoint, err, errVar, t):  # driver.py:207-209
    return observations.FakeObservation(state, Npoints=npoint, error=err, errorVar=errVar, tmax=(t))


def read_obs(filen):  # driver.py:211-213
    return observations.Observation_FromFile(filename=filen, Npoints=100)


def save_obs(obs, true_state, label):  # driver.py:215-222 (writes err, not rv, in column 3)
    col1 = obs.t / 1.720e-2
    col2 = obs.rv / 3.355e-5
    col3 = obs.err / 3.355e-5
    h = _hash(true_state, label)
    fn = 'obs_{ha}.vels'.format(ha=h.hexdigest())
    np.savetxt(fn, np.c_[col1, col2, col3])
    return fn


def efficacy(Niter, AC, clocktimes):  # driver.py:412-414
    return Niter / ((clocktimes[-1] - clocktimes[1]).total_seconds() * np.max(AC))


def calc_kstatistic(chain1, chain2):  # driver.py:423-425
    from scipy import stats

    return [stats.ks_2samp(chain1[:, i], chain2[:, i]) for i in range(chain1.shape[1])]


def integrated_time(x, c=5.0):
    """Integrated autocorrelation time of x [n_steps][n_walkers] (walker-averaged ACF, Sokal
    automatic window M = smallest m with m >= c * tau(m))."""
    x = np.asarray(x, dtype=np.float64)
    if x.ndim == 1:
        x = x[:, None]
    n = x.shape[0]
    y = x - x.mean(0)
    f = np.fft.rfft(y, n=2 * n, axis=0)
    acf = np.fft.irfft(f * np.conjugate(f), axis=0)[:n].mean(1)
    if acf[0] <= 0:
        return float("nan")
    acf /= acf[0]
    taus = 2.0 * np.cumsum(acf) - 1.0
    m = np.arange(len(taus)) < c * taus
    window = int(np.argmin(m)) if not m.all() else len(taus) - 1
    return float(taus[window])


def ess(chain_steps_walkers_params):
    """ESS per parameter of a [n_steps][n_walkers][P] ensemble chain: n_steps * n_walkers / tau."""
    c = np.asarray(chain_steps_walkers_params)
    n, w, P = c.shape
    taus = np.array([integrated_time(c[:, :, p]) for p in range(P)])
    return n * w / taus, taus

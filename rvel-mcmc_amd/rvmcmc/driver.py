"""Run orchestration and chain diagnostics (mirror of the non-plotting parts of /root/reference/driver.py).

Kept: McmcBundle (driver.py:20-33), auto_correlation (:37-43), writing_to_log (:45-53),
run_mh / run_emcee / run_smala (:57-147), pre_eps_smala (:149-169), run_alsmala (:171-202), create_obs / read_obs /
save_obs (:207-222), the non-plotting part of return_trimmed_results (:265-333, trimmed_results),
efficacy (:412-414), calc_kstatistic (:423-425), load_data / save_data / save_aux_* (:429-448), the
per-parameter "AC time" of plot_ACTimes / inLinePlotEmceeAcTimes (:343-410).
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


def run_alsmala(label, Niter, true_state, obs, eps, alpha, bern_a, bern_b, printing_every=40):  # driver.py:171-202
    """Full SMALA step with probability exp(-bern_a i / Niter), else the cheap derivative-reusing
    step (bern_b is unused, as in the reference)."""
    alsmala = mcmc.Alsmala(true_state, obs, eps, alpha)
    chain = np.zeros((Niter + 1, alsmala.state.Nvars))
    chainlogp = np.zeros(Niter + 1)
    tries = 0
    clocktimes = [datetime.utcnow()]
    chainlogp[0] = true_state.get_logp(obs)
    chain[0] = true_state.get_params()
    for i in range(Niter):
        if np.exp(-bern_a * i / Niter) > np.random.uniform():
            tries += bool(alsmala.step())
        else:
            tries += bool(alsmala.step_mala())
        chainlogp[i + 1] = alsmala.state.get_logp(obs)
        chain[i + 1] = alsmala.state.get_params()
        if i % printing_every == 1:
            clocktimes.append(datetime.utcnow())
    clocktimes.append(datetime.utcnow())
    print("Acceptance rate: %.2f%%" % ((tries / float(Niter)) * 100))
    return McmcBundle(alsmala, chain, chainlogp, clocktimes, obs, Niter, true_state), _hash(true_state, label)


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


def writing_to_log(obj, name, logging):  # driver.py:45-53 (the reference's file name is a NameError)
    """Append every element of obj, space separated, as one line of the file log<name>."""
    if not logging:
        return
    with open("log{r}".format(r=name), "a") as f:
        f.write(" ".join("{v}".format(v=v) for _, v in np.ndenumerate(np.asarray(obj, dtype=object))) + " \n")


def pre_eps_smala(true_state, obs, eps, alpha, Niter, rng=None, max_rounds=50):  # driver.py:149-169
    """Tune SMALA's eps until a trial run of Niter accepted steps has an acceptance rate in
    [0.52, 0.68]: outside it, eps moves down (rate too low) or up (too high) by
    |N(0.065, 0.025)| * 8 |rate - 0.6| (positive draws only), as the reference's recursion does;
    iterative here, with a bound on the rounds."""
    rng = rng if rng is not None else np.random
    for _ in range(max_rounds):
        smala = mcmc.Smala(true_state, obs, eps, alpha)
        print("Trying out eps = {e}".format(e=eps))
        tries = 0
        for i in range(Niter):
            tries += smala.step_force()
        rate = float(Niter) / tries
        print("Acc. Rate was {a}".format(a=rate))
        if 0.52 <= rate <= 0.68:
            return eps
        mod = 0.0
        while mod <= 0.0:
            mod = rng.normal(loc=0.065, scale=0.025) * 8. * abs(rate - 0.6)
        eps = eps - mod if rate < 0.52 else eps + mod
    return eps


def trimmed_results(bundle, burn_in_fraction, take_every_n=1):
    """The non-plotting part of return_trimmed_results (driver.py:265-333): the chain after the
    burn-in fraction (per walker block for an emcee bundle, whose chain stacks Niter/Nwalkers
    iterations of each walker), thinned to every n-th index, as (states, chainlogp, average state)."""
    Niter, chain, chainlogp = bundle.mcmc_Niter, bundle.mcmc_chain, bundle.mcmc_chainlogp
    base = bundle.mcmc.state
    if bundle.mcmc_is_emcee:
        per = Niter // bundle.mcmc_Nwalkers
        idx = [c for w in range(bundle.mcmc_Nwalkers) for c in range(int(w * per + per * burn_in_fraction), (w + 1) * per)]
    else:
        idx = list(range(int(Niter * burn_in_fraction), Niter))
    idx = [c for c in idx if c % take_every_n == 0]
    states = []
    for c in idx:
        s = base.deepcopy()
        s.set_params(chain[c])
        states.append(s)
    avg = base.deepcopy()
    avg.set_params(np.mean(np.asarray(chain)[idx], axis=0))
    return states, np.asarray(chainlogp)[idx], avg


def load_data(name, h):  # driver.py:429-430
    return np.load('{n}_{h}.npy'.format(n=name, h=h.hexdigest()))


def save_data(dat, name, h):  # driver.py:432-433
    np.save('{n}_{h}'.format(n=name, h=h.hexdigest()), dat)


def _save_aux(h, true_state, line):
    with open('aux_{h}'.format(h=h.hexdigest()), "w") as f:
        f.write('initial = ' + str(true_state.planets))
        f.write("\n" + line)


def save_aux_smala(h, true_state, label, Niter, eps, alpha):  # driver.py:435-438
    _save_aux(h, true_state, "label, Niter, Eps, Alpha = '{l}', {n}, {e}, {a}".format(l=label, n=Niter, e=eps, a=alpha))


def save_aux_emcee(h, true_state, label, Niter, Nwalkers, scal):  # driver.py:440-443
    _save_aux(h, true_state, "label, Niter, Nwalkers, Scale = '{l}', {n}, {s}, {t}".format(l=label, n=Niter, s=Nwalkers,
                                                                                           t=scal))


def save_aux_mh(h, true_state, label, Niter, scal, step):  # driver.py:445-448
    _save_aux(h, true_state, "label, Niter, Scale, Stepsize = '{l}', {n}, {s}, {t}".format(l=label, n=Niter, s=scal,
                                                                                           t=step))


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


# The notebooks' older names for the same functions ((Ex)HD155358.ipynb,
# (Ex)Full Test + Usage Example.ipynb, generator.py); they return (bundle, hash) like run_*.
createEns = run_emcee
createMH = run_mh
createSMALA = run_smala
createALSMALA = run_alsmala
createObs = CreateObs = create_obs
ReadObs = read_obs
saveData = save_data
loadData = load_data
saveAuxSmala = save_aux_smala
saveAuxEmcee = save_aux_emcee
saveAuxMH = save_aux_mh

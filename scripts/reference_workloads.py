"""The reference's three benchmark workloads, run through this framework's reference-named API.

mcmc_benchmark_mh.py, mcmc_benchmark_emcee.py and mcmc_benchmark_smala.py are Python-2 scripts
(print statements, REBOUND, corner plots) that cannot run here; what a user switching over needs
is the same workload on the same API.  Each function below sets up the script's state,
observations and sampler settings (file:line cited), runs the sampler loop with the script's
step_force() pattern, and reports what the script prints (acceptance rate, the reference's
"AC time" per parameter) plus wall time.  Plots are out of scope.

Named stand-ins for inputs the reference tree lacks:
  * TEST_3-2_COMPACT.vels (mcmc_benchmark_emcee.py:35, mcmc_benchmark_smala.py:35) is not in the
    reference: each script's own commented-out FakeObservation line is used instead
    (mcmc_benchmark_emcee.py:34, mcmc_benchmark_smala.py:34), seeded.
  * mcmc_benchmark_smala.py:51 calls mcmc.Smala(true_state, obs) without eps and alpha (a
    TypeError against mcmc.py:127); the values of generator.py:43 (eps 0.12, alpha 1.4) are used.

Usage: python scripts/reference_workloads.py [--scale 0.05] [mh emcee smala]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd")]

import mcmc  # noqa: E402  (the reference's module names, rvel-mcmc_amd/*.py)
import observations  # noqa: E402
import state  # noqa: E402
from rvmcmc import driver  # noqa: E402


def _ac_times(chain):
    return [driver.ac_time(chain[:, i]) for i in range(chain.shape[1])]


def mh_workload(scale=1.0, seed=2017):
    np.random.seed(seed)
    true_state = state.State(planets=[{"m": 1.2e-3, "a": 0.88, "h": 0.218, "k": 0.015, "l": 0.3},
                                      {"m": 2.1e-3, "a": 1.44 + 0.11, "h": 0.16, "k": 0.02, "l": 2.2}])  # :32
    obs = observations.FakeObservation(true_state, Npoints=200, error=1.5e-4, errorVar=2.5e-5, tmax=120.)  # :34
    mh = mcmc.Mh(true_state, obs)  # :51
    mh.set_scales({"m": 1.e-3, "a": 0.3, "h": 0.5, "k": 0.5, "l": np.pi / 2.})  # :52
    mh.step_size = 10.0e-3  # :53
    Niter = max(2, int(6000 * scale))  # :54
    chain = np.zeros((Niter, mh.state.Nvars))
    tries = 0
    t0 = time.perf_counter()
    for i in range(Niter):
        tries += mh.step_force()
        chain[i] = mh.state.get_params()
    dt = time.perf_counter() - t0
    return {"workload": "mcmc_benchmark_mh.py", "Niter": Niter, "acceptance_rate": Niter / tries,
            "ac_times": _ac_times(chain), "wall_s": dt, "logl_evals_per_s": tries / dt}


def emcee_workload(scale=1.0, seed=2017):
    np.random.seed(seed)
    true_state = state.State(planets=[{"m": 0.94e-3, "a": 0.226, "h": -0.045, "k": -0.015, "l": 1.265},
                                      {"m": 1.965e-3, "a": 0.307, "h": -0.035, "k": -0.00, "l": 1.76}])  # :33
    obs = observations.FakeObservation(true_state, Npoints=200, error=1.5e-4, errorVar=2.5e-5, tmax=(30))  # :34
    Nwalkers = 32  # :50
    ens = mcmc.Ensemble(true_state, obs, scales={"m": 1.5e-3, "a": 0.3, "h": 0.1, "k": 0.1, "l": np.pi / 2.},
                        nwalkers=Nwalkers)  # :51
    Niter = max(2 * Nwalkers, int(25000 * scale))  # :52
    n_it = Niter // Nwalkers
    chain = np.zeros((Niter, ens.state.Nvars))
    chainlogp = np.zeros(Niter)
    t0 = time.perf_counter()
    for i in range(n_it):  # :55-60 (walker j's samples fill the block j*Niter/Nwalkers + i)
        ens.step_force()
        for j in range(Nwalkers):
            chain[j * n_it + i] = ens.states[j]
            chainlogp[j * n_it + i] = ens.lnprob[j]
    dt = time.perf_counter() - t0
    return {"workload": "mcmc_benchmark_emcee.py", "Niter": n_it * Nwalkers, "iterations": n_it,
            "errors": ens.totalErrorCount, "acceptance_rate": float(ens.sampler.acceptance_fraction().mean().item()),
            "ac_times": _ac_times(chain), "wall_s": dt, "logl_evals_per_s": ens.sampler.nevals / dt,
            "finite_lnprob": bool(np.isfinite(chainlogp[:n_it * Nwalkers]).all())}


def smala_workload(scale=1.0, seed=2017):
    np.random.seed(seed)
    true_state = state.State(planets=[{"m": 0.9e-3, "a": 0.226, "h": -0.06, "k": -0.015, "l": 1.3},
                                      {"m": 1.85e-3, "a": 0.3057, "h": -0.03, "k": -0.01, "l": 1.75}])  # :32
    obs = observations.FakeObservation(true_state, Npoints=60, error=1.5e-4, errorVar=2.5e-5, tmax=(30))  # :34
    smala = mcmc.Smala(true_state, obs, 0.12, 1.4)  # :51 with generator.py:43's eps, alpha
    Niter = max(2, int(4200 * scale))  # :52
    chain = np.zeros((Niter, smala.state.Nvars))
    chainlogp = np.zeros(Niter)
    tries = 0
    t0 = time.perf_counter()
    for i in range(Niter):
        tries += smala.step_force()
        chain[i] = smala.state.get_params()
        chainlogp[i] = smala.state.logp
    dt = time.perf_counter() - t0
    return {"workload": "mcmc_benchmark_smala.py", "Niter": Niter, "acceptance_rate": Niter / tries,
            "ac_times": _ac_times(chain), "wall_s": dt, "steps_per_s": tries / dt,
            "finite_logp": bool(np.isfinite(chainlogp).all())}


WORKLOADS = {"mh": mh_workload, "emcee": emcee_workload, "smala": smala_workload}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--scale", type=float, default=0.05, help="fraction of each script's Niter")
    ap.add_argument("which", nargs="*", default=list(WORKLOADS))
    a = ap.parse_args(argv)
    out = []
    for w in a.which:
        r = WORKLOADS[w](a.scale)
        print(json.dumps(r), flush=True)
        out.append(r)
    return out


if __name__ == "__main__":
    main()

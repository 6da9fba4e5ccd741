"""Dump the bench ensemble (bench.py's setup, resolve off) at a few iterations: calibration data
for the adaptive-resolution estimate."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from rvmcmc import engine  # noqa: E402
from rvmcmc.ensemble import EnsembleSampler  # noqa: E402
from rvmcmc.observations import FakeObservation  # noqa: E402
from rvmcmc.state import State  # noqa: E402
from conftest import S2_PLANETS, S2_SCALES  # noqa: E402

state = State(planets=[dict(p) for p in S2_PLANETS])
state.integrator = engine.IntegratorConfig(resolve_tol=0.0)
np.random.seed(2017)
obs = FakeObservation(state, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
scales = np.array([S2_SCALES[k] for k in state.get_rawkeys()])
X0 = state.get_params()[None] + 0.1e-2 * scales * np.random.normal(size=(4096, state.Nvars))
ens = EnsembleSampler(4096, state, obs, seed=2017)
ens.set_positions(X0)
ens.compute_lnprob()
out = {}
for it in range(1, 2001):
    ens.step()
    if it in (3, 10, 23, 100, 500, 2000):
        out[f"it{it}"] = ens.gather_positions()
os.makedirs("gpurun_out", exist_ok=True)
np.savez_compressed("gpurun_out/bench_ensemble.npz", tf=obs.tf, tb=obs.tb, rvf=obs.rvf, rvb=obs.rvb,
                    errorf=obs.errorf, errorb=obs.errorb, **out)
print("saved", list(out))

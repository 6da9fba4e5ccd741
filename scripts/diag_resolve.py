"""Diagnose refinement counts per iteration on the bench ensemble (bench.py's setup)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from rvmcmc import engine  # noqa: E402
from rvmcmc.ensemble import EnsembleSampler  # noqa: E402
from rvmcmc.observations import FakeObservation  # noqa: E402
from rvmcmc.state import State  # noqa: E402
from conftest import S2_PLANETS, S2_SCALES  # noqa: E402

torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
state = State(planets=[dict(p) for p in S2_PLANETS])
state.integrator = engine.IntegratorConfig()
np.random.seed(2017)
obs = FakeObservation(state, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
scales = np.array([S2_SCALES[k] for k in state.get_rawkeys()])
X0 = state.get_params()[None] + 0.1e-2 * scales * np.random.normal(size=(4096, state.Nvars))
ens = EnsembleSampler(4096, state, obs, seed=2017, device=dev)
ens.set_positions(X0)
ens.compute_lnprob()
print("lnprob", ens.check_faults())
for it in range(25):
    ens.step()
    f = ens.check_faults()
    P = ens.gather_positions()
    print(it, f["refined"], "spread a1", float(np.std(P[:, 1])), float(np.std(P[:, 6])), "lnp min",
          float(ens.gather_lnprob().min()))

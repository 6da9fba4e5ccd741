"""The bench's sampler at the steady state of its own chain: the bench setup (bench.py: 2-planet
synthetic, 101 epochs, 4096 walkers) started from the ensemble after 2000 iterations
(scripts/probe/ens_it2000.npy, from scripts/dump_bench_ensemble.py) instead of the initial ball;
iterations/s and evaluations/s with the adaptive resolution off and on, and its counters."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from conftest import S2_PLANETS  # noqa: E402
from rvmcmc import engine  # noqa: E402
from rvmcmc.ensemble import EnsembleSampler  # noqa: E402
from rvmcmc.observations import FakeObservation  # noqa: E402
from rvmcmc.state import State  # noqa: E402


def run(resolve_tol, levels=(4, 5, 6, 7), resolve_max=None, iters=int(os.environ.get("ITERS", "30")), warm=3):
    if resolve_max is None:
        resolve_max = engine.IntegratorConfig().resolve_max
    state = State(planets=[dict(p) for p in S2_PLANETS])
    state.integrator = engine.IntegratorConfig(resolve_tol=resolve_tol, levels=tuple(levels), resolve_max=resolve_max)
    np.random.seed(2017)
    obs = FakeObservation(state, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    X = np.load(os.path.join(ROOT, "scripts/probe/ens_it2000.npy"))
    ens = EnsembleSampler(len(X), state, obs, seed=2017)
    ens.set_positions(X)
    ens.compute_lnprob()
    for _ in range(warm):
        ens.step()
    torch.cuda.synchronize()
    f0 = ens.check_faults()
    ens.plan.time_kernels(iters)
    t0 = time.perf_counter()
    for _ in range(iters):
        ens.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    km, kr = ens.plan.kernel_times()
    f = ens.check_faults()
    return dict(resolve_tol=resolve_tol, resolve_max=resolve_max, levels=list(levels), walkers=len(X), iterations=iters, ms_per_iteration=1e3 * dt / iters,
                evals_per_s=len(X) * iters / dt, speculative=bool(ens.speculating()), faults=f,
                faults_warm=f0, logl_kernel_ms=float(np.mean(km)) if len(km) else None,
                refine_kernel_ms=float(np.mean(kr)) if len(kr) else None,
                refine_kernel_ms_quantiles=[float(v) for v in np.quantile(kr, [0, .25, .5, .75, 1])] if len(kr) else None,
                lib=os.environ.get("RVM_LIB_PATH", "default"))


if __name__ == "__main__":
    # specs "LEVELS:TOL[:RMAX]", e.g. 4,5,6,7:5e-7:4 (default: the bench's levels, resolution off / on)
    specs = sys.argv[1:] or ["4,5,6,7:0", "4,5,6,7:5e-7"]
    for sp in specs:
        f = sp.split(":")
        print(json.dumps(run(float(f[1]), tuple(int(v) for v in f[0].split(",")), int(f[2]) if len(f) > 2 else None)),
              flush=True)

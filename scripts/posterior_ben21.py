"""Posterior (statistical) parity with the reference's own SMALA run on TEST_2-1_COMPACT.vels.

The reference's mcmc_benchmark_smala.py run "Ben-2-1" (plotArchive/Ben's 2-1/log_Ben-2-1) logged
the RV curves of 45 states drawn from the second half of its SMALA chain (RDMGHOSTS lines, fixture
G5 = tests/golden/g5_ghosts.npz, 1000 times linspace(tb[0], tf[-1])).  Here the same posterior is
sampled with the device affine ensemble from the run's start state (fixture G3's planets), and the
model RV curves of our posterior samples at the same 1000 times are compared with the ghosts:
per time, the ghosts' mean against our posterior mean in units of our posterior sd, and the ratio
of the ghosts' sd to ours.  Prints one JSON line.  Usage: python scripts/posterior_ben21.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd")]
import torch  # noqa: E402

from rvmcmc import engine  # noqa: E402
from rvmcmc.ensemble import EnsembleSampler  # noqa: E402
from rvmcmc.observations import Observation_FromFile  # noqa: E402
from rvmcmc.state import State  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")
SCALES = {"m": 1.5e-3, "a": 0.3, "h": 0.1, "k": 0.1, "l": np.pi / 2.}  # mcmc_benchmark_emcee.py:51


def main(W=2048, burn=1500, keep=500, thin=10, seed=7):
    g = json.load(open(os.path.join(GOLDEN, "golden.json")))["G3"]
    gh = np.load(os.path.join(GOLDEN, "g5_ghosts.npz"))
    t, rv_ref = gh["t"], gh["rv"]
    obs = Observation_FromFile(os.path.join(GOLDEN, "TEST_2-1_COMPACT.vels"), Npoints=g["Npoints"])
    s = State(planets=[dict(p) for p in g["planets"]])
    rng = np.random.default_rng(seed)
    sc = np.array([SCALES[k] for k in s.get_rawkeys()])
    X0 = s.get_params()[None] + 1e-3 * sc * rng.standard_normal((W, s.Nvars))
    ens = EnsembleSampler(W, s, obs, seed=seed)
    ens.set_positions(X0)
    t0 = time.perf_counter()
    for _ in range(burn):
        ens.step()
    samples = []
    for i in range(keep):
        ens.step()
        if i % thin == 0:
            samples.append(torch.cat(ens.pos, 1).clone())
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    X = torch.cat(samples, 1)                                   # [P][n] free parameters
    # model RV of every sample at the ghosts' 1000 times (one plan over those epochs)
    dt, mult, hint = s.integrator.plan_args(s.planets)
    plan = engine.LoglPlan(t, np.zeros_like(t), np.ones_like(t), 1.0, len(s.planets), dt, mult, X.shape[1],
                           period_hint=hint)
    lp, st, rv = plan.logl(s.param_map().to_kernel(X), want_rv=True)
    ok = (st == 0).cpu().numpy()
    rv = rv.cpu().numpy()[:, ok]                                 # [1000][n_ok]
    m_o, s_o = rv.mean(1), rv.std(1)
    m_r, s_r = rv_ref.mean(0), rv_ref.std(0)
    z = np.abs(m_r - m_o) / s_o
    ratio = s_r / s_o
    out = {"walkers": W, "burn_in_iterations": burn, "samples": int(ok.sum()), "wall_s": wall,
           "acceptance": float(ens.acceptance_fraction().mean().item()),
           "ghosts": int(rv_ref.shape[0]),
           "mean_diff_in_our_sd": {"median": float(np.median(z)), "p95": float(np.percentile(z, 95)),
                                   "max": float(z.max())},
           "sd_ratio_ref_over_ours": {"median": float(np.median(ratio)), "p5": float(np.percentile(ratio, 5)),
                                      "p95": float(np.percentile(ratio, 95))},
           "our_sd_m_per_s_median": float(np.median(s_o) / 3.355e-5),
           "ref_sd_m_per_s_median": float(np.median(s_r) / 3.355e-5)}
    print(json.dumps(out), flush=True)
    return out


if __name__ == "__main__":
    main()

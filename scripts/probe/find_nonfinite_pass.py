"""Search (CPU, oracle) for prior-passing S2 walkers whose adaptive halving passes blow up
(status NONFINITE from a halving pass): random extreme systems -- masses up to ~e^7 x S2's,
semi-major axes within a factor e, eccentricities up to 0.99 -- with hill_factor 0 (no encounter
exit), resolve_max 2 to keep the search cheap.  The two walkers it finds (trials 26 and 33 of seed
5) are tests/test_gpu_contract.py's NONFINITE_WALKERS."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("oracle", "rvel-mcmc_amd", "tests")]
import oracle as O  # noqa: E402
from conftest import S2_PLANETS, s2_obs_oracle  # noqa: E402
from rvmcmc import engine  # noqa: E402


def main():
    obs = s2_obs_oracle()
    cfg = engine.IntegratorConfig()
    dt, mult, _ = cfg.plan_args(S2_PLANETS)
    tol, _, guard, _ = cfg.resolve(S2_PLANETS)
    rng = np.random.default_rng(5)
    base = O.pal_params(S2_PLANETS)
    for trial in range(34):
        n = 64
        P = np.repeat(base[None], n, 0)
        P[:, :, 0] *= np.exp(rng.uniform(0, 7, (n, 2)))
        P[:, :, 1] *= np.exp(rng.uniform(-1, 1, (n, 2)))
        P[:, :, 2] = rng.uniform(-0.99, 0.99, (n, 2))
        P[:, :, 3] = rng.uniform(-0.99, 0.99, (n, 2))
        bad = P[:, :, 2] ** 2 + P[:, :, 3] ** 2 >= 1
        P[:, :, 2][bad] *= 0.5
        P[:, :, 3][bad] *= 0.5
        if trial not in (26, 33):
            continue
        out = O.logl_whx_adapt_batch(P, 2, obs, dt, mult, tol, 2, 0.0, ecc_guard=guard)
        for i in np.nonzero(out[1] == 3)[0]:
            print(f"trial {trial} walker {i}: stages {out[2][i].tolist()}\n{np.array2string(P[i][:, :5], precision=8)}")


if __name__ == "__main__":
    main()

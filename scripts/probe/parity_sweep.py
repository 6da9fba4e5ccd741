"""Probe (GPU + the oracle's IAS15 on the host): accept-decision parity against IAS15 at steady states
with more walkers than the GPU tests use (tests/test_gpu_ias15_decisions.py's stretch_parity:
speculative iterations of the real sampler, every decision and every OK proposal's logL against
the IAS15 restatement).  HD155358 and the 3-planet system after 1000 device iterations of W walkers,
the bench chain from its iteration-2000 ensemble over more iterations.  Prints one report per case.
usage: parity_sweep.py [W] [iterations]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("rvel-mcmc_amd", "oracle", "tests")]
import oracle as O  # noqa: E402
import test_gpu_ias15_decisions as T  # noqa: E402
from conftest import S2_PLANETS, s2_obs_oracle  # noqa: E402


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    cases = []
    planets, obs = T._hd()
    cases.append(("HD155358", planets, obs))
    np.random.seed(2017)
    p3 = [dict(p) for p in S2_PLANETS] + [dict(T.THIRD)]
    cases.append(("3planet", p3, O.fake_obs(p3, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)))
    for name, planets, obs in cases:
        X0 = T._burned_in(planets, obs, W, 1000)
        tally, info = T.stretch_parity(f"sweep/steady-state {name} {W} walkers", planets, obs, W, 0.0,
                                       iterations=iters, warm=0, roundoff=True, X0=X0)
        print(json.dumps({"case": name, "walkers": W, **tally.report(**info)}, default=str), flush=True)
    X0 = np.load(os.path.join(ROOT, "scripts", "probe", "ens_it2000.npy"))
    tally, info = T.stretch_parity("sweep/steady-state S2 4096 walkers", S2_PLANETS, s2_obs_oracle(), len(X0), 0.0,
                                   iterations=2 * iters, warm=0, roundoff=True, X0=X0)
    print(json.dumps({"case": "S2 (bench chain, iteration 2000)", "walkers": len(X0), **tally.report(**info)},
                     default=str), flush=True)


if __name__ == "__main__":
    main()

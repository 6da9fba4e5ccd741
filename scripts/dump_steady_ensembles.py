"""Steady-state ensembles of the HD155358 and 3-planet chains (the device sampler, 512 walkers,
1000 iterations from the tight ball: the procedure of tests/test_gpu_ias15_decisions.py
_burned_in), saved for the CPU studies of the adaptive resolution's certain-reject bound on those
systems (tests/test_ias15_parity_harness.py, scripts/probe/cut_ratio_study.py):
scripts/probe/ens_hd155358_it1000.npy and ens_3planet_it1000.npy ([512][Nvars], State order)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("rvel-mcmc_amd", "oracle", "tests")]
OUT = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "scripts", "probe")  # (gpurun_out/ on a GPU box)


def main():
    from test_gpu_ias15_decisions import THIRD, _burned_in, _hd

    import oracle as O
    from conftest import S2_PLANETS

    planets, obs = _hd()
    np.save(os.path.join(OUT, "ens_hd155358_it1000.npy"), _burned_in(planets, obs, 512, 1000))
    np.random.seed(2017)
    planets = [dict(p) for p in S2_PLANETS] + [dict(THIRD)]
    obs = O.fake_obs(planets, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    np.save(os.path.join(OUT, "ens_3planet_it1000.npy"), _burned_in(planets, obs, 512, 1000))
    print("saved")


if __name__ == "__main__":
    main()

"""Config 3 (BASELINE.json): HD155358.vels 2-planet fit with the affine sampler, plus an
independent batched-MH run, for posterior (statistical) parity.

The reference's own posterior summaries for this data set are in (Ex)HD155358.ipynb (emcee,
40 walkers, cell 12: mean of 50 post-burn-in samples; cell 19: best SMALA sample).  Prints one
JSON line with posterior means / standard deviations of both samplers, the KS statistics between
them, the reference's reported means and timing.  Usage: python scripts/posterior_hd155358.py
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd")]
import torch  # noqa: E402

from rvmcmc import driver  # noqa: E402
from rvmcmc.ensemble import EnsembleSampler  # noqa: E402
from rvmcmc.mcmc import MhChains  # noqa: E402
from rvmcmc.observations import Observation_FromFile  # noqa: E402
from rvmcmc.state import State  # noqa: E402

SOL = [6.57730330e-01, -9.72263877e-02, -7.82798396e-02, 8.84031737e-04, 4.42804990e+00,
       1.04404207e+00, -2.05622789e-02, -1.08797961e-01, 8.30379710e-04, 1.49919861e+00]
# (Ex)HD155358.ipynb cell 12: "Resulting average params state", order a,h,k,m,l per planet
REF_MEAN = [6.57839047e-01, -1.01399218e-01, -7.91210835e-02, 8.83846740e-04, 4.43076459e+00,
            1.04392356e+00, -1.65660093e-02, -1.04423913e-01, 8.31166528e-04, 1.45003290e+00]


def main(W=4096, iters=600, mh_steps=3000):
    obs = Observation_FromFile(os.path.join(ROOT, "tests", "golden", "HD155358.vels"), Npoints=100)
    # the notebook's Python-2 dict order is a, h, k, m, l
    planets = [{"a": SOL[0], "h": SOL[1], "k": SOL[2], "m": SOL[3], "l": SOL[4]},
               {"a": SOL[5], "h": SOL[6], "k": SOL[7], "m": SOL[8], "l": SOL[9]}]
    s = State(planets=planets)
    sc = {"m": 5.5e-6, "a": 0.001, "h": 0.02, "k": 0.02, "l": np.pi / 4.}  # (Ex)HD155358.ipynb cell 7
    scales = np.array([sc[k] for k in s.get_rawkeys()])
    rng = np.random.default_rng(2017)
    X0 = s.get_params()[None] + 1e-3 * scales * rng.standard_normal((W, s.Nvars))
    ens = EnsembleSampler(W, s, obs, seed=7)
    ens.set_positions(X0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    burn = iters // 2
    chain = []
    for i in range(iters):
        ens.step()
        if i >= burn:
            chain.append(torch.cat(ens.pos, 1).t().clone())
    torch.cuda.synchronize()
    t_ens = time.perf_counter() - t0
    C = torch.stack(chain).cpu().numpy()                     # [steps][W][P]
    flat = C.reshape(-1, s.Nvars)
    mean_e, sd_e = flat.mean(0), flat.std(0)
    ess, taus = driver.ess(C)
    # independent check: batched MH from the affine posterior's spread
    mh = MhChains(s, obs, sd_e, 0.5, W, X0=C[-1].T.copy(), seed=11)
    t1 = time.perf_counter()
    mchain = []
    for i in range(mh_steps):
        mh.step()
        if i >= mh_steps // 2 and i % 10 == 0:
            mchain.append(mh.X.t().clone())
    torch.cuda.synchronize()
    t_mh = time.perf_counter() - t1
    M = torch.stack(mchain).cpu().numpy().reshape(-1, s.Nvars)
    from scipy import stats

    ks = [float(stats.ks_2samp(flat[::97, p], M[::97, p]).statistic) for p in range(s.Nvars)]
    out = {"keys": s.get_rawkeys(), "affine_mean": mean_e.tolist(), "affine_sd": sd_e.tolist(),
           "mh_mean": M.mean(0).tolist(), "mh_sd": M.std(0).tolist(), "ks_affine_vs_mh": ks,
           "reference_mean_cell12": REF_MEAN,
           "ref_minus_ours_in_sd": ((np.array(REF_MEAN) - mean_e) / sd_e).tolist(),
           "affine_seconds": t_ens, "affine_evals_per_s": W * iters / t_ens, "tau": taus.tolist(),
           "ess_per_s": float(ess.min() / t_ens * 2), "mh_seconds": t_mh,
           "mh_acceptance": float(mh.accepted.double().mean().item() / mh_steps),
           "affine_acceptance": float(ens.acceptance_fraction().mean().item())}
    print(json.dumps(out))
    return out


if __name__ == "__main__":
    main()

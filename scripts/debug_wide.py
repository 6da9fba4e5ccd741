"""Dump GPU statuses/logL for the wide-ball parity case (debug aid)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import oracle as O  # noqa: E402
from conftest import S2_PLANETS, s2_obs_oracle  # noqa: E402
from rvmcmc import engine  # noqa: E402

obs = s2_obs_oracle()
rng = np.random.default_rng(3)
P = np.repeat(O.pal_params(S2_PLANETS)[None], 256, 0)
P[:, :, :5] *= 1 + 0.6 * rng.standard_normal((256, 2, 5))
P[0, 0, 1] = 0.02
P[1, 1, 0] = 5e-6
P[2, 0, 2], P[2, 0, 3] = 0.8, 0.6
P[3, 1, 1] = P[3, 0, 1] * 1.01
dt = engine.min_period(S2_PLANETS) / 24.0
t, rv, er = engine.obs_arrays(obs)
plan = engine.LoglPlan(t, rv, er, obs.Npoints, 2, dt, 4, 256)
out = {}
for nl in (1, 4):
    plan = engine.LoglPlan(t, rv, er, obs.Npoints, 2, dt, nl, 256)
    K = torch.as_tensor(np.concatenate([P[:, p, :5].T for p in range(2)], 0).copy(), device="cuda")
    lp, st, rvo = plan.logl(K, want_rv=True)
    torch.cuda.synchronize()
    out[f"lp{nl}"] = lp.cpu().numpy()
    out[f"st{nl}"] = st.cpu().numpy()
    out[f"rv{nl}"] = rvo.cpu().numpy()
np.savez(os.path.join(ROOT, "gpurun_out", "debug_wide.npz"), P=P, **out)
print("saved")

"""Level-split vs LDS-coupled layout: per-epoch model RVs of the same walkers (diagnostic)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import oracle as O  # noqa: E402
from conftest import S2_PLANETS, s2_obs_oracle  # noqa: E402
from test_gpu_logl import _ball, _plan, _run  # noqa: E402

obs = s2_obs_oracle()
W = int(sys.argv[1]) if len(sys.argv) > 1 else 4128
plan, dt = _plan(obs, S2_PLANETS, max_walkers=W)
P = _ball(S2_PLANETS, W, seed=21)
big, st_big, rv_big = _run(plan, P, want_rv=True)
t = np.concatenate([obs.tf, obs.tb]) if hasattr(obs, "tf") else None
for i in (0, 1, 31, 32, 1000, W - 1):
    one, st1, rv1 = _run(plan, P[i:i + 1], want_rv=True)
    d = rv1[:, 0] - rv_big[:, i]
    nz = np.nonzero(d)[0]
    print(i, one[0], big[i], one[0] - big[i], "n_diff_epochs", len(nz), "first", nz[:8], "max", np.abs(d).max(),
          flush=True)
ref, sref = O.logl_whx_batch(P[[0, 1000]], 2, obs, dt, (4, 5, 6, 7))
print("oracle", ref, "big", big[[0, 1000]])

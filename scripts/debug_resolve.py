"""Debug: adaptive resolution on the wide ball in the level-split layout (one 6144-walker launch)
under three settings against the oracle restatement of each."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import test_gpu_resolve as T  # noqa: E402
from conftest import s2_obs_oracle  # noqa: E402

obs = s2_obs_oracle()
W = 6144
X = T.wide_walkers(W)
for res in ((0.0, 0), (T.TOL, 0), (T.TOL, 1), (T.TOL, 4)):
    plan, dt, mult = T._plan(obs, W, resolve=res)
    got, st = T._run(plan, X)
    f = plan.faults(reset=True)
    ref, st_ref, rf, est, margin = T._adapt_oracle(T._oracle_P(X), obs, dt, mult, res[0], res[1])
    mism = np.nonzero(st != st_ref)[0]
    ok = (st == 0) & (st_ref == 0)
    with np.errstate(invalid="ignore"):
        err = np.abs(got - ref) / np.maximum(1, np.abs(ref))
    big = np.nonzero(ok & (err > 1e-9))[0]
    print(res, f, "status mismatches", len(mism), "logl>1e-9", len(big), "groups", sorted(set((mism // 32).tolist()))[:20])
    pairs = {}
    for i in mism:
        k = (int(st[i]), int(st_ref[i]), int(i % 32 >= 16))
        pairs[k] = pairs.get(k, 0) + 1
    print("   (dev, ref, upper half):count", pairs)
    # per group: did the oracle refine any walker of the group (in either direction)?
    g = np.arange(W) // 32
    team = np.zeros(W // 32, bool)
    np.logical_or.at(team, g, rf.sum(axis=1) > 0)
    print("   mismatch groups with oracle refinement:", int(team[np.unique(mism // 32)].sum()), "of",
          len(np.unique(mism // 32)), "; groups refining:", int(team.sum()))

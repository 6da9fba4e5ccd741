"""Cost of rv_out (the SMALA stencil's per-epoch model RVs) on a likelihood launch: the same
S2-ball launch with and without it, at the SMALA stencil size and the sampler's half size.
Usage: python scripts/probe/rvout_cost.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import oracle as O  # noqa: E402
from conftest import S2_PLANETS, s2_obs_oracle  # noqa: E402
from rvmcmc import engine  # noqa: E402


def main():
    obs = s2_obs_oracle()
    cfg = engine.IntegratorConfig()
    dt, mult, hint = cfg.plan_args(S2_PLANETS)
    t, rv, er = engine.obs_arrays(obs)
    for W in (2048, 5376):
        plan = engine.LoglPlan(t, rv, er, obs.Npoints, 2, dt, mult, W, period_hint=hint)
        rng = np.random.default_rng(0)
        P = np.repeat(O.pal_params(S2_PLANETS)[None], W, 0)
        P[:, :, :5] *= 1 + 1e-3 * rng.standard_normal((W, 2, 5))
        K = torch.as_tensor(np.concatenate([P[:, p, :5].T for p in range(2)], 0).copy(), device="cuda")
        out = {}
        for want in (False, True):
            for _ in range(3):
                plan.logl(K, want_rv=want)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                plan.logl(K, want_rv=want)
            e1.record()
            torch.cuda.synchronize()
            out["rv_out" if want else "plain"] = e0.elapsed_time(e1) / 10
        print(W, {k: round(v, 4) for k, v in out.items()}, "ms/launch", flush=True)


if __name__ == "__main__":
    main()

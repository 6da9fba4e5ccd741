"""Diagnose one proposal the device leaves UNRESOLVED (GPU + oracle): its logL / status alone and
in batches (the launch layouts differ by walker count), for several resolve_max, with the
refinement kernel's split exchange on and off, next to the oracle's walker-level rule and IAS15.
Usage: diag_walker.py '<JSON list of free-parameter rows of the S2 state>'"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("rvel-mcmc_amd", "oracle", "tests")]
import torch  # noqa: E402

import ias15_parity as IP  # noqa: E402
import oracle as O  # noqa: E402
from conftest import S2_PLANETS, s2_obs_oracle  # noqa: E402
from rvmcmc import engine  # noqa: E402
from rvmcmc.state import State  # noqa: E402


def main():
    rows = np.array(json.loads(sys.argv[1]), dtype=np.float64)
    s = State(planets=[dict(p) for p in S2_PLANETS])
    pm = s.param_map()
    obs = s2_obs_oracle()
    hill = s.hillRadiusFactor
    cfg = engine.IntegratorConfig()
    dt, mult, hint = cfg.plan_args(S2_PLANETS)
    tol, rmax0, guard, _ = cfg.resolve(S2_PLANETS)
    P = IP.to_oracle(pm, rows)
    li, si = IP.ias15_logl(P, 2, obs, hill)
    la, sa, rf, est, _ = O.logl_whx_adapt_batch(P, 2, obs, dt, mult, tol, 12, hill, ecc_guard=guard)
    print(json.dumps({"oracle_adapt": la.tolist(), "status": sa.tolist(), "stages": rf.tolist(),
                      "ias15": li.tolist(), "ias15_status": si.tolist()}), flush=True)
    t = np.concatenate([obs.tf, obs.tb])
    rv = np.concatenate([obs.rvf, obs.rvb])
    sg = np.concatenate([obs.errorf, obs.errorb])
    rng = np.random.default_rng(0)
    for split in ("1", "0"):
        if split == "0":
            os.environ["RVM_REFINE_SPLIT"] = "0"
        for rmax in (4, 8, 12):
            for W in (1, 64, 1024, 3072):
                plan = engine.LoglPlan(t, rv, sg, obs.Npoints, 2, dt, mult, max(W, 64), torch.device("cuda", 0), hint, False,
                                       (tol, rmax, guard, True))
                X = np.repeat(rows[:1], W, axis=0)
                if W > 64:  # the row among tight-ball walkers (others settle early)
                    X[1:] = s.get_params()[None] + 1e-4 * rng.standard_normal((W - 1, X.shape[1]))
                Xd = torch.as_tensor(np.ascontiguousarray(X.T), device="cuda")
                lp, st, _ = plan.logl(pm.to_kernel(Xd), hill_factor=hill)
                torch.cuda.synchronize()
                f = plan.faults(reset=True)
                print(json.dumps({"split": split, "resolve_max": rmax, "W": W, "logl0": float(lp[0].item()),
                                  "status0": int(st[0].item()), "faults": f}), flush=True)
                del plan


if __name__ == "__main__":
    main()

"""Config 1 (reference-API single-chain Mh, mcmc_benchmark_mh.py) taken apart: the single-walker
likelihood launch on config 1's observation set (200 points) timed with HIP events -- resolution off
and on, with the plan's counters, and the Mh chain's wall time per step after a warm-up.
Usage: python scripts/probe/config1_probe.py"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from conftest import S2_PLANETS as S2  # noqa: E402
from rvmcmc import engine, mcmc  # noqa: E402
from rvmcmc.observations import FakeObservation  # noqa: E402
from rvmcmc.state import State  # noqa: E402


def launch_times(plan, K, n=30):
    lp, st, _ = plan.logl(K)
    torch.cuda.synchronize()
    plan.faults(reset=True)
    out = []
    for _ in range(n):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        plan.logl(K, out=lp, status=st)
        e1.record()
        torch.cuda.synchronize()
        out.append(e0.elapsed_time(e1))
    fl = plan.faults(reset=True)
    return float(np.median(out)), fl["refined"] / n, int(st[0])


def main():
    torch.cuda.set_device(0)
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in S2])
    obs = FakeObservation(s, Npoints=200, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    cfg = engine.IntegratorConfig()
    dt, mult, hint = cfg.plan_args(S2)
    t = np.concatenate([obs.tf, obs.tb])
    rv = np.concatenate([obs.rvf, obs.rvb])
    er = np.concatenate([obs.errorf, obs.errorb])
    X = np.array([[p[k] for k in ("m", "a", "h", "k", "l")] for p in S2]).reshape(-1)
    K = torch.as_tensor(X[:, None].copy(), device="cuda")
    for name, res in [("off", (0.0, 0)), ("on", cfg.resolve(S2))]:
        plan = engine.LoglPlan(t, rv, er, 200, 2, dt, mult, 1, period_hint=hint, resolve=res)
        ms, ref, st = launch_times(plan, K)
        print(json.dumps({"launch": "1 walker", "resolve": name, "ms_median": ms, "refined_per_launch": ref,
                          "status": st, "ext_mult": plan.ext_mult}), flush=True)
    for spec, tol in ((1, None), (3, None), (1, 0.0)):
        np.random.seed(2017)
        s = State(planets=[dict(p) for p in S2])
        if tol is not None:
            s.integrator = engine.IntegratorConfig(resolve_tol=tol)
        obs = FakeObservation(s, Npoints=200, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
        mh = mcmc.Mh(s, obs, speculate=spec)
        mh.set_scales({"m": 1.e-3, "a": 0.3, "h": 0.5, "k": 0.5, "l": np.pi / 2.})
        mh.step_size = 10.0e-3
        for _ in range(20):
            mh.step_force()
        torch.cuda.synchronize()
        tries = 0
        t0 = time.perf_counter()
        for _ in range(200):
            tries += mh.step_force()
        el = time.perf_counter() - t0
        print(json.dumps({"mh": spec, "resolve_tol": tol, "accepted_steps_per_s": 200 / el, "logl_evals_per_s": tries / el,
                          "ms_per_eval": 1e3 * el / tries}), flush=True)


if __name__ == "__main__":
    main()

"""Kernel micro-benchmark: one rvm_logl_batch launch on the S2 workload, timed with HIP events,
plus a T1 spot check against the oracle.  Usage: python scripts/kbench.py [W ...]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import oracle as O  # noqa: E402
from conftest import S2_PLANETS, s2_obs_oracle  # noqa: E402
from rvmcmc import _lib, engine  # noqa: E402

_lib.LIB_PATH = os.environ.get("RVM_LIB", _lib.LIB_PATH)  # A/B runs against another build


def main():
    Ws = [int(a) for a in sys.argv[1:]] or [2048, 4096]
    # LEVELS: "4" (harmonic 1..4) or "4,5,6,7" (multipliers); SPO: base steps per shortest orbit
    lv = os.environ.get("LEVELS", "4,5,6,7")
    nl = tuple(int(v) for v in lv.split(",")) if "," in lv else int(lv)
    spo = float(os.environ.get("SPO", "8"))
    obs = s2_obs_oracle()
    planets = [dict(p) for p in S2_PLANETS]
    if os.environ.get("NPL") == "3":  # config 5's added planet
        planets.append({"m": 1e-3, "a": 2.6, "h": 0.05, "k": 0.0, "l": 1.0})
    npl = len(planets)
    pmin = engine.min_period(planets)
    dt = pmin / spo
    t, rv, er = engine.obs_arrays(obs)
    plan = engine.LoglPlan(t, rv, er, obs.Npoints, npl, dt, nl, max(Ws), period_hint=pmin)
    rng = np.random.default_rng(0)
    for W in Ws:
        P = np.repeat(O.pal_params(planets)[None], W, 0)
        P[:, :, :5] *= 1 + float(os.environ.get("BALL", "1e-3")) * rng.standard_normal((W, npl, 5))
        K = torch.as_tensor(np.concatenate([P[:, p, :5].T for p in range(npl)], 0).copy(), device="cuda")
        lp, st, _ = plan.logl(K)
        torch.cuda.synchronize()
        times = []
        for _ in range(int(os.environ.get("REPS", "20"))):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            plan.logl(K, out=lp, status=st)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        idx = np.arange(0, W, max(1, W // 16))
        ref, sref = O.logl_whx_batch(P[idx], npl, obs, dt, nl)
        got = lp.cpu().numpy()[idx]
        err = np.max(np.abs(got - ref) / np.maximum(1, np.abs(ref)))
        ms = float(np.median(times))
        print(f"W={W} nl={nl} spo={spo:g}: {ms:.3f} ms/launch  {W / ms * 1e3:.3e} evals/s  T1 err {err:.2e}  "
              f"steps {plan.info()}", flush=True)


if __name__ == "__main__":
    main()

"""T2 of the likelihood over the bench's own ensemble (reference physics), fixed step vs adaptive.

Input: profiles/r03_bench_ensemble.npz -- the bench sampler's walkers (bench.py's setup, 4096
walkers, the kernel's own FakeObservation data) at iterations 23 (end of the timed window), 100
and 2000 (the ESS run's regime), dumped on the GPU by scripts/dump_bench_ensemble.py.  For a sample
of walkers at each iteration: |logL - logL_IAS15| with the plan's fixed step (resolve_tol = 0,
round 2's kernel algorithm) and with the adaptive resolution (IntegratorConfig defaults), both
from the oracle's restatements (T1-pinned to the kernel).  One JSON line per iteration.
Usage: python scripts/t2_bench_posterior.py [n_walkers] > profiles/r03_t2_bench_posterior.jsonl"""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as O  # noqa: E402
from conftest import S2_PLANETS  # noqa: E402
from rvmcmc import engine  # noqa: E402


def par(fn, P, nt=os.cpu_count() or 8):
    idx = np.array_split(np.arange(len(P)), nt)
    with ThreadPoolExecutor(nt) as ex:
        parts = list(ex.map(lambda ix: fn(P[ix]), idx))
    return [np.concatenate([p[k] for p in parts]) for k in range(len(parts[0]))]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    d = np.load(os.path.join(ROOT, "profiles", "r03_bench_ensemble.npz"))
    obs = O.OracleObs(tf=d["tf"], tb=d["tb"], rvf=d["rvf"], rvb=d["rvb"], errorf=d["errorf"], errorb=d["errorb"],
                      Npoints=100)
    cfg = engine.IntegratorConfig()
    dt, mult, _ = cfg.plan_args(S2_PLANETS)
    for key in ("it23", "it100", "it2000"):
        X = d[key][:n]
        P = np.zeros((len(X), 2, 7))
        P[:, :, :5] = X.reshape(-1, 2, 5)
        li, si = par(lambda p: O.logl_ias15_batch(p, 2, obs), P)
        lf, sf = par(lambda p: O.logl_whx_batch(p, 2, obs, dt, mult), P)
        la, sa, rf, _, _ = par(lambda p: O.logl_whx_adapt_batch(p, 2, obs, dt, mult, cfg.resolve_tol, cfg.resolve_max),
                               P)
        ok_f, ok_a = (sf == 0) & (si == 0), (sa == 0) & (si == 0)
        ef, ea = np.abs(lf - li)[ok_f], np.abs(la - li)[ok_a]
        print(json.dumps({
            "iteration": int(key[2:]), "walkers": len(X),
            "spread_over_scales": np.round(X.std(0) / np.array([1.5e-3, .3, .1, .1, np.pi / 2] * 2), 4).tolist(),
            "fixed_step": {"max_abs_dlogl": float(ef.max()), "n_above_1e-6": int((ef > 1e-6).sum()),
                           "p99": float(np.quantile(ef, .99)), "status_mismatch": int((sf != si).sum())},
            "adaptive": {"resolve_tol": cfg.resolve_tol, "resolve_max": cfg.resolve_max,
                         "max_abs_dlogl": float(ea.max()), "n_above_1e-6": int((ea > 1e-6).sum()),
                         "status_mismatch": int((sa != si).sum()),
                         "walker_directions_refined": int((rf > 0).sum()), "work_factor": float((2.0 ** rf).mean())},
        }), flush=True)


if __name__ == "__main__":
    main()

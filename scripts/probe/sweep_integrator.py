"""Integrator settings vs T2 and refinement work, on the bench's own walker slots (CPU, oracle).

For each candidate (levels, steps_per_orbit): the oracle's adaptive restatement
(oracle.logl_whx_adapt_batch, the kernel's algorithm incl. the extension level and the eccentricity
guard) over the 6144 slots of a speculative stretch iteration (scripts/probe/make_slots.py), against
IAS15 (the reference physics).  Reports max |dlogL| over OK proposals, count above 1e-6, status
mismatches, the stage histogram (0 plan step, 1 extension, 1 + r halvings) and the main-pass steps
per shortest period ((sum(mult) + ext) * steps_per_orbit: what one level-split launch integrates).
Usage: python scripts/probe/sweep_integrator.py slots.npz [n] [levels:spo ...]"""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
    f = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 6144
    cands = sys.argv[3:] or ["4,5,6,7:8", "4,5,6,7:7", "3,4,5,6:8", "3,4,5,6:7"]
    d = np.load(f)
    obs = O.OracleObs(tf=d["tf"], tb=d["tb"], rvf=d["rvf"], rvb=d["rvb"], errorf=d["errorf"], errorb=d["errorb"],
                      Npoints=100)
    X = d["K"][:n] if "K" in d else d["it2000"][:n]
    P = np.zeros((len(X), 2, 7))
    P[:, :, :5] = X.reshape(-1, 2, 5)
    li, si = par(lambda p: O.logl_ias15_batch(p, 2, obs), P)
    for c in cands:
        lv, spo = c.split(":")
        cfg = engine.IntegratorConfig(levels=tuple(int(x) for x in lv.split(",")), steps_per_orbit=float(spo))
        dt, mult, _ = cfg.plan_args(S2_PLANETS)
        tol, rmax, guard, _ = cfg.resolve(S2_PLANETS)
        la, sa, rf, _, _ = par(lambda p: O.logl_whx_adapt_batch(p, 2, obs, dt, mult, tol, rmax, ecc_guard=guard), P)
        ok = (sa == 0) & (si == 0)
        e = np.abs(la - li)[ok]
        ext = O.ext_multiplier(mult, rmax)
        hist = np.bincount(rf.ravel(), minlength=rmax + 2)
        print(json.dumps({
            "slots": os.path.basename(f), "n": len(X), "levels": list(mult), "steps_per_orbit": float(spo),
            "ext": ext, "main_pass_steps_per_Pmin": (sum(mult) + ext) * float(spo),
            "max_abs_dlogl": float(e.max()), "n_above_1e-6": int((e > 1e-6).sum()),
            "n_above_5e-7": int((e > 5e-7).sum()),
            "status_mismatch": int((sa != si).sum()), "stage_hist": hist.tolist(),
            "halving_directions": int((rf >= 2).sum()),
        }), flush=True)


if __name__ == "__main__":
    main()

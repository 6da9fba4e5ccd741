"""Study (CPU, oracle): would a sixth Richardson level (9 steps per base step, joined to the five
the main pass already has) settle the directions the extension leaves to a halving pass?  On the
6144 slots of a speculative iteration from the bench chain's iteration-2000 ensemble
(scripts/probe/slots_it2000.npz): walkers the adaptive rule halves (stage >= 2 in either
direction), their |logL - logL_IAS15| with the plan's levels (4..7), with the extension (4..8), with
a sixth level (4..9) and (4..10), and |logL(4..9) - logL(4..8)| as the candidate bound.
Output: profiles/r03t_sixth_level_study.json.  Usage: python scripts/probe/sixth_level_study.py"""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("rvel-mcmc_amd", "oracle", "tests")]
import oracle as O  # noqa: E402
from conftest import S2_PLANETS  # noqa: E402
from rvmcmc import engine  # noqa: E402


def par(fn, P, nt=os.cpu_count() or 8):
    idx = np.array_split(np.arange(len(P)), nt)
    with ThreadPoolExecutor(nt) as ex:
        parts = list(ex.map(lambda ix: fn(P[ix]), idx))
    return [np.concatenate([p[k] for p in parts]) for k in range(len(parts[0]))]


def main():
    d = np.load(os.path.join(ROOT, "scripts", "probe", "slots_it2000.npz"))
    obs = O.OracleObs(tf=d["tf"], tb=d["tb"], rvf=d["rvf"], rvb=d["rvb"], errorf=d["errorf"], errorb=d["errorb"],
                      Npoints=100)
    X = d["K"]
    P = np.zeros((len(X), 2, 7))
    P[:, :, :5] = X.reshape(-1, 2, 5)
    cfg = engine.IntegratorConfig()
    dt, mult, _ = cfg.plan_args(S2_PLANETS)
    tol, rmax, guard, _ = cfg.resolve(S2_PLANETS)
    la, sa, rf, _, _ = par(lambda p: O.logl_whx_adapt_batch(p, 2, obs, dt, mult, tol, rmax, ecc_guard=guard), P)
    h = (rf >= 2).any(axis=1) & (sa == 0)
    Ph = P[h]
    li, si = par(lambda p: O.logl_ias15_batch(p, 2, obs), Ph)
    L = {}
    for name, m in (("4..7", (4, 5, 6, 7)), ("4..8", (4, 5, 6, 7, 8)), ("4..9", (4, 5, 6, 7, 8, 9)),
                    ("4..10", (4, 5, 6, 7, 8, 9, 10))):
        L[name] = par(lambda p: O.logl_whx_batch(p, 2, obs, dt, m), Ph)[0]
    ok = si == 0
    out = {"slots": "slots_it2000", "walkers_halved": int(h.sum()), "ias15_ok": int(ok.sum())}
    for k, v in L.items():
        e = np.abs(v - li)[ok]
        out[f"err_{k}"] = {"max": float(np.nanmax(e)), "p90": float(np.nanquantile(e, .9)),
                           "n_above_1e-6": int((e > 1e-6).sum())}
    b = np.abs(L["4..9"] - L["4..8"])[ok]
    e6 = np.abs(L["4..9"] - li)[ok]
    for k in (2.5e-7, 5e-7, 1e-6):
        sel = b <= k
        out[f"bound_{k:g}"] = {"settled": int(sel.sum()), "max_err_settled": float(e6[sel].max()) if sel.any() else None}
    print(json.dumps(out))


if __name__ == "__main__":
    main()

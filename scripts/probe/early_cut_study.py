"""Study (CPU, oracle): the certain-reject test right after the extension (rvoracle.c EARLY_CUT)
against today's rule (the test only after a halving pass), on stretch proposals formed from the
bench chain's iteration-2000 ensemble (profiles/r03_bench_ensemble.npz: half 0 proposes against
half 1, z / j / u drawn as emcee 2.2.1 does, lnp0 = IAS15 logL of the current walker).  Reports
the stage histogram (0 plan step, 1 extension, 1 + r halvings), the cuts, and -- the correctness
check -- how many cut proposals IAS15's logL would have accepted (must be 0).
Usage: RVO_LIB=<EARLY_CUT build> python scripts/probe/early_cut_study.py   (once per build)"""
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
        parts = list(ex.map(lambda ix: fn(P[ix], ix), idx))
    return [np.concatenate([p[k] for p in parts]) for k in range(len(parts[0]))]


def main():
    d = np.load(os.path.join(ROOT, "profiles", "r03_bench_ensemble.npz"))
    obs = O.OracleObs(tf=d["tf"], tb=d["tb"], rvf=d["rvf"], rvb=d["rvb"], errorf=d["errorf"], errorb=d["errorb"],
                      Npoints=100)
    key = sys.argv[1] if len(sys.argv) > 1 else "it2000"
    E = d[key]
    n = len(E) // 2
    X, C = E[:n], E[n:]
    rng = np.random.default_rng(7)
    z = ((2.0 - 1.0) * rng.random(n) + 1.0) ** 2 / 2.0
    j = rng.integers(0, n, n)
    u = rng.random(n)
    Q = C[j] - z[:, None] * (C[j] - X)

    def rows(A):
        P = np.zeros((len(A), 2, 7))
        P[:, :, :5] = A.reshape(-1, 2, 5)
        return P

    l0, _ = par(lambda p, ix: O.logl_ias15_batch(p, 2, obs), rows(X))
    li, si = par(lambda p, ix: O.logl_ias15_batch(p, 2, obs), rows(Q))
    cfg = engine.IntegratorConfig()
    dt, mult, _ = cfg.plan_args(S2_PLANETS)
    tol, rmax, guard, _ = cfg.resolve(S2_PLANETS)
    ctx = dict(mode=np.ones(n, dtype=np.int32), dim=10, z=z, u=u, lnp0=l0)
    la, sa, rf, _, _, cut = par(lambda p, ix: O.logl_whx_adapt_batch(
        p, 2, obs, dt, mult, tol, rmax, ecc_guard=guard,
        ctx=dict(ctx, **{k: np.asarray(ctx[k])[ix] for k in ("mode", "z", "u", "lnp0")})), rows(Q))
    acc_ias = 9.0 * np.log(z) + li - l0 > np.log(u)
    acc_dev = 9.0 * np.log(z) + la - l0 > np.log(u)
    cutw = cut.any(axis=1)
    ok = (sa == 0) & (si == 0) & ~cutw
    print(json.dumps({
        "lib": os.path.basename(os.environ.get("RVO_LIB", "liboracle.so")), "ensemble": key, "proposals": n,
        "stage_hist": np.bincount(rf.ravel(), minlength=rmax + 2).tolist(),
        "halving_directions": int((rf >= 2).sum()), "deepest": int(rf.max()),
        "cut_walkers": int(cutw.sum()), "cut_but_ias15_accepts": int((cutw & acc_ias).sum()),
        "decisions_differ": int((acc_dev != acc_ias).sum()),
        "max_abs_dlogl_ok_uncut": float(np.abs(la - li)[ok].max()),
    }), flush=True)


if __name__ == "__main__":
    main()

"""Study (CPU, oracle): the certain-reject cut's eccentricity guard factor (oracle CUT_ECC_FACTOR,
kernel RVM_CUT_ECC_FACTOR) -- what it costs and what it protects.  For the steady-state ensembles of
HD155358, the 3-planet system and the bench chain (scripts/probe/ens_*.npy) it draws stretch moves
(fresh z, partner, u per iteration from one ensemble), takes the reference decision on IAS15 logL, and
runs the adaptive restatement with the sampler's accept inputs (the cut on) for each guard factor
(1 - e_cut) = f (1 - e_guard); f = 0: no guard.  Per factor: decisions that differ from the
reference's (beyond MARGIN of it, same status), walker-directions cut, the stages reached (the
refinement work), and the three walkers of tests/golden/cut_guard_walkers.json.
usage: cut_guard_study.py [iterations] [factors, comma-separated] [k: past the guard the bound after
the extension is chi2 - min(k d, 100 est); 0 = chi2 - 100 est] [systems] [1: past the guard, pass 1's
change is measured against the extension's RV instead of the main pass's] -> JSON lines."""
import ctypes as C
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("rvel-mcmc_amd", "oracle", "tests", "scripts/probe")]
import ias15_parity as IP  # noqa: E402
import oracle as O  # noqa: E402
from conftest import GOLDEN  # noqa: E402
from encounter_rule_study import system  # noqa: E402
from rvmcmc import engine  # noqa: E402
from rvmcmc.state import State  # noqa: E402


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    factors = [float(f) for f in (sys.argv[2] if len(sys.argv) > 2 else "0,0.6712,0.5,0.4,0.3").split(",")]
    gk = float(sys.argv[3]) if len(sys.argv) > 3 else 10.0  # past the guard: chi2 - min(gk d, 100 est)
    systems = sys.argv[4].split(",") if len(sys.argv) > 4 else ["hd155358", "3planet", "s2"]
    prev_ext = int(sys.argv[5]) if len(sys.argv) > 5 else 0  # past the guard, pass 1's change against the extension
    L = O.lib()
    L.rvo_study_set_cut_factor.argtypes = [C.c_double]
    L.rvo_study_set_guard_k.argtypes = [C.c_double]
    L.rvo_study_set_guard_k(gk)
    L.rvo_study_set_prev_ext(prev_ext)
    nt = IP.n_threads()
    with open(os.path.join(GOLDEN, "cut_guard_walkers.json")) as f:
        fixture = json.load(f)["walkers"]
    for name in systems:
        planets, obs, X = system(name)
        s = State(planets=[dict(p) for p in planets])
        pm = s.param_map()
        npl, dim = pm.n_planets, s.Nvars
        cfg = engine.IntegratorConfig()
        dt, mult, _ = cfg.plan_args(planets)
        tol, rmax, guard, _ = cfg.resolve(planets)
        rng = np.random.default_rng(23)
        n = len(X) // 2
        lnx = IP.ias15_logl(IP.to_oracle(pm, X), npl, obs)[0]
        Q, Z, U, L0 = [], [], [], []
        for _ in range(iters):
            for h in (0, 1):
                x, c = (X[:n], X[n:]) if h == 0 else (X[n:], X[:n])
                q, z = IP.stretch_proposal(x, c, rng.random(n), rng.random(n))
                Q.append(q)
                Z.append(z)
                U.append(rng.random(n))
                L0.append(lnx[:n] if h == 0 else lnx[n:])
        Q, Z, U, L0 = np.concatenate(Q), np.concatenate(Z), np.concatenate(U), np.concatenate(L0)
        P = IP.to_oracle(pm, Q)
        lq, sq = IP.ias15_logl(P, npl, obs)
        with np.errstate(invalid="ignore", divide="ignore"):
            d_ref = (dim - 1.0) * np.log(Z) + lq - L0
            acc_ref = d_ref > np.log(U)
            near = np.abs(d_ref - np.log(U)) < IP.MARGIN
        e = np.sqrt(np.max(P[:, :, 2] ** 2 + P[:, :, 3] ** 2, axis=1))
        chunks = [ix for ix in np.array_split(np.arange(len(P)), nt) if len(ix)]
        for f in factors:
            L.rvo_study_set_cut_factor(f)

            def one(ix):
                ctx = dict(mode=np.ones(len(ix), dtype=np.int32), dim=dim, z=Z[ix], u=U[ix], lnp0=L0[ix])
                return O.logl_whx_adapt_batch(P[ix], npl, obs, dt, mult, tol, rmax, ecc_guard=guard, ctx=ctx)

            with ThreadPoolExecutor(nt) as ex:
                parts = list(ex.map(one, chunks))
            lo, st, stage, _, _, cut = (np.concatenate([p[k] for p in parts]) for k in range(6))
            with np.errstate(invalid="ignore", divide="ignore"):
                acc = ~cut.any(axis=1) & ((dim - 1.0) * np.log(Z) + lo - L0 > np.log(U))
            bad = np.nonzero((acc != acc_ref) & ~near & (st == sq))[0]
            ec = 1.0 - (1.0 - guard) * f
            row = {"system": name, "factor": f, "guard_k": gk, "prev_ext": prev_ext, "e_cut": ec if f > 0 else None, "proposals": int(len(P)),
                   "decisions_differing": int(len(bad)), "differing_e": [round(float(e[i]), 3) for i in bad],
                   "walkers_cut": int(cut.any(axis=1).sum()), "guarded_walkers": int((e > ec).sum()) if f > 0 else 0,
                   "direction_stages_sum": int(stage.sum()),
                   "walkers_stage_ge3": int((stage.max(axis=1) >= 3).sum()),
                   "walkers_stage_ge4": int((stage.max(axis=1) >= 4).sum())}
            if name == "hd155358":
                ok = 0
                for r in fixture:
                    Pf = np.array([r["params"]])
                    ctx = dict(mode=np.ones(1, dtype=np.int32), dim=10, z=np.array([r["z"]]), u=np.array([r["u"]]),
                               lnp0=np.array([r["lnp0"]]))
                    lf, sf, _, _, _, cf = O.logl_whx_adapt_batch(Pf, 2, obs, dt, mult, tol, rmax, ecc_guard=guard,
                                                                 ctx=ctx)
                    ok += int(sf[0] == 0 and not cf[0].any() and 9.0 * np.log(r["z"]) + lf[0] - r["lnp0"] > np.log(r["u"]))
                row["fixture_walkers_accepted"] = ok
            print(json.dumps(row), flush=True)
    L.rvo_study_set_cut_factor(-1.0)
    L.rvo_study_set_guard_k(10.0)
    L.rvo_study_set_prev_ext(0)


if __name__ == "__main__":
    main()

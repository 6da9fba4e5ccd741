"""Study (CPU, oracle): the walker-directions of the steady-state sampler's launches that need a
SECOND halving pass (the ~30-40 % of steady-state iterations whose refinement kernel takes ~1.05 ms
instead of ~0.63 ms, profiles/r05b_bench.json kernel_ms_quantiles).  For each such direction
(and, for calibration, every direction one halving pass settles): per-epoch Richardson RVs of the
main pass (levels 4..7 at the plan's step), pass 1 (8, 10, 12, 14) and pass 2 (16 .. 28); pass 1's
estimate est1 (its r against the three finer levels' r3), its step-doubling change d1 against the
main pass's RV (what the kernel's lower bound uses; asymptotically 2^8 - 1 = 255 x pass 1's own
error), and pass 1's actual error against IAS15 -- whether a cheaper settle test than pass 2 would
hold T2 for them.  usage: pass2_study.py [iterations]  -> JSON lines."""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("rvel-mcmc_amd", "oracle", "tests")]
import ias15_parity as IP  # noqa: E402
import oracle as O  # noqa: E402
from conftest import S2_PLANETS, s2_obs_oracle  # noqa: E402
from philox_ref import stretch_uniforms  # noqa: E402
from rvmcmc import engine  # noqa: E402
from rvmcmc.state import State  # noqa: E402


def curves(P, obs, dt, d):
    """per-epoch RVs of one walker, direction d, in the oracle's epoch order: main, pass 1, pass 1's
    r3, pass 2, IAS15; and the direction's observations."""
    planets = [{"m": P[p, 0], "a": P[p, 1], "h": P[p, 2], "k": P[p, 3], "l": P[p, 4]} for p in range(len(P))]
    t, o, e = (obs.tf, obs.rvf, obs.errorf) if d == 0 else (obs.tb, obs.rvb, obs.errorb)
    out = {}
    for key, mult in (("r0", (4, 5, 6, 7)), ("r1", (8, 10, 12, 14)), ("r1_3", (10, 12, 14)),
                      ("r2", (16, 20, 24, 28)), ("x5", (8, 10, 12, 14, 15)), ("x7", (8, 9, 10, 11, 12, 13, 14)),
                      ("x6", (9, 10, 11, 12, 13, 14)), ("x6b", (8, 10, 12, 14, 9, 11))):
        out[key] = O.whx_rv(planets, t, dt, mult, 1.0)[0]
    out["ias"] = O.get_rv_ias15(planets, t, 1.0)[0]
    return out, o, e * e


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    s = State(planets=[dict(p) for p in S2_PLANETS])
    obs = s2_obs_oracle()
    pm = s.param_map()
    dim = s.Nvars
    X0 = np.load(os.path.join(ROOT, "scripts", "probe", "ens_it2000.npy"))
    n = len(X0) // 2
    cfg = engine.IntegratorConfig()
    dt, mult, _ = cfg.plan_args(S2_PLANETS)
    tol, rmax, guard, _ = cfg.resolve(S2_PLANETS)
    nt = os.cpu_count() or 8
    N = obs.Npoints

    def adapt(A, ctx=None):
        P = IP.to_oracle(pm, A)
        idx = [ix for ix in np.array_split(np.arange(len(P)), nt) if len(ix)]

        def one(ix):
            c = None if ctx is None else {k: (v[ix] if isinstance(v, np.ndarray) else v) for k, v in ctx.items()}
            return O.logl_whx_adapt_batch(P[ix], 2, obs, dt, mult, tol, rmax, 1.0, ecc_guard=guard, ctx=c)

        with ThreadPoolExecutor(nt) as ex:
            parts = list(ex.map(one, idx))
        return [np.concatenate([p[k] for p in parts]) for k in range(len(parts[0]))]

    pos = [X0[:n].copy(), X0[n:].copy()]
    lnp = [adapt(p)[0] for p in pos]
    rows = []
    for it in range(iters):
        u1, u2, u3 = stretch_uniforms(2017, 0, n, it, 0)
        q0, z0 = IP.stretch_proposal(pos[0], pos[1], u1, u2, 2.0)
        ctx0 = dict(mode=np.ones(n, dtype=np.int32), dim=dim, z=z0, u=u3, lnp0=lnp[0])
        l0, s0, rf0, est0, _, cut0 = adapt(q0, ctx0)
        with np.errstate(invalid="ignore"):
            acc0 = (dim - 1.0) * np.log(z0) + l0 - lnp[0] > np.log(u3)
        v1, v2, v3 = stretch_uniforms(2017, n, n, it, 1)
        zz = ((2.0 - 1.0) * v1 + 1) ** 2 / 2.0
        j = np.clip(np.floor(v2 * n).astype(int), 0, n - 1)
        ca, cb = pos[0][j], q0[j]
        qa = ca - zz[:, None] * (ca - pos[1])
        qb = cb - zz[:, None] * (cb - pos[1])
        ctx1 = dict(mode=np.ones(2 * n, dtype=np.int32), dim=dim, z=np.concatenate([zz, zz]),
                    u=np.concatenate([v3, v3]), lnp0=np.concatenate([lnp[1], lnp[1]]))
        l1, s1, rf1, est1, _, cut1 = adapt(np.concatenate([qa, qb]), ctx1)
        Q = np.concatenate([q0, qa, qb])
        rf = np.concatenate([rf0, rf1])
        cut = np.concatenate([cut0, cut1])
        # directions settled by one halving (stage 2) or needing two (stage 3), not cut
        for slot, d in zip(*np.nonzero((rf >= 2) & (cut == 0))):
            P = IP.to_oracle(pm, Q[slot:slot + 1])[0]
            c, o, s2 = curves(P, obs, dt, d)
            chi = {k: float(np.sum((c[k] - o) ** 2 / s2)) / N for k in ("r0", "r1", "r2", "ias")}
            e1 = float(np.sum(np.abs((c["r1"] - c["r1_3"]) * (c["r1"] + c["r1_3"] - 2 * o)) / s2)) / N
            d1 = float(np.sum(np.abs((c["r1"] - c["r0"]) * (c["r1"] + c["r0"] - 2 * o)) / s2)) / N
            def chg(a, b):
                return float(np.sum(np.abs((c[a] - c[b]) * (c[a] + c[b] - 2 * o)) / s2)) / N / (0.5 * tol)

            for k in ("x5", "x7", "x6b"):
                chi[k] = float(np.sum((c[k] - o) ** 2 / s2)) / N
            rows.append({"it": it, "slot": int(slot), "dir": int(d), "stage": int(rf[slot, d]),
                         "x5_d_over_tol": chg("x5", "r1"), "x5_err": abs(chi["x5"] - chi["ias"]),
                         "x7_est_over_tol": chg("x7", "x6"), "x7_err": abs(chi["x7"] - chi["ias"]),
                         "x6b_d_over_tol": chg("x6b", "r1"), "x6b_err": abs(chi["x6b"] - chi["ias"]),
                         "est1_over_tol": e1 / (0.5 * tol), "d1_over_tol": d1 / (0.5 * tol),
                         "err1": abs(chi["r1"] - chi["ias"]), "err2": abs(chi["r2"] - chi["ias"]),
                         "err0": abs(chi["r0"] - chi["ias"])})
        print(json.dumps({"it": it, "pass1_dirs": int(((rf == 2) & (cut == 0)).sum()),
                          "pass2_dirs": int(((rf >= 3) & (cut == 0)).sum())}), flush=True)
        pos[0] = np.where(acc0[:, None], q0, pos[0])
        lnp[0] = np.where(acc0, l0, lnp[0])
        pick = acc0[j]
        q1 = np.where(pick[:, None], qb, qa)
        l1s = np.where(pick, l1[n:], l1[:n])
        with np.errstate(invalid="ignore"):
            acc1 = (dim - 1.0) * np.log(zz) + l1s - lnp[1] > np.log(v3)
        pos[1] = np.where(acc1[:, None], q1, pos[1])
        lnp[1] = np.where(acc1, l1s, lnp[1])
    for r in rows:
        if r["stage"] >= 3:
            print(json.dumps(r))
    for cand, key in (("x5", "x5_d_over_tol"), ("x7", "x7_est_over_tol"), ("x6b", "x6b_d_over_tol")):
        for st in (2, 3):
            R = [r for r in rows if r["stage"] == st]
            if not R:
                continue
            ok = [r for r in R if r[key] <= 1.0]
            print(json.dumps({"candidate": cand, "stage": st, "dirs": len(R), "settled": len(ok),
                              "max_err_settled": max([r[cand + "_err"] for r in ok], default=0.0),
                              "max_err_all": max(r[cand + "_err"] for r in R)}))
    R = [r for r in rows if r["stage"] == 2]
    if R:
        ratio = np.array([r["err1"] / max(r["d1_over_tol"] * 0.5 * tol, 1e-300) for r in R])
        print(json.dumps({"pass1_settled_dirs": len(R), "max_err1": max(r["err1"] for r in R),
                          "err1_over_d1_max": float(ratio.max()), "err1_over_d1_p99": float(np.quantile(ratio, 0.99)),
                          "d1_over_tol_max": max(r["d1_over_tol"] for r in R)}))


if __name__ == "__main__":
    main()

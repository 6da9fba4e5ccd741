"""Study (CPU, oracle): the walker-directions of a steady-state chain that need two or more halving
passes (HD155358 by default: the ensemble of test_stretch_vs_ias15_steady_state_other_systems).
For each such direction (not cut): per pass rf = 0 (the plan's step) .. 4 the estimate est_rf (the
chi2 change when the coarsest level is dropped, / npoints / tol_dir: the kernel's settle test is
est <= 1), the step-doubling change against the previous pass, and the pass's actual error
|chi2 - chi2_IAS15| / npoints -- whether the passes these walkers climb are needed for T2, or the
estimate over-reads; and the same for a three-level pass (the coarsest three levels of the pass,
6 x 2^rf steps per base step at most: est3, err3).
usage: deep_walker_study.py [iterations] [hd155358|s2]  -> JSON lines."""
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


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    system = sys.argv[2] if len(sys.argv) > 2 else "hd155358"
    if system == "hd155358":
        from test_gpu_ias15_decisions import _hd

        planets, obs = _hd()
        X0 = np.load(os.path.join(ROOT, "scripts", "probe", "ens_hd155358_it1000.npy"))
    else:
        planets, obs = S2_PLANETS, s2_obs_oracle()
        X0 = np.load(os.path.join(ROOT, "scripts", "probe", "ens_it2000.npy"))
    s = State(planets=[dict(p) for p in planets])
    pm = s.param_map()
    dim = s.Nvars
    n = len(X0) // 2
    cfg = engine.IntegratorConfig()
    dt, mult, _ = cfg.plan_args(planets)
    tol, rmax, guard, _ = cfg.resolve(planets)
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

    def analyse(P, d):
        pl = [{"m": P[p, 0], "a": P[p, 1], "h": P[p, 2], "k": P[p, 3], "l": P[p, 4]} for p in range(len(P))]
        t, o, e = (obs.tf, obs.rvf, obs.errorf) if d == 0 else (obs.tb, obs.rvb, obs.errorb)
        s2 = e * e
        ias = O.get_rv_ias15(pl, t, 1.0)[0]
        c_ias = float(np.sum((ias - o) ** 2 / s2)) / N
        row, prev = [], None
        for rf in range(5):
            m = tuple(int(k) << rf for k in mult)
            r = O.whx_rv(pl, t, dt, m, 1.0)[0]
            r3 = O.whx_rv(pl, t, dt, m[1:], 1.0)[0]
            est = float(np.sum(np.abs((r - r3) * (r + r3 - 2 * o)) / s2)) / N / (0.5 * tol)
            dch = None if prev is None else float(np.sum(np.abs((r - prev) * (r + prev - 2 * o)) / s2)) / N / (0.5 * tol)
            c = float(np.sum((r - o) ** 2 / s2)) / N
            e = {"rf": rf, "est_over_tol": est, "change_over_tol": dch, "err": abs(c - c_ias)}
            if rf >= 1:  # (a three-level pass: the coarsest three of the four, max 6 x 2^rf per base step)
                r3l = O.whx_rv(pl, t, dt, m[:3], 1.0)[0]
                r3d = O.whx_rv(pl, t, dt, m[1:3], 1.0)[0]
                e["est3_over_tol"] = float(np.sum(np.abs((r3l - r3d) * (r3l + r3d - 2 * o)) / s2)) / N / (0.5 * tol)
                e["err3"] = abs(float(np.sum((r3l - o) ** 2 / s2)) / N - c_ias)
            row.append(e)
            prev = r
        return row

    pos = [X0[:n].copy(), X0[n:].copy()]
    lnp = [adapt(p)[0] for p in pos]
    for it in range(iters):
        u1, u2, u3 = stretch_uniforms(2017, 0, n, it, 0)
        q0, z0 = IP.stretch_proposal(pos[0], pos[1], u1, u2, 2.0)
        ctx0 = dict(mode=np.ones(n, dtype=np.int32), dim=dim, z=z0, u=u3, lnp0=lnp[0])
        l0, s0, rf0, _, _, cut0 = adapt(q0, ctx0)
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
        l1, s1, rf1, _, _, cut1 = adapt(np.concatenate([qa, qb]), ctx1)
        Q = np.concatenate([q0, qa, qb])
        rf = np.concatenate([rf0, rf1])
        cut = np.concatenate([cut0, cut1])
        for slot, d in zip(*np.nonzero((rf >= 3) & ((cut & 1) == 0))):
            P = IP.to_oracle(pm, Q[slot:slot + 1])[0]
            print(json.dumps({"it": it, "slot": int(slot), "dir": int(d), "stage": int(rf[slot, d]),
                              "e": [float(np.hypot(P[p, 2], P[p, 3])) for p in range(len(P))],
                              "passes": analyse(P, d)}), flush=True)
        pos[0] = np.where(acc0[:, None], q0, pos[0])
        lnp[0] = np.where(acc0, l0, lnp[0])
        pick = acc0[j]
        q1 = np.where(pick[:, None], qb, qa)
        l1s = np.where(pick, l1[n:], l1[:n])
        with np.errstate(invalid="ignore"):
            acc1 = (dim - 1.0) * np.log(zz) + l1s - lnp[1] > np.log(v3)
        pos[1] = np.where(acc1[:, None], q1, pos[1])
        lnp[1] = np.where(acc1, l1s, lnp[1])


if __name__ == "__main__":
    main()

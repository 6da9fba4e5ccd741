"""Study (CPU, oracle): can the walkers of a steady-state launch that need a halving pass be picked
BEFORE the launch, from their parameters alone?  If every launch's halving walkers were among the
K slots a cheap score ranks first, pass 1 of those K could run on the CUs the main launch leaves idle
(16 of 256 at 6144 slots) and the refinement kernel would replay it instead of integrating it after
the main pass ("start pass 1 on the main launch's idle CUs").

For the speculative stretch iterations of the bench chain from scripts/probe/ens_it2000.npy (as
pass2_study.py forms them): the slots whose walker needs halving pass 1 (oracle rvo_logl_whx_adapt
stage >= 2 in a direction, not cut before it), and per score the rank of the worst such slot -- the
K that would have caught them all.  Scores: tau = min over planets of P (1 - e)^1.5 (the quickest
pericentre passage), max e, and the eccentricity-guard factor.
usage: pass1_predictor_study.py [iterations] -> JSON lines."""
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


def scores(P):
    """P [n][planets][5] (m, a, h, k, l) -> dict of per-slot scores (higher = more likely to halve)"""
    m, a, h, k = P[..., 0], P[..., 1], P[..., 2], P[..., 3]
    e = np.sqrt(h * h + k * k)
    per = np.where(a > 0, np.abs(a) ** 1.5 / np.sqrt(1.0 + m), np.inf)
    with np.errstate(invalid="ignore", divide="ignore"):
        tau = per * np.clip(1.0 - e, 1e-6, None) ** 1.5
        # closest possible approach of the pair: a_o (1 - e_o) - a_i (1 + e_i), relative to a_i
        gap = (a[:, 1] * (1 - e[:, 1]) - a[:, 0] * (1 + e[:, 0])) / a[:, 0]
    return {"inv_tau": 1.0 / np.min(tau, axis=1), "max_e": np.max(e, axis=1), "neg_gap": -gap,
            "inv_tau_x_gap": (1.0 / np.min(tau, axis=1)) * np.exp(-np.clip(gap, -5, 5) * 4.0)}


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 3
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
        # a slot halves when a direction reached stage >= 2 (cut walkers stop at their stage)
        halving = np.any(rf >= 2, axis=1)
        deep = np.any(rf >= 3, axis=1)
        P = IP.to_oracle(pm, Q)
        sc = scores(P)
        out = {"it": it, "slots": int(len(Q)), "halving_slots": int(halving.sum()), "pass2_slots": int(deep.sum()),
               "cut_slots": int((cut != 0).any(axis=1).sum()) if cut.ndim > 1 else int((cut != 0).sum())}
        for name, v in sc.items():
            order = np.argsort(-np.nan_to_num(v, nan=np.inf), kind="stable")
            rank = np.empty(len(order), dtype=np.int64)
            rank[order] = np.arange(len(order))
            out[f"K_all_halving_{name}"] = int(rank[halving].max()) + 1 if halving.any() else 0
            out[f"K_all_pass2_{name}"] = int(rank[deep].max()) + 1 if deep.any() else 0
            out[f"halving_in_top512_{name}"] = int((rank[halving] < 512).sum())
        print(json.dumps(out), flush=True)
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

"""Study (CPU, oracle): the walker slots of the steady-state sampler's speculative launches
(scripts/probe/steady_bench.py's chain: ens_it2000.npy, seed 2017, 6144 slots per iteration -- half
0's proposals and half 1's against both outcomes of its partner) through the walker-level rule with
the sampler's accept inputs (certain rejects), restated by the oracle.  Per iteration: how many
slots reach each stage, and for the slots that need two or more halving passes their extension
change d, final logL against their current lnp, and whether the accept test passes -- which walkers
make half of the steady state's refinement launches take a second pass (GPU trace, r04n)."""
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
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    s = State(planets=[dict(p) for p in S2_PLANETS])
    obs = s2_obs_oracle()  # (bench.py's FakeObservation, restated on the CPU)
    pm = s.param_map()
    dim = s.Nvars
    X0 = np.load(os.path.join(ROOT, "scripts", "probe", "ens_it2000.npy"))
    W = len(X0)
    n = W // 2
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
        # half 0 against half 1 (as the speculative launch's slots [0, n))
        u1, u2, u3 = stretch_uniforms(2017, 0, n, it, 0)
        q0, z0 = IP.stretch_proposal(pos[0], pos[1], u1, u2, 2.0)
        ctx0 = dict(mode=np.ones(n, dtype=np.int32), dim=dim, z=z0, u=u3, lnp0=lnp[0])
        l0, s0, rf0, _, _, cut0 = adapt(q0, ctx0)
        with np.errstate(invalid="ignore"):
            acc0 = (dim - 1.0) * np.log(z0) + l0 - lnp[0] > np.log(u3)
        # half 1 against both outcomes of its partner (slots [n, 3n))
        v1, v2, v3 = stretch_uniforms(2017, n, n, it, 1)
        zz = ((2.0 - 1.0) * v1 + 1) ** 2 / 2.0
        j = np.clip(np.floor(v2 * n).astype(int), 0, n - 1)
        ca, cb = pos[0][j], q0[j]
        qa = ca - zz[:, None] * (ca - pos[1])
        qb = cb - zz[:, None] * (cb - pos[1])
        ctx1 = dict(mode=np.ones(2 * n, dtype=np.int32), dim=dim, z=np.concatenate([zz, zz]),
                    u=np.concatenate([v3, v3]), lnp0=np.concatenate([lnp[1], lnp[1]]))
        l1, s1, rf1, _, _, cut1 = adapt(np.concatenate([qa, qb]), ctx1)
        rf = np.concatenate([rf0, rf1]).max(axis=1)
        cc = np.concatenate([cut0, cut1])
        cut = (cc & 1).any(axis=1)
        jumped = (cc & 2).any(axis=1)  # (study build with -DJUMP_T: the walker started at rf = 2)
        # latency of the launch's refinement in units of one rf = 1 pass: the deepest walker's passes
        units = np.where(rf >= 2, 2.0 ** (rf - 1) * 2 - np.where(jumped, 2, 1), 0)  # sum_{r=r0}^{rf-1} 2^(r-1)
        lall = np.concatenate([l0, l1])
        z3 = np.concatenate([z0, zz, zz])
        u3a = np.concatenate([u3, v3, v3])
        lp0 = np.concatenate([lnp[0], lnp[1], lnp[1]])
        with np.errstate(invalid="ignore", divide="ignore"):
            dacc = (dim - 1.0) * np.log(z3) + lall - lp0 - np.log(u3a)
        deep = np.nonzero(rf >= 3)[0]
        print(json.dumps({"it": it, "stage_hist": np.bincount(rf, minlength=6).tolist(), "cut": int(cut.sum()),
                          "jumped": int(jumped.sum()), "refine_units": float(units.max()),
                          "deep_slots": [{"slot": int(i), "stage": int(rf[i]), "cut": bool(cut[i]),
                                          "accept_margin": float(dacc[i]), "logl": float(lall[i]),
                                          "lnp0": float(lp0[i])} for i in deep]}), flush=True)
        # the chain goes on with half 0's decisions, then half 1's variant by its partner's decision
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

"""Study (CPU, oracle): replay the proposals of tests/test_gpu_ias15_decisions.py's wide-ball and
steady-state tests (the same Philox draws; the chain follows the oracle's own decisions, which are
the device's wherever the two agree) and report, per proposal the walker-level rule (oracle
rvo_logl_whx_adapt, plain launch: no accept inputs) leaves UNRESOLVED or more than 1e-6 from IAS15,
its stages, estimates and IAS15 logL.  Usage: replay_parity.py wide|steady [resolve_max]"""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("rvel-mcmc_amd", "oracle", "tests")]
import ias15_parity as IP  # noqa: E402
import oracle as O  # noqa: E402
from conftest import S2_PLANETS, S2_SCALES, s2_obs_oracle  # noqa: E402
from philox_ref import stretch_uniforms  # noqa: E402
from rvmcmc import engine  # noqa: E402
from rvmcmc.state import State  # noqa: E402


def par(fn, P, nt=os.cpu_count() or 8):
    idx = [ix for ix in np.array_split(np.arange(len(P)), nt) if len(ix)]
    with ThreadPoolExecutor(nt) as ex:
        parts = list(ex.map(lambda ix: fn(P[ix]), idx))
    return [np.concatenate([p[k] for p in parts]) for k in range(len(parts[0]))]


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "wide"
    rmax = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    obs = s2_obs_oracle()
    s = State(planets=[dict(p) for p in S2_PLANETS])
    pm = s.param_map()
    dim = s.Nvars
    scales = np.array([S2_SCALES[k] for k in s.get_rawkeys()])
    if which == "wide":
        W = 2048
        X0 = s.get_params()[None] + 0.6 * scales * np.random.default_rng(3).standard_normal((W, dim))
    else:
        X0 = np.load(os.path.join(ROOT, "scripts", "probe", "ens_it2000.npy"))
        W = len(X0)
    n = W // 2
    hill = s.hillRadiusFactor
    cfg = engine.IntegratorConfig()
    dt, mult, _ = cfg.plan_args(S2_PLANETS)
    tol, _, guard, _ = cfg.resolve(S2_PLANETS)
    seed = 2017

    def adapt(A):
        return par(lambda p: O.logl_whx_adapt_batch(p, 2, obs, dt, mult, tol, rmax, hill, ecc_guard=guard),
                   IP.to_oracle(pm, A))

    pos = [X0[:n].copy(), X0[n:].copy()]
    lnp = [adapt(p)[0] for p in pos]
    for it in range(2):
        for h in (0, 1):
            c = pos[1 - h]
            u1, u2, u3 = stretch_uniforms(seed, h * n, n, it, h)
            q, z = IP.stretch_proposal(pos[h], c, u1, u2, 2.0)
            la, sa, rf, est, mg = adapt(q)
            li, si = IP.ias15_logl(IP.to_oracle(pm, q), 2, obs, hill)
            ok = (sa == 0) & (si == 0)
            bad = np.nonzero((sa == O.ORACLE_UNRESOLVED) | (ok & (np.abs(la - li) > 1e-6)) | (rf.max(1) >= int(os.environ.get('DEEP', 99))))[0]
            for i in bad:
                print(json.dumps({"it": it, "half": h, "i": int(i), "status": int(sa[i]), "ias15_status": int(si[i]),
                                  "logl": float(la[i]), "logl_ias15": float(li[i]), "stages": rf[i].tolist(),
                                  "est": est[i].tolist(), "q": q[i].tolist()}), flush=True)
            print(json.dumps({"it": it, "half": h, "statuses": np.bincount(sa, minlength=5).tolist(),
                              "stage_hist": np.bincount(rf.ravel(), minlength=rmax + 2).tolist(),
                              "max_dlogl_ok": float(np.max(np.abs(la - li)[ok])) if ok.any() else 0.0}), flush=True)
            with np.errstate(invalid="ignore"):
                acc = (dim - 1.0) * np.log(z) + la - lnp[h] > np.log(u3)
            pos[h] = np.where(acc[:, None], q, pos[h])
            lnp[h] = np.where(acc, la, lnp[h])


if __name__ == "__main__":
    main()

"""Study (CPU, oracle): how deep the walker-level adaptive resolution goes on plain likelihood
launches (no sampler accept inputs, so no certain rejects) of a 0.6-wide ball around S2 and of
stretch proposals between its members -- the regime of tests/test_gpu_ias15_decisions.py's wide-ball
test -- for resolve_max 4 / 6 / 8: the stage histogram (0 the plan's step, 1 the extension,
1 + r a halving pass r) and the statuses (4 = UNRESOLVED).  One JSON line per (set, resolve_max)."""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("rvel-mcmc_amd", "oracle", "tests")]
import oracle as O  # noqa: E402
from conftest import S2_PLANETS, S2_SCALES, s2_obs_oracle  # noqa: E402
from rvmcmc import engine  # noqa: E402
from rvmcmc.state import State  # noqa: E402


def par(fn, P, nt=os.cpu_count() or 8):
    idx = np.array_split(np.arange(len(P)), nt)
    with ThreadPoolExecutor(nt) as ex:
        parts = list(ex.map(lambda ix: fn(P[ix]), idx))
    return [np.concatenate([p[k] for p in parts]) for k in range(len(parts[0]))]


def main():
    obs = s2_obs_oracle()
    s = State(planets=[dict(p) for p in S2_PLANETS])
    scales = np.array([S2_SCALES[k] for k in s.get_rawkeys()])
    W = 2048
    X0 = s.get_params()[None] + 0.6 * scales * np.random.default_rng(3).standard_normal((W, s.Nvars))
    n = W // 2
    X, C = X0[:n], X0[n:]
    r2 = np.random.default_rng(7)
    z = ((2.0 - 1.0) * r2.random(n) + 1.0) ** 2 / 2.0
    j = r2.integers(0, n, n)
    Q = C[j] - z[:, None] * (C[j] - X)

    def rows(A):
        P = np.zeros((len(A), 2, 7))
        P[:, :, :5] = A.reshape(-1, 2, 5)
        return P

    cfg = engine.IntegratorConfig()
    dt, mult, _ = cfg.plan_args(S2_PLANETS)
    tol, _, guard, _ = cfg.resolve(S2_PLANETS)
    for A, name in ((X0, "0.6-wide ball, 2048 walkers"), (Q, "stretch proposals between its halves, 1024")):
        for rmax in (4, 6, 8):
            la, sa, rf, _, _ = par(lambda p: O.logl_whx_adapt_batch(p, 2, obs, dt, mult, tol, rmax, ecc_guard=guard),
                                   rows(A))
            print(json.dumps({"set": name, "resolve_max": rmax, "statuses": np.bincount(sa, minlength=5).tolist(),
                              "unresolved": int((sa == O.ORACLE_UNRESOLVED).sum()),
                              "stage_hist": np.bincount(rf.ravel(), minlength=rmax + 2).tolist()}), flush=True)


if __name__ == "__main__":
    main()

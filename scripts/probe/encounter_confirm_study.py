"""Study (CPU, oracle): a finer pass confirms every encounter (VERDICT r5 item 2's rule) -- the
oracle's study switch rvo_study_set_enc_confirm: 0 = the product rule (an encounter only the main
pass's coarser levels see refines on, the finest level's or a halving pass's ends the walker),
1 = the main pass's finest level refines on too (the extension or pass 1 decides), 2 = besides, a
halving pass's encounter ends the walker only when the stage before it saw one, 3 = rule 1 and the
extension's encounter refines on too, 4 = rule 3 and a halving pass's encounter needs the previous
halving pass's.  For the steady-state
stretch proposals of a system (encounter_rule_study.py's draws) it reports, per rule, the status pairs
against the IAS15 restatement (2/0: the device ends ENCOUNTER and REBOUND integrates; 0/2 the other
way), the 2/0 pairs' densely sampled closest approach, and the stages the walker-directions reached
(the cost).  usage: encounter_confirm_study.py {hd155358|3planet|s2} [n_iterations] -> JSON lines."""
import json
import os
import sys
from concurrent.futures import ThreadPoolExecutor

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("rvel-mcmc_amd", "oracle", "tests", "scripts/probe")]
import ias15_parity as IP  # noqa: E402
import oracle as O  # noqa: E402
from encounter_rule_study import level_ratio, system  # noqa: E402
from rvmcmc import engine  # noqa: E402
from rvmcmc.state import State  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "hd155358"
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    planets, obs, X = system(name)
    s = State(planets=[dict(p) for p in planets])
    pm = s.param_map()
    npl = pm.n_planets
    cfg = engine.IntegratorConfig()
    dt, mult, _ = cfg.plan_args(planets)
    tol, rmax, guard, _ = cfg.resolve(planets)
    rng = np.random.default_rng(11)
    n = len(X) // 2
    Q = []
    for _ in range(iters):
        for h in (0, 1):
            x, c = (X[:n], X[n:]) if h == 0 else (X[n:], X[:n])
            q, _ = IP.stretch_proposal(x, c, rng.random(n), rng.random(n))
            Q.append(q)
    P = IP.to_oracle(pm, np.concatenate(Q))
    _, st_ref = IP.ias15_logl(P, npl, obs)
    nt = IP.n_threads()
    chunks = [ix for ix in np.array_split(np.arange(len(P)), nt) if len(ix)]
    L = O.lib()
    for rule in (0, 1, 2, 3, 4):
        L.rvo_study_set_enc_confirm(rule)
        with ThreadPoolExecutor(nt) as ex:
            parts = list(ex.map(lambda ix: O.logl_whx_adapt_batch(P[ix], npl, obs, dt, mult, tol, rmax,
                                                                   ecc_guard=guard), chunks))
        st = np.concatenate([p[1] for p in parts])
        stage = np.concatenate([p[2] for p in parts])
        e20 = np.nonzero((st == IP.ST_ENC) & (st_ref == IP.ST_OK))[0]
        e02 = np.nonzero((st == IP.ST_OK) & (st_ref == IP.ST_ENC))[0]
        truth = [level_ratio(P[i:i + 1], npl, obs, dt / 32, 1) for i in e20]
        smax = stage.max(axis=1)
        print(json.dumps({"system": name, "rule": rule, "proposals": int(len(P)),
                          "device_encounters": int((st == IP.ST_ENC).sum()),
                          "ias15_encounters": int((st_ref == IP.ST_ENC).sum()),
                          "enc_2_0": int(len(e20)), "enc_2_0_outside_exit_distance": int(sum(t >= 1 for t in truth)),
                          "enc_2_0_truth": sorted(round(t, 4) for t in truth), "enc_0_2": int(len(e02)),
                          "other_pairs": int(((st != st_ref) & ~np.isin(np.arange(len(P)), np.r_[e20, e02])).sum()),
                          "unresolved": int((st == 4).sum()),
                          "walkers_by_deepest_stage": {str(k): int((smax == k).sum()) for k in range(int(smax.max()) + 1)},
                          "direction_stages_sum": int(stage.sum())}), flush=True)
    L.rvo_study_set_enc_confirm(0)


if __name__ == "__main__":
    main()

"""Study (CPU, oracle): how the kernel's encounter calls compare with REBOUND's.

The reference ends a proposal when a pair comes inside exit_min_distance at an IAS15 step end
(state.py:46; mcmc.py:30-34, 119-121).  The kernel (and its oracle mirror rvo_logl_whx_adapt) tests
the exit distance at every kick of its Wisdom-Holman levels, whose positions near a close approach
carry the level's discretisation error.  For the steady-state stretch proposals of a system
(scripts/probe/ens_*_it1000.npy, stretch moves with fresh draws) this script takes every proposal
the adaptive restatement ends ENCOUNTER and reports, per proposal:
  ias15     -- the IAS15 restatement's status (2 = it raises Encounter too),
  truth     -- the closest approach over the span on a trajectory sampled 32x finer than the plan's
               step (one WH level at dt / 32), as a multiple of the exit distance,
  main      -- the same on the main pass's finest level (mult 7), ext on the extension level (8),
  p1, p2    -- on the finest level of halving passes 1 and 2 (mult 14, 28).
Every ratio is the smallest pair distance the level's kicks saw / the exit distance (< 1: that level
calls the encounter).  usage: encounter_rule_study.py {hd155358|3planet|s2} [n_iterations] -> JSON."""
import ctypes as C
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
from rvmcmc import engine  # noqa: E402
from rvmcmc.state import State  # noqa: E402


def system(name):
    from test_gpu_ias15_decisions import THIRD, _hd

    if name == "hd155358":
        planets, obs = _hd()
        X = np.load(os.path.join(ROOT, "scripts", "probe", "ens_hd155358_it1000.npy"))
    elif name == "3planet":
        np.random.seed(2017)
        planets = [dict(p) for p in S2_PLANETS] + [dict(THIRD)]
        obs = O.fake_obs(planets, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
        X = np.load(os.path.join(ROOT, "scripts", "probe", "ens_3planet_it1000.npy"))
    else:
        planets, obs = S2_PLANETS, s2_obs_oracle()
        X = np.load(os.path.join(ROOT, "scripts", "probe", "ens_it2000.npy"))
    return planets, obs, X


def level_ratio(P1, npl, obs, dt, sub):
    """smallest pair distance / exit distance on one WH level (sub steps per base step dt)."""
    L = O.lib()
    L.rvo_debug_min_ratio.restype = C.c_double
    L.rvo_debug_min_ratio.argtypes = [C.c_int]
    L.rvo_debug_min_ratio(1)
    O.logl_whx_seq_batch(P1, npl, obs, dt, [sub])
    return float(np.sqrt(L.rvo_debug_min_ratio(1)))


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
    mult = list(mult)
    fin = max(mult)
    rng = np.random.default_rng(11)
    n = len(X) // 2
    Q = []
    for _ in range(iters):
        for h in (0, 1):
            x, c = (X[:n], X[n:]) if h == 0 else (X[n:], X[:n])
            q, _ = IP.stretch_proposal(x, c, rng.random(n), rng.random(n))
            Q.append(q)
    Q = np.concatenate(Q)
    P = IP.to_oracle(pm, Q)
    nt = IP.n_threads()
    chunks = [ix for ix in np.array_split(np.arange(len(P)), nt) if len(ix)]
    with ThreadPoolExecutor(nt) as ex:
        parts = list(ex.map(lambda ix: O.logl_whx_adapt_batch(P[ix], npl, obs, dt, mult, tol, rmax,
                                                               ecc_guard=guard)[1], chunks))
    st_dev = np.concatenate(parts)
    _, st_ref = IP.ias15_logl(P, npl, obs)
    enc = np.nonzero(st_dev == IP.ST_ENC)[0]

    def one(i):
        P1 = P[i:i + 1]
        return dict(i=int(i), ias15=int(st_ref[i]), truth=level_ratio(P1, npl, obs, dt / 32, 1),
                    main=level_ratio(P1, npl, obs, dt, fin), ext=level_ratio(P1, npl, obs, dt, fin + 1),
                    p1=level_ratio(P1, npl, obs, dt, 2 * fin), p2=level_ratio(P1, npl, obs, dt, 4 * fin),
                    lv0=[level_ratio(P1, npl, obs, dt, m) for m in mult],
                    lv1=[level_ratio(P1, npl, obs, dt, 2 * m) for m in mult],
                    lv2=[level_ratio(P1, npl, obs, dt, 4 * m) for m in mult],
                    lv3=[level_ratio(P1, npl, obs, dt, 8 * m) for m in mult])

    # (one thread: rvo_debug_min_ratio is thread-local, but keep the oracle calls simple)
    rows = [one(i) for i in enc]
    # the unanimity rule (round 6): a pass ends the walker ENCOUNTER only when every level of it saw
    # the exit distance; a pass whose levels disagree sends the walker to the next pass
    for r in rows:
        r["unanimous_stage"] = None
        r["unanimous_enc"] = None
        for p, key in enumerate(("lv0", "lv1", "lv2", "lv3")):
            f = [v < 1.0 for v in r[key]]
            if all(f) or not any(f):
                r["unanimous_stage"], r["unanimous_enc"] = p, all(f)
                break
    rule = dict(enc_2_0_after=sum(1 for r in rows if r["ias15"] == 0 and r["unanimous_enc"]),
                enc_2_0_after_outside=sum(1 for r in rows if r["ias15"] == 0 and r["unanimous_enc"] and r["truth"] >= 1),
                enc_0_2_new=sum(1 for r in rows if r["ias15"] == 2 and r["unanimous_enc"] is False),
                undecided_after_pass3=sum(1 for r in rows if r["unanimous_enc"] is None),
                stage_counts={str(p): sum(1 for r in rows if r["unanimous_stage"] == p) for p in range(4)})
    out = dict(system=name, proposals=int(len(P)), device_encounters=int(len(enc)),
               ias15_encounters=int((st_ref == IP.ST_ENC).sum()),
               enc_2_0=int(((st_dev == IP.ST_ENC) & (st_ref == IP.ST_OK)).sum()),
               enc_0_2=int(((st_dev == IP.ST_OK) & (st_ref == IP.ST_ENC)).sum()), unanimity_rule=rule, rows=rows)
    print(json.dumps(out))


if __name__ == "__main__":
    main()

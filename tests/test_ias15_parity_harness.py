"""CPU check of the reference-physics decision harness (tests/ias15_parity.py) with the oracle's
restatement of the kernel algorithm (rvo_whx) standing in for the device: the IAS15-driven emcee
restatement and the WH-driven one must make the same decisions on a small S2 ensemble, and the
tally must count exemptions and mismatches as documented."""
import numpy as np

import ias15_parity as IP
import oracle as O
from conftest import S2_PLANETS, S2_SCALES, s2_obs_oracle
from philox_ref import stretch_uniforms


def test_stretch_harness_whx_vs_ias15():
    from rvmcmc.state import State

    s = State(planets=[dict(p) for p in S2_PLANETS])
    pm = s.param_map()
    obs = s2_obs_oracle()
    dt, mult, _ = s.integrator.plan_args(s.planets)
    W, dim, n = 64, s.Nvars, 32
    scales = np.array([S2_SCALES[k] for k in s.get_rawkeys()])
    X = s.get_params()[None] + 1e-3 * scales * np.random.default_rng(0).standard_normal((W, dim))
    pos = [X[:n].copy(), X[n:].copy()]
    lw = [O.logl_whx_batch(IP.to_oracle(pm, p), 2, obs, dt, mult)[0] for p in pos]
    li = [IP.ias15_logl(IP.to_oracle(pm, p), 2, obs)[0] for p in pos]
    tally = IP.Tally("harness")
    for it in range(2):
        for h in (0, 1):
            u1, u2, u3 = stretch_uniforms(7, h * n, n, it, h)
            q, z = IP.stretch_proposal(pos[h], pos[1 - h], u1, u2)
            lqw, sqw = O.logl_whx_batch(IP.to_oracle(pm, q), 2, obs, dt, mult)
            lqi, sqi = IP.ias15_logl(IP.to_oracle(pm, q), 2, obs)
            dw = (dim - 1.0) * np.log(z) + lqw - lw[h]
            di = (dim - 1.0) * np.log(z) + lqi - li[h]
            acc_w, acc_i = dw > np.log(u3), di > np.log(u3)
            tally.add(acc_w, acc_i, np.abs(di - np.log(u3)), sqw, sqi, lqw, lqi)
            pos[h] = np.where(acc_w[:, None], q, pos[h])
            lw[h] = np.where(acc_w, lqw, lw[h])
            li[h] = np.where(acc_w, lqi, li[h])
    rep = tally.report()
    assert rep["decisions"] == 2 * W and rep["mismatches_not_exempt"] == 0
    assert rep["max_abs_dlogl_ok_proposals"] < 5e-8
    assert 0 < rep["accepted_ias15"] < rep["decisions"]


def test_tally_counts_exemptions():
    t = IP.Tally("counts")
    acc_dev = np.array([1, 0, 1, 0, 1], bool)
    acc_ref = np.array([1, 1, 0, 0, 0], bool)
    margin = np.array([1.0, 1e-7, 1.0, 1.0, 1.0])    # walker 1 near the margin
    st_dev = np.array([0, 0, 2, 0, 0])                # walker 2: encounter on one side only
    st_ref = np.array([0, 0, 0, 0, 0])
    t.add(acc_dev, acc_ref, margin, st_dev, st_ref)
    r = t.report()
    assert r["exempt_near_margin"] == 1 and r["exempt_status_disagreement"] == 1
    assert r["differing_but_exempt"] == 2 and r["mismatches_not_exempt"] == 1 and t.mismatch == [4]
    t2 = IP.Tally("explained")
    t2.add(acc_dev[4:], acc_ref[4:], margin[4:], st_dev[4:], st_ref[4:], explained=np.array([True]))
    assert t2.report()["mismatches_not_exempt"] == 0 and t2.disagree_explained == 1

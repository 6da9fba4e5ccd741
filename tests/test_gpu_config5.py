"""BASELINE config 5 on one GPU: the 8192-walker shard of the 65536-walker 3-planet ensemble.

The 8-GPU run is the driver's (RCCL complementary-half all-gather, rvmcmc/ensemble.py); the
sharded index layout is covered by tests/test_dist_gloo.py::test_config5_layout_world8.  Here one
rank's shard runs on the production path for several iterations, then
  * a 128-walker subset of its positions is checked against the oracle restatement of the kernel
    algorithm (T1, tests/test_gpu_logl.py) and against IAS15, the reference physics (T2,
    |dlogL| <= 1e-6 on sampler-visited states as tests/test_gpu_ias15_decisions.py);
  * the sampler's stored lnprob (from its fused / speculative launches) equals one plain launch
    over all 8192 positions and single-walker launches, bit for bit.
"""
import json

import numpy as np
import pytest

import ias15_parity as IP
import oracle as O
from conftest import S2_PLANETS, S2_SCALES
from test_gpu_resolve import assert_t1_adaptive

pytestmark = pytest.mark.gpu

THIRD = {"m": 1e-3, "a": 2.6, "h": 0.05, "k": 0.0, "l": 1.0}  # scripts/configs_bench.py config 5
T2_ABS = 1e-6


def test_config5_shard_8192_walkers():
    import torch

    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.state import State

    planets = [dict(p) for p in S2_PLANETS] + [dict(THIRD)]
    np.random.seed(2017)
    obs = O.fake_obs(planets, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    s = State(planets=[dict(p) for p in planets])
    pm = s.param_map()
    W = 8192
    rng = np.random.default_rng(7)
    scales = np.array([S2_SCALES[k] for k in s.get_rawkeys()])
    X0 = s.get_params()[None] + 1e-3 * scales * rng.standard_normal((W, s.Nvars))
    ens = EnsembleSampler(W, s, obs, seed=2024)
    ens.set_positions(X0)
    for _ in range(4):
        ens.step()
    torch.cuda.synchronize()
    X = ens.gather_positions()
    lnp = ens.gather_lnprob()
    acc = ens.naccepted.cpu().numpy()
    assert np.isfinite(lnp).all()
    assert 0.05 < acc.mean() / 4 < 0.95

    # one plain launch over the whole shard reproduces the sampler's stored values bit for bit
    K = pm.to_kernel(torch.as_tensor(np.ascontiguousarray(X.T), device="cuda"))
    lp_all, st_all, _ = ens.plan.logl(K, hill_factor=ens.hill_factor)
    lp_all = lp_all.cpu().numpy()
    np.testing.assert_array_equal(lp_all, lnp)
    for i in (0, 15, 16, 4095, 4096, W - 1):
        one, _, _ = ens.plan.logl(K[:, i:i + 1].contiguous(), hill_factor=ens.hill_factor)
        assert one.item() == lnp[i], i

    idx = np.r_[0:32, 2048:2080, 4096:4128, W - 32:W]
    P = IP.to_oracle(pm, X[idx])
    plan = ens.plan  # (the default IntegratorConfig: adaptive resolution on)
    assert plan.resolve_tol > 0 and plan.ext_mult == O.ext_multiplier(plan.mult, plan.resolve_max)
    rf, _ = assert_t1_adaptive(lnp[idx], st_all.cpu().numpy()[idx], P, 3, obs, plan.dt, plan.mult, plan.resolve_tol,
                               plan.resolve_max, ecc_guard=plan.ecc_guard)
    ias, st_ias = IP.ias15_logl(P, 3, obs, ens.hill_factor)
    assert (st_ias == 0).all()
    d2 = np.abs(lnp[idx] - ias)
    print(json.dumps({"test": "config5 shard", "walkers": W, "iterations": 4, "acceptance": float(acc.mean() / 4),
                      "speculative": bool(ens.speculating()), "t2_max_abs_dlogl": float(d2.max()),
                      "t2_subset": int(len(idx)),
                      "subset_directions_extended": int((rf == 1).sum()), "subset_directions_halved": int((rf >= 2).sum())}))
    assert d2.max() <= T2_ABS

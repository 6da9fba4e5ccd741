"""Fused MH and SMALA steps against their multi-launch paths.

* rvm_mh_step: proposal (Philox), walker logL and MH accept in ONE likelihood launch, against
  rvm_mh_propose + rvm_logl_batch + rvm_mh_accept with the same draws (mcmc.py:107-121).
* rvm_smala_stencil_logl + rvm_smala_derive_accept (rvm_smala_metric_accept for the exact
  Hessian): the proposal's central-difference stencil formed inside the likelihood launch, and the
  metric + accept in one kernel, against rvm_fd_params + rvm_logl_batch + rvm_smala_derive +
  rvm_smala_accept (mcmc.py:167-187).
Chains, logp, accept counters and (SMALA) every cache entry must be bit-identical.
"""
import numpy as np
import pytest

from conftest import S2_PLANETS, S2_SCALES, s2_obs_oracle

pytestmark = pytest.mark.gpu

MH_SCALES = {"m": 1.e-3, "a": 0.3, "h": 0.5, "k": 0.5, "l": np.pi / 2.}  # mcmc_benchmark_mh.py:52


def _state(case):
    from rvmcmc import state

    planets = [dict(p) for p in S2_PLANETS]
    kw = {}
    if case == "fixed_params":
        kw = dict(ignore_params=[["h"], ["k", "l"]])
    elif case == "three_planets":
        planets.append({"m": 1e-3, "a": 2.6, "h": 0.05, "k": 0.0, "l": 1.0})
    elif case == "inclined":
        planets[0]["ix"], planets[0]["iy"] = 0.05, -0.03
        planets[1]["ix"], planets[1]["iy"] = -0.02, 0.04
    return state.State(planets=planets, **kw)


# level_split: 6144 chains -> 384 (walker group, direction) units, the level-split launch layout
@pytest.mark.parametrize("case,n,step,iters", [("s2", 256, 1e-3, 4), ("fixed_params", 256, 1e-3, 4),
                                               ("wide", 256, 3e-2, 4), ("three_planets", 128, 1e-3, 3),
                                               ("inclined", 128, 1e-3, 3), ("level_split", 6144, 1e-3, 2)])
def test_fused_mh_step_matches_three_launch_path(case, n, step, iters):
    import torch

    from rvmcmc.mcmc import MhChains

    s = _state(case)
    obs = s2_obs_oracle()
    runs = []
    for fused in (True, False):
        mh = MhChains(s, obs, MH_SCALES, step, n, seed=11)
        for _ in range(iters):
            mh.step(fused=fused)
        torch.cuda.synchronize()
        runs.append((mh.X.cpu().numpy(), mh.lnp.cpu().numpy(), mh.accepted.cpu().numpy()))
    for a, b in zip(runs[0], runs[1]):
        np.testing.assert_array_equal(a, b)
    acc = runs[0][2].sum() / (n * iters)
    print(f"[mh fused {case}] chains {n} iterations {iters} acceptance {acc:.3f} "
          f"non-finite lnp {int((~np.isfinite(runs[0][1])).sum())}")
    assert 0.0 < acc < 1.0
    if case == "wide":
        assert acc < 0.5


@pytest.mark.parametrize("case,hessian", [("s2", "gauss-newton"), ("fixed_params", "gauss-newton"),
                                          ("three_planets", "gauss-newton"), ("s2", "exact"),
                                          ("many", "gauss-newton")])
def test_fused_smala_step_matches_separate_launches(case, hessian):
    import torch

    from rvmcmc.smala import SmalaChains

    s = _state("s2" if case == "many" else case)
    obs = s2_obs_oracle()
    C_ = 256 if case == "many" else 16  # 256 chains: config 4's stencil launch (5376 walkers)
    rng = np.random.default_rng(2)
    scales = np.array([S2_SCALES.get(k, 1e-2) for k in s.get_rawkeys()])
    X0 = (s.get_params()[None] + 1e-3 * scales * rng.standard_normal((C_, s.Nvars))).T.copy()
    runs = []
    for fused in (True, False):
        sm = SmalaChains(s, obs, eps=0.5, alpha=1e3, n_chains=C_, X0=X0, seed=9, hessian=hessian)
        for _ in range(3):
            sm.step(fused=fused)
        torch.cuda.synchronize()
        cache = {k: v.cpu().numpy() for k, v in sm.cache.items() if k != "_c"}
        runs.append((sm.X.cpu().numpy(), sm.accepted.cpu().numpy(), sm.failures.cpu().numpy(), cache))
    for a, b in zip(runs[0][:3], runs[1][:3]):
        np.testing.assert_array_equal(a, b)
    for k in runs[0][3]:
        np.testing.assert_array_equal(runs[0][3][k], runs[1][3][k], err_msg=k)
    print(f"[smala fused {case} {hessian}] chains {C_} accepted {int(runs[0][1].sum())} of {3 * C_}")
    assert runs[0][1].sum() > 0

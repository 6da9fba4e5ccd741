"""Throughput of every BASELINE.json config on one GPU (bench.py keeps the headline config).

  config 2: affine stretch, 1024 walkers, 2-planet synthetic (101 epochs)
  config 2w: the headline workload (4096 walkers) from a wide initial ball
  config 3: affine stretch, 4096 walkers, HD155358.vels (122 epochs)
  config 4: SMALA, 256 chains, 10-dim 2-planet, FD gradient/metric (21 logL per chain-step)
  config 5: affine stretch, 3-planet synthetic, 8192 walkers per GPU (= 65536 over 8 GPUs);
            the third planet is named here (not in the reference): {m 1e-3, a 2.6, h 0.05, k 0, l 1}
  config 1: the reference-API single-chain Mh (mcmc_benchmark_mh.py), steps/s
  config 1b: batched MH chains (MhChains, fused rvm_mh_step), 4096 chains; 1bu / 4u: the same
            with the separate propose / logL / accept launches (before the fusion)

The affine configs (2, 2w, 3, 5) and SMALA (4) are timed at their chain's steady state, after a
burn-in of BURN_IN iterations (RVM_CONFIGS_BURN_IN, default 3000; SMALA a third of it), as the
headline bench.py is; the window from the tight ball of rounds 1-5 stays as `ball_window`
(`first_steps` for SMALA).

Prints one JSON line per config.  Usage: python scripts/configs_bench.py [config ...]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd")]
import torch  # noqa: E402

from rvmcmc import mcmc  # noqa: E402
from rvmcmc.ensemble import EnsembleSampler  # noqa: E402
from rvmcmc.observations import FakeObservation, Observation_FromFile  # noqa: E402
from rvmcmc.smala import SmalaChains  # noqa: E402
from rvmcmc.state import State  # noqa: E402

S2 = [{"m": 1.2e-3, "a": 0.88, "h": 0.218, "k": 0.015, "l": 0.3},
      {"m": 2.1e-3, "a": 1.55, "h": 0.16, "k": 0.02, "l": 2.2}]
THIRD = {"m": 1e-3, "a": 2.6, "h": 0.05, "k": 0.0, "l": 1.0}
SCALES = {"m": 1.5e-3, "a": 0.3, "h": 0.1, "k": 0.1, "l": np.pi / 2.}
# iterations before the steady-state window (bench.py burns in 4000; RVM_CONFIGS_BURN_IN overrides)
BURN_IN = int(os.environ.get("RVM_CONFIGS_BURN_IN", "3000"))
# (studies) base steps per shortest period for every config's plan (IntegratorConfig.steps_per_orbit)
if os.environ.get("RVM_CONFIGS_SPO"):
    import dataclasses

    from rvmcmc import engine

    engine.DEFAULT_CONFIG = dataclasses.replace(engine.DEFAULT_CONFIG,
                                                steps_per_orbit=float(os.environ["RVM_CONFIGS_SPO"]))


def _window(ens, steps, warmup):
    for _ in range(warmup):
        ens.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        ens.step()
    torch.cuda.synchronize()
    return time.perf_counter() - t0


def _affine(state, obs, W, steps=20, warmup=3, ball=1e-3, burn_in=BURN_IN, steady_steps=100):
    """The ball window (iterations warmup .. warmup + steps from the tight ball: rounds 1-5's figure,
    now a side figure) and, after a burn-in, the chain's steady state (the
    headline bench times its steady state too, bench.py); the top-level rate is the steady state's."""
    sc = np.array([SCALES[k] for k in state.get_rawkeys()])
    X0 = state.get_params()[None] + ball * sc * np.random.normal(size=(W, state.Nvars))
    ens = EnsembleSampler(W, state, obs, seed=1)
    ens.set_positions(X0)
    ens.compute_lnprob()
    dt = _window(ens, steps, warmup)
    ball_win = {"walker_logl_evals_per_s": W * steps / dt, "ms_per_iteration": 1e3 * dt / steps,
                "iterations": [warmup, warmup + steps]}
    out = {"ball_window": ball_win}
    if burn_in > 0:
        done = warmup + steps
        for _ in range(max(0, burn_in - done)):
            ens.step()
        torch.cuda.synchronize()
        ens.check_faults()
        ens.plan.faults(reset=True)
        t0 = dict(ens.plan.totals)  # (running totals: the sampler's periodic checks reset the counters)
        dt = _window(ens, steady_steps, 3)
        ens.plan.faults(reset=True)
        f = {k: ens.plan.totals[k] - t0[k] for k in t0}
        first = max(burn_in, done) + 3
        out.update({"walker_logl_evals_per_s": W * steady_steps / dt, "ms_per_iteration": 1e3 * dt / steady_steps,
                    "timed_window": [first, first + steady_steps], "window": "steady state (after the burn-in)",
                    "refined_per_iteration": f["refined"] / (steady_steps + 3),
                    "faults_in_window": {k: v for k, v in f.items() if v and k not in ("refined", "truncated", "skipped")}})
    else:
        out.update(ball_win)
        out["window"] = "ball"
    out.update({"acceptance": float(ens.acceptance_fraction().mean().item()), "plan_steps": ens.plan.info()})
    return out


def config2():
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in S2])
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    return {"config": "2: affine, 1024 walkers, 2-planet synthetic", **_affine(s, obs, 1024)}


def config2w():
    """the same workload from a wide ball (x100 the tight one) to expose prior /
    encounter exits and the kernel's general-solver paths (eccentric, close orbits)."""
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in S2])
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    out = _affine(s, obs, 4096, ball=1e-1)
    return {"config": "2w: affine, 4096 walkers, 2-planet synthetic, wide ball (0.1 x scales)", **out}


def config3():
    np.random.seed(2017)
    sol = [6.57730330e-01, -9.72263877e-02, -7.82798396e-02, 8.84031737e-04, 4.42804990e+00,
           1.04404207e+00, -2.05622789e-02, -1.08797961e-01, 8.30379710e-04, 1.49919861e+00]
    s = State(planets=[{"m": sol[3], "a": sol[0], "h": sol[1], "k": sol[2], "l": sol[4]},
                       {"m": sol[8], "a": sol[5], "h": sol[6], "k": sol[7], "l": sol[9]}])
    obs = Observation_FromFile(os.path.join(ROOT, "tests", "golden", "HD155358.vels"), Npoints=100)
    return {"config": "3: affine, 4096 walkers, HD155358.vels", **_affine(s, obs, 4096)}


def config4(chains=256, steps=100, fused=True, burn_in=None, steady_steps=400):
    """SMALA config 4; timed after a burn-in of the chains (the steady state; the first `steps` steps
    from the start are reported as a side figure).  The steady window is 400 steps: its mean is set by
    rare steps whose centres climb to halving passes 4-5 (median ~0.65 ms, a few steps of 3-7 ms,
    scripts/probe/smala_tail_probe.py), so a short window's mean varies by tens of per cent."""
    burn_in = max(0, BURN_IN // 3) if burn_in is None else burn_in
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in S2])
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    sm = SmalaChains(s, obs, eps=0.5, alpha=1e3, n_chains=chains, seed=0)
    sm.step(fused=fused)
    torch.cuda.synchronize()

    def window(n):
        # (an event on the launch stream after each step: the steps' own durations, for their spread --
        # a step whose centres need a second halving pass takes about twice as long)
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
        # (the burn-in's steps are enqueued without a wait: the clock starts once they have run --
        # rounds 6's first steady-state figures timed their tail too, 2.6 / 1.2 ms per step against
        # the steps' own 0.8, scripts/probe/smala_host_probe.py)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        evs[0].record()
        for i in range(n):
            sm.step(fused=fused)
            evs[i + 1].record()
        torch.cuda.synchronize()
        return time.perf_counter() - t0, np.array([evs[i].elapsed_time(evs[i + 1]) for i in range(n)])

    dt0, _ = window(steps)
    first = {"chain_steps_per_s": chains * steps / dt0, "ms_per_step": 1e3 * dt0 / steps, "steps": [1, 1 + steps]}
    for _ in range(max(0, burn_in - steps - 1)):
        sm.step(fused=fused)
    dt, per = window(steady_steps)
    start = max(burn_in, steps + 1)
    P = s.Nvars
    how = ("fused: propose + stencil logL launch + derive/accept kernel" if fused else
           "separate propose / fd / logL / derive / accept launches")
    return {"config": f"4: SMALA, 256 chains, 10-dim, FD (2P+1 = 21 logL per chain-step), {how}",
            "chain_steps_per_s": chains * steady_steps / dt,
            "walker_logl_evals_per_s": chains * steady_steps * (2 * P + 1) / dt,
            "ms_per_step": 1e3 * dt / steady_steps, "acceptance": float(sm.accepted.double().mean().item() / sm.iteration),
            "window": "steady state (after the burn-in)", "timed_window": [start, start + steady_steps],
            "first_steps": first,
            "step_ms_quantiles": [float(v) for v in np.quantile(per, [0, 0.25, 0.5, 0.75, 0.9, 1.0])],
            "step_ms_quantile_levels": [0, 0.25, 0.5, 0.75, 0.9, 1.0]}


def config4x(chains=256, steps=5):
    """config 4 with the reference's metric: exact gradient + Hessian (rvm_logl_derivs, one
    hyper-dual integration per chain and parameter pair: P(P+1)/2 = 55 per chain-step)."""
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in S2])
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    sm = SmalaChains(s, obs, eps=0.5, alpha=1e3, n_chains=chains, seed=0, hessian="exact")
    sm.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        sm.step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"config": "4x: SMALA, 256 chains, 10-dim, exact gradient + Hessian (hyper-dual, 55 pair integrations)",
            "chain_steps_per_s": chains * steps / dt, "ms_per_step": 1e3 * dt / steps,
            "acceptance": float(sm.accepted.double().mean().item() / sm.iteration)}


def config4u():
    return config4(fused=False)


def config1b(chains=4096, steps=200, fused=True):
    """Batched MH (MhChains: mcmc.py:107-121 for every chain at once), 4096 chains on the
    2-planet synthetic config, mcmc_benchmark_mh.py:52 scales, step 1e-3."""
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in S2])
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    mh = mcmc.MhChains(s, obs, {"m": 1.e-3, "a": 0.3, "h": 0.5, "k": 0.5, "l": np.pi / 2.}, 1e-3, chains, seed=0)
    for _ in range(3):
        mh.step(fused=fused)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        mh.step(fused=fused)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    how = "fused (rvm_mh_step, one launch)" if fused else "propose / logL / accept launches"
    return {"config": f"1b: batched MH, {chains} chains, 2-planet synthetic, {how}",
            "chain_steps_per_s": chains * steps / dt, "ms_per_step": 1e3 * dt / steps,
            "acceptance": float(mh.accepted.double().mean().item() / mh.iteration)}


def config1bu():
    return config1b(fused=False)


def config5(W=8192):
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in S2] + [dict(THIRD)])
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    return {"config": "5: affine, 3-planet synthetic, 8192 walkers per GPU (65536 / 8)", **_affine(s, obs, W)}


def config1(steps=200, speculate=1):
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in S2])
    obs = FakeObservation(s, Npoints=200, error=1.5e-4, errorVar=2.5e-5, tmax=120.)   # mcmc_benchmark_mh.py:34
    mh = mcmc.Mh(s, obs, speculate=speculate)
    mh.set_scales({"m": 1.e-3, "a": 0.3, "h": 0.5, "k": 0.5, "l": np.pi / 2.})       # :52
    mh.step_size = 10.0e-3                                                            # :53
    tries = 0
    t0 = time.perf_counter()
    for _ in range(steps):
        tries += mh.step_force()
    dt = time.perf_counter() - t0
    return {"config": "1: reference-API Mh, single chain (mcmc_benchmark_mh.py)" +
            (f", speculative x{speculate} (bit-identical chain)" if speculate > 1 else ""),
            "accepted_steps_per_s": steps / dt, "logl_evals_per_s": tries / dt, "acceptance": steps / tries}


def config1s():
    return config1(speculate=int(os.environ.get("RVM_SPECULATE", "3")))


def main():
    which = sys.argv[1:] or ["2", "2w", "3", "4", "4u", "4x", "5", "1", "1s", "1b", "1bu"]
    table = {"1": config1, "2": config2, "2w": config2w, "3": config3, "4": config4, "4u": config4u, "4x": config4x,
             "5": config5, "1s": config1s, "1b": config1b, "1bu": config1bu}
    for c in which:
        out = table[c]()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()

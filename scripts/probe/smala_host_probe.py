"""Probe (GPU): is config 4 (SMALA FD, 256 chains) at its steady state bound by the GPU or by the host?
After a burn-in, times a window of steps by the wall clock and by HIP events between the steps (their
sum is the GPU's stream time), and profiles the host side of the same window (cProfile, top entries
by cumulative time).  usage: smala_host_probe.py [burn_in] [steps] -> JSON lines."""
import cProfile
import io
import json
import os
import pstats
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "scripts")]
import torch  # noqa: E402

import configs_bench as CB  # noqa: E402
from rvmcmc.observations import FakeObservation  # noqa: E402
from rvmcmc.smala import SmalaChains  # noqa: E402
from rvmcmc.state import State  # noqa: E402


def window(sm, n, prof=None):
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(n + 1)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs[0].record()
    if prof:
        prof.enable()
    for i in range(n):
        sm.step()
        evs[i + 1].record()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    if prof:
        prof.disable()
    wall = time.perf_counter() - t0
    per = np.array([evs[i].elapsed_time(evs[i + 1]) for i in range(n)])
    return wall, t_enq, per


def main():
    burn = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in CB.S2])
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    sm = SmalaChains(s, obs, eps=0.5, alpha=1e3, n_chains=256, seed=0)
    sm.step()
    wall, enq, per = window(sm, 100)
    print(json.dumps({"window": "first", "wall_ms_per_step": 1e3 * wall / 100, "enqueue_ms_per_step": 1e3 * enq / 100,
                      "gpu_ms_per_step": float(per.mean())}), flush=True)
    for _ in range(burn - 101):
        sm.step()
    pr = cProfile.Profile()
    wall, enq, per = window(sm, steps, pr)
    print(json.dumps({"window": "steady", "wall_ms_per_step": 1e3 * wall / steps, "enqueue_ms_per_step": 1e3 * enq / steps,
                      "gpu_ms_per_step": float(per.mean()), "gpu_ms_quantiles": np.quantile(per, [0, .5, .9, 1]).round(3).tolist()}),
          flush=True)
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats("cumulative").print_stats(18)
    print(buf.getvalue())


if __name__ == "__main__":
    main()

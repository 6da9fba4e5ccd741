"""Probe (GPU): config 4's heavy tail at its steady state (scripts/configs_bench.py config 4: median
step ~0.65 ms, mean 1.8-3 ms).  Burns the 256 SMALA chains in, then times STEPS steps one by one (HIP
events) with the centres' adaptive plan's counters per step (refinement passes, certain rejects,
floor settles, UNRESOLVED), and saves the proposals (the centres) of the slowest steps for an oracle
replay (scripts/probe/smala_tail_replay.py).  usage: smala_tail_probe.py [burn_in] [steps] -> JSON lines,
gpurun_out/smala_tail_slow.npz."""
import json
import os
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


def main():
    burn = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in CB.S2])
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    sm = SmalaChains(s, obs, eps=0.5, alpha=1e3, n_chains=256, seed=0)
    t0 = time.perf_counter()
    for i in range(burn):
        sm.step()
        if i % 200 == 0:
            torch.cuda.synchronize()
            print(json.dumps({"burn": i, "s": round(time.perf_counter() - t0, 1)}), flush=True)
    plan = sm._center_plan()
    with torch.cuda.stream(sm._side):
        plan.faults(reset=True)
    rows, keep = [], []
    for i in range(steps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        sm.step()
        e1.record()
        torch.cuda.synchronize()
        with torch.cuda.stream(sm._side):
            f = plan.faults(reset=True)
        ms = e0.elapsed_time(e1)
        rows.append({"step": burn + i, "ms": ms, **f})
        keep.append((ms, sm.Xs.cpu().numpy().copy()))
    ms = np.array([r["ms"] for r in rows])
    print(json.dumps({"steps": steps, "ms_mean": float(ms.mean()), "ms_quantiles": np.quantile(ms, [0, .25, .5, .75, .9, .99, 1]).round(3).tolist()}))
    for r in sorted(rows, key=lambda r: -r["ms"])[:20]:
        print(json.dumps(r))
    slow = sorted(keep, key=lambda k: -k[0])[:8]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez(os.path.join(ROOT, "gpurun_out", "smala_tail_slow.npz"), ms=np.array([k[0] for k in slow]),
             Xs=np.stack([k[1] for k in slow]), keys=np.array(s.get_rawkeys()))


if __name__ == "__main__":
    main()

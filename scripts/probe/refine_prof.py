"""Where the refinement kernel's time goes at the bench chain's steady state (the RVM_PROFILE build,
scripts/probe/librvmcmc_prof.so from `make -C rvel-mcmc_amd profile`): the steady-state sampler of
scripts/probe/steady_bench.py, and for each iteration the refinement launch's span on the device
clock and its slowest wave -- prologue (walker state re-derived, schedule staged), the pass loop
(cycles in segments per step, in epoch handling, in the eager / team / split hand-offs), the tail
after it -- with the shader clock it ran at (rvm_refine.hip RVM_PROFILE record)."""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from conftest import S2_PLANETS  # noqa: E402
from rvmcmc import _lib, engine  # noqa: E402

SLOTS, MAXW = 20, 4096


def main():
    _lib.LIB_PATH = os.environ.get("RVM_LIB_PATH") or os.path.join(ROOT, "scripts", "probe", "librvmcmc_prof.so")
    lib = _lib.load()
    lib.rvm_rprof_copy.argtypes = [C.c_void_p, C.c_size_t]
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.observations import FakeObservation
    from rvmcmc.state import State

    state = State(planets=[dict(p) for p in S2_PLANETS])
    state.integrator = engine.IntegratorConfig(resolve_tol=5e-7)
    np.random.seed(2017)
    obs = FakeObservation(state, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    X = np.load(os.path.join(ROOT, "scripts/probe/ens_it2000.npy"))
    ens = EnsembleSampler(len(X), state, obs, seed=2017)
    ens.set_positions(X)
    ens.compute_lnprob()
    for _ in range(3):
        ens.step()
    torch.cuda.synchronize()
    buf = np.zeros(MAXW * SLOTS, dtype=np.uint64)
    rows = []
    for it in range(int(os.environ.get("ITERS", "40"))):
        lib.rvm_rprof_clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ens.step()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        assert lib.rvm_rprof_copy(buf.ctypes.data, buf.nbytes) == 0
        b = buf.reshape(MAXW, SLOTS).astype(np.int64)
        b = b[b[:, 3] != 0]
        if not len(b):
            continue
        t_launch0 = b[:, 0].min()
        span = (b[:, 3].max() - t_launch0) / 100.0  # us
        busy = b[b[:, 6] > 0]
        i = int(np.argmax(b[:, 3]))
        w = b[i]
        us = lambda x: float(x) / 100.0  # noqa: E731
        clk = float(w[7] + w[8]) / max(1.0, (w[2] - w[0]) * 10.0)  # cycles per ns = GHz
        out = {"it": it, "wall_ms": 1e3 * wall, "span_us": span, "waves": int(len(b)), "busy_waves": int(len(busy)),
               "tasks": int(len(set((b[:, 9] & 0xFFFF).tolist()))),
               "slowest": {"entry_us": us(w[0] - t_launch0), "prologue_us": us(w[1] - w[0]),
                           "loop_us": us(w[2] - w[1]), "tail_us": us(w[3] - w[2]),
                           "seg_kcyc": w[4] / 1e3, "epoch_kcyc": w[5] / 1e3, "wait_kcyc": w[12] / 1e3,
                           "steps": int(w[6]), "cyc_per_step": float(w[4]) / max(1, w[6]), "ghz": clk,
                           "team": int((w[9] >> 16) & 0xF), "own": int((w[9] >> 20) & 0xF) - 1,
                           "level": int((w[9] >> 24) & 0xF) - 1, "passes": int(w[10])}}
        if len(busy):
            cps = busy[:, 4] / np.maximum(1, busy[:, 6])
            out["busy_cyc_per_step_median"] = float(np.median(cps))
            out["busy_cyc_per_step_max"] = float(cps.max())
            out["busy_steps_max"] = int(busy[:, 6].max())
            out["busy_prologue_us_median"] = float(np.median(busy[:, 1] - busy[:, 0]) / 100.0)
            # cycles from entry: list sizes read, schedule staged, slot index + draws, rows loaded,
            # walker state set up, pass loop
            out["busy_prologue_kcyc_median"] = [float(np.median(busy[:, c]) / 1e3) for c in (13, 14, 16, 17, 15, 7)]
            crit = busy[int(np.argmax(busy[:, 6]))]
            out["critical"] = {"steps": int(crit[6]), "cyc_per_step": float(crit[4]) / max(1, crit[6]),
                               "seg_kcyc": crit[4] / 1e3, "epoch_kcyc": crit[5] / 1e3, "wait_kcyc": crit[12] / 1e3,
                               "prologue_us": float(crit[1] - crit[0]) / 100.0, "loop_us": float(crit[2] - crit[1]) / 100.0,
                               "level": int((crit[9] >> 24) & 0xF) - 1, "team": int((crit[9] >> 16) & 0xF)}
        # per team (0 = A: pass 1, 1 = B: pass 2 concurrently, then the rest): when its last wave
        # ended, and its longest-integrating wave's breakdown
        for tm in (0, 1):
            bt = b[((b[:, 9] >> 16) & 0xF) == tm]
            if not len(bt):
                continue
            wt = bt[int(np.argmax(bt[:, 6]))]
            out[f"team{tm}"] = {"end_us": us(bt[:, 3].max() - t_launch0), "loop_end_us": us(bt[:, 2].max() - t_launch0),
                                "steps": int(wt[6]), "seg_kcyc": wt[4] / 1e3, "epoch_kcyc": wt[5] / 1e3,
                                "wait_kcyc": wt[12] / 1e3, "loop_us": us(wt[2] - wt[1]),
                                "loop_start_us": us(wt[1] - t_launch0), "passes": int(wt[10])}
        rows.append(out)
        print(json.dumps(out), flush=True)
    if rows:
        S = [r["slowest"] for r in rows]
        print(json.dumps({"summary": True, "iterations": len(rows),
                          "span_us_median": float(np.median([r["span_us"] for r in rows])),
                          "slowest_prologue_us_median": float(np.median([s["prologue_us"] for s in S])),
                          "slowest_loop_us_median": float(np.median([s["loop_us"] for s in S])),
                          "slowest_tail_us_median": float(np.median([s["tail_us"] for s in S])),
                          "slowest_cyc_per_step_median": float(np.median([s["cyc_per_step"] for s in S])),
                          "slowest_epoch_share_median": float(np.median(
                              [s["epoch_kcyc"] / max(1e-9, s["seg_kcyc"] + s["epoch_kcyc"] + s["wait_kcyc"]) for s in S])),
                          "slowest_wait_kcyc_median": float(np.median([s["wait_kcyc"] for s in S])),
                          "slowest_ghz_median": float(np.median([s["ghz"] for s in S])),
                          "lib": os.path.basename(_lib.LIB_PATH)}), flush=True)


if __name__ == "__main__":
    main()

"""Timeline of the level-split layout from the RVM_PROFILE build (make -C rvel-mcmc_amd profile):
per wave the realtime (100 MHz) at start, at the end of its integration, after its arrival
atomic, and at its end; per unit which level arrived last and how long its combine took.
Usage: python scripts/probe/prof_levelsplit.py [W]  (plain S2 launch; W = 6144 -> level-split)"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

import oracle as O  # noqa: E402
from conftest import S2_PLANETS, s2_obs_oracle  # noqa: E402
from rvmcmc import _lib, engine  # noqa: E402

SLOTS, MAXW = 18, 4096


def main():
    W = int(sys.argv[1]) if len(sys.argv) > 1 else 6144
    _lib.LIB_PATH = os.path.join(ROOT, "scripts", "probe", "librvmcmc_prof.so")
    lib = _lib.load()
    lib.rvm_prof_copy.argtypes = [C.c_void_p, C.c_size_t]
    obs = s2_obs_oracle()
    dt, mult, hint = engine.IntegratorConfig().plan_args(S2_PLANETS)
    t, rv, er = engine.obs_arrays(obs)
    plan = engine.LoglPlan(t, rv, er, obs.Npoints, 2, dt, mult, W, period_hint=hint)
    rng = np.random.default_rng(0)
    P = np.repeat(O.pal_params(S2_PLANETS)[None], W, 0)
    P[:, :, :5] *= 1 + 1e-3 * rng.standard_normal((W, 2, 5))
    K = torch.as_tensor(np.concatenate([P[:, p, :5].T for p in range(2)], 0).copy(), device="cuda")
    for _ in range(3):
        plan.logl(K)
    torch.cuda.synchronize()
    out = {"W": W, "runs": []}
    for rep in range(3):
        lib.rvm_prof_clear()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        plan.logl(K)
        e1.record()
        torch.cuda.synchronize()
        buf = np.zeros(MAXW * SLOTS, dtype=np.uint64)
        assert lib.rvm_prof_copy(buf.ctypes.data, buf.nbytes) == 0
        b = buf.reshape(MAXW, SLOTS).astype(np.int64)
        b = b[b[:, 6] != 0]
        t0 = b[:, 5].min()
        us = lambda x: (x - t0) / 100.0  # noqa: E731
        lvl = b[:, 7] & 0xFF
        arr = b[:, 13] & 0xFF
        unit = b[:, 13] >> 8
        fin = arr == 3
        r = {"event_us": 1e3 * e0.elapsed_time(e1), "waves": int(len(b)), "span_us": float(us(b[:, 6].max())),
             "start_spread_us": float(us(b[:, 5].max())),
             "last_integration_end_us": float(us(b[:, 11].max())),
             "integration_end_us_by_level": {int(k): [float(np.percentile(us(b[lvl == k, 11]), q)) for q in (0, 50, 100)]
                                              for k in range(4)},
             "last_arriver_level_hist": np.bincount(lvl[fin], minlength=4).tolist(),
             "finisher_fence_atomic_us": [float(np.percentile((b[fin, 12] - b[fin, 11]) / 100.0, q)) for q in (50, 100)],
             "finisher_combine_us": [float(np.percentile((b[fin, 6] - b[fin, 12]) / 100.0, q)) for q in (50, 100)],
             "nonfinisher_fence_atomic_us": [float(np.percentile((b[~fin, 12] - b[~fin, 11]) / 100.0, q)) for q in (50, 100)],
             "unit_first_to_last_integration_end_us": None}
        spread = []
        for u in np.unique(unit):
            m = unit == u
            spread.append((b[m, 11].max() - b[m, 11].min()) / 100.0)
        r["unit_first_to_last_integration_end_us"] = [float(np.percentile(spread, q)) for q in (0, 50, 100)]
        # start times by block type: type-B blocks are the first nB blocks of the grid
        out["runs"].append(r)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""Cost of the adaptive resolution on the bench's own walker slots: one plain likelihood launch
over the 6144 slots of a speculative stretch iteration (scripts/probe/make_slots.py; the bench's
observation set), timed with HIP events, resolution off vs on, with the plan's counters (passes =
extension + halving walker-direction passes).  Usage: python scripts/probe/resolve_cost.py
scripts/probe/slots_it23.npz [...]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "tests")]
import torch  # noqa: E402

from conftest import S2_PLANETS  # noqa: E402
from rvmcmc import engine  # noqa: E402


def main():
    for f in sys.argv[1:]:
        d = np.load(f)
        t = np.concatenate([d["tf"], d["tb"]])
        rv = np.concatenate([d["rvf"], d["rvb"]])
        er = np.concatenate([d["errorf"], d["errorb"]])
        X = d["K"]
        W = len(X)
        cfg = engine.IntegratorConfig()
        dt, mult, hint = cfg.plan_args(S2_PLANETS)
        K = torch.as_tensor(np.ascontiguousarray(X.T), device="cuda")
        for res in [(0.0, 0), cfg.resolve(S2_PLANETS)]:
            plan = engine.LoglPlan(t, rv, er, 100, 2, dt, mult, W, period_hint=hint, resolve=res)
            lp, st, _ = plan.logl(K)
            torch.cuda.synchronize()
            plan.faults(reset=True)
            times = []
            for _ in range(10):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                plan.logl(K, out=lp, status=st)
                e1.record()
                torch.cuda.synchronize()
                times.append(e0.elapsed_time(e1))
            fl = plan.faults(reset=True)
            s = st.cpu().numpy()
            print(json.dumps({"slots": os.path.basename(f), "resolve": list(res), "ext_mult": plan.ext_mult,
                              "ms_median": float(np.median(times)), "ms_min": float(np.min(times)),
                              "passes_per_launch": fl["refined"] / 10, "unresolved_per_launch": fl["unresolved"] / 10,
                              "status_counts": np.bincount(s, minlength=5).tolist()}), flush=True)


if __name__ == "__main__":
    main()

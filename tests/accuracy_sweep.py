"""Accuracy/cost sweep of the kernel algorithm (Richardson-extrapolated WH, oracle restatement)
against the IAS15 restatement: for each (n_levels, steps_per_orbit) prints max |dlogL| over a
walker ball and the schedule cost (critical-path steps = finest level; total steps = all levels).
Test tooling (imports oracle/); not collected by pytest.  Usage: python tests/accuracy_sweep.py"""
import itertools
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from conftest import S2_PLANETS, s2_obs_oracle  # noqa: E402  (puts oracle/ on sys.path)
import oracle as O  # noqa: E402


def steps(obs, dt):
    out = 0
    for t in (np.sort(np.asarray(obs.tf)), np.sort(-np.asarray(obs.tb))):
        prev = 0.0
        for x in t:
            out += int(np.ceil((x - prev) / dt - 1e-9)) if x > prev else 0
            prev = x
    return out


def main():
    golden = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden.json")))
    sol = golden["G2"]["sol"]
    hd = [{"m": sol[3], "a": sol[0], "h": sol[1], "k": sol[2], "l": sol[4]},
          {"m": sol[8], "a": sol[5], "h": sol[6], "k": sol[7], "l": sol[9]}]
    hd_obs = O.obs_from_file(os.path.join(os.path.dirname(__file__), "golden", "HD155358.vels"), Npoints=100)
    cases = [("S2", S2_PLANETS, s2_obs_oracle()), ("HD", hd, hd_obs)]
    W = int(os.environ.get("W", "16"))
    grid = [(4, 24), (3, 24), (3, 32), (3, 40), (5, 16), (5, 20), (6, 12), (6, 16), (4, 20), (4, 16)]
    if len(sys.argv) > 1:
        # "nl,spo" (harmonic levels 1..nl) or "m1-m2-...@spo" (level multiplier sequence)
        grid = []
        for a in sys.argv[1:]:
            if "@" in a:
                seq, spo = a.split("@")
                grid.append((tuple(int(v) for v in seq.split("-")), float(spo)))
            else:
                nl, spo = a.split(",")
                grid.append((int(nl), float(spo)))
    for name, planets, obs in cases:
        pmin = min(2 * np.pi * np.sqrt(p["a"] ** 3 / (1 + p["m"])) for p in planets)
        rng = np.random.default_rng(1)
        base = O.pal_params(planets)
        params = np.repeat(base[None], W, 0)
        params[:, :, :5] *= 1 + 1e-3 * rng.standard_normal((W, len(planets), 5))
        ref, st_ref = O.logl_ias15_batch(params, len(planets), obs, hill_factor=1.0)
        ok = st_ref == 0
        for nl, spo in grid:
            dt = pmin / spo
            got, st = O.logl_whx_batch(params, len(planets), obs, dt, nl, hill_factor=1.0)
            err = np.max(np.abs(got[ok] - ref[ok]))
            s1 = steps(obs, dt)
            mult = list(range(1, nl + 1)) if isinstance(nl, int) else list(nl)
            print(json.dumps({"case": name, "levels": mult, "spo": spo, "max_abs_dlogl": float(err),
                              "sum_abs_w": float(np.abs(O.richardson_weights(nl)).sum()),
                              "critical_steps": s1 * max(mult), "total_steps": s1 * sum(mult)}), flush=True)


if __name__ == "__main__":
    main()

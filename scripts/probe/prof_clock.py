"""Shader clock and cycles per WH step per Richardson level, from the RVM_PROFILE build
(make -C rvel-mcmc_amd profile -> scripts/probe/librvmcmc_prof.so).

Each wave records s_memtime (shader cycles) and s_memrealtime (100 MHz) at its start and end, so
cycles / realtime is the clock the wave actually ran at, and segment cycles / (mult x base steps)
is the cost of one step on that level.  Answers: is a launch issue-bound (cycles per step grow
when two waves share a SIMD) or clock-bound (the clock drops under full-chip fp64 load)?
Usage: [RESOLVE=5e-7,4] [BALL=1e-3] python scripts/probe/prof_clock.py W [W ...]   (S2 workload)"""
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


def pct(x):
    return [round(float(np.percentile(x, q)), 3) for q in (0, 50, 100)]


def run(lib, W):
    obs = s2_obs_oracle()
    dt, mult, hint = engine.IntegratorConfig().plan_args(S2_PLANETS)
    t, rv, er = engine.obs_arrays(obs)
    # RESOLVE="tol,max": an adaptive plan (its extension level runs as a fifth level of the split
    # layout, or as a concurrent wave of the one-group-per-block layout)
    rs = os.environ.get("RESOLVE")
    resolve = (float(rs.split(",")[0]), int(rs.split(",")[1])) if rs else (0.0, 0)
    plan = engine.LoglPlan(t, rv, er, obs.Npoints, 2, dt, mult, W, period_hint=hint, resolve=resolve)
    info = plan.info()
    nbase = [info["steps_fwd"], info["steps_bwd"]]
    rng = np.random.default_rng(0)
    P = np.repeat(O.pal_params(S2_PLANETS)[None], W, 0)
    P[:, :, :5] *= 1 + float(os.environ.get("BALL", "1e-3")) * rng.standard_normal((W, 2, 5))
    K = torch.as_tensor(np.concatenate([P[:, p, :5].T for p in range(2)], 0).copy(), device="cuda")
    for _ in range(3):
        plan.logl(K)
    torch.cuda.synchronize()
    lib.rvm_prof_clear()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    plan.logl(K)
    e1.record()
    torch.cuda.synchronize()
    buf = np.zeros(MAXW * SLOTS, dtype=np.uint64)
    assert lib.rvm_prof_copy(buf.ctypes.data, buf.nbytes) == 0
    b = buf.reshape(MAXW, SLOTS).astype(np.int64)
    used = (b[:, 6] != 0) & (b[:, 4] != 0)
    gw = np.nonzero(used)[0]
    b = b[used]
    lvl = b[:, 7] & 0xFF
    d = (b[:, 7] >> 8) & 0xFF
    m = (b[:, 7] >> 16) & 0xFF
    cyc = b[:, 4] - b[:, 0]
    rt_us = (b[:, 6] - b[:, 5]) / 100.0
    ok = rt_us > 1.0
    out = {"W": W, "event_us": 1e3 * e0.elapsed_time(e1), "waves": int(len(b)), "steps_fwd_bwd": nbase,
           "clock_ghz": pct(cyc[ok] / rt_us[ok] / 1e3), "span_us": float((b[:, 6].max() - b[:, 5].min()) / 100.0)}
    # placement from HW_REG_HW_ID (simd [5:4]): which wave slots of a block share a SIMD
    simd = (b[:, 10] >> 4) & 3
    wpb = 8 if W > 4096 else (5 if rs else 4)
    blk, wv = gw // wpb, gw % wpb
    pairs = {}
    for bk in np.unique(blk):
        sel = blk == bk
        for s_ in np.unique(simd[sel]):
            k = str(sorted(wv[sel][simd[sel] == s_].tolist()))
            pairs[k] = pairs.get(k, 0) + 1
    out["waves_sharing_a_simd"] = pairs
    steps = m * np.where(d == 0, nbase[0], nbase[1])
    for k in sorted(set(lvl.tolist())):
        s = lvl == k
        t0 = b[:, 5].min()
        out[f"level{k}"] = {"mult": int(m[s][0]), "seg_cycles_per_step": pct(b[s, 2] / steps[s]),
                            "wave_us": pct(rt_us[s]), "total_kcyc": pct(cyc[s] / 1e3),
                            "prologue_kcyc": pct((b[s, 1] - b[s, 0]) / 1e3),
                            "pro_params_pal_setup_stage_barrier_kcyc": [
                                pct(x / 1e3) for x in
                                (b[s, 14] - b[s, 0], b[s, 15] - b[s, 14], b[s, 16] - b[s, 15], b[s, 17] - b[s, 16],
                                 b[s, 1] - b[s, 17])], "epochs_kcyc": pct(b[s, 3] / 1e3),
                            "rest_kcyc": pct((cyc[s] - (b[s, 1] - b[s, 0]) - b[s, 2] - b[s, 3]) / 1e3),
                            "start_us": pct((b[s, 5] - t0) / 100.0), "end_us": pct((b[s, 6] - t0) / 100.0),
                            "redo": int(b[s, 8].sum())}
        # level-split waves: the end of the integration (o[11]) and a combiner's arrival (o[12]:
        # every epoch consumed, verdict next)
        if np.any(b[s, 11] != 0):
            out[f"level{k}"]["integ_end_us"] = pct((b[s, 11] - t0) / 100.0)
        if np.any(b[s, 12] != 0):
            out[f"level{k}"]["comb_arrival_us"] = pct((b[s, 12] - t0) / 100.0)
    # level-split: per unit, the combiner's arrival against the last of its levels' integration
    # ends (o[13] >> 8 = unit): the time the combiner needs after its last input
    if np.any(b[:, 11] != 0):
        unit = (b[:, 13] >> 8) & 0xFFFF
        t0 = b[:, 5].min()
        lag, own = [], []
        for u in np.unique(unit[b[:, 12] != 0]):
            su = unit == u
            cmb = su & (lvl == 0)
            if not np.any(cmb):
                continue
            last = b[su, 11].max()
            lag.append((b[cmb, 12].max() - last) / 100.0)
            own.append((b[cmb, 12].max() - b[cmb, 11].max()) / 100.0)
        out["comb_after_last_level_us"] = pct(np.array(lag))
        out["comb_after_own_level_us"] = pct(np.array(own))
    return out


def main():
    _lib.LIB_PATH = os.path.join(ROOT, "scripts", "probe", "librvmcmc_prof.so")
    lib = _lib.load()
    lib.rvm_prof_copy.argtypes = [C.c_void_p, C.c_size_t]
    for a in sys.argv[1:] or ["2048", "6144"]:
        print(json.dumps(run(lib, int(a))), flush=True)


if __name__ == "__main__":
    main()

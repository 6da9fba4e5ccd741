"""Per-wave timing breakdown of rvm::logl_kernel from the RVM_PROFILE build
(make -C rvel-mcmc_amd profile -> scripts/probe/librvmcmc_prof.so).
Usage: python scripts/probe/prof_kernel.py [W]   (S2 workload, default integrator)"""
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
    slots = os.environ.get("SLOTS")  # (e.g. scripts/probe/slots_it2000.npz: a steady-state launch's slots)
    KS = np.load(slots)["K"] if slots else None
    W = int(sys.argv[1]) if len(sys.argv) > 1 else (len(KS) if KS is not None else 2048)
    assert W <= 8192
    _lib.LIB_PATH = os.path.join(ROOT, "scripts", "probe", "librvmcmc_prof.so")
    lib = _lib.load()
    lib.rvm_prof_copy.argtypes = [C.c_void_p, C.c_size_t]
    obs = s2_obs_oracle()
    cfg = engine.IntegratorConfig()
    dt, mult, hint = cfg.plan_args(S2_PLANETS)
    t, rv, er = engine.obs_arrays(obs)
    res = cfg.resolve(S2_PLANETS) if os.environ.get("RESOLVE", "0") == "1" else (0.0, 0)
    plan = engine.LoglPlan(t, rv, er, obs.Npoints, 2, dt, mult, W, period_hint=hint, resolve=res)
    rng = np.random.default_rng(0)
    P = np.repeat(O.pal_params(S2_PLANETS)[None], W, 0)
    P[:, :, :5] *= 1 + float(os.environ.get("BALL", "1e-3")) * rng.standard_normal((W, 2, 5))
    K = torch.as_tensor(np.concatenate([P[:, p, :5].T for p in range(2)], 0).copy(), device="cuda")
    if KS is not None:
        K = torch.as_tensor(np.ascontiguousarray(KS[:W].T), device="cuda")
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
    used = b[:, 4] != 0
    b = b[used]
    lvl = b[:, 7] & 0xFF
    out = {"W": W, "event_ms": e0.elapsed_time(e1), "waves": int(used.sum()),
           "realtime_span_us": float((b[:, 6].max() - b[:, 5].min()) / 100.0)}  # s_memrealtime: 100 MHz
    for k in sorted(set(lvl.tolist())):
        m = lvl == k
        tot = b[m, 4] - b[m, 0]
        out[f"level{k}"] = {"mult": int((b[m, 7][0] >> 16)), "total_kcyc": float(np.median(tot) / 1e3),
                            "prologue_kcyc": float(np.median(b[m, 1] - b[m, 0]) / 1e3),
                            "segments_kcyc": float(np.median(b[m, 2]) / 1e3),
                            "epochs_kcyc": float(np.median(b[m, 3]) / 1e3),
                            "tail_kcyc": float(np.median(tot - (b[m, 1] - b[m, 0]) - b[m, 2] - b[m, 3]) / 1e3),
                            "max_total_kcyc": float(tot.max() / 1e3),
                            "segments_redone_mean": float(b[m, 8].mean()), "segments": int(b[m, 9].max())}
    rt = (b[:, 6] - b[:, 5]) / 100.0
    out["wave_realtime_us"] = {"min": float(rt.min()), "median": float(np.median(rt)), "max": float(rt.max())}
    tot = b[:, 4] - b[:, 0]
    slow = np.argsort(tot)[::-1][:6]
    out["slowest_waves"] = [{"level_mult": int((b[i, 7] >> 16) & 0xFF), "dir": int((b[i, 7] >> 8) & 0xFF),
                             "total_kcyc": float(tot[i] / 1e3), "segments_kcyc": float(b[i, 2] / 1e3),
                             "epochs_kcyc": float(b[i, 3] / 1e3), "redo": int(b[i, 8])} for i in slow]
    out["start_spread_us"] = float((b[:, 5].max() - b[:, 5].min()) / 100.0)
    # placement (HW_REG_HW_ID, gfx9 layout): wave_id [3:0], simd [5:4], cu [11:8], sh [12], se [15:13]
    hw = b[:, 10]
    simd, cu, sh, se = (hw >> 4) & 3, (hw >> 8) & 15, (hw >> 12) & 1, (hw >> 13) & 7
    gidx = np.nonzero(used)[0]
    wv = gidx % int(os.environ.get("WPB_WAVES", "4"))  # wave index within its block
    out["wave_in_block_vs_simd"] = {int(k): np.bincount(simd[wv == k], minlength=4).tolist() for k in sorted(set(wv.tolist()))}
    key = (se * 2 + sh) * 16 + cu
    mult = (b[:, 7] >> 16) & 0xFF
    load = {}
    for k, s_, m_ in zip(key.tolist(), simd.tolist(), mult.tolist()):
        load.setdefault((k, s_), []).append(m_)
    per = [sum(v) for v in load.values()]
    out["simd_load_mult_sum"] = {"max": int(max(per)), "hist": {str(x): per.count(x) for x in sorted(set(per))}}
    out["cus_used"] = int(len(set(key.tolist())))
    fails = np.zeros(12, dtype=np.uint64)
    lib.rvm_prof_fail_copy.argtypes = [C.c_void_p]
    if lib.rvm_prof_fail_copy(fails.ctypes.data) == 0 and fails.any():
        f = fails.reshape(4, 3).astype(np.float64)
        out["gated_rare"] = {"wave_steps_second_halley": int(f[3, 0]), "wave_steps_kepler_rare": int(f[3, 1]),
                             "lanes_kepler_rare": int(f[3, 2])}
        out["first_halley_step"] = {f"NT{6 + i}": {"lane_drifts": int(f[i, 0]),
                                                   "z_beyond_bound": float(f[i, 1] / max(f[i, 0], 1)),
                                                   "not_accepted": float(f[i, 2] / max(f[i, 0], 1))}
                                    for i in range(3) if f[i, 0] > 0}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

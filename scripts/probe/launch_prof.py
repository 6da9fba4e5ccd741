"""Where one likelihood launch's time goes, per wave (the RVM_PROFILE build,
scripts/probe/librvmcmc_prof.so): the affine sampler of scripts/configs_bench.py config CFG (2: 1024
walkers, 2 planets; 5: 8192 walkers, 3 planets) from its ball, a few iterations, then for the last
launch of each iteration: its waves' start / end on the real-time clock, and the slowest wave's level,
prologue, segment and epoch-handling cycles, steps (the level's multiplier x base steps) and redone
segments.  usage: launch_prof.py CFG -> JSON lines."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "scripts")]
import torch  # noqa: E402

from rvmcmc import _lib  # noqa: E402

SLOTS, MAXW = 18, 4096


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "2"
    _lib.LIB_PATH = os.path.join(ROOT, "scripts", "probe", "librvmcmc_prof.so")
    lib = _lib.load()
    lib.rvm_prof_copy.argtypes = [C.c_void_p, C.c_size_t]
    import configs_bench as CB
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.observations import FakeObservation
    from rvmcmc.state import State

    np.random.seed(2017)
    planets = [dict(p) for p in CB.S2] + ([dict(CB.THIRD)] if cfg == "5" else [])
    s = State(planets=planets)
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    W = 8192 if cfg == "5" else 1024
    sc = np.array([CB.SCALES[k] for k in s.get_rawkeys()])
    X0 = s.get_params()[None] + 1e-3 * sc * np.random.normal(size=(W, s.Nvars))
    ens = EnsembleSampler(W, s, obs, seed=1)
    ens.set_positions(X0)
    ens.compute_lnprob()
    for _ in range(3):
        ens.step()
    torch.cuda.synchronize()
    buf = np.zeros(MAXW * SLOTS, dtype=np.uint64)
    for it in range(4):
        lib.rvm_prof_clear()
        torch.cuda.synchronize()
        ens.step()
        torch.cuda.synchronize()
        assert lib.rvm_prof_copy(buf.ctypes.data, buf.nbytes) == 0
        b = buf.reshape(MAXW, SLOTS).astype(np.int64)
        b = b[b[:, 4] != 0]
        t0 = b[:, 5].min()
        end = (b[:, 6] - t0) / 100.0
        i = int(np.argmax(end))
        w = b[i]
        tot = w[4] - w[0]
        print(json.dumps({"it": it, "waves": int(len(b)), "span_us": float(end.max()),
                          "start_us_max": float((b[:, 5] - t0).max() / 100.0),
                          "slowest": {"mult": int((w[7] >> 16) & 0xFF), "level": int(w[7] & 0xFF), "dir": int((w[7] >> 8) & 0xFF),
                                      "total_kcyc": tot / 1e3, "prologue_kcyc": (w[1] - w[0]) / 1e3,
                                      "segments_kcyc": w[2] / 1e3, "epochs_kcyc": w[3] / 1e3, "redo": int(w[8]),
                                      "epochs": int(w[9]), "ghz": float(tot) / max(1.0, (w[6] - w[5]) * 10.0)},
                          "segments_kcyc_by_level_max": {int(m): float(b[((b[:, 7] >> 16) & 0xFF) == m, 2].max() / 1e3)
                                                         for m in sorted(set(((b[:, 7] >> 16) & 0xFF).tolist()))}}),
              flush=True)


if __name__ == "__main__":
    main()

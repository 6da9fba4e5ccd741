"""Per-iteration timing of the likelihood kernel at the bench chain's steady state (the RVM_PROFILE
build, scripts/probe/librvmcmc_prof.so from `make -C rvel-mcmc_amd profile` or `profile-fails`):
the steady-state sampler of scripts/probe/steady_bench.py, and for each iteration the slowest wave
of its likelihood launch (level, direction, segment / epoch cycles, redone segments) next to the
medians, and the iteration's wall time -- what makes some launches twice as long as others.
With the profile-fails build the Kepler first-step failure counts of each launch as well."""
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

SLOTS, MAXW = 18, 4096


def main():
    _lib.LIB_PATH = os.path.join(ROOT, "scripts", "probe", "librvmcmc_prof.so")
    lib = _lib.load()
    lib.rvm_prof_copy.argtypes = [C.c_void_p, C.c_size_t]
    lib.rvm_prof_fail_copy.argtypes = [C.c_void_p]
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.observations import FakeObservation
    from rvmcmc.state import State

    state = State(planets=[dict(p) for p in S2_PLANETS])
    state.integrator = engine.IntegratorConfig(resolve_tol=float(os.environ.get("TOL", "5e-7")))
    np.random.seed(2017)
    obs = FakeObservation(state, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    X = np.load(os.path.join(ROOT, "scripts/probe/ens_it2000.npy"))
    ens = EnsembleSampler(len(X), state, obs, seed=2017)
    ens.set_positions(X)
    ens.compute_lnprob()
    for _ in range(3):
        ens.step()
    torch.cuda.synchronize()
    ens.plan.time_kernels(64)
    buf = np.zeros(MAXW * SLOTS, dtype=np.uint64)
    for it in range(int(os.environ.get("ITERS", "30"))):
        lib.rvm_prof_clear()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ens.step()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        assert lib.rvm_prof_copy(buf.ctypes.data, buf.nbytes) == 0
        b = buf.reshape(MAXW, SLOTS).astype(np.int64)
        b = b[b[:, 4] != 0]
        rt = (b[:, 6] - b[:, 5]) / 100.0
        tot = b[:, 4] - b[:, 0]
        i = int(np.argmax(rt))
        out = {"it": it, "wall_ms": 1e3 * wall, "waves": int(len(b)), "wave_rt_us_max": float(rt.max()),
               "wave_rt_us_median": float(np.median(rt)),
               "slowest": {"mult": int((b[i, 7] >> 16) & 0xFF), "flags": int(b[i, 7] & 0xFF),
                           "dir": int((b[i, 7] >> 8) & 0xFF), "total_kcyc": float(tot[i] / 1e3),
                           "segments_kcyc": float(b[i, 2] / 1e3), "epochs_kcyc": float(b[i, 3] / 1e3),
                           "redo": int(b[i, 8])},
               "segments_kcyc_median": float(np.median(b[:, 2]) / 1e3),
               "segments_kcyc_max": float(b[:, 2].max() / 1e3), "redo_max": int(b[:, 8].max())}
        fails = np.zeros(12, dtype=np.uint64)
        if lib.rvm_prof_fail_copy(fails.ctypes.data) == 0 and fails.any():
            f = fails.reshape(4, 3).astype(np.int64)
            out["wave_steps_second_halley"], out["wave_steps_kepler_rare"], out["lanes_kepler_rare"] = \
                [int(v) for v in f[3]]
        print(json.dumps(out), flush=True)
    main_ms, ref_ms = ens.plan.kernel_times(64)
    print(json.dumps({"logl_kernel_ms": main_ms.tolist(), "refine_kernel_ms": ref_ms.tolist(),
                      "faults": ens.check_faults()}), flush=True)


if __name__ == "__main__":
    main()

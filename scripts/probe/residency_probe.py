"""Are a launch's blocks co-resident?  (timing build, scripts/probe/librvmcmc_prof.so.)  Runs config 5
(scripts/configs_bench.py: 3 planets, 8192 walkers, the two-launch stretch step) for a few iterations
and reports, for the last likelihood launch, the start times of its waves (rvm_prof, the 100 MHz real
time at each wave's start): with every block resident at once they start within a few microseconds;
with two rounds the second half starts when the first half ends."""
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
    _lib.LIB_PATH = os.path.join(ROOT, "scripts", "probe", "librvmcmc_prof.so")
    lib = _lib.load()
    lib.rvm_prof_copy.argtypes = [C.c_void_p, C.c_size_t]
    import configs_bench as CB
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.observations import FakeObservation
    from rvmcmc.state import State

    np.random.seed(2017)
    s = State(planets=[dict(p) for p in CB.S2] + [dict(CB.THIRD)])
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    W = 8192
    sc = np.array([CB.SCALES[k] for k in s.get_rawkeys()])
    X0 = s.get_params()[None] + 1e-3 * sc * np.random.normal(size=(W, s.Nvars))
    ens = EnsembleSampler(W, s, obs, seed=1)
    ens.set_positions(X0)
    ens.compute_lnprob()
    for _ in range(3):
        ens.step()
    torch.cuda.synchronize()
    buf = np.zeros(MAXW * SLOTS, dtype=np.uint64)
    for it in range(3):
        lib.rvm_prof_clear()
        torch.cuda.synchronize()
        ens.step()  # (two half-step launches: the record holds the second's waves)
        torch.cuda.synchronize()
        assert lib.rvm_prof_copy(buf.ctypes.data, buf.nbytes) == 0
        b = buf.reshape(MAXW, SLOTS).astype(np.int64)
        b = b[b[:, 4] != 0]
        st = (b[:, 5] - b[:, 5].min()) / 100.0
        en = (b[:, 6] - b[:, 5].min()) / 100.0
        print(json.dumps({"it": it, "waves": int(len(b)), "start_us_quantiles": np.quantile(st, [0, .25, .5, .75, .9, 1]).round(1).tolist(),
                          "end_us_quantiles": np.quantile(en, [0, .25, .5, .75, .9, 1]).round(1).tolist(),
                          "waves_starting_after_50us": int((st > 50).sum())}), flush=True)


if __name__ == "__main__":
    main()

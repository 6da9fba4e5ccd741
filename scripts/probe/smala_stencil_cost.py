"""Why the SMALA stencil launch (config 4) is slower than a ball launch of the same size: time
the likelihood launch on the real stencil after a few SMALA steps, on the stencil of the initial
point, and on an S2 ball of the same walker count.  Usage: python scripts/probe/smala_stencil_cost.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd")]
import torch  # noqa: E402

from rvmcmc import _lib, smala  # noqa: E402
from rvmcmc.observations import FakeObservation  # noqa: E402
from rvmcmc.state import State  # noqa: E402

S2 = [{"m": 1.2e-3, "a": 0.88, "h": 0.218, "k": 0.015, "l": 0.3},
      {"m": 2.1e-3, "a": 1.55, "h": 0.16, "k": 0.02, "l": 2.2}]


def time_launch(state, obs, K, pmap, reps=10):
    for _ in range(2):
        state.get_logp_batch(obs, K, hill_factor=1.0, want_rv=True, pmap=pmap)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        lp, st, _ = state.get_logp_batch(obs, K, hill_factor=1.0, want_rv=True, pmap=pmap)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, np.bincount(st.cpu().numpy(), minlength=4).tolist()


def stencil_of(sm, X):
    P, C = X.shape
    fl = torch.as_tensor(smala.fd_floor_vector(sm.state), device=X.device)
    out = torch.empty((P, (2 * P + 1) * C), dtype=torch.float64, device=X.device)
    _lib.check(_lib.load().rvm_fd_params(P, C, X.contiguous().data_ptr(), float(sm.rel_step), fl.data_ptr(),
                                         out.data_ptr(), _lib.stream_handle()), "rvm_fd_params")
    return out


def main():
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in S2])
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    sm = smala.SmalaChains(s, obs, eps=0.5, alpha=1e3, n_chains=256, seed=0)
    X0 = sm.X.clone()
    for _ in range(10):
        sm.step()
    torch.cuda.synchronize()
    W = 21 * 256
    rng = np.random.default_rng(0)
    ball = torch.as_tensor(s.get_params()[:, None] * (1 + 1e-3 * rng.standard_normal((s.Nvars, W))), device="cuda")
    for name, K in (("stencil after 10 steps", stencil_of(sm, sm.X)), ("stencil of the start", stencil_of(sm, X0)),
                    ("S2 ball", ball)):
        ms, hist = time_launch(s, obs, K.contiguous(), sm.pmap)
        print(f"{name:24s} W={K.shape[1]} {ms:.4f} ms  status {hist}", flush=True)
    X = sm.X.cpu().numpy()
    print("chain spread (rel std per param):", np.round(X.std(1) / np.abs(X.mean(1)), 4).tolist())


if __name__ == "__main__":
    main()

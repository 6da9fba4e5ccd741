"""Where a SMALA step's time goes (config 4: 256 chains, 10-dim): logL launch vs torch linalg."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd")]
import torch  # noqa: E402

from rvmcmc import smala  # noqa: E402
from rvmcmc.observations import FakeObservation  # noqa: E402
from rvmcmc.state import State  # noqa: E402

S2 = [{"m": 1.2e-3, "a": 0.88, "h": 0.218, "k": 0.015, "l": 0.3},
      {"m": 2.1e-3, "a": 1.55, "h": 0.16, "k": 0.02, "l": 2.2}]


def timed(fn, n=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3, out


def main():
    np.random.seed(2017)
    s = State(planets=[dict(p) for p in S2])
    obs = FakeObservation(s, Npoints=100, error=1.5e-4, errorVar=2.5e-5, tmax=120.)
    sm = smala.SmalaChains(s, obs, eps=0.5, alpha=1e3, n_chains=256, seed=0)
    X = sm.X
    ms_fd, (lp, g, H, st) = timed(lambda: smala.fd_logp_grad_metric(sm.state, obs, X, sm.rel_step, sm.pmap, 1.0))
    A = (-H).permute(2, 0, 1).contiguous()
    ms_eigh, _ = timed(lambda: torch.linalg.eigh(A))
    ms_chol, _ = timed(lambda: torch.linalg.cholesky_ex(A @ A.transpose(1, 2) + torch.eye(10, device=A.device, dtype=A.dtype)))
    ms_step, _ = timed(lambda: sm.step())
    P = sm.state.Nvars
    stencil = torch.empty((P, (2 * P + 1) * 256), dtype=torch.float64, device=X.device)
    ms_logl, _ = timed(lambda: sm.state.get_logp_batch(obs, stencil.copy_(X.repeat(1, 2 * P + 1)), hill_factor=1.0,
                                                       want_rv=True, pmap=sm.pmap))
    print(dict(step_ms=ms_step, fd_logp_grad_metric_ms=ms_fd, logl_launch_5376_ms=ms_logl,
               eigh_ms=ms_eigh, cholesky_ms=ms_chol))


if __name__ == "__main__":
    main()

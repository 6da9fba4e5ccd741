"""Find the proposals a sampler run reports NONFINITE: the HD155358 posterior run
(scripts/posterior_hd155358.py) on the three-launch half-step path (bit-identical to the fused and
speculative paths), whose proposals are materialised; dumps them to gpurun_out/nonfinite.npz."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "scripts")]
import torch  # noqa: E402

from rvmcmc import engine  # noqa: E402
from rvmcmc.ensemble import EnsembleSampler  # noqa: E402
from rvmcmc.observations import Observation_FromFile  # noqa: E402
from rvmcmc.state import State  # noqa: E402
import posterior_hd155358 as PH  # noqa: E402

engine.FAULT_CHECK_EVERY = 0
obs = Observation_FromFile(os.path.join(ROOT, "tests", "golden", "HD155358.vels"), Npoints=100)
S = PH.SOL
planets = [{"a": S[0], "h": S[1], "k": S[2], "m": S[3], "l": S[4]}, {"a": S[5], "h": S[6], "k": S[7], "m": S[8], "l": S[9]}]
s = State(planets=planets)
sc = {"m": 5.5e-6, "a": 0.001, "h": 0.02, "k": 0.02, "l": np.pi / 4.}
scales = np.array([sc[k] for k in s.get_rawkeys()])
rng = np.random.default_rng(2017)
W = 4096
X0 = s.get_params()[None] + 1e-3 * scales * rng.standard_normal((W, s.Nvars))
ens = EnsembleSampler(W, s, obs, seed=7)
ens.set_positions(X0)
ens.speculating = lambda: False
ens.fused = False
found = []
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 600):
    if ens.lnp[0] is None:
        ens.compute_lnprob()
    A, B = ens.pos
    for h, (X, Y) in enumerate(((A, B), (B, A))):
        ens.half_step(X, ens.lnp[h], Y, h)
        st = ens._status.cpu().numpy()
        bad = np.nonzero(st == 3)[0]
        if len(bad):
            q = ens._q.t().cpu().numpy()[bad]
            found.append((it, h, bad, q))
            print("iteration", it, "half", h, "walkers", bad.tolist(), "q", q.tolist(), flush=True)
    ens.iteration += 1
    if found and len(found) >= 3:
        break
os.makedirs("gpurun_out", exist_ok=True)
np.savez("gpurun_out/nonfinite.npz", q=np.concatenate([f[3] for f in found]) if found else np.zeros((0, 10)),
         keys=np.array(s.get_rawkeys()))
print("found", sum(len(f[2]) for f in found))

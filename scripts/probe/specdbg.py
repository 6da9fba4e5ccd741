import sys, os
sys.path[:0]=['tests','rvel-mcmc_amd','oracle']
import numpy as np
from test_gpu_samplers import _state_and_obs
from rvmcmc import mcmc
s, obs = _state_and_obs()
runs=[]
for spec in (1, 8):
    np.random.seed(11)
    mh = mcmc.Mh(s, obs, speculate=spec)
    mh.set_scales({"m": 1.e-3, "a": 0.3, "h": 0.5, "k": 0.5, "l": np.pi / 2.})
    mh.step_size = 4e-2
    out=[]
    for _ in range(60):
        r = mh.step(); out.append((r, mh.state.logp, mh.state.get_params()[:2].tolist()))
    runs.append(out)
[print(i, a, "|", b) for i,(a,b) in enumerate(zip(*runs)) if a != b][:3]

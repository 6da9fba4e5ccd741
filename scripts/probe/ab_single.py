"""Single-walker and batch logL of the same walkers under the library named by RVM_LIB."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from rvmcmc import _lib  # noqa: E402

_lib.LIB_PATH = os.environ.get("RVM_LIB", _lib.LIB_PATH)
from conftest import S2_PLANETS, s2_obs_oracle  # noqa: E402
from test_gpu_logl import _ball, _plan, _run  # noqa: E402

obs = s2_obs_oracle()
W = 4128
plan, dt = _plan(obs, S2_PLANETS, max_walkers=W)
P = _ball(S2_PLANETS, W, seed=21)
for i in (0, 1, 32):
    one, _, _ = _run(plan, P[i:i + 1])
    print("before big", i, repr(one[0]), flush=True)
plan2, _ = _plan(obs, S2_PLANETS, max_walkers=64)
for i in (0, 1, 32):
    one, _, _ = _run(plan2, P[i:i + 1])
    print("small plan", i, repr(one[0]), flush=True)
big, _, _ = _run(plan, P)
for i in (0, 1, 32):
    one, _, _ = _run(plan, P[i:i + 1])
    print(os.path.basename(_lib.LIB_PATH), i, repr(one[0]), repr(big[i]), flush=True)

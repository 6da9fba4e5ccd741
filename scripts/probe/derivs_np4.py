"""Probe: 4-planet exact derivatives vs central differences of the oracle at several steps."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np
import oracle as O
from conftest import S2_PLANETS
from test_gpu_derivs import _case, _gpu_derivs, fd_derivs, sigma_steps, scaled_errors, fd_of_gradient, _kernel_params
from test_gpu_logl import LEVELS

extra = [{"m": 1e-3, "a": 2.6, "h": 0.05, "k": 0.0, "l": 1.0}, {"m": 5e-4, "a": 3.9, "h": 0.0, "k": 0.03, "l": 4.0}]
for npl in (3, 4):
    planets = (S2_PLANETS + extra)[:npl]
    np.random.seed(5)
    obs = O.fake_obs(planets, Npoints=30, error=1.5e-4, errorVar=2.5e-5, tmax=40.)
    plan, dt, Pw = _case(planets, obs, W=2)
    lp, g, H, st = _gpu_derivs(plan, Pw)
    x = _kernel_params(Pw[0:1], 5)[:, 0]
    for sc in (2.0, 1.0, 0.4):
        d = sc * sigma_steps(H[:, :, 0], x, 5)
        f0, gf, Hf = fd_derivs(lambda P: O.logl_whx_batch(P, npl, obs, dt, LEVELS)[0], x, npl, 5, d=d)
        eg, eH = scaled_errors(g[:, 0], H[:, :, 0], gf, Hf)
        _, eHg = scaled_errors(g[:, 0], H[:, :, 0], g[:, 0], fd_of_gradient(plan, x, d))
        s_ = np.sqrt(np.abs(np.diag(H[:, :, 0])))
        worst = int(np.argmax(np.abs(g[:, 0] - gf) / s_))
        print(npl, sc, "grad %.2e (worst row %d)  hess-vs-FD(grad) %.2e  hess-vs-2nd %.2e" % (eg, worst, eHg, eH))

"""Debug: GPU hyper-dual derivatives vs central differences of the oracle (per parameter)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import numpy as np
import torch
import oracle as O
from conftest import S2_PLANETS
from test_gpu_derivs import fd_derivs, _kernel_params, sigma_steps, scaled_errors
from rvmcmc import engine

def run(planets, tmax, npts, label, inclined=False):
    np.random.seed(1)
    obs = O.fake_obs(planets, Npoints=npts, error=1.5e-4, errorVar=2.5e-5, tmax=tmax)
    pmin = engine.min_period(planets)
    dt = pmin / 8
    t, rv, er = engine.obs_arrays(obs)
    plan = engine.LoglPlan(t, rv, er, obs.Npoints, len(planets), dt, (4, 5, 6, 7), 64, period_hint=pmin, inclined=inclined)
    Pw = np.repeat(O.pal_params(planets)[None], 1, 0)
    R = 7 if inclined else 5
    if inclined:
        Pw[:, :, 5] = 0.05 + 0.01 * np.arange(len(planets))[None, :]
        Pw[:, :, 6] = -0.03
    K = torch.as_tensor(_kernel_params(Pw, R), device="cuda")
    lp, g, H, st = plan.derivs(K, list(range(K.shape[0])))
    torch.cuda.synchronize()
    g = g.cpu().numpy()[:, 0]; H = H.cpu().numpy()[:, :, 0]
    x = _kernel_params(Pw, R)[:, 0]
    f0, gf, Hf = fd_derivs(lambda P: O.logl_whx_batch(P, len(planets), obs, dt, (4, 5, 6, 7), has_inc=int(inclined))[0], x, len(planets), R, d=sigma_steps(H, x, R))
    f0b, gfb, Hfb = fd_derivs(lambda P: O.logl_whx_batch(P, len(planets), obs, dt, (4, 5, 6, 7), has_inc=int(inclined))[0], x, len(planets), R, d=0.3*sigma_steps(H, x, R))
    print('scaled errors', scaled_errors(g, H, gf, Hf))
    print(label, "logl", lp.item(), f0)
    for i in range(len(x)):
        print(f"  {i}: g {g[i]: .10e} fd {gf[i]: .10e} {gfb[i]: .10e}  Hii {H[i,i]: .8e} fd {Hf[i,i]: .8e} {Hfb[i,i]: .8e}")
    s_ = np.sqrt(np.abs(np.diag(H)))
    e = np.abs(H - Hf) / np.outer(s_, s_)
    i, j = np.unravel_index(np.argmax(e), e.shape)
    print("worst H entry", i, j, H[i, j], Hf[i, j], Hfb[i, j], e[i, j])

run(S2_PLANETS, 30., 20, "2 planets")
run(S2_PLANETS[:1], 30., 20, "1 planet inclined", inclined=True)
run(S2_PLANETS, 30., 20, "2 planets inclined", inclined=True)

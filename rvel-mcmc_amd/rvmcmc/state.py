"""State: the reference's planet-parameter container, with its likelihood on the GPU.

Mirrors /root/reference/state.py (Python 2): same constructor, same free-parameter bookkeeping
(ignore_vars with the reference's `x not in ignore_vars` semantics, so a str works as a set of
characters), same vector API, same priorHard thresholds and same get_logp caching.  What
changed is underneath: REBOUND + IAS15 are replaced by the librvmcmc HIP kernel
(Wisdom-Holman + Richardson extrapolation), and a batched entry point
`get_logp_batch` evaluates many parameter vectors in one launch.

Deliberate differences:
  * priorHard does not print; it logs at DEBUG level.
  * get_logp_d_dd / get_chi2_d_dd return the exact derivatives of the kernel's own discrete
    integrator (rvm_logl_derivs, hyper-dual forward mode) where the reference integrates REBOUND's
    order-1/order-2 variational equations alongside IAS15 (state.py:218-294); method="fd" gives
    the SMALA fast path's central-difference gradient + Gauss-Newton Hessian instead.
  * Python 3 dict order defines the parameter order (insertion order); the reference ran on
    Python 2 dicts.
"""
from __future__ import annotations

import copy
import logging

import numpy as np

from . import engine

log = logging.getLogger(__name__)


class Encounter(Exception):
    """Raised when a pair of bodies comes closer than exit_min_distance (rebound.Encounter)."""


class State(object):
    def __init__(self, planets, ignore_vars=[], ignore_params=None):  # state.py:8-31
        self.planets = planets
        self.logp = None
        self.logp_d = None
        self.logp_dd = None
        self.planets_vars = []
        self.Nvars = 0
        self.hillRadiusMax = 0.0
        self.hillRadiusFactor = 1.
        self.ignore_vars = ignore_vars
        self.ignore_params = ignore_params
        self.integrator = engine.DEFAULT_CONFIG
        for p, planet in enumerate(planets):
            planet_vars = [x for x in planet.keys() if (x not in ignore_vars)]
            if ignore_params is not None:
                for o in range(len(ignore_params[p])):
                    planet_vars.remove(ignore_params[p][o])
            self.planets_vars.append(planet_vars)
            self.Nvars += len(planet_vars)

    # -- free-parameter bookkeeping (state.py:124-207) ------------------------------------------
    def _is_free(self, i, k):
        if k in self.ignore_vars:
            return False
        if self.ignore_params is not None and k in self.ignore_params[i]:
            return False
        return True

    def shift_params(self, vec):
        self.logp = None
        if len(vec) != self.Nvars:
            raise AttributeError("vector has wrong length")
        varindex = 0
        for i, planet in enumerate(self.planets):
            for k in planet.keys():
                if self._is_free(i, k):
                    self.planets[i][k] += vec[varindex]
                    varindex += 1

    def get_params(self):
        params = np.zeros(self.Nvars)
        parindex = 0
        for i, planet in enumerate(self.planets):
            for k in planet.keys():
                if self._is_free(i, k):
                    params[parindex] = self.planets[i][k]
                    parindex += 1
        return params

    def set_params(self, vec):
        self.logp = None
        if len(vec) != self.Nvars:
            raise AttributeError("vector has wrong length")
        varindex = 0
        for i, planet in enumerate(self.planets):
            for k in planet.keys():
                if self._is_free(i, k):
                    self.planets[i][k] = vec[varindex]
                    varindex += 1

    def get_keys(self):
        keys = [""] * self.Nvars
        parindex = 0
        for i, planet in enumerate(self.planets):
            for k in planet.keys():
                if self._is_free(i, k):
                    keys[parindex] = "$%s_%d$" % (k, i)
                    parindex += 1
        return keys

    def get_rawkeys(self):
        keys = [""] * self.Nvars
        parindex = 0
        for i, planet in enumerate(self.planets):
            for k in planet.keys():
                if self._is_free(i, k):
                    keys[parindex] = k
                    parindex += 1
        return keys

    def deepcopy(self):  # state.py:212-213 -- NOTE: resets hillRadiusFactor to 1.0, as the reference does
        s = State(copy.deepcopy(self.planets), copy.deepcopy(self.ignore_vars),
                  ignore_params=copy.deepcopy(self.ignore_params))
        s.integrator = self.integrator
        return s

    def priorHard(self):  # state.py:299-315
        for i, planet in enumerate(self.planets):
            if planet["a"] <= 0.02:
                log.debug("Invalid state was proposed (a)")
                return True
            if planet["m"] <= 5e-6:
                log.debug("Invalid state was proposed (m)")
                return True
            if ("h" in planet) or ("k" in planet):
                if planet["h"] ** 2 + planet["k"] ** 2 >= 1.0:
                    log.debug("Invalid state was proposed (h & k)")
                    return True
            if ("ix" in planet) or ("iy" in planet):
                if planet["ix"] ** 2 + planet["iy"] ** 2 >= 4.0:
                    log.debug("Invalid state was proposed (ix & iy)")
                    return True
        return False

    # -- likelihood -------------------------------------------------------------------------------
    @staticmethod
    def lnprior(theta):  # state.py:115-119 (the reference's emcee-style flat prior on one planet's m, a, h, k, l)
        m, a, h, k, l = theta
        if (1e-7 < m < 0.1) and (1e-2 < a < 500.0) and ((h ** 2 + k ** 2) < 1.0) and (-2 * np.pi < l < 2 * np.pi):
            return 0.0
        return -np.inf

    def var_pindex_vname(self, vindex):  # state.py:218-225: free-parameter index -> (planet index + 1, key)
        vi = 0
        for pindex, p in enumerate(self.planets_vars):
            for v in p:
                if vindex == vi:
                    return pindex + 1, v
                vi += 1
        return None

    def param_map(self):
        return engine.ParamMap(self)

    def hill_radius_max(self):
        """state.py:42-44 (not used by the kernel, which recomputes it per walker)."""
        r = 0.0
        for p in self.planets:
            r = max(r, p["a"] * (p["m"] / 3.0) ** (1.0 / 3.0))
        self.hillRadiusMax = r
        return r

    def _plan(self, obs, max_walkers=1, device=None):
        dt, mult, hint = self.integrator.plan_args(self.planets)
        return engine.plan_for(obs, len(self.planets), dt, mult, max_walkers, device, hint,
                               engine.is_inclined(self.planets), self.integrator.resolve(self.planets))

    def get_rv(self, times):
        """state.py:61-73: model RV (star barycentric vx) at `times`; raises Encounter."""
        import torch

        times = np.asarray(times, dtype=np.float64)

        class _T:  # a throw-away observation set carrying only the epochs
            pass

        o = _T()
        o.tf, o.tb = times, np.zeros(0)
        o.rvf, o.rvb = np.zeros(len(times)), np.zeros(0)
        o.errorf, o.errorb = np.ones(len(times)), np.zeros(0)
        o.Npoints = 1
        plan = self._plan(o)
        K = torch.as_tensor(self.param_map().vector_to_kernel_np(self.get_params()), device=plan.device)[:, None]
        _, st, rv = plan.logl(K.contiguous(), hill_factor=self.hillRadiusFactor, want_rv=True)
        st = int(st.item())
        if st == 2:
            raise Encounter("Two particles had a close encounter (d<exit_min_distance).")
        return rv[:, 0].cpu().numpy()

    def get_rv_plotting(self, obs, Npoints=1000):  # state.py:78-84
        times = np.linspace(obs.tb[0], obs.tf[len(obs.tf) - 1], Npoints)
        return times, self.get_rv(times)

    def _eval(self, obs):
        import torch

        plan = self._plan(obs)
        K = torch.as_tensor(self.param_map().vector_to_kernel_np(self.get_params()), device=plan.device)[:, None]
        lp, st, _ = plan.logl(K.contiguous(), hill_factor=self.hillRadiusFactor)
        return float(lp.item()), int(st.item())

    def get_chi2(self, obs):  # state.py:89-98
        lp, st = self._eval(obs)
        if st == 2:
            raise Encounter("Two particles had a close encounter (d<exit_min_distance).")
        if st == 3:  # (the reference would hand emcee a NaN, which it refuses)
            from ._lib import RvmError

            raise RvmError("non-finite chi2 on the GPU (RVM_STATUS_NONFINITE)")
        if st == 4:
            log.warning("walker not resolved to the plan's tolerance after the last refinement (UNRESOLVED): "
                        "logp = -inf")
        return -lp

    def get_logp(self, obs):  # state.py:103-110
        if self.priorHard():
            return -np.inf
        softlnpri = 0.0
        if self.logp is None:
            self.logp = -self.get_chi2(obs)
        return self.logp + softlnpri

    def get_logp_batch(self, obs, X, hill_factor=None, want_rv=False, pmap=None):
        """Batched get_logp: X is a float64 device tensor [Nvars][W] of free-parameter vectors.

        Returns (logp[W], status[W], rv[n_obs][W] | None); prior / encounter / non-finite walkers
        get -inf (status 1 / 2 / 3) instead of an exception."""
        pmap = pmap or self.param_map()
        plan = self._plan(obs, max_walkers=X.shape[1], device=X.device)
        K = pmap.to_kernel(X)
        hf = self.hillRadiusFactor if hill_factor is None else hill_factor
        return plan.logl(K, hill_factor=hf, want_rv=want_rv)

    # -- derivatives (state.py:218-294) -------------------------------------------------------------
    def get_logp_d_dd_batch(self, obs, X, hill_factor=None, pmap=None):
        """Exact logp, gradient and Hessian for a batch of free-parameter vectors X [Nvars][C]
        (float64 device tensor): rvm_logl_derivs, the hyper-dual counterpart of the reference's
        order-1/order-2 variational particles.  Returns (logp[C], grad[P][C], hess[P][P][C], status[C])."""
        pmap = pmap or self.param_map()
        plan = self._plan(obs, device=X.device)
        hf = self.hillRadiusFactor if hill_factor is None else hill_factor
        return plan.derivs(pmap.to_kernel(X), pmap.slots, hill_factor=hf)

    def get_chi2_d_dd(self, obs):  # state.py:253-288
        """(chi2, dchi2, d2chi2) ÷ obs.Npoints at the current parameters; raises Encounter."""
        import torch

        x = torch.as_tensor(self.get_params(), dtype=torch.float64, device=engine.default_device())[:, None]
        lp, g, H, st = self.get_logp_d_dd_batch(obs, x)
        st = int(st[0].item())
        if st == 2:
            raise Encounter("Two particles had a close encounter (d<exit_min_distance).")
        return -float(lp[0].item()), -g[:, 0].cpu().numpy(), -H[:, :, 0].cpu().numpy()

    def get_logp_d_dd(self, obs, method="exact", rel_step=1e-6):  # state.py:290-294
        """logp, its gradient and its Hessian (cached like the reference until set_params/shift_params).

        method="exact" (default, the reference's semantics): exact derivatives of the likelihood
        (rvm_logl_derivs).  method="fd": the SMALA fast path's central differences with the
        Gauss-Newton Hessian (rvmcmc.smala.fd_logp_grad_metric)."""
        if self.logp is None or self.logp_d is None:
            if method == "fd":
                from .smala import fd_logp_grad_metric
                import torch

                x = torch.as_tensor(self.get_params(), dtype=torch.float64, device=engine.default_device())[:, None]
                lp, g, H, st = fd_logp_grad_metric(self, obs, x, rel_step=rel_step)
                if int(st[0].item()) == 2:
                    raise Encounter("Two particles had a close encounter (d<exit_min_distance).")
                self.logp = float(lp[0].item())
                self.logp_d = g[:, 0].cpu().numpy()
                self.logp_dd = H[:, :, 0].cpu().numpy()
            elif method == "exact":
                chi, chi_d, chi_dd = self.get_chi2_d_dd(obs)
                self.logp, self.logp_d, self.logp_dd = -chi, -chi_d, -chi_dd
            else:
                raise ValueError("method must be 'exact' or 'fd'")
        return self.logp, self.logp_d, self.logp_dd

"""SMALA (simplified manifold MALA with the SoftAbs metric), mcmc.py:126-187.

The reference takes logp, its gradient and its Hessian from REBOUND's 1st/2nd-order variational
equations (state.py:229-294).  Here (north-star: "SMALA with finite-difference grad logL") every
derivative comes from ONE batched likelihood launch over the central-difference stencil
(2P+1 parameter vectors per chain, `rvm_fd_params`):

  grad_p logp  = (logp(x + e_p) - logp(x - e_p)) / (2 e_p)
  J[e, p]      = (rv_e(x + e_p) - rv_e(x - e_p)) / (2 e_p)      (per-epoch model RV Jacobian)
  H            = -(2 / Npoints) J^T diag(1/sigma^2) J          (Gauss-Newton Hessian of logp)

The SoftAbs metric G = Q diag(lambda coth(alpha lambda)) Q^T of eig(-H) (mcmc.py:135-139), the
drift mu = x + eps^2/2 G^-1 grad, the proposal x* = mu + eps chol(G^-1) z, and the Gaussian
q-ratio (mcmc.py:144-187) follow the reference.  The Gauss-Newton Hessian drops the
residual * d2rv term of the exact Hessian, so per-step parity with the reference SMALA is not
defined; parity is statistical.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib, engine

# relative FD step and per-key absolute floors (h, k and l can be ~0)
FD_REL_STEP = 1e-6
FD_FLOOR = {"m": 1e-4, "a": 1e-2, "h": 1e-2, "k": 1e-2, "l": 1.0, "ix": 1e-2, "iy": 1e-2}


def _torch():
    import torch

    return torch


def fd_floor_vector(state):
    return np.array([FD_FLOOR.get(k, 1e-2) for k in state.get_rawkeys()], dtype=np.float64)


def fd_logp_grad_metric(state, obs, X, rel_step=FD_REL_STEP, pmap=None, hill_factor=None):
    """X: [P][C] float64 device tensor -> (logp[C], grad[P][C], H[P][P][C], status[C])."""
    torch = _torch()
    lib = _lib.load()
    P, C_ = X.shape
    pmap = pmap or state.param_map()
    fl = torch.as_tensor(fd_floor_vector(state), device=X.device)
    S = 2 * P + 1
    stencil = torch.empty((P, S * C_), dtype=torch.float64, device=X.device)
    _lib.check(lib.rvm_fd_params(P, C_, X.contiguous().data_ptr(), float(rel_step), fl.data_ptr(),
                                 stencil.data_ptr(), _lib.stream_handle()), "rvm_fd_params")
    # the stencil on the fixed-step plan (every point of a chain with the same steps:
    # SmalaChains._fixed_plan), the centres' logp from the adaptive one
    it = state.integrator
    dt, mult, hint = it.plan_args(state.planets)
    plan = engine.plan_for(obs, len(state.planets), dt, mult, S * C_, X.device, hint, engine.is_inclined(state.planets),
                           (0.0, 0))
    hf = state.hillRadiusFactor if hill_factor is None else hill_factor
    lp, st, rv = plan.logl(pmap.to_kernel(stencil), hill_factor=hf, want_rv=True)
    if it.resolve()[0] > 0.0:
        lpc, stc, _ = state.get_logp_batch(obs, X.contiguous(), hill_factor=hill_factor, pmap=pmap)
        lp[:C_].copy_(lpc)
        st[:C_].copy_(stc)
    lp = lp.view(S, C_)
    st = st.view(S, C_)
    rv = rv.view(-1, S, C_)
    ax = torch.maximum(X.abs(), fl[:, None])
    eps = rel_step * ax                                       # [P][C]
    # the stencil kernel forms x +/- eps exactly as below; use the realised step for the divisor
    xp = X + eps
    xm = X - eps
    den = (xp - xm)                                           # [P][C]
    idx_p = torch.arange(P, device=X.device) * 2 + 1
    grad = (lp[idx_p] - lp[idx_p + 1]) / den                  # [P][C]
    J = (rv[:, idx_p, :] - rv[:, idx_p + 1, :]) / den[None]   # [E][P][C]
    t, rvo, er = engine.obs_arrays(obs)
    w = torch.as_tensor(1.0 / (er * er), device=X.device)     # [E]
    H = -(2.0 / float(obs.Npoints)) * torch.einsum("epc,e,eqc->pqc", J, w, J)
    # a chain is usable only if its whole stencil evaluated cleanly
    bad = (st != 0).any(0)
    status = torch.where(bad, torch.where(st[0] != 0, st[0], torch.full_like(st[0], 2)), st[0])
    return lp[0], grad, H, status


class SmalaChains:
    """C independent SMALA chains on the device (config 4: 256 chains).

    Per step (mcmc.py:167-187 for every chain at once): rvm_smala_propose, one likelihood launch
    over the (2P+1)-point stencil of the proposals (rvm_fd_params + rvm_logl_batch with rv_out),
    rvm_smala_derive (gradient, Gauss-Newton Hessian, SoftAbs metric by a per-chain Jacobi
    eigen-solver, Cholesky, drift) and rvm_smala_accept.  No host synchronisation in step().

    hessian="exact": the reference's metric -- exact gradient and Hessian of logp from
    rvm_logl_derivs (state.py:253-294) and rvm_smala_metric -- instead of the FD stencil and the
    Gauss-Newton Hessian (BASELINE config 4 names the FD variant)."""

    def __init__(self, initial_state, obs, eps, alpha, n_chains, X0=None, seed=0, device=None, rel_step=FD_REL_STEP,
                 hessian="gauss-newton"):
        torch = _torch()
        self.state = initial_state.deepcopy()
        self.obs = obs
        self.eps = float(eps)
        self.alpha = float(alpha)
        self.P = self.state.Nvars
        if self.P > _lib.RVM_SMALA_MAX_PARAMS:
            raise ValueError(f"SMALA supports at most {_lib.RVM_SMALA_MAX_PARAMS} free parameters")
        self.n = int(n_chains)
        if hessian not in ("gauss-newton", "exact"):
            raise ValueError("hessian must be 'gauss-newton' or 'exact'")
        self.hessian = hessian
        self.rel_step = float(rel_step)
        self.seed = int(seed)
        self.device = torch.device(device) if device is not None else engine.default_device()
        self.lib = _lib.load()
        self.pmap = self.state.param_map()
        self.floor = torch.as_tensor(fd_floor_vector(self.state), device=self.device)
        _, _, er = engine.obs_arrays(obs)
        self.inv_sigma2 = torch.as_tensor(1.0 / (er * er), device=self.device)
        self.n_obs = len(er)
        if X0 is None:
            X0 = np.tile(self.state.get_params()[:, None], (1, self.n))
        self.X = torch.as_tensor(np.asarray(X0, dtype=np.float64), device=self.device).contiguous()
        S = 2 * self.P + 1
        self.stencil = torch.empty((self.P, S * self.n), dtype=torch.float64, device=self.device)
        self.Xs = torch.empty_like(self.X)
        self.cache = self._new_cache()
        self.prop = self._new_cache()
        self.accepted = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        self.failures = torch.zeros(self.n, dtype=torch.int32, device=self.device)
        self.iteration = 0
        self._derive_into(self.X, self.cache)

    def _new_cache(self):
        torch = _torch()
        P, C, dev = self.P, self.n, self.device
        d = dict(lp=torch.empty(C, dtype=torch.float64, device=dev),
                 grad=torch.empty((P, C), dtype=torch.float64, device=dev),
                 mu=torch.empty((P, C), dtype=torch.float64, device=dev),
                 L=torch.empty((P * P, C), dtype=torch.float64, device=dev),
                 G=torch.empty((P * P, C), dtype=torch.float64, device=dev),
                 logdet=torch.empty(C, dtype=torch.float64, device=dev),
                 ok=torch.zeros(C, dtype=torch.int32, device=dev))
        d["_c"] = _lib.SmalaCache(*[d[k].data_ptr() for k in ("lp", "grad", "mu", "L", "G", "logdet", "ok")])
        return d

    def _fixed_plan(self, max_walkers):
        """The plan of the stencil's neighbour points: the state's integrator with the adaptive
        resolution off.  Finite differences need every point of a chain's stencil integrated with
        the same steps -- a refinement of some points but not others (per-walker decisions) would
        put the resolution's change, up to the bound, into the difference quotient -- and the
        gradient and metric only shape the proposal (the MH test keeps the target exact); the
        chain's logp itself comes from the adaptive plan (_center_logl)."""
        it = self.state.integrator
        dt, mult, hint = it.plan_args(self.state.planets)
        return engine.plan_for(self.obs, len(self.state.planets), dt, mult, max_walkers, self.device, hint,
                               engine.is_inclined(self.state.planets), (0.0, 0))

    def _center_plan(self):
        """The adaptive plan of the chains' own logp (on the side stream: _center_start), created at
        the size the centre launch needs and kept, so its fault counters are the ones read."""
        torch = _torch()
        if getattr(self, "_side", None) is None:
            self._side = torch.cuda.Stream(device=self.device)
        with torch.cuda.stream(self._side):
            self._cplan = self.state._plan(self.obs, max_walkers=self.n, device=self.device)
        return self._cplan

    def _center_start(self, X):
        """Start the centres' logp on the adaptive plan (T2: the value the accept test uses) on a
        side stream, concurrently with the stencil launch on the fixed-step plan: both launches are
        latency-bound and together fill a fraction of the CUs, so the centres' main pass, extension
        and halving passes hide behind the stencil.  Returns what _center_join needs (None when the
        resolution is off: the stencil's own centre values are the fixed-step logp)."""
        torch = _torch()
        if self.state.integrator.resolve()[0] <= 0.0:
            return None
        plan = self._center_plan()
        main = torch.cuda.current_stream(self.device)
        ready = torch.cuda.Event()
        ready.record(main)
        with torch.cuda.stream(self._side):
            self._side.wait_event(ready)
            lpc, stc, _ = plan.logl(self.pmap.to_kernel(X), hill_factor=1.0)
            done = torch.cuda.Event()
            done.record(self._side)
        return lpc, stc, done

    def _center_join(self, pending, lp, st):
        """Overwrite the stencil centres' logp / status (walkers 0 .. C-1) with the side stream's."""
        if pending is None:
            return
        torch = _torch()
        lpc, stc, done = pending
        main = torch.cuda.current_stream(self.device)
        main.wait_event(done)
        lp[:self.n].copy_(lpc)
        st[:self.n].copy_(stc)
        lpc.record_stream(main)  # (allocated on the side stream, last read on this one)
        stc.record_stream(main)

    def _center_logl(self, X, lp, st):
        self._center_join(self._center_start(X), lp, st)

    def _stencil_logl(self, X, fused=True, join=True):
        """logp, status [(2P+1) C] and model RVs [n_obs][(2P+1) C] over the central-difference
        stencil of X: one launch that forms the stencil in the likelihood kernel's prologue
        (rvm_smala_stencil_logl), or rvm_fd_params + rvm_logl_batch (fused=False; same bits), both
        on the fixed-step plan (_fixed_plan); the centres' logp then from the adaptive plan
        (join=False, fused only: not copied in; returned as the pending launch, or None)."""
        torch = _torch()
        S = 2 * self.P + 1
        plan = self._fixed_plan(S * self.n)
        pending = self._center_start(X)
        if not fused:
            _lib.check(self.lib.rvm_fd_params(self.P, self.n, X.data_ptr(), self.rel_step, self.floor.data_ptr(),
                                              self.stencil.data_ptr(), _lib.stream_handle()), "rvm_fd_params")
            lp, st, rv = plan.logl(self.pmap.to_kernel(self.stencil), hill_factor=1.0, want_rv=True)
            self._plan_keep = plan
            self._center_join(pending, lp, st)
            return lp, st, rv
        if getattr(self, "_st_bufs", None) is None:
            self._st_bufs = (torch.empty(S * self.n, dtype=torch.float64, device=self.device),
                             torch.empty(S * self.n, dtype=torch.int32, device=self.device),
                             torch.empty((self.n_obs, S * self.n), dtype=torch.float64, device=self.device))
        lp, st, rv = self._st_bufs
        with torch.cuda.device(self.device):
            _lib.check(self.lib.rvm_smala_stencil_logl(plan._h, C.byref(self.pmap.c_map()), self.P, self.n,
                                                       X.data_ptr(), self.rel_step, self.floor.data_ptr(), 1.0,
                                                       lp.data_ptr(), st.data_ptr(), rv.data_ptr(),
                                                       _lib.stream_handle()), "rvm_smala_stencil_logl")
        self._plan_keep = plan  # the launch's plan stays alive with the sampler
        if not join:
            return lp, st, rv, pending
        self._center_join(pending, lp, st)
        return lp, st, rv

    def _derive_into(self, X, cache, fused=True):
        st_h = _lib.stream_handle()
        if self.hessian == "exact":
            pending = self._center_start(X)  # (the adaptive logp beside the derivative launch)
            lp, g, H, st = self.state.get_logp_d_dd_batch(self.obs, X, hill_factor=1.0, pmap=self.pmap)
            self._center_join(pending, lp, st)
            _lib.check(self.lib.rvm_smala_metric(self.P, self.n, X.data_ptr(), lp.data_ptr(), st.data_ptr(),
                                                 g.data_ptr(), H.data_ptr(), self.alpha, self.eps,
                                                 C.byref(cache["_c"]), st_h), "rvm_smala_metric")
            self._keep = (lp, g, H, st)  # alive until the stream has consumed them
            return
        lp, st, rv = self._stencil_logl(X, fused)
        _lib.check(self.lib.rvm_smala_derive(self.P, self.n, self.n_obs, X.data_ptr(), self.rel_step,
                                             self.floor.data_ptr(), lp.data_ptr(), st.data_ptr(), rv.data_ptr(),
                                             self.inv_sigma2.data_ptr(), float(self.obs.Npoints), self.alpha,
                                             self.eps, C.byref(cache["_c"]), st_h), "rvm_smala_derive")

    def checkpoint(self, path):
        """Chains, counters, iteration and seed to an .npz.  The per-chain derivative caches are not
        stored: restore() re-derives them from the chains (the same launches, so the same values)."""
        np.savez(path, X=self.X.cpu().numpy(), accepted=self.accepted.cpu().numpy(),
                 failures=self.failures.cpu().numpy(), iteration=self.iteration, seed=self.seed, eps=self.eps,
                 alpha=self.alpha, hessian=self.hessian)

    def restore(self, path):
        torch = _torch()
        d = np.load(path)
        if d["X"].shape != tuple(self.X.shape) or str(d["hessian"]) != self.hessian:
            raise ValueError("checkpoint was written for a different sampler configuration")
        self.X = torch.as_tensor(d["X"], device=self.device).contiguous()
        self.accepted = torch.as_tensor(d["accepted"], device=self.device).contiguous()
        self.failures = torch.as_tensor(d["failures"], device=self.device).contiguous()
        self.iteration, self.seed = int(d["iteration"]), int(d["seed"])
        self.eps, self.alpha = float(d["eps"]), float(d["alpha"])
        self._derive_into(self.X, self.cache)

    @property
    def linalg_failures(self):
        return int(self.failures.sum().item())

    def step(self, z=None, u=None, fused=True):
        """One SMALA step of every chain; z [C][P] / u [C] inject the normals / uniforms.

        fused=True (default): three launches -- rvm_smala_propose, the stencil likelihood launch
        (rvm_smala_stencil_logl; exact: rvm_logl_derivs) and rvm_smala_derive_accept
        (rvm_smala_metric_accept) -- with the centres on the adaptive plan, rvm_smala_derive_sides
        beside the centres' launch and rvm_smala_center_accept after it; fused=False runs the separate
        fd / logl / derive / accept launches (bit-identical; 256 chains: 523k vs 485k chain-steps/s fused vs separate,
        profiles/r02h_configs.jsonl).  The plan is looked up per step for the current stream
        (State._plan -> engine.plan_for), so any stream is safe."""
        st_h = _lib.stream_handle()
        zp = 0
        if z is not None:
            self._z = z.t().contiguous()
            zp = self._z.data_ptr()
        up = 0
        if u is not None:
            self._u = u.contiguous()
            up = self._u.data_ptr()
        _lib.check(self.lib.rvm_smala_propose(self.P, self.n, 0, self.X.data_ptr(), C.byref(self.cache["_c"]),
                                              self.eps, self.seed, self.iteration, zp, self.Xs.data_ptr(), st_h),
                   "rvm_smala_propose")
        cur, prop = C.byref(self.cache["_c"]), C.byref(self.prop["_c"])
        if fused and self.hessian == "exact":
            pending = self._center_start(self.Xs)  # (the logp the accept uses: adaptive resolution)
            lp, g, H, st = self.state.get_logp_d_dd_batch(self.obs, self.Xs, hill_factor=1.0, pmap=self.pmap)
            self._center_join(pending, lp, st)
            _lib.check(self.lib.rvm_smala_metric_accept(self.P, self.n, 0, self.X.data_ptr(), self.Xs.data_ptr(),
                                                        lp.data_ptr(), st.data_ptr(), g.data_ptr(), H.data_ptr(),
                                                        self.alpha, self.eps, cur, prop, self.seed, self.iteration,
                                                        up, self.accepted.data_ptr(), self.failures.data_ptr(),
                                                        st_h), "rvm_smala_metric_accept")
            self._keep = (lp, g, H, st)
            self.iteration += 1
            self._periodic_faults()
            return
        if fused:
            lp, st, rv, pending = self._stencil_logl(self.Xs, join=False)
            if pending is not None:
                # the proposal's derivatives and metric from the stencil's sides while the centres'
                # adaptive launch (and its halving passes) still runs on the side stream; the accept
                # once it is done, with the centres' own logp and status (no copies; same bits)
                torch = _torch()
                _lib.check(self.lib.rvm_smala_derive_sides(
                    self.P, self.n, self.n_obs, self.Xs.data_ptr(), self.rel_step, self.floor.data_ptr(),
                    lp.data_ptr(), st.data_ptr(), rv.data_ptr(), self.inv_sigma2.data_ptr(),
                    float(self.obs.Npoints), self.alpha, self.eps, prop, st_h), "rvm_smala_derive_sides")
                lpc, stc, done = pending
                main = torch.cuda.current_stream(self.device)
                main.wait_event(done)
                _lib.check(self.lib.rvm_smala_center_accept(
                    self.P, self.n, 0, self.X.data_ptr(), self.Xs.data_ptr(), lpc.data_ptr(), stc.data_ptr(), cur,
                    prop, self.eps, self.seed, self.iteration, up, self.accepted.data_ptr(),
                    self.failures.data_ptr(), st_h), "rvm_smala_center_accept")
                lpc.record_stream(main)  # (allocated on the side stream, last read on this one)
                stc.record_stream(main)
                self.iteration += 1
                self._periodic_faults()
                return
            _lib.check(self.lib.rvm_smala_derive_accept(
                self.P, self.n, 0, self.n_obs, self.X.data_ptr(), self.Xs.data_ptr(), self.rel_step,
                self.floor.data_ptr(), lp.data_ptr(), st.data_ptr(), rv.data_ptr(), self.inv_sigma2.data_ptr(),
                float(self.obs.Npoints), self.alpha, self.eps, cur, prop, self.seed, self.iteration, up,
                self.accepted.data_ptr(), self.failures.data_ptr(), st_h), "rvm_smala_derive_accept")
            self.iteration += 1
            self._periodic_faults()
            return
        self._derive_into(self.Xs, self.prop, fused=False)
        _lib.check(self.lib.rvm_smala_accept(self.P, self.n, 0, self.X.data_ptr(), C.byref(self.cache["_c"]),
                                             self.Xs.data_ptr(), C.byref(self.prop["_c"]), self.eps, self.seed,
                                             self.iteration, up, self.accepted.data_ptr(), self.failures.data_ptr(),
                                             st_h), "rvm_smala_accept")
        self.iteration += 1
        self._periodic_faults()


    def _periodic_faults(self):  # (engine.periodic_fault_check over both plans)
        every = getattr(self, "fault_check_every", engine.FAULT_CHECK_EVERY)
        if every and self.iteration % every == 0:
            self.check_faults()

    def check_faults(self):
        """rvm_plan_faults of the chains' plans (the centres' adaptive one, on its side stream, and the
        stencil's fixed-step one): raises on hand-off timeouts / NONFINITE / UNRESOLVED results;
        returns the adaptive plan's counters."""
        torch = _torch()
        name = type(self).__name__
        if self.hessian == "gauss-newton":
            self._fixed_plan((2 * self.P + 1) * self.n).check_faults(name)
        if self.state.integrator.resolve()[0] <= 0.0:
            self.last_faults = {}
            return self.last_faults
        plan = getattr(self, "_cplan", None) or self._center_plan()
        with torch.cuda.stream(self._side):
            self.last_faults = plan.check_faults(name)
        return self.last_faults


class Smala:
    """mcmc.py:126-187 with the reference's host-side control flow and numpy global RNG."""

    def __init__(self, initial_state, obs, eps, alp):
        from .mcmc import Mcmc  # noqa: F401 (class hierarchy mirrors the reference)

        self.state = initial_state.deepcopy()
        self.obs = obs
        self.epsilon = eps
        self.alpha = alp

    def step_force(self):
        tries = 1
        while self.step() == False:  # noqa: E712
            tries += 1
        return tries

    def softabs(self, hessians):  # mcmc.py:135-139
        lam, Q = np.linalg.eigh(-0.5 * (hessians + hessians.T))
        with np.errstate(divide="ignore", invalid="ignore"):
            lam_twig = np.where(np.abs(self.alpha * lam) < 1e-8, 1.0 / self.alpha, lam * 1. / np.tanh(self.alpha * lam))
        return np.dot(Q, np.dot(np.diag(lam_twig), Q.T))

    def generate_proposal(self):  # mcmc.py:144-153
        logp, logp_d, logp_dd = self.state.get_logp_d_dd(self.obs)
        Ginv = np.linalg.inv(self.softabs(logp_dd))
        Ginvsqrt = np.linalg.cholesky(Ginv)
        mu = self.state.get_params() + (self.epsilon) ** 2 * np.dot(Ginv, logp_d) / 2.
        newparams = mu + self.epsilon * np.dot(Ginvsqrt, np.random.normal(0., 1., self.state.Nvars))
        prop = self.state.deepcopy()
        prop.set_params(newparams)
        return prop

    def transitionProbability(self, state_from, state_to):  # mcmc.py:158-162
        from scipy import stats

        logp, logp_d, logp_dd = state_from.get_logp_d_dd(self.obs)
        Ginv = np.linalg.inv(self.softabs(logp_dd))
        mu = state_from.get_params() + (self.epsilon) ** 2 * np.dot(Ginv, logp_d) / 2.
        return stats.multivariate_normal.logpdf(state_to.get_params(), mean=mu, cov=(self.epsilon) ** 2 * Ginv)

    def step(self):  # mcmc.py:167-187
        from .state import Encounter

        try:
            stateStar = self.generate_proposal()
            if stateStar.priorHard():
                return False
            q_ts_t = self.transitionProbability(self.state, stateStar)
            q_t_ts = self.transitionProbability(stateStar, self.state)
        except Encounter:
            return False
        except np.linalg.LinAlgError:
            return False  # the reference quit()s the process here (mcmc.py:179-183); we reject
        if np.exp(stateStar.logp - self.state.logp + q_t_ts - q_ts_t) > np.random.uniform():
            self.state = stateStar
            return True
        return False


class Alsmala(Smala):
    """mcmc.py:191-230: SMALA whose cheap "MALA" step reuses the current state's derivatives --
    the proposal inherits logp_d / logp_dd, only its logp is evaluated (one likelihood launch
    instead of a derivative launch).  driver.run_alsmala mixes the two steps with probability
    exp(-bern_a i / Niter) of a full SMALA step.  As in the reference, a state accepted by the
    cheap step keeps the inherited (stale) derivatives, and get_logp_d_dd returns them while its
    logp is cached."""

    def generate_proposal_mala(self):  # mcmc.py:195-206
        self.state.get_logp(self.obs)
        logp_d, logp_dd = self.state.logp_d, self.state.logp_dd
        Ginv = np.linalg.inv(self.softabs(logp_dd))
        Ginvsqrt = np.linalg.cholesky(Ginv)
        mu = self.state.get_params() + (self.epsilon) ** 2 * np.dot(Ginv, logp_d) / 2.
        newparams = mu + self.epsilon * np.dot(Ginvsqrt, np.random.normal(0., 1., self.state.Nvars))
        prop = self.state.deepcopy()
        prop.set_params(newparams)
        prop.logp_d = logp_d
        prop.logp_dd = logp_dd
        return prop

    def transitionProbability_mala(self, state_from, state_to):  # mcmc.py:208-212
        from scipy import stats

        state_from.get_logp(self.obs)
        logp_d, logp_dd = state_from.logp_d, state_from.logp_dd
        Ginv = np.linalg.inv(self.softabs(logp_dd))
        mu = state_from.get_params() + (self.epsilon) ** 2 * np.dot(Ginv, logp_d) / 2.
        return stats.multivariate_normal.logpdf(state_to.get_params(), mean=mu, cov=(self.epsilon) ** 2 * Ginv)

    def step_mala(self):  # mcmc.py:214-230
        from .state import Encounter

        if self.state.logp_d is None:  # no derivatives yet: the reference would fail on None
            self.state.get_logp_d_dd(self.obs)
        try:
            stateStar = self.generate_proposal_mala()
            if stateStar.priorHard():
                return False
            q_ts_t = self.transitionProbability_mala(self.state, stateStar)
            q_t_ts = self.transitionProbability_mala(stateStar, self.state)
        except Encounter:
            return False
        except np.linalg.LinAlgError:
            return False  # the reference quit()s (mcmc.py:226-229); we reject
        if np.exp(stateStar.logp - self.state.logp + q_t_ts - q_ts_t) > np.random.uniform():
            self.state = stateStar
            return True
        return False

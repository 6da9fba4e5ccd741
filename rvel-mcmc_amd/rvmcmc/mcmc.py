"""Samplers with the reference's API (mirror of /root/reference/mcmc.py), GPU underneath.

* Mcmc / step_force           mcmc.py:12-25
* lnprob(x, e)                mcmc.py:28-35   (scalar callback; any exception -> -inf)
* Ensemble                    mcmc.py:40-75   (emcee 2.2.1 stretch move; here the whole ensemble
                                               lives on the GPU, see ensemble.EnsembleSampler)
* Mh                          mcmc.py:80-121  (single chain, host RNG as the reference)
* Alsmala                     mcmc.py:191-230 (SMALA with cheap derivative-reusing MALA steps)
* Smala                       mcmc.py:126-187 (SoftAbs SMALA on State.get_logp_d_dd: exact
                                               derivatives, rvm_logl_derivs)
* MhChains                    batched independent MH chains on the device (new; the batched
                              counterpart of Mh, one logL launch per step for all chains)
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib, engine
from .ensemble import EnsembleSampler
from .state import Encounter


class Mcmc(object):
    def __init__(self, initial_state, obs):
        self.state = initial_state.deepcopy()  # NOTE: resets hillRadiusFactor to 1.0 (state.py:212-213)
        self.obs = obs

    def step(self):
        return True

    def step_force(self):
        tries = 1
        while self.step() == False:  # noqa: E712 (reference semantics)
            tries += 1
        return tries


def lnprob(x, e):
    """mcmc.py:28-35: emcee-style callback; every exception maps to -inf."""
    e.state.set_params(x)
    try:
        logp = e.state.get_logp(e.obs)
    except Exception:
        return -np.inf
    return logp


def _scales_vector(state, scales):
    """mcmc.py:70-75 / 98-103: dict keyed by parameter name -> vector; an array is taken as is."""
    if not isinstance(scales, dict):
        v = np.asarray(scales, dtype=np.float64)
        if v.shape != (state.Nvars,):
            raise ValueError("scales array must have Nvars entries")
        return v.copy()
    out = np.ones(state.Nvars)
    for i, k in enumerate(state.get_rawkeys()):
        if k in scales:
            out[i] = scales[k]
    return out


class Ensemble(Mcmc):
    """mcmc.py:40-75 -- same constructor and step() contract; emcee replaced by the device sampler."""

    def __init__(self, initial_state, obs, scales, nwalkers=10, seed=None):
        super(Ensemble, self).__init__(initial_state, obs)
        self.set_scales(scales)
        self.nwalkers = nwalkers
        self.states = [self.state.get_params() for i in range(nwalkers)]
        self.previous_states = [self.state.get_params() for i in range(nwalkers)]
        self.lnprob = None
        self.totalErrorCount = 0
        for i, s in enumerate(self.states):
            shift = 0.1e-2 * self.scales * np.random.normal(size=self.state.Nvars)
            self.states[i] += shift
        if seed is None:
            seed = int(np.random.randint(0, 2 ** 62))
        self.sampler = EnsembleSampler(nwalkers, self.state, obs, seed=seed)
        self.sampler.set_positions(np.array(self.states))

    def step(self):
        self.previous_states = self.states
        self.sampler.step()
        self.states = list(self.sampler.gather_positions())
        self.lnprob = self.sampler.gather_lnprob()
        for i in range(len(self.states)):
            for j in range(len(self.states[0])):
                if self.previous_states[i][j] != self.states[i][j]:
                    return True
        return False

    def set_scales(self, scales):
        self.scales = _scales_vector(self.state, scales)


class Mh(Mcmc):
    """mcmc.py:80-121 -- one chain, numpy global RNG in the reference's draw order.

    speculate = K > 1 (opt-in): the single chain is launch-latency-bound (one 1-walker likelihood
    launch per proposal), so K proposals are generated ahead -- with exactly the draws the
    sequential chain would make if they were all rejected (normal, then a uniform only for a
    proposal that passes priorHard) -- and evaluated in ONE launch.  step() then consumes them in
    order with the reference's test; at the first acceptance (or at an encounter, after which the
    reference draws no uniform) the rest is dropped and the global RNG is rewound to where the
    sequential chain would be.  The chain, the logp values and the RNG stream are bit-identical to
    speculate=1, provided nothing else draws from np.random between step() calls; flush() puts
    the RNG back where the sequential chain has it (e.g. after the last step)."""

    def __init__(self, initial_state, obs, speculate=1):
        super(Mh, self).__init__(initial_state, obs)
        self._buf = []
        self.step_size = 3e-5
        self.speculate = int(speculate)

    @property
    def step_size(self):
        return self._step_size

    @step_size.setter
    def step_size(self, v):
        self._step_size = v
        self._buf = []  # proposals drawn ahead used the old step size

    def generate_proposal(self):
        prop = self.state.deepcopy()
        shift = self.step_size * self.scales * np.random.normal(size=self.state.Nvars)
        prop.shift_params(shift)
        return prop

    def set_scales(self, scales):
        self.scales = _scales_vector(self.state, scales)
        self._buf = []

    def step(self):
        if self.speculate > 1:
            return self._step_speculative()
        while True:
            try:
                logp = self.state.get_logp(self.obs)
                proposal = self.generate_proposal()
                if proposal.priorHard():
                    return False
                logp_proposal = proposal.get_logp(self.obs)
                if np.exp(logp_proposal - logp) > np.random.uniform():
                    self.state = proposal
                    return True
                return False
            except Encounter:
                return False

    def flush(self):
        """Drop the proposals drawn ahead and put the global RNG where the sequential chain would
        have it (call before drawing from np.random yourself between steps)."""
        if self._buf:
            np.random.set_state(self._rng_consumed)
            self._buf = []

    def _fill(self):
        import torch

        self._base_logp = self.state.get_logp(self.obs)
        entries, live = [], []
        for _ in range(self.speculate):
            prop = self.generate_proposal()
            after_normal = np.random.get_state()
            if prop.priorHard():
                entries.append([prop, True, after_normal, None, None, 0])
                continue
            u = np.random.uniform()
            entries.append([prop, False, after_normal, u, np.random.get_state(), 0])
            live.append(entries[-1])
        # one launch per plan: a proposal's own scalar get_logp would use the plan of its own
        # (gridded) base step and resolution settings (its eccentricity guard included), so
        # proposals are grouped by the whole plan key to give bit-identical values
        groups = {}
        for e in live:
            it = e[0].integrator
            groups.setdefault((it.plan_args(e[0].planets), it.resolve(e[0].planets)), []).append(e)
        for grp in groups.values():
            X = torch.as_tensor(np.array([e[0].get_params() for e in grp]).T.copy(), device=engine.default_device())
            lp, st, _ = grp[0][0].get_logp_batch(self.obs, X)
            lp, st = lp.cpu().numpy(), st.cpu().numpy()
            for e, l, s_ in zip(grp, lp, st):
                e[0].logp = float(l)
                e[5] = int(s_)
        self._buf = entries

    def _step_speculative(self):
        if not self._buf:
            self._fill()
        prop, prior_bad, after_normal, u, after_u, status = self._buf.pop(0)
        self._rng_consumed = after_normal if prior_bad else after_u
        if prior_bad:
            return False
        if status == _lib.RVM_STATUS_ENCOUNTER:  # Encounter raised before the uniform is drawn
            np.random.set_state(after_normal)
            self._buf = []
            return False
        if np.exp(prop.logp - self._base_logp) > u:
            self.state = prop
            np.random.set_state(after_u)
            self._buf = []
            return True
        return False


class MhChains:
    """n_chains independent Gaussian random-walk MH chains, all resident on the device.

    Per step ONE launch for all chains (rvm_mh_step: the likelihood kernel forms each chain's
    proposal in its prologue and runs the accept on the lane that finishes the chain), or with
    injected draws a proposal kernel, one likelihood launch and an accept kernel (mcmc.py:89-121
    semantics per chain; priorHard / Encounter proposals are rejected through logp = -inf)."""

    def __init__(self, initial_state, obs, scales, step_size, n_chains, X0=None, seed=0, device=None):
        import torch

        self.state = initial_state.deepcopy()
        self.obs = obs
        self.dim = self.state.Nvars
        self.n = int(n_chains)
        self.step_size = float(step_size)
        self.seed = int(seed)
        self.iteration = 0
        self.device = torch.device(device) if device is not None else engine.default_device()
        self.lib = _lib.load()
        self.pmap = self.state.param_map()
        dt, mult, hint = self.state.integrator.plan_args(self.state.planets)
        self.plan = engine.plan_for(obs, self.pmap.n_planets, dt, mult, self.n, self.device, hint, self.pmap.inclined,
                                    self.state.integrator.resolve(self.state.planets))
        self.scales = torch.as_tensor(_scales_vector(self.state, scales), device=self.device)
        if X0 is None:
            X0 = np.tile(self.state.get_params()[:, None], (1, self.n))
        self.X = torch.as_tensor(np.asarray(X0, dtype=np.float64), device=self.device).contiguous()
        self.lnp, _, _ = self.plan.logl(self.pmap.to_kernel(self.X), hill_factor=self.state.hillRadiusFactor)
        self.lnp = self.lnp.clone()
        self.Q = torch.empty_like(self.X)
        self.accepted = torch.zeros(self.n, dtype=torch.int32, device=self.device)

    def checkpoint(self, path):
        """Chains, their logp, accept counters, iteration and seed to an .npz; a restored sampler
        continues bit-identically (Philox draws keyed by seed, iteration and chain)."""
        np.savez(path, X=self.X.cpu().numpy(), lnp=self.lnp.cpu().numpy(), accepted=self.accepted.cpu().numpy(),
                 iteration=self.iteration, seed=self.seed, step_size=self.step_size)

    def restore(self, path):
        import torch

        d = np.load(path)
        if d["X"].shape != tuple(self.X.shape):
            raise ValueError("checkpoint was written for a different number of chains or parameters")
        self.X = torch.as_tensor(d["X"], device=self.device).contiguous()
        self.lnp = torch.as_tensor(d["lnp"], device=self.device).contiguous()
        self.accepted = torch.as_tensor(d["accepted"], device=self.device).contiguous()
        self.iteration, self.seed, self.step_size = int(d["iteration"]), int(d["seed"]), float(d["step_size"])
        self.Q = torch.empty_like(self.X)

    def step(self, draws_propose=None, draws_accept=None, fused=True):
        """One MH step of every chain: (fused=True, the default, with Philox draws) ONE launch,
        rvm_mh_step: proposal, likelihood and accept fused; or (fused=False, or injected draws) the
        propose / likelihood / accept launches; bit-identical for the same draws.  In the
        level-split layout every level wave of a walker forms its proposal in its prologue; the
        walker's planet lanes share the Box-Muller draws (rvm_logl.hip), and the fused launch is
        ahead (4096 chains: 15.3-15.6M vs 14.8-15.1M chain-steps/s, profiles/r02h_configs.jsonl).
        On the stream the chains were built on (engine.check_stream)."""
        import torch

        engine.check_stream(self.plan, "MhChains.step")

        st = _lib.stream_handle()
        if fused and draws_propose is None and draws_accept is None:
            with torch.cuda.device(self.device):
                _lib.check(self.lib.rvm_mh_step(self.plan._h, C.byref(self.pmap.c_map()), self.dim, self.n, 0,
                                                self.X.data_ptr(), self.lnp.data_ptr(), self.scales.data_ptr(),
                                                self.step_size, self.seed, self.iteration,
                                                float(self.state.hillRadiusFactor), 0, 0, self.accepted.data_ptr(),
                                                st), "rvm_mh_step")
            self.iteration += 1
            engine.periodic_fault_check(self, self.plan)
            return
        _lib.check(self.lib.rvm_mh_propose(self.dim, self.n, 0, self.X.data_ptr(), self.scales.data_ptr(),
                                           self.step_size, self.seed, self.iteration,
                                           draws_propose.data_ptr() if draws_propose is not None else 0,
                                           self.Q.data_ptr(), st), "rvm_mh_propose")
        lnp_new, _, _ = self.plan.logl(self.pmap.to_kernel(self.Q), hill_factor=self.state.hillRadiusFactor)
        _lib.check(self.lib.rvm_mh_accept(self.dim, self.n, 0, self.X.data_ptr(), self.lnp.data_ptr(),
                                          self.Q.data_ptr(), lnp_new.data_ptr(), self.seed, self.iteration,
                                          draws_accept.data_ptr() if draws_accept is not None else 0,
                                          self.accepted.data_ptr(), st), "rvm_mh_accept")
        self.iteration += 1
        engine.periodic_fault_check(self, self.plan)

    def check_faults(self):
        """rvm_plan_faults of the chains' plan: raises on hand-off timeouts / NONFINITE results."""
        self.last_faults = self.plan.check_faults(type(self).__name__)
        return self.last_faults


from .smala import Alsmala, Smala, SmalaChains  # noqa: E402  (re-export with the reference's module layout)

__all__ = ["Mcmc", "lnprob", "Ensemble", "Mh", "MhChains", "Smala", "Alsmala", "SmalaChains", "EnsembleSampler"]

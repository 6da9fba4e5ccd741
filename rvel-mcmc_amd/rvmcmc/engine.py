"""Batched likelihood engine: torch device tensors in, the HIP kernel through the C ABI.

`LoglPlan` owns one `rvm_plan` (epoch schedule + observation data resident in HBM) and launches
`rvm_logl_batch` on the caller's current torch stream.  `ParamMap` maps a reference-style
`State` (dict-of-planets, free parameters in dict order, state.py:8-31 / 124-207) onto the
kernel's canonical SoA layout [5 * n_planets][n_walkers] with per-planet order m, a, h, k, l
(7 rows with ix, iy for inclined systems).
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib

KERNEL_KEYS = ("m", "a", "h", "k", "l")
KERNEL_KEYS_INCLINED = KERNEL_KEYS + ("ix", "iy")
SUPPORTED_KEYS = set(KERNEL_KEYS_INCLINED)


def level_multipliers(levels) -> tuple:
    """int n -> the harmonic sequence (1, ..., n); a sequence -> its distinct positive ints."""
    if isinstance(levels, (int, np.integer)):
        mult = tuple(range(1, int(levels) + 1))
    else:
        mult = tuple(int(m) for m in levels)
    if not 1 <= len(mult) <= _lib.RVM_MAX_LEVELS:
        raise ValueError(f"1..{_lib.RVM_MAX_LEVELS} Richardson levels supported, got {len(mult)}")
    if len(set(mult)) != len(mult) or min(mult) < 1 or max(mult) > 64:
        raise ValueError("level multipliers must be distinct integers in 1..64")
    return mult


DT_GRID = 16  # base-step grid points per factor of two (IntegratorConfig.step_for)
ECC_GRID = 64  # the eccentricity guard's reference eccentricity is rounded to multiples of 1/ECC_GRID


@dataclass(frozen=True)
class IntegratorConfig:
    """Wisdom-Holman + Richardson settings.

    steps_per_orbit: base steps per shortest orbital period of the reference state
                     (dt = P_min / steps_per_orbit) unless `dt` is given explicitly.
    levels:          Richardson level multipliers: level k integrates every epoch-to-epoch
                     segment with mult[k] x its base steps (step dt/mult[k]); an int n means the
                     harmonic sequence 1..n.  The default (4, 5, 6, 7) at steps_per_orbit = 8
                     (steps P/32 .. P/56) keeps |logL - logL_IAS15| <= ~2e-9 on the benchmark
                     configs (T2 tier; the tests enforce 5e-8) with the shortest longest-level
                     integration of the sequences we measured.
    """

    steps_per_orbit: float = 8.0
    levels: tuple = (4, 5, 6, 7)
    dt: Optional[float] = None
    # adaptive resolution (rvm_config.resolve_tol / resolve_max): a walker-direction
    # whose estimated extrapolation error exceeds resolve_tol / 2 (in logL) gets the extension level
    # and, if that does not settle it, passes with every step halved, up to resolve_max times -- the
    # plan's step is fixed from the sampler's initial state, the reference's IAS15 adapts to every
    # proposal.  Measured against IAS15 on the bench chain's own proposals (iteration 23 / 2000) and
    # a 0.6-wide ball: max |dlogL| 1.8e-7 / 7.0e-7 / 3.3e-7 with the eccentricity guard below (the
    # fixed step: 668 of 6144 steady-state proposals above 1e-6).  Cost on the bench (the extension
    # as a fifth level, certain rejects cut after it): 0.53 ms per iteration against 0.375 with the
    # fixed step; at the chain's steady state 6.2 ms against 0.69.  resolve_tol = 0
    # turns it off (the round-2 fixed-step algorithm).
    resolve_tol: float = 5e-7
    resolve_max: int = 12
    # eccentricity guard (rvm_plan_set_verify_eccentricity): walkers whose pericentre passage is more
    # than this factor quicker than the plan's reference orbit's always get the extension -- the
    # estimate under-read on such orbits (all three T2 misses it left at the bench chain's steady
    # state had e >= 0.295 against the reference's 0.218; the guard at 1.1 -> e > 0.266 removes them,
    # DESIGN.md §3).  0: off.
    verify_speedup: float = 1.1
    # certain-reject test (rvm_plan_set_certain_reject; fused sampler launches only): a proposal whose
    # accept test fails even at the upper bound on its logL that both directions' lower bounds on
    # chi2 give stops refining and is rejected.  The bound of an open direction is EMPIRICAL (chi2
    # less the change its last stage brought, capped at 100 x its estimate; measured error / estimate
    # <= 57, and no cut proposal was an IAS15 accept in the studies of DESIGN.md §3 item 5;
    # tests/test_ias15_parity_harness.py re-checks it on every CPU run).  False: every open walker
    # refines to the tolerance (slower at the steady state, no heuristic in the decision).
    certain_reject: bool = True

    @property
    def mult(self) -> tuple:
        return level_multipliers(self.levels)

    @property
    def n_levels(self) -> int:
        return len(self.mult)

    def step_for(self, planets) -> float:
        """Base step: P_min / steps_per_orbit rounded to the nearest point of the grid
        2^(k/DT_GRID) (within 2.2 % of nominal; the error scales as h^8, T2 margins cover it), so
        that the states a sampler visits share a few plans instead of one plan per state (the
        scalar State API builds its plan from the state's own orbits)."""
        if self.dt is not None:
            return float(self.dt)
        raw = min_period(planets) / float(self.steps_per_orbit)
        return 2.0 ** (round(math.log2(raw) * DT_GRID) / DT_GRID)

    def resolve(self, planets=None) -> tuple:
        """(resolve_tol, resolve_max, eccentricity guard, certain_reject) for plan_for / LoglPlan; the
        guard (0: off) from the plan's reference planets: the eccentricity whose pericentre passage is
        verify_speedup times quicker, (1 - e)^-3/2 = verify_speedup (1 - e_ref)^-3/2."""
        return float(self.resolve_tol), int(self.resolve_max), self.ecc_guard(planets), bool(self.certain_reject)

    def ecc_guard(self, planets) -> float:
        """The guard from the reference planets' largest eccentricity, rounded to the grid
        ECC_GRID (as step_for grids the step): the scalar State API plans from each state's own
        planets, and a guard that varied continuously would give every state a plan of its own."""
        if not planets or not (self.verify_speedup > 0.0) or not (self.resolve_tol > 0.0):
            return 0.0
        e_ref = max(float(np.hypot(p.get("h", 0.0), p.get("k", 0.0))) for p in planets)
        e_ref = round(e_ref * ECC_GRID) / ECC_GRID
        if not e_ref < 1.0:
            return 0.0
        return float(1.0 - (self.verify_speedup * (1.0 - e_ref) ** -1.5) ** (-2.0 / 3.0))

    def plan_args(self, planets):
        """(dt, level multipliers, period hint) for plan_for / LoglPlan; the hint (Stumpff series
        length per level: speed only) follows the gridded step, so it is shared as well."""
        dt = self.step_for(planets)
        hint = dt * float(self.steps_per_orbit) if self.dt is None else min_period(planets)
        return dt, self.mult, hint


def is_inclined(planets) -> bool:
    """An inclined plan is needed when any planet dict carries ix / iy (REBOUND adds z then)."""
    return any(("ix" in p) or ("iy" in p) for p in planets)


DEFAULT_CONFIG = IntegratorConfig()


def min_period(planets) -> float:
    """Shortest Keplerian period (code units, G = M_star = 1) of a list of planet dicts."""
    best = math.inf
    for p in planets:
        a = float(p["a"])
        m = float(p.get("m", 0.0))
        if a > 0:
            best = min(best, 2.0 * math.pi * math.sqrt(a ** 3 / (1.0 + max(m, 0.0))))
    if not math.isfinite(best):
        raise ValueError("cannot derive an integrator step: no planet with a > 0")
    return best


def _torch():
    import torch

    return torch


def default_device():
    torch = _torch()
    if not torch.cuda.is_available():
        raise _lib.RvmError("no HIP device visible: the likelihood runs only on the GPU (no CPU fallback)")
    return torch.device("cuda", torch.cuda.current_device())


class LoglPlan:
    """rvm_plan for one observation set on one device."""

    def __init__(self, t, rv, sigma, npoints, n_planets, dt, levels=4, max_walkers=4096, device=None,
                 period_hint=0.0, inclined=False, resolve=(0.0, 0)):
        torch = _torch()
        self.lib = _lib.load()
        self.device = torch.device(device) if device is not None else default_device()
        t = np.ascontiguousarray(np.asarray(t, dtype=np.float64))
        rv = np.ascontiguousarray(np.asarray(rv, dtype=np.float64))
        sigma = np.ascontiguousarray(np.asarray(sigma, dtype=np.float64))
        if not (len(t) == len(rv) == len(sigma)):
            raise ValueError("t, rv and sigma must have the same length")
        self.n_obs = len(t)
        self.n_planets = int(n_planets)
        self.dt = float(dt)
        self.mult = level_multipliers(levels)
        self.n_levels = len(self.mult)
        self.period_hint = float(period_hint)
        self.inclined = bool(inclined)
        self.rows = (7 if self.inclined else 5) * self.n_planets
        self.npoints = float(npoints)
        self.max_walkers = int(max_walkers)
        self.resolve_tol, self.resolve_max = float(resolve[0]), int(resolve[1])
        self.ecc_guard = float(resolve[2]) if len(resolve) > 2 else 0.0
        self.certain_reject = bool(resolve[3]) if len(resolve) > 3 else True
        lm = (C.c_int32 * _lib.RVM_MAX_LEVELS)(*self.mult)
        cfg = _lib.RvmConfig(self.n_planets, self.dt, self.n_levels, self.npoints, lm, self.period_hint,
                             int(self.inclined), self.resolve_tol, self.resolve_max)
        handle = C.c_void_p()
        dp = C.POINTER(C.c_double)
        with torch.cuda.device(self.device):
            rc = self.lib.rvm_plan_create(C.byref(cfg), t.ctypes.data_as(dp), rv.ctypes.data_as(dp),
                                          sigma.ctypes.data_as(dp), self.n_obs, self.max_walkers, C.byref(handle))
        _lib.check(rc, "rvm_plan_create")
        self._h = handle
        ext = C.c_int32()
        _lib.check(self.lib.rvm_plan_extension(self._h, C.byref(ext)), "rvm_plan_extension")
        self.ext_mult = ext.value  # the adaptive resolution's extension level (0: none)
        if self.ecc_guard > 0.0:
            _lib.check(self.lib.rvm_plan_set_verify_eccentricity(self._h, self.ecc_guard),
                       "rvm_plan_set_verify_eccentricity")
        if not self.certain_reject:
            _lib.check(self.lib.rvm_plan_set_certain_reject(self._h, 0), "rvm_plan_set_certain_reject")

    def faults(self, reset=False, stream=None) -> dict:
        """rvm_plan_counters: the plan's counters (synchronises the stream): hand-off timeouts, NONFINITE
        and UNRESOLVED results, refinement passes, refinements cut short on a certain reject,
        directions settled at their roundoff floor; reset=True zeroes them and restores the hand-off
        workspace."""
        vals = (C.c_int64 * _lib.RVM_N_COUNTERS)()
        _lib.check(self.lib.rvm_plan_counters(self._h, int(bool(reset)), vals, _lib.RVM_N_COUNTERS,
                                              _lib.stream_handle(stream)), "rvm_plan_counters")
        f = dict(handoff_timeouts=vals[0], nonfinite=vals[1], unresolved=vals[2], refined=vals[3],
                 truncated=vals[4], floor_settled=vals[5], skipped=vals[6])
        if reset:  # (running totals over every reset: the samplers' periodic checks reset the counters)
            tot = self.__dict__.setdefault("totals", dict.fromkeys(f, 0))
            for k, v in f.items():
                tot[k] += v
        return f

    def check_faults(self, what="plan", stream=None, group=None) -> dict:
        """Raise RvmError on hand-off timeouts, NONFINITE results, or (a plan that refines, resolve_max
        > 0) UNRESOLVED results since the last check: emcee raises on a NaN log-probability
        (mcmc.py:28-35 / emcee 2.2.1), and neither a stalled hand-off nor a walker the adaptive
        resolution could not bring within its bound may pass as an ordinary rejection.  Returns the
        counters (then reset).  group: a torch.distributed group whose ranks check together (the
        counts are summed over it, so every rank raises, or none -- a rank raising alone would leave
        the others blocked in the sampler's next collective)."""
        f = self.faults(reset=True, stream=stream)
        bad = [f["handoff_timeouts"], f["nonfinite"], f["unresolved"] if self.resolve_max > 0 else 0]
        if group is not None:
            torch = _torch()
            dist = torch.distributed
            dev = self.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
            t = torch.tensor(bad, dtype=torch.int64, device=dev)
            dist.all_reduce(t, group=group)
            bad = [int(v) for v in t.cpu()]
        if any(bad):
            raise _lib.RvmError(f"{what}: {bad[0]} level-split hand-off timeout(s), {bad[1]} non-finite "
                                f"log-likelihood(s), {bad[2]} walker(s) not resolved to the plan's tolerance after "
                                f"{self.resolve_max} halvings on the GPU (rvm_plan_faults"
                                f"{', summed over the ranks' if group is not None else ''})")
        return f

    def time_kernels(self, max_launches):
        """rvm_plan_time_kernels: the next max_launches evaluations on this plan record HIP events
        around their likelihood and refinement kernels (read with kernel_times)."""
        _lib.check(self.lib.rvm_plan_time_kernels(self._h, int(max_launches)), "rvm_plan_time_kernels")

    def kernel_times(self, max_launches=4096):
        """(likelihood kernel ms [n], refinement kernel ms [n]) of the evaluations timed since
        time_kernels (waits for them); timing stops."""
        a = (C.c_float * max_launches)()
        b = (C.c_float * max_launches)()
        n = C.c_int32()
        _lib.check(self.lib.rvm_plan_kernel_times(self._h, a, b, int(max_launches), C.byref(n)), "rvm_plan_kernel_times")
        return np.array(a[:n.value], dtype=np.float64), np.array(b[:n.value], dtype=np.float64)

    def set_handoff_timeout(self, seconds):
        _lib.check(self.lib.rvm_plan_set_handoff_timeout(self._h, float(seconds)), "rvm_plan_set_handoff_timeout")

    def info(self):
        vals = [C.c_int32() for _ in range(4)]
        _lib.check(self.lib.rvm_plan_info(self._h, *[C.byref(v) for v in vals]), "rvm_plan_info")
        return dict(steps_fwd=vals[0].value, steps_bwd=vals[1].value, epochs_fwd=vals[2].value,
                    epochs_bwd=vals[3].value)

    def logl(self, params, hill_factor=1.0, want_rv=False, out=None, status=None, rv_out=None, stream=None):
        """params: float64 device tensor [5*n_planets][W] ([7*n_planets][W] for an inclined plan) ->
        (logl[W], status[W], rv|None).

        rv (if requested) is [n_obs][W], rows in the plan's input epoch order."""
        torch = _torch()
        if params.dtype != torch.float64 or params.device != self.device or params.dim() != 2:
            raise ValueError("params must be a 2-D float64 tensor on the plan's device")
        if params.shape[0] != self.rows:
            raise ValueError(f"params must have {self.rows} rows (m,a,h,k,l{',ix,iy' if self.inclined else ''} "
                             f"per planet)")
        params = params.contiguous()
        W = params.shape[1]
        if W > self.max_walkers:
            raise ValueError(f"{W} walkers exceed the plan's max_walkers={self.max_walkers}")
        if out is None:
            out = torch.empty(W, dtype=torch.float64, device=self.device)
        if status is None:
            status = torch.empty(W, dtype=torch.int32, device=self.device)
        rvp = 0
        if want_rv:
            if rv_out is None:
                rv_out = torch.empty((self.n_obs, W), dtype=torch.float64, device=self.device)
            rvp = rv_out.data_ptr()
        with torch.cuda.device(self.device):
            rc = self.lib.rvm_logl_batch(self._h, W, params.data_ptr(), float(hill_factor), out.data_ptr(),
                                         status.data_ptr(), rvp, _lib.stream_handle(stream))
        _lib.check(rc, "rvm_logl_batch")
        return out, status, (rv_out if want_rv else None)

    def derivs(self, params, dir_rows, hill_factor=1.0, stream=None):
        """Exact logp, gradient and Hessian (rvm_logl_derivs; state.py:218-294 get_chi2_d_dd /
        get_logp_d_dd): params [rows][C] float64 device tensor, dir_rows = kernel rows of the
        free parameters (ParamMap.slots).  Returns (logl[C], grad[P][C], hess[P][P][C], status[C]);
        gradient and Hessian are NaN where status != 0."""
        torch = _torch()
        if params.dtype != torch.float64 or params.device != self.device or params.dim() != 2:
            raise ValueError("params must be a 2-D float64 tensor on the plan's device")
        if params.shape[0] != self.rows:
            raise ValueError(f"params must have {self.rows} rows")
        params = params.contiguous()
        C_ = params.shape[1]
        rows = np.ascontiguousarray(np.asarray(dir_rows, dtype=np.int32))
        P = len(rows)
        f64 = dict(dtype=torch.float64, device=self.device)
        lp = torch.empty(C_, **f64)
        grad = torch.empty((P, C_), **f64)
        hess = torch.empty((P, P, C_), **f64)
        st = torch.empty(C_, dtype=torch.int32, device=self.device)
        nb = int(self.lib.rvm_logl_derivs_workspace_bytes(C_, P))
        ws = torch.empty(max(nb, 8), dtype=torch.uint8, device=self.device)
        with torch.cuda.device(self.device):
            rc = self.lib.rvm_logl_derivs(self._h, C_, params.data_ptr(), P, rows.ctypes.data_as(C.POINTER(C.c_int32)),
                                          float(hill_factor), lp.data_ptr(), grad.data_ptr(), hess.data_ptr(),
                                          st.data_ptr(), ws.data_ptr(), _lib.stream_handle(stream))
        _lib.check(rc, "rvm_logl_derivs")
        return lp, grad, hess, st

    def stretch_half_step(self, pmap, X0, lnp0, c_aos, s0_begin, a, seed, iteration, half, hill_factor=1.0,
                          lnp_new=None, status=None, accepted=None, X0_aos=None, stream=None):
        """Fused emcee stretch half-step (rvm_stretch_half_step): propose against the complement
        c_aos [n1][dim] (walker-major), walker logL of the proposals, accept -- one launch.  X0
        [dim][n0] and lnp0 [n0] are updated in place, and X0_aos [n0][dim] (optional, the
        walker-major mirror of X0) too; lnp_new / status (optional) receive the proposals' logl."""
        torch = _torch()
        for t in (X0, lnp0, c_aos) + ((X0_aos,) if X0_aos is not None else ()):
            if t.dtype != torch.float64 or t.device != self.device or not t.is_contiguous():
                raise ValueError("X0, lnp0, c_aos, X0_aos must be contiguous float64 tensors on the plan's device")
        dim, n0 = X0.shape
        if c_aos.dim() != 2 or c_aos.shape[1] != dim or lnp0.shape != (n0,):
            raise ValueError("shape mismatch between X0 [dim][n0], lnp0 [n0] and c_aos [n1][dim]")
        if X0_aos is not None and X0_aos.shape != (n0, dim):
            raise ValueError("X0_aos must be [n0][dim]")
        if n0 > self.max_walkers:
            raise ValueError(f"{n0} walkers exceed the plan's max_walkers={self.max_walkers}")
        with torch.cuda.device(self.device):
            rc = self.lib.rvm_stretch_half_step(
                self._h, C.byref(pmap.c_map()), dim, n0, int(s0_begin), X0.data_ptr(),
                X0_aos.data_ptr() if X0_aos is not None else 0, lnp0.data_ptr(), c_aos.shape[0], c_aos.data_ptr(),
                float(a), int(seed), int(iteration), int(half), float(hill_factor),
                lnp_new.data_ptr() if lnp_new is not None else 0, status.data_ptr() if status is not None else 0,
                accepted.data_ptr() if accepted is not None else 0, _lib.stream_handle(stream))
        _lib.check(rc, "rvm_stretch_half_step")

    def stretch_iteration_begin(self, pmap, X0, lnp0, X1, c0_aos, c1_aos, s0_begin, s1_begin, a, seed, iteration,
                                lnp_spec, status_spec, dec, hill_factor=1.0, accepted0=None, stream=None, lnp1=None):
        """First launch of a speculative stretch iteration (rvm_stretch_iteration_begin): half 0's
        half-step (X0 [dim][n], lnp0 [n] updated in place, decisions to dec [n]) and half 1's
        proposals from X1 [dim][n] against both possible positions of their partners, logl of all
        3 n slots to lnp_spec / status_spec [3 n].  c0_aos / c1_aos: both halves walker-major
        [n_half][dim] as at the start of the iteration (unchanged until the end call).  lnp1 [n]
        (optional): half 1's log-probabilities, the accept inputs of its slots."""
        torch = _torch()
        for t in (X0, lnp0, X1, c0_aos, c1_aos, lnp_spec):
            if t.dtype != torch.float64 or t.device != self.device or not t.is_contiguous():
                raise ValueError("X0, lnp0, X1, c0_aos, c1_aos, lnp_spec must be contiguous float64 tensors on the "
                                 "plan's device")
        dim, n = X0.shape
        n_half = c0_aos.shape[0]
        if X1.shape != (dim, n) or lnp0.shape != (n,) or c0_aos.shape != (n_half, dim) or c1_aos.shape != (n_half, dim):
            raise ValueError("shape mismatch between X0/X1 [dim][n], lnp0 [n] and c0_aos/c1_aos [n_half][dim]")
        if lnp_spec.shape != (3 * n,) or status_spec.shape != (3 * n,) or dec.shape != (n,):
            raise ValueError("lnp_spec / status_spec must be [3 n], dec [n]")
        if lnp1 is not None and (lnp1.dtype != torch.float64 or lnp1.device != self.device or lnp1.shape != (n,)
                                 or not lnp1.is_contiguous()):
            raise ValueError("lnp1 must be a contiguous float64 [n] tensor on the plan's device")
        if status_spec.dtype != torch.int32 or dec.dtype != torch.int32:
            raise ValueError("status_spec and dec must be int32")
        if 3 * n > self.max_walkers:
            raise ValueError(f"3 x {n} walker slots exceed the plan's max_walkers={self.max_walkers}")
        with torch.cuda.device(self.device):
            rc = self.lib.rvm_stretch_iteration_begin(
                self._h, C.byref(pmap.c_map()), dim, n, int(s0_begin), int(s1_begin), X0.data_ptr(), lnp0.data_ptr(),
                X1.data_ptr(), lnp1.data_ptr() if lnp1 is not None else 0, n_half, c0_aos.data_ptr(), c1_aos.data_ptr(),
                float(a), int(seed), int(iteration),
                float(hill_factor), lnp_spec.data_ptr(), status_spec.data_ptr(), dec.data_ptr(),
                accepted0.data_ptr() if accepted0 is not None else 0, _lib.stream_handle(stream))
        _lib.check(rc, "rvm_stretch_iteration_begin")

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            self.lib.rvm_plan_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def stretch_iteration_end(X0, X0_aos, dec, dec_all, X1, X1_aos, lnp1, c0_aos, c1_aos, lnp_spec, status_spec,
                          s0_begin, s1_begin, a, seed, iteration, accepted1=None, lnp_new=None, status_new=None,
                          stream=None):
    """Second launch of a speculative stretch iteration (rvm_stretch_iteration_end): half 1's
    accepts with the logl variant its partner's decision (dec_all [n_half], global order)
    selects; X1 [dim][n], lnp1, the mirrors X0_aos / X1_aos [n][dim] (nullable) updated."""
    torch = _torch()
    lib = _lib.load()
    dim, n = X1.shape
    n_half = c0_aos.shape[0]
    if X0.shape != (dim, n) or lnp1.shape != (n,) or dec.shape != (n,) or dec_all.shape != (n_half,):
        raise ValueError("shape mismatch in stretch_iteration_end")
    for t in (X0_aos, X1_aos):
        if t is not None and t.shape != (n, dim):
            raise ValueError("mirrors must be [n][dim]")
    ptr = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
    with torch.cuda.device(X1.device):
        rc = lib.rvm_stretch_iteration_end(dim, n, int(s0_begin), int(s1_begin), X0.data_ptr(), ptr(X0_aos),
                                           dec.data_ptr(), dec_all.data_ptr(), X1.data_ptr(), ptr(X1_aos),
                                           lnp1.data_ptr(), n_half, c0_aos.data_ptr(), c1_aos.data_ptr(),
                                           lnp_spec.data_ptr(), status_spec.data_ptr(), float(a), int(seed),
                                           int(iteration), ptr(accepted1), ptr(lnp_new), ptr(status_new),
                                           _lib.stream_handle(stream))
    _lib.check(rc, "rvm_stretch_iteration_end")


def obs_arrays(obs):
    """Observation -> (t, rv, sigma) concatenated as tf then tb (rv_out rows follow this order)."""
    t = np.concatenate([np.asarray(obs.tf, dtype=np.float64), np.asarray(obs.tb, dtype=np.float64)])
    rv = np.concatenate([np.asarray(obs.rvf, dtype=np.float64), np.asarray(obs.rvb, dtype=np.float64)])
    er = np.concatenate([np.asarray(obs.errorf, dtype=np.float64), np.asarray(obs.errorb, dtype=np.float64)])
    return t, rv, er


FAULT_CHECK_EVERY = 256  # sampler iterations between automatic rvm_plan_faults checks (0: never)


def periodic_fault_check(sampler, plan):
    """Every `fault_check_every` iterations (a sampler attribute, default FAULT_CHECK_EVERY) read the
    plan's counters and raise on a hand-off timeout or a NONFINITE result (LoglPlan.check_faults):
    the check synchronises the stream, so it is amortised over many iterations rather than run per
    step; `sampler.check_faults()` runs it on demand."""
    every = getattr(sampler, "fault_check_every", FAULT_CHECK_EVERY)
    if plan is not None and every and sampler.iteration % every == 0:
        sampler.last_faults = plan.check_faults(type(sampler).__name__, group=fault_group(sampler))


def fault_group(sampler):
    """The process group whose ranks must check a sampler's faults together (None on one rank)."""
    return getattr(sampler, "group", None) if getattr(sampler, "world", 1) > 1 else None


PLAN_CACHE_SIZE = 32  # plans kept per observation set


def check_stream(plan, what="sampler"):
    """A sampler's plan came from plan_for on the stream current at its construction, and a plan's
    workspace (direction slots, hand-off slots) is single-stream: stepping the sampler from
    another stream could share that workspace with a concurrent launch.  Raise instead."""
    want = getattr(plan, "stream", None)
    if want is None or plan.device.type != "cuda":
        return
    cur = _torch().cuda.current_stream(plan.device).cuda_stream
    if int(cur) != want:
        raise RuntimeError(f"{what}: stepped on another stream than the one it was built on (its plan's "
                           f"workspace is single-stream, include/rvmcmc.h); build one sampler per stream")


def plan_for(obs, n_planets, dt, levels, max_walkers, device=None, period_hint=0.0, inclined=False,
             resolve=(0.0, 0)) -> LoglPlan:
    """Cached LoglPlan on an Observation object (keyed by device, the caller's current stream and
    the integrator settings: a plan's workspace is single-stream, include/rvmcmc.h)."""
    torch = _torch()
    dev = torch.device(device) if device is not None else default_device()
    cache = obs.__dict__.setdefault("_rvm_plans", {})
    mult = level_multipliers(levels)
    stream = torch.cuda.current_stream(dev).cuda_stream if dev.type == "cuda" else 0
    resolve = (float(resolve[0]), int(resolve[1]), float(resolve[2]) if len(resolve) > 2 else 0.0,
               bool(resolve[3]) if len(resolve) > 3 else True)
    key = (str(dev), int(stream), int(n_planets), float(dt), mult, float(period_hint), bool(inclined), resolve)
    plan = cache.pop(key, None)
    if plan is None or plan.max_walkers < max_walkers:
        t, rv, er = obs_arrays(obs)
        cap = max(int(max_walkers), plan.max_walkers * 2 if plan else 0, 64)
        plan = LoglPlan(t, rv, er, obs.Npoints, n_planets, dt, mult, cap, dev, period_hint, inclined, resolve)
        plan.stream = int(stream)
    cache[key] = plan  # most recently used last
    while len(cache) > PLAN_CACHE_SIZE:  # bounded: the least recently used plan is dropped (freed
        cache.pop(next(iter(cache)))      # when no sampler holds it any more)
    return plan


class ParamMap:
    """Free-parameter vectors of a State  <->  kernel SoA parameter blocks.

    The free parameters of a State are its planets' keys in dict order minus ignore_vars /
    ignore_params (state.py:26-31, 143-155).  The kernel wants every planet's m, a, h, k, l (and
    ix, iy when any planet carries an inclination key: an inclined plan); non-free values are
    taken from the State's planets (missing h/k/l/ix/iy default to 0 as REBOUND's Pal
    constructor does)."""

    def __init__(self, state):
        self.n_planets = len(state.planets)
        if not 1 <= self.n_planets <= _lib.RVM_MAX_PLANETS:
            raise ValueError(f"1..{_lib.RVM_MAX_PLANETS} planets supported, got {self.n_planets}")
        self.inclined = any(("ix" in p) or ("iy" in p) for p in state.planets)
        keys = KERNEL_KEYS_INCLINED if self.inclined else KERNEL_KEYS
        R = len(keys)
        self.rows_per_planet = R
        base = np.zeros(R * self.n_planets)
        for i, p in enumerate(state.planets):
            unknown = set(p.keys()) - SUPPORTED_KEYS
            if unknown:
                raise ValueError(f"planet {i}: unsupported keys {sorted(unknown)} (Pal elements m,a,h,k,l,ix,iy)")
            if "a" not in p:
                raise ValueError(f"planet {i}: 'a' is required")
            for j, k in enumerate(keys):
                base[R * i + j] = float(p.get(k, 0.0))
        self.base = base
        slots = []
        for i, planet in enumerate(state.planets):
            for k in planet.keys():
                if state._is_free(i, k):
                    slots.append(R * i + keys.index(k))
        self.slots = np.asarray(slots, dtype=np.int64)
        self.n_free = len(slots)
        # free parameters already in kernel order (all keys free, kernel order): no remapping
        self.identity = self.n_free == R * self.n_planets and bool(np.all(self.slots == np.arange(self.n_free)))
        self._dev_cache = {}

    def to_kernel(self, X):
        """X: float64 device tensor [n_free][W] -> kernel params [R*np][W] (R = 5, or 7 if inclined)."""
        torch = _torch()
        if self.identity and X.is_contiguous():
            return X
        key = str(X.device)
        if key not in self._dev_cache:
            self._dev_cache[key] = (torch.as_tensor(self.base, device=X.device),
                                    torch.as_tensor(self.slots, device=X.device))
        base, slots = self._dev_cache[key]
        W = X.shape[1]
        K = base[:, None].expand(-1, W).clone()
        if self.n_free:
            K.index_copy_(0, slots, X)
        return K

    def c_map(self):
        """rvm_param_map for the fused stretch half-step (row -> free index, or fixed value)."""
        if getattr(self, "_c_map", None) is None:
            m = _lib.ParamMapC()
            m.n_rows = len(self.base)
            for r in range(_lib.RVM_MAX_PARAM_ROWS):
                m.src[r] = -1
                m.base[r] = float(self.base[r]) if r < len(self.base) else 0.0
            for k, r in enumerate(self.slots.tolist()):
                m.src[r] = k
            self._c_map = m
        return self._c_map

    def vector_to_kernel_np(self, x):
        k = self.base.copy()
        k[self.slots] = np.asarray(x, dtype=np.float64)
        return k

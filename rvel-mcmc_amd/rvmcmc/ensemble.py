"""Device-resident affine-invariant ensemble sampler (emcee 2.2.1 stretch move).

The reference drives emcee 2.2.1's EnsembleSampler (mcmc.py:40-65; version from script.sh:9) with
threads=1 and a serial map over `lnprob`.  emcee is not vendored; its published algorithm
(EnsembleSampler.sample + _propose_stretch) is restated here with the ensemble
kept in HBM as SoA [dim][W] float64 and every walker-logL of a half-step evaluated by one launch of
the HIP likelihood kernel:

    for (S0, S1) in [(first half, second half), (second half, first half)]:
        z  = ((a - 1) u1 + 1)^2 / a            (a = 2)
        j  = floor(u2 |S1|)
        q  = c_j - z (c_j - x)
        lnpdiff = (dim - 1) ln z + lnp(q) - lnp(x) ;  accept if lnpdiff > ln u3
    (S1 of the second half-step is the already-updated first half.)

Random numbers are counter-based (Philox4x32-10, keyed by seed, iteration, half and GLOBAL walker
index), so a run is reproducible and identical for any number of ranks.

Multi-GPU (one process per GPU, torch.distributed over RCCL/xGMI): each rank owns a contiguous
slice of each half; before each half-step the complement half's positions are all-gathered
(dim x W/2 float64 -- the only collective on the data path).  The fused half-step reads the
complement walker-major ([W/2][dim], one contiguous row per gathered c_j); each half keeps a
walker-major mirror next to its [dim][n] positions, updated by the same launch on accept, so the
gather needs no re-layout.
"""
from __future__ import annotations

import numpy as np

from . import _lib, engine


def _torch():
    import torch

    return torch


class DeviceOps:
    """The three per-half-step operations on the GPU, through librvmcmc.so: stretch proposal,
    batched walker log-likelihood (the HIP kernel), stretch accept.  (The distributed tests inject
    numpy restatements of these three to exercise the sharding logic on CPU with gloo.)"""

    def __init__(self, sampler):
        torch = _torch()
        self.s = sampler
        self.lib = _lib.load()
        st = sampler.state
        dt, mult, hint = st.integrator.plan_args(st.planets)
        # room for the 3 n walker slots of a speculative iteration (iteration_begin)
        self.plan = engine.plan_for(sampler.obs, sampler.pmap.n_planets, dt, mult, 3 * sampler.nloc,
                                    sampler.device, hint, sampler.pmap.inclined, st.integrator.resolve(st.planets))
        self.timing = None  # set to [] to collect (start_event, end_event, n_walkers) per logL launch
        self.track_status = False  # set True to histogram per-walker statuses (costs a small kernel)
        self.status_counts = torch.zeros(4, dtype=torch.int64, device=sampler.device)

    def propose(self, X0, c, half, q, z, draws=None):
        s = self.s
        _lib.check(self.lib.rvm_stretch_propose(s.dim, s.nloc, s.global_begin(half), X0.data_ptr(), s.halfk,
                                                c.data_ptr(), s.a, s.seed, s.iteration, half,
                                                draws.data_ptr() if draws is not None else 0, q.data_ptr(),
                                                z.data_ptr(), _lib.stream_handle()), "rvm_stretch_propose")

    def logl(self, X, out=None, status=None):
        torch = _torch()
        K = self.s.pmap.to_kernel(X)
        if self.timing is not None:  # HIP events on the launch stream, around the likelihood launch only
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        lp, st, _ = self.plan.logl(K, hill_factor=self.s.hill_factor, out=out, status=status)
        if self.timing is not None:
            e1.record()
            self.timing.append((e0, e1, X.shape[1]))
        if self.track_status:
            self.status_counts.index_add_(0, st.long(), torch.ones_like(st, dtype=torch.int64))
        return lp, st

    def fused_half_step(self, X0, X0_aos, lnp0, c_aos, half, lnp_new, status, accepted):
        """propose + logl + accept in one likelihood launch (rvm_stretch_half_step), bit-identical
        to the three-launch sequence with Philox draws.  c_aos: the complement walker-major
        [n1][dim]; X0_aos: this half's walker-major mirror (updated on accept with X0)."""
        torch = _torch()
        s = self.s
        if self.timing is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        self.plan.stretch_half_step(s.pmap, X0, lnp0, c_aos, s.global_begin(half), s.a, s.seed, s.iteration,
                                    half, s.hill_factor, lnp_new=lnp_new, status=status, accepted=accepted,
                                    X0_aos=X0_aos)
        if self.timing is not None:
            e1.record()
            self.timing.append((e0, e1, X0.shape[1]))
        if self.track_status:
            self.status_counts.index_add_(0, status.long(), torch.ones_like(status, dtype=torch.int64))

    def speculation_pays(self):
        """Whether one launch of 3 n walker slots (a whole speculative iteration) beats two
        half-step launches of n, by the launch shape of launch_logl (rvm_logl.hip): a wave group of
        64/L walkers per direction, one block per group while two blocks per group fit the CUs (the
        longest level alone on its SIMD), else two groups per block with mirrored levels (SIMD
        loads mult[i] + mult[nl-1-i]), one block per CU at a time, or the level-split layout (SIMD
        loads max(m3, m2 + m0, 2 m1)) when its blocks fit the CUs."""
        torch = _torch()
        s = self.s
        n_cu = torch.cuda.get_device_properties(s.device).multi_processor_count
        npl = s.pmap.n_planets
        wpb = 64 // (1 if npl == 1 else (2 if npl == 2 else 4))
        mult = list(self.plan.mult)
        t1 = max(mult)
        t2 = max(mult[i] + mult[-1 - i] for i in range(len(mult)))

        def units(W):
            g = -(-W // wpb)
            if 2 * g <= n_cu or 2 * len(mult) * 64 > 512:
                return t1 * -(-2 * g // n_cu)
            c = t2 * -(-g // n_cu)
            # level-split layout (four increasing levels, one round of g + ceil(2g / 8) blocks; the
            # plan of a speculative sampler has its workspace: 2 g > n_cu here)
            if len(mult) == 4 and all(a < b for a, b in zip(mult, mult[1:])) and g + -(-2 * g // 8) <= n_cu:
                c = min(c, max(mult[3], mult[2] + mult[0], 2 * mult[1]))
            return c

        return units(3 * s.nloc) < 2 * units(s.nloc)

    def iteration_begin(self, c0, c1):
        """rvm_stretch_iteration_begin on the sampler's buffers (half 0 updated, all 3 n logl)."""
        torch = _torch()
        s = self.s
        n = s.nloc
        if self.timing is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        self.plan.stretch_iteration_begin(s.pmap, s.pos[0], s.lnp[0], s.pos[1], c0, c1, s.global_begin(0),
                                          s.global_begin(1), s.a, s.seed, s.iteration, s._lnp_spec, s._st_spec,
                                          s._dec, hill_factor=s.hill_factor, accepted0=s.naccepted[:n], lnp1=s.lnp[1])
        if self.timing is not None:
            e1.record()
            self.timing.append((e0, e1, 3 * n))
        if self.track_status:
            st = s._st_spec[:n]
            self.status_counts.index_add_(0, st.long(), torch.ones_like(st, dtype=torch.int64))

    def iteration_end(self, c0, c1, dec_all):
        """rvm_stretch_iteration_end: half 1's accepts, both walker-major mirrors refreshed."""
        torch = _torch()
        s = self.s
        n = s.nloc
        engine.stretch_iteration_end(s.pos[0], s.pos_aos[0], s._dec, dec_all, s.pos[1], s.pos_aos[1], s.lnp[1], c0, c1,
                                     s._lnp_spec, s._st_spec, s.global_begin(0), s.global_begin(1), s.a, s.seed,
                                     s.iteration, accepted1=s.naccepted[n:], lnp_new=s._lnp_new, status_new=s._status)
        if self.track_status:
            self.status_counts.index_add_(0, s._status.long(), torch.ones_like(s._status, dtype=torch.int64))

    def accept(self, X0, lnp0, q, lnp_new, z, half, accepted, draws=None):
        s = self.s
        _lib.check(self.lib.rvm_stretch_accept(s.dim, s.nloc, s.global_begin(half), X0.data_ptr(), lnp0.data_ptr(),
                                               q.data_ptr(), lnp_new.data_ptr(), z.data_ptr(), s.seed, s.iteration,
                                               half, draws.data_ptr() if draws is not None else 0,
                                               accepted.data_ptr(), _lib.stream_handle()), "rvm_stretch_accept")


class EnsembleSampler:
    def __init__(self, nwalkers, state, obs, a=2.0, seed=0, device=None, hill_factor=None, group=None,
                 pmap=None, ops=None):
        torch = _torch()
        dim = state.Nvars
        if nwalkers % 2 != 0:
            raise ValueError("The number of walkers must be even.")
        if nwalkers < 2 * dim:
            raise ValueError("The number of walkers needs to be more than twice the dimension of your parameter space.")
        self.k = int(nwalkers)
        self.dim = dim
        self.comm_timing = None  # set to [] to collect HIP events around the collectives (N > 1)
        self.a = float(a)
        self.seed = int(seed) & ((1 << 64) - 1)
        self.state = state
        self.obs = obs
        self.pmap = pmap or state.param_map()
        self.hill_factor = state.hillRadiusFactor if hill_factor is None else float(hill_factor)
        self.device = torch.device(device) if device is not None else engine.default_device()
        # distributed layout: rank r owns walkers [r*nloc, (r+1)*nloc) of each half
        self.group = group
        if group is not None or (torch.distributed.is_available() and torch.distributed.is_initialized()):
            self.rank = torch.distributed.get_rank(group)
            self.world = torch.distributed.get_world_size(group)
        else:
            self.rank, self.world = 0, 1
        self.halfk = self.k // 2
        if self.halfk % self.world != 0:
            raise ValueError("nwalkers/2 must be divisible by the world size")
        self.nloc = self.halfk // self.world
        self.iteration = 0
        self.ops = ops(self) if ops is not None else DeviceOps(self)
        self.plan = getattr(self.ops, "plan", None)
        n = self.nloc
        f64 = dict(dtype=torch.float64, device=self.device)
        self._q = torch.empty((dim, n), **f64)
        self._z = torch.empty(n, **f64)
        self._lnp_new = torch.empty(n, **f64)
        self._status = torch.empty(n, dtype=torch.int32, device=self.device)
        self._c_full = torch.empty((dim, self.halfk), **f64)
        self._gather = torch.empty(self.world * dim * n, **f64) if self.world > 1 else None
        self._gather_aos = torch.empty((self.halfk, dim), **f64) if self.world > 1 else None
        # both halves' walker-major mirrors in one buffer (pos_aos[h] are views of it): at N > 1 a
        # speculative iteration gathers both with ONE all-gather
        self._aos_pair = torch.empty((2, n, dim), **f64)
        self.pos_aos = [self._aos_pair[0], self._aos_pair[1]]
        self._gather_pair = torch.empty(self.world * 2 * n * dim, **f64) if self.world > 1 else None
        self._c01 = torch.empty((2, self.halfk, dim), **f64) if self.world > 1 else None
        self._aos_stale = True  # pos_aos (walker-major mirrors for the fused path) out of date
        self.naccepted = torch.zeros(2 * n, dtype=torch.int32, device=self.device)
        self.nevals = 0
        # speculative whole iterations (iteration_begin / iteration_end, bit-identical to two
        # half-steps): None = when the launch shape says they pay, True / False to force
        self.speculative = None
        self.nevals_speculative = 0  # walker-logL evaluations of the variants not taken
        self._lnp_spec = torch.empty(3 * n, **f64)
        self._st_spec = torch.empty(3 * n, dtype=torch.int32, device=self.device)
        self._dec = torch.zeros(n, dtype=torch.int32, device=self.device)
        self._dec_all = torch.empty(self.halfk, dtype=torch.int32, device=self.device) if self.world > 1 else None
        self._spec_pays = None
        # one launch per half-step (rvm_stretch_half_step) unless draws are injected or the ops
        # (e.g. the CPU restatements of the distributed tests) provide only the three-step path
        self.fused = hasattr(self.ops, "fused_half_step")

    @property
    def timing(self):
        return getattr(self.ops, "timing", None)

    @timing.setter
    def timing(self, v):
        self.ops.timing = v

    # ---- global <-> local indexing ------------------------------------------------------------
    def global_begin(self, half):
        return half * self.halfk + self.rank * self.nloc

    def local_slices(self):
        """Global walker indices owned by this rank (first-half slice, second-half slice)."""
        return (slice(self.global_begin(0), self.global_begin(0) + self.nloc),
                slice(self.global_begin(1), self.global_begin(1) + self.nloc))

    def lnprob(self, X, out=None, status=None):
        lp, st = self.ops.logl(X, out=out, status=status)
        self.nevals += X.shape[1]
        return lp, st

    def _complement(self, Xc):
        """Full complement half [dim][W/2] in global order (all-gather over ranks)."""
        torch = _torch()
        if self.world == 1:
            return Xc
        torch.distributed.all_gather_into_tensor(self._gather, Xc.contiguous().view(-1), group=self.group)
        g = self._gather.view(self.world, self.dim, self.nloc)
        self._c_full.copy_(g.permute(1, 0, 2).reshape(self.dim, self.halfk))
        return self._c_full

    def _complement_aos(self, other):
        """Full complement half walker-major [W/2][dim] in global order: this rank's mirror, or
        the all-gather of every rank's (rank r holds walkers [r nloc, (r+1) nloc) of the half, so
        the gathered blocks are already in global order: no re-layout copy)."""
        torch = _torch()
        if self.world == 1:
            return self.pos_aos[other]
        torch.distributed.all_gather_into_tensor(self._gather_aos, self.pos_aos[other], group=self.group)
        return self._gather_aos

    def _set_aos(self, a0, a1):
        self._aos_pair[0].copy_(a0)
        self._aos_pair[1].copy_(a1)
        self.pos_aos = [self._aos_pair[0], self._aos_pair[1]]

    def _refresh_aos(self):
        self._set_aos(self.pos[0].t(), self.pos[1].t())
        self._aos_stale = False

    def half_step(self, X0, lnp0, Xc, half, draws_propose=None, draws_accept=None):
        """Update this rank's slice X0 = pos[half] [dim][nloc] (in place) against the complement
        half Xc = pos[1 - half]."""
        n = self.nloc
        if self.fused and draws_propose is None and draws_accept is None:
            if X0 is not self.pos[half] or Xc is not self.pos[1 - half]:
                raise ValueError("the fused half-step updates the sampler's own halves (pos[half], pos[1 - half])")
            if self._aos_stale:
                self._refresh_aos()
            c = self._complement_aos(1 - half)
            self.ops.fused_half_step(X0, self.pos_aos[half], lnp0, c, half, self._lnp_new, self._status,
                                     self.naccepted[half * n:(half + 1) * n])
            self.nevals += n
            return
        c = self._complement(Xc)
        self._aos_stale = True
        self.ops.propose(X0, c, half, self._q, self._z, draws_propose)
        self.lnprob(self._q, out=self._lnp_new, status=self._status)
        self.ops.accept(X0, lnp0, self._q, self._lnp_new, self._z, half, self.naccepted[half * n:(half + 1) * n],
                        draws_accept)

    # ---- ensemble state ------------------------------------------------------------------------
    def set_positions(self, X_global):
        """X_global: [W][dim] array-like of ALL walkers (every rank passes the same array); this
        rank keeps its two slices as contiguous device tensors [dim][nloc]."""
        torch = _torch()
        Xg = torch.as_tensor(np.asarray(X_global, dtype=np.float64), device=self.device)
        if Xg.shape != (self.k, self.dim):
            raise ValueError(f"positions must be [{self.k}][{self.dim}]")
        s0, s1 = self.local_slices()
        self.pos = [Xg[s0].t().contiguous(), Xg[s1].t().contiguous()]
        self._set_aos(Xg[s0], Xg[s1])
        self._aos_stale = False
        self.lnp = [None, None]

    def compute_lnprob(self):
        self.lnp = [self.lnprob(self.pos[h])[0].clone() for h in (0, 1)]
        for h in (0, 1):
            self.check_initial(self.lnp[h])

    def speculating(self):
        """Whether step() runs speculative whole iterations (see `speculative`)."""
        if not (self.fused and hasattr(self.ops, "iteration_begin")):
            return False
        if self.speculative is not None:
            return bool(self.speculative)
        if self._spec_pays is None:
            self._spec_pays = bool(self.ops.speculation_pays())
        return self._spec_pays

    def step(self):
        """One emcee iteration (both half-steps) over this rank's walkers (on the stream the sampler
        was built on: engine.check_stream)."""
        engine.check_stream(self.plan, "EnsembleSampler.step")
        if self.lnp[0] is None:
            self.compute_lnprob()
        if self.speculating():
            self._speculative_iteration()
        else:
            A, B = self.pos
            self.half_step(A, self.lnp[0], B, 0)
            self.half_step(B, self.lnp[1], A, 1)
        self.iteration += 1
        engine.periodic_fault_check(self, self.plan)

    def check_faults(self):
        """Raise on level-split hand-off timeouts or NONFINITE log-likelihoods since the last check
        (rvm_plan_faults; also run every FAULT_CHECK_EVERY iterations by step()); returns the
        counters, including walker-directions refined by the adaptive resolution."""
        self.last_faults = self.plan.check_faults(type(self).__name__, group=engine.fault_group(self))
        return self.last_faults

    def gather_mirrors(self):
        """Both halves' walker-major mirrors [W/2][dim] in global order: this rank's own at N = 1,
        else one all-gather of the pair buffer re-laid out by one copy."""
        torch = _torch()
        if self._aos_stale:
            self._refresh_aos()
        if self.world == 1:
            return self.pos_aos[0], self.pos_aos[1]
        torch.distributed.all_gather_into_tensor(self._gather_pair, self._aos_pair.view(-1), group=self.group)
        g = self._gather_pair.view(self.world, 2, self.nloc, self.dim)
        self._c01.view(2, self.world, self.nloc, self.dim).copy_(g.permute(1, 0, 2, 3))
        return self._c01[0], self._c01[1]

    def _speculative_iteration(self):
        """Both half-steps as one launch over 3 nloc walker slots (half 0, and half 1 against both
        possible positions of each partner) plus a small accept launch; bit-identical to two
        half_step calls.  Collectives (N > 1): the two halves' walker-major mirrors before the
        launch (one all-gather of the pair buffer, re-laid out by one copy), half 0's decisions
        between the two launches."""
        torch = _torch()
        ct = self.comm_timing is not None and self.world > 1
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)] if ct else None
        if ct:
            ev[0].record()
        c0, c1 = self.gather_mirrors()
        if ct:
            ev[1].record()
        dec_all = self._dec if self.world == 1 else self._dec_all
        self.ops.iteration_begin(c0, c1)
        if self.world > 1:
            if ct:
                ev[2].record()
            # (every rank's half-0 decisions: this is where a rank waits for the slowest rank's
            # likelihood and refinement kernels)
            torch.distributed.all_gather_into_tensor(self._dec_all, self._dec, group=self.group)
            if ct:
                ev[3].record()
                self.comm_timing.append(ev)
        self.ops.iteration_end(c0, c1, dec_all)
        self.nevals += 2 * self.nloc
        self.nevals_speculative += self.nloc

    def gather_positions(self):
        """All walkers [W][dim] on every rank (host numpy), global order."""
        torch = _torch()
        loc = [p.t().contiguous() for p in self.pos]  # [nloc][dim]
        if self.world == 1:
            return torch.cat(loc, 0).cpu().numpy()
        out = []
        for h in (0, 1):
            buf = torch.empty((self.world * self.nloc, self.dim), dtype=torch.float64, device=self.device)
            torch.distributed.all_gather_into_tensor(buf, loc[h], group=self.group)
            out.append(buf)
        return torch.cat(out, 0).cpu().numpy()

    def gather_lnprob(self):
        torch = _torch()
        if self.world == 1:
            return torch.cat(self.lnp, 0).cpu().numpy()
        out = []
        for h in (0, 1):
            buf = torch.empty(self.world * self.nloc, dtype=torch.float64, device=self.device)
            torch.distributed.all_gather_into_tensor(buf, self.lnp[h].contiguous(), group=self.group)
            out.append(buf)
        return torch.cat(out, 0).cpu().numpy()

    def _gather_int(self, local):
        """[2*nloc] per-rank counters (half 0 slice | half 1 slice) -> [W] in global order."""
        torch = _torch()
        n = self.nloc
        if self.world == 1:
            return local.cpu().numpy()
        out = []
        for h in (0, 1):
            buf = torch.empty(self.world * n, dtype=local.dtype, device=self.device)
            torch.distributed.all_gather_into_tensor(buf, local[h * n:(h + 1) * n].contiguous(), group=self.group)
            out.append(buf)
        return torch.cat(out).cpu().numpy()

    def checkpoint(self, path):
        """Save the whole ensemble (every rank takes part; rank 0 writes path, an .npz): positions
        [W][dim] and lnprob [W] in global order, accept counters, iteration, seed and stretch scale.
        With counter-based draws keyed by (seed, iteration, half, global walker) a restored sampler
        continues bit-identically, on any number of ranks (checkpoint / resume)."""
        pos, lnp, acc = self.gather_positions(), self.gather_lnprob(), self._gather_int(self.naccepted)
        if self.rank == 0:
            np.savez(path, positions=pos, lnprob=lnp, naccepted=acc, iteration=self.iteration, seed=self.seed,
                     a=self.a, nwalkers=self.k, dim=self.dim)

    def restore(self, path):
        """Load a checkpoint written by checkpoint() (same nwalkers and dim; any world size)."""
        torch = _torch()
        d = np.load(path)
        if int(d["nwalkers"]) != self.k or int(d["dim"]) != self.dim:
            raise ValueError("checkpoint was written for a different ensemble size or dimension")
        self.set_positions(d["positions"])
        s0, s1 = self.local_slices()
        lnp = torch.as_tensor(d["lnprob"], device=self.device)
        self.lnp = [lnp[s0].contiguous(), lnp[s1].contiguous()]
        acc = torch.as_tensor(d["naccepted"].astype(np.int32), device=self.device)
        self.naccepted = torch.cat([acc[s0], acc[s1]]).contiguous()
        self.iteration = int(d["iteration"])
        self.seed = int(d["seed"])
        self.a = float(d["a"])

    def check_initial(self, lnp):
        torch = _torch()
        if bool(torch.isnan(lnp).any()):
            raise ValueError("The initial lnprob was NaN.")

    def acceptance_fraction(self):
        return self.naccepted.double() / max(self.iteration, 1)

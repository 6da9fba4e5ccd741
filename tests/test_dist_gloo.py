"""Multi-process (world_size 2, gloo, CPU) test of the sharded affine sampler's orchestration.

The production path shards walkers over ranks and all-gathers the complement half over RCCL
(ensemble.EnsembleSampler).  Here the same EnsembleSampler runs with torch.distributed gloo on
CPU tensors; its three device operations (stretch proposal, walker logL, accept) are replaced
by numpy restatements (emcee 2.2.1 stretch semantics with the device's Philox draws restated in
tests/philox_ref.py, and an analytic Gaussian logL).  The run must be bit-identical to the
single-process run: the RNG is keyed by global walker index and the complement is gathered in
global order.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import S2_PLANETS, S2_SCALES
from philox_ref import stretch_uniforms

W = 48
ITERS = 4
SEED = 12345


class NumpyOps:
    """CPU restatement of DeviceOps (test double; the product has no CPU path)."""

    def __init__(self, sampler):
        self.s = sampler
        self.timing = None
        self.mu = np.array(sampler.state.get_params())
        self.sd = 1e-3 * np.abs(self.mu) + 1e-4

    def propose(self, X0, c, half, q, z, draws=None):
        s = self.s
        u1, u2, _ = stretch_uniforms(s.seed, s.global_begin(half), s.nloc, s.iteration, half)
        zz = ((s.a - 1.0) * u1 + 1.0) * ((s.a - 1.0) * u1 + 1.0) / s.a
        j = np.minimum(np.floor(u2 * s.halfk).astype(np.int64), s.halfk - 1)
        C = c.numpy()
        x = X0.numpy()
        q.copy_(torch.from_numpy(C[:, j] - zz[None, :] * (C[:, j] - x)))
        z.copy_(torch.from_numpy(zz))

    def logl(self, X, out=None, status=None):
        x = X.numpy()
        lp = -0.5 * np.sum(((x - self.mu[:, None]) / self.sd[:, None]) ** 2, axis=0)
        lp = torch.from_numpy(lp)
        if out is None:
            out = torch.empty_like(lp)
        if status is None:
            status = torch.zeros(lp.shape[0], dtype=torch.int32)
        out.copy_(lp)
        status.zero_()
        return out, status

    def accept(self, X0, lnp0, q, lnp_new, z, half, accepted, draws=None):
        s = self.s
        _, _, u3 = stretch_uniforms(s.seed, s.global_begin(half), s.nloc, s.iteration, half)
        lnpdiff = (s.dim - 1.0) * np.log(z.numpy()) + lnp_new.numpy() - lnp0.numpy()
        acc = lnpdiff > np.log(u3)
        acc_t = torch.from_numpy(acc)
        X0[:, acc_t] = q[:, acc_t]
        lnp0[acc_t] = lnp_new[acc_t]
        accepted += acc_t.to(torch.int32)


class FusedNumpyOps(NumpyOps):
    """NumpyOps plus the fused half-step's contract (rvm_stretch_half_step): the complement arrives
    walker-major [W/2][dim] (gathered from the ranks' walker-major mirrors, no re-layout) and the
    half's mirror X0_aos is kept in step with X0."""

    def fused_half_step(self, X0, X0_aos, lnp0, c_aos, half, lnp_new, status, accepted):
        s = self.s
        assert c_aos.shape == (s.halfk, s.dim) and X0_aos.shape == (s.nloc, s.dim)
        np.testing.assert_array_equal(X0_aos.numpy(), X0.t().numpy())  # mirror in step before
        q = torch.empty_like(X0)
        z = torch.empty(s.nloc, dtype=torch.float64)
        self.propose(X0, c_aos.t().contiguous(), half, q, z)
        self.logl(q, out=lnp_new, status=status)
        self.accept(X0, lnp0, q, lnp_new, z, half, accepted)
        X0_aos.copy_(X0.t())


class SpecNumpyOps(FusedNumpyOps):
    """FusedNumpyOps plus the speculative iteration's contract (rvm_stretch_iteration_begin /
    _end): both halves arrive walker-major and gathered (c0, c1, as at the start of the
    iteration); begin does half 0's half-step and evaluates half 1's proposals against both
    possible positions of their partners; end takes half 0's decisions in global order (dec_all)
    and accepts half 1 with the variant they select."""

    def speculation_pays(self):
        return True

    def _half0_proposals_all(self, C0, C1):
        """Every half-0 walker's proposal [halfk][dim] from its own draws (keys 0 .. halfk-1)."""
        s = self.s
        u1, u2, _ = stretch_uniforms(s.seed, 0, s.halfk, s.iteration, 0)
        zz = ((s.a - 1.0) * u1 + 1.0) * ((s.a - 1.0) * u1 + 1.0) / s.a
        j = np.minimum(np.floor(u2 * s.halfk).astype(np.int64), s.halfk - 1)
        return C1[j] - zz[:, None] * (C1[j] - C0)

    def _half1_draws(self):
        s = self.s
        u1, u2, u3 = stretch_uniforms(s.seed, s.global_begin(1), s.nloc, s.iteration, 1)
        zz = ((s.a - 1.0) * u1 + 1.0) * ((s.a - 1.0) * u1 + 1.0) / s.a
        j = np.minimum(np.floor(u2 * s.halfk).astype(np.int64), s.halfk - 1)
        return zz, j, u3

    def iteration_begin(self, c0, c1):
        s = self.s
        n = s.nloc
        assert c0.shape == c1.shape == (s.halfk, s.dim)
        C0, C1 = c0.numpy().copy(), c1.numpy().copy()
        dec0 = s.naccepted[:n].clone()
        lnp_new = torch.empty(n, dtype=torch.float64)
        st = torch.empty(n, dtype=torch.int32)
        q = torch.empty_like(s.pos[0])
        z = torch.empty(n, dtype=torch.float64)
        self.propose(s.pos[0], c1.t().contiguous(), 0, q, z)
        self.logl(q, out=lnp_new, status=st)
        self.accept(s.pos[0], s.lnp[0], q, lnp_new, z, 0, s.naccepted[:n])
        s._dec.copy_((s.naccepted[:n] - dec0).to(torch.int32))
        s._lnp_spec[:n] = lnp_new
        zz, j, _ = self._half1_draws()
        Q0 = self._half0_proposals_all(C0, C1)
        x1 = s.pos[1].numpy()
        for v, C in enumerate((C0, Q0)):
            qv = C[j].T - zz[None, :] * (C[j].T - x1)
            s._lnp_spec[(1 + v) * n:(2 + v) * n] = self.logl(torch.from_numpy(qv))[0]
        s._st_spec.zero_()

    def iteration_end(self, c0, c1, dec_all):
        s = self.s
        n = s.nloc
        assert dec_all.shape == (s.halfk,)
        C0, C1 = c0.numpy(), c1.numpy()
        zz, j, u3 = self._half1_draws()
        v = dec_all.numpy()[j].astype(bool)
        lnew = np.where(v, s._lnp_spec[2 * n:].numpy(), s._lnp_spec[n:2 * n].numpy())
        c = np.where(v[:, None], self._half0_proposals_all(C0, C1)[j], C0[j])
        x1 = s.pos[1].numpy()
        q = c.T - zz[None, :] * (c.T - x1)
        acc = torch.from_numpy((s.dim - 1.0) * np.log(zz) + lnew - s.lnp[1].numpy() > np.log(u3))
        s.pos[1][:, acc] = torch.from_numpy(q)[:, acc]
        s.lnp[1][acc] = torch.from_numpy(lnew)[acc]
        s.naccepted[n:] += acc.to(torch.int32)
        for h in (0, 1):
            s.pos_aos[h].copy_(s.pos[h].t())


THIRD = {"m": 1e-3, "a": 2.6, "h": 0.05, "k": 0.0, "l": 1.0}  # scripts/configs_bench.py config 5
DEFAULT = dict(W=W, planets=S2_PLANETS, iters=ITERS)
# BASELINE config 5: 65536 walkers, 3 planets, sharded 8 ways (8192 walkers = 4096 per half per rank)
CONFIG5 = dict(W=65536, planets=S2_PLANETS + [THIRD], iters=2)


def _initial_positions(state, W):
    rng = np.random.default_rng(3)
    scales = np.array([S2_SCALES[k] for k in state.get_rawkeys()])
    return state.get_params()[None] + 1e-3 * scales * rng.standard_normal((W, state.Nvars))


def _run_sampler(fused=False, ckpt=None, cfg=DEFAULT):
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.state import State

    W_, iters = cfg["W"], cfg["iters"]
    state = State(planets=[dict(p) for p in cfg["planets"]])
    ops = {False: NumpyOps, True: FusedNumpyOps, "spec": SpecNumpyOps}
    ens = EnsembleSampler(W_, state, obs=None, seed=SEED, device="cpu", ops=ops[fused])
    assert ens.fused == bool(fused) and ens.speculating() == (fused == "spec")
    ens.set_positions(_initial_positions(state, W_))
    ens.compute_lnprob()
    if ckpt is None:
        for _ in range(iters):
            ens.step()
    else:  # half the iterations, checkpoint, continue in a fresh sampler from the file
        for _ in range(iters // 2):
            ens.step()
        ens.checkpoint(ckpt)
        if dist.is_initialized():
            dist.barrier()
        ens = EnsembleSampler(W_, state, obs=None, seed=0, device="cpu", ops=ops[fused])
        ens.restore(ckpt)
        for _ in range(iters - iters // 2):
            ens.step()
    return ens.gather_positions(), ens.gather_lnprob(), ens.naccepted.clone()


def _worker(rank, world, port, out_dir, fused=False, ckpt=False, cfg=DEFAULT):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pos, lnp, acc = _run_sampler(fused, os.path.join(out_dir, "ckpt.npz") if ckpt else None, cfg)
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), pos=pos, lnp=lnp, acc=acc.numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,fused", [(2, False), (4, False), (2, True), (4, True), (1, "spec"), (2, "spec"),
                                         (4, "spec")])
def test_sharded_ensemble_bit_identical_to_single_process(tmp_path, world, fused):
    """Three-launch path (SoA complement, all-gather + re-layout), fused path (walker-major
    complement gathered from the mirrors) and speculative whole iterations (both halves gathered,
    half 0's decisions all-gathered between the two launches): every world size gives the
    single-process three-launch run."""
    pos1, lnp1, acc1 = _run_sampler()
    if fused:
        pf, lf, af = _run_sampler(fused=fused)
        np.testing.assert_array_equal(pf, pos1)
        np.testing.assert_array_equal(lf, lnp1)
        np.testing.assert_array_equal(af.numpy(), acc1.numpy())
        if world == 1:
            return
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), fused), nprocs=world, join=True)
    accs = []
    for r in range(world):
        d = np.load(tmp_path / f"rank{r}.npz")
        np.testing.assert_array_equal(d["pos"], pos1)   # every rank sees the same global ensemble
        np.testing.assert_array_equal(d["lnp"], lnp1)
        accs.append(d["acc"])
    # acceptance counters: rank r owns slices r of each half
    n = W // 2 // world
    got = np.concatenate([np.concatenate([a[:n] for a in accs]), np.concatenate([a[n:] for a in accs])])
    np.testing.assert_array_equal(got, acc1.numpy())
    assert 0 < acc1.sum() < W * ITERS


@pytest.mark.parametrize("world", [1, 2])
def test_checkpoint_resume_is_bit_identical(tmp_path, world):
    """Checkpoint after half the iterations, restore into a new sampler, continue: the same
    ensemble as the uninterrupted run (SURVEY.md §5 checkpoint / resume; counter-based draws)."""
    pos1, lnp1, acc1 = _run_sampler()
    if world == 1:
        pos, lnp, acc = _run_sampler(ckpt=str(tmp_path / "ckpt.npz"))
        np.testing.assert_array_equal(acc.numpy(), acc1.numpy())
    else:
        mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), False, True), nprocs=world, join=True)
        d = np.load(tmp_path / "rank0.npz")
        pos, lnp = d["pos"], d["lnp"]
    np.testing.assert_array_equal(pos, pos1)
    np.testing.assert_array_equal(lnp, lnp1)


@pytest.mark.parametrize("fused", [True, "spec"])
def test_config5_layout_world8(tmp_path, fused):
    """BASELINE config 5's sharded layout: 65536 walkers of the 3-planet system over 8 ranks
    (rank r owns walkers [4096 r, 4096 (r + 1)) of each 32768-walker half; Philox keys = global
    indices; complements all-gathered in global order).  Every rank's gathered ensemble, lnprob
    and its slices of the accept counters equal the single-process run (the RCCL path itself is
    unmeasured on hardware: the driver's 8-GPU node runs it)."""
    world = 8
    pos1, lnp1, acc1 = _run_sampler(fused=fused, cfg=CONFIG5)
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), fused, False, CONFIG5), nprocs=world, join=True)
    W_ = CONFIG5["W"]
    n = W_ // 2 // world
    accs = []
    for r in range(world):
        d = np.load(tmp_path / f"rank{r}.npz")
        np.testing.assert_array_equal(d["pos"], pos1)
        np.testing.assert_array_equal(d["lnp"], lnp1)
        assert d["acc"].shape == (2 * n,)
        accs.append(d["acc"])
    got = np.concatenate([np.concatenate([a[:n] for a in accs]), np.concatenate([a[n:] for a in accs])])
    np.testing.assert_array_equal(got, acc1.numpy())
    assert 0 < acc1.sum() < W_ * CONFIG5["iters"]


def test_sampler_rejects_bad_sizes():
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.state import State

    state = State(planets=[dict(p) for p in S2_PLANETS])
    with pytest.raises(ValueError):
        EnsembleSampler(W + 1, state, None, device="cpu", ops=NumpyOps)   # odd (emcee 2.2.1)
    with pytest.raises(ValueError):
        EnsembleSampler(18, state, None, device="cpu", ops=NumpyOps)      # < 2 * dim

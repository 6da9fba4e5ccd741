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


def _initial_positions(state):
    rng = np.random.default_rng(3)
    scales = np.array([S2_SCALES[k] for k in state.get_rawkeys()])
    return state.get_params()[None] + 1e-3 * scales * rng.standard_normal((W, state.Nvars))


def _run_sampler(fused=False, ckpt=None):
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.state import State

    state = State(planets=[dict(p) for p in S2_PLANETS])
    ens = EnsembleSampler(W, state, obs=None, seed=SEED, device="cpu", ops=FusedNumpyOps if fused else NumpyOps)
    assert ens.fused == fused
    ens.set_positions(_initial_positions(state))
    ens.compute_lnprob()
    if ckpt is None:
        for _ in range(ITERS):
            ens.step()
    else:  # half the iterations, checkpoint, continue in a fresh sampler from the file
        for _ in range(ITERS // 2):
            ens.step()
        ens.checkpoint(ckpt)
        if dist.is_initialized():
            dist.barrier()
        ens = EnsembleSampler(W, state, obs=None, seed=0, device="cpu", ops=FusedNumpyOps if fused else NumpyOps)
        ens.restore(ckpt)
        for _ in range(ITERS - ITERS // 2):
            ens.step()
    return ens.gather_positions(), ens.gather_lnprob(), ens.naccepted.clone()


def _worker(rank, world, port, out_dir, fused=False, ckpt=False):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pos, lnp, acc = _run_sampler(fused, os.path.join(out_dir, "ckpt.npz") if ckpt else None)
        np.savez(os.path.join(out_dir, f"rank{rank}.npz"), pos=pos, lnp=lnp, acc=acc.numpy())
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,fused", [(2, False), (4, False), (2, True), (4, True)])
def test_sharded_ensemble_bit_identical_to_single_process(tmp_path, world, fused):
    """Three-launch path (SoA complement, all-gather + re-layout) and fused path (walker-major
    complement gathered from the mirrors): every world size gives the single-process run."""
    pos1, lnp1, acc1 = _run_sampler()
    if fused:
        pf, lf, af = _run_sampler(fused=True)
        np.testing.assert_array_equal(pf, pos1)
        np.testing.assert_array_equal(lf, lnp1)
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


def test_sampler_rejects_bad_sizes():
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.state import State

    state = State(planets=[dict(p) for p in S2_PLANETS])
    with pytest.raises(ValueError):
        EnsembleSampler(W + 1, state, None, device="cpu", ops=NumpyOps)   # odd (emcee 2.2.1)
    with pytest.raises(ValueError):
        EnsembleSampler(18, state, None, device="cpu", ops=NumpyOps)      # < 2 * dim

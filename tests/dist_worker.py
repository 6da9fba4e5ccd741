"""Worker of tests/test_gpu_a_dist.py (not a test module): one rank of the affine sampler with the
real HIP DeviceOps, over gloo on 127.0.0.1, on cuda:0.  Writes rank 0's gathered state to the
output .npz.  Usage: python dist_worker.py RANK WORLD PORT WALKERS ITERS OUT"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "rvel-mcmc_amd"), os.path.join(ROOT, "oracle"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    rank, world, port, W, iters, out = (int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]),
                                        int(sys.argv[5]), sys.argv[6])
    import torch
    import torch.distributed as dist

    from conftest import S2_PLANETS, S2_SCALES, s2_obs_oracle
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.state import State

    torch.cuda.set_device(0)
    group = None
    if world > 1:
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    s = State(planets=[dict(p) for p in S2_PLANETS])
    obs = s2_obs_oracle()
    scales = np.array([S2_SCALES[k] for k in s.get_rawkeys()])
    X0 = s.get_params()[None] + 1e-3 * scales * np.random.default_rng(11).standard_normal((W, s.Nvars))
    ens = EnsembleSampler(W, s, obs, seed=2027, group=group)
    ens.set_positions(X0)
    ens.compute_lnprob()
    for _ in range(iters):
        ens.step()
    faults = ens.check_faults()  # raises on hand-off timeouts / NONFINITE
    pos, lnp, acc = ens.gather_positions(), ens.gather_lnprob(), ens._gather_int(ens.naccepted)
    if rank == 0:
        np.savez(out, positions=pos, lnprob=lnp, naccepted=acc, speculative=ens.speculating(), nloc=ens.nloc,
                 world=ens.world, refined=faults["refined"], unresolved=faults["unresolved"])
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()

"""Probe (GPU + oracle): a stretch decision of the device sampler that its own plain-launch logL does
not reproduce (tests/test_gpu_ias15_decisions.py stretch_parity's self-consistency check).  Runs the
HD155358 steady state (W walkers after 1000 device iterations) for a few iterations and, for every
proposal whose device decision differs from (dim-1) log z + logL_plain - lnp0 > log u, prints the
device's statuses and values, and the oracle's adaptive restatement of the same proposal with and
without the sampler's accept inputs (its certain-reject cut).  usage: decision_mismatch_probe.py [W] [iters]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, d) for d in ("rvel-mcmc_amd", "oracle", "tests")]
import ias15_parity as IP  # noqa: E402
import oracle as O  # noqa: E402
import test_gpu_ias15_decisions as T  # noqa: E402
from philox_ref import stretch_uniforms  # noqa: E402


def main():
    import torch
    from rvmcmc import engine
    from rvmcmc.ensemble import EnsembleSampler
    from rvmcmc.state import State

    W = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    burn = int(sys.argv[3]) if len(sys.argv) > 3 else 1000
    planets, obs = T._hd()
    X0 = T._burned_in(planets, obs, W, burn)
    s = State(planets=[dict(p) for p in planets])
    pm = s.param_map()
    dim = s.Nvars
    ens = EnsembleSampler(W, s, obs, seed=2017)
    ens.set_positions(X0)
    ens.compute_lnprob()
    torch.cuda.synchronize()
    n, hill = ens.nloc, ens.hill_factor
    cfg = s.integrator
    dt, mult, _ = cfg.plan_args(planets)
    tol, rmax, guard, _ = cfg.resolve(planets)
    found = 0
    for _ in range(iters):
        it = ens.iteration
        before = [p.t().cpu().numpy().copy() for p in ens.pos]
        lnp_dev = [l.cpu().numpy().copy() for l in ens.lnp]
        ens.plan.faults(reset=True)
        ens.step()
        torch.cuda.synchronize()
        f = ens.plan.faults(reset=True)
        after = [p.t().cpu().numpy() for p in ens.pos]
        lnp_after = [l.cpu().numpy() for l in ens.lnp]
        for h in (0, 1):
            c = before[1] if h == 0 else after[0]
            u1, u2, u3 = stretch_uniforms(ens.seed, ens.global_begin(h), n, it, h)
            q, z = IP.stretch_proposal(before[h], c, u1, u2, ens.a)
            lq_dev, sq_dev = T._device_logl(ens.plan, pm, q, hill)
            with np.errstate(invalid="ignore"):
                d_dev = (dim - 1.0) * np.log(z) + lq_dev - lnp_dev[h]
            acc_dev = np.any(after[h] != before[h], axis=1)
            bad = np.nonzero(acc_dev != (d_dev > np.log(u3)))[0]
            for i in bad:
                found += 1
                P = IP.to_oracle(pm, q[i:i + 1])
                plain = O.logl_whx_adapt_batch(P, len(planets), obs, dt, mult, tol, rmax, hill, ecc_guard=guard)
                ctx = dict(mode=np.ones(1, dtype=np.int32), dim=dim, z=z[i:i + 1], u=u3[i:i + 1],
                           lnp0=lnp_dev[h][i:i + 1])
                cutr = O.logl_whx_adapt_batch(P, len(planets), obs, dt, mult, tol, rmax, hill, ecc_guard=guard, ctx=ctx)
                ias = IP.ias15_logl(P, len(planets), obs, hill)[0]
                print(json.dumps({"it": it, "half": h, "i": int(i), "acc_sampler": bool(acc_dev[i]),
                                  "logl_plain_device": float(lq_dev[i]), "status_plain_device": int(sq_dev[i]),
                                  "lnp0": float(lnp_dev[h][i]), "lnp_after": float(lnp_after[h][i]),
                                  "log_u_minus_dimlogz": float(np.log(u3[i]) - (dim - 1.0) * np.log(z[i])),
                                  "margin_plain": float(d_dev[i] - np.log(u3[i])),
                                  "oracle_plain": {"logl": float(plain[0][0]), "status": int(plain[1][0]),
                                                   "stage": plain[2][0].tolist()},
                                  "oracle_with_cut": {"logl": float(cutr[0][0]), "status": int(cutr[1][0]),
                                                      "stage": cutr[2][0].tolist(), "cut": cutr[5][0].tolist()},
                                  "ias15_logl": float(ias[0]), "faults": f, "oracle_params": P[0].tolist(),
                                  "z": float(z[i]), "u": float(u3[i])}), flush=True)
    print(json.dumps({"mismatches": found, "walkers": W, "iterations": iters}))


if __name__ == "__main__":
    main()

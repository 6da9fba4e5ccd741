"""The real HIP sampler at world size 2 (mcmc.py:52,59; emcee 2.2.1's complement read, SURVEY
App. A.6): two ranks over gloo, both on cuda:0, each with its own device context, 4096 walkers per
rank (2048 per half: the speculative 6144-slot launch of the bench), against one rank with all
8192 walkers (half-step launches).  Positions, lnprob and accept counters must be bit-identical (Philox draws keyed by
global walker index), and no walker NONFINITE / no hand-off timeout (check_faults in the worker).

The ranks run as child processes (tests/dist_worker.py) started before this pytest process touches
the GPU: the module sorts first among the GPU tests.  RCCL itself (the driver's 8-GPU runs) is not
exercised here: two ranks cannot share one device under RCCL.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(world, W, iters, out, timeout=240):
    port = _free_port()
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_worker.py"), str(r), str(world), str(port),
                               str(W), str(iters), out], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
        logs.append(o.decode(errors="replace"))
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    return np.load(out)


def test_world2_real_device_ops_bit_identical_to_one_rank(tmp_path):
    import torch

    assert not torch.cuda.is_initialized(), "run before any GPU call of this process (module sorts first)"
    two = _run(2, 8192, 3, str(tmp_path / "w2.npz"))
    one = _run(1, 8192, 3, str(tmp_path / "w1.npz"))
    assert int(two["world"]) == 2 and int(one["world"]) == 1
    # 4096 walkers per rank take the speculative launch; one rank with 8192 runs the half steps
    # (tests/test_gpu_samplers.py proves those two bit-identical on one rank)
    assert bool(two["speculative"])
    np.testing.assert_array_equal(two["positions"], one["positions"])
    np.testing.assert_array_equal(two["lnprob"], one["lnprob"])
    np.testing.assert_array_equal(two["naccepted"], one["naccepted"])
    assert 0 < two["naccepted"].sum() < 3 * 8192
    assert np.isfinite(two["lnprob"]).all()
    print(f"world 2 == world 1 over 3 iterations of 8192 walkers; refined walker-directions "
          f"{int(two['refined'])} (rank 0) / {int(one['refined'])}")

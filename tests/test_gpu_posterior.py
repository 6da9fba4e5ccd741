"""Config 3 posterior parity: HD155358.vels, 4096-walker affine ensemble on the GPU.

Statistical parity in the reference's own style (its notebooks compare samplers with KS tests and
print posterior means):
  * the reference's reported posterior mean ((Ex)HD155358.ipynb cell 12, emcee, 50 post-burn-in
    samples) lies within 1 posterior standard deviation of ours for every parameter;
  * our two independent samplers (affine stretch and batched MH) agree: KS < 0.1 per marginal
    and |mean difference| < 0.25 sd.
"""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_hd155358_posterior_parity():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import posterior_hd155358 as P

    out = P.main(W=4096, iters=600, mh_steps=3000)
    sd = np.array(out["affine_sd"])
    assert np.all(np.abs(out["ref_minus_ours_in_sd"]) < 1.0), out["ref_minus_ours_in_sd"]
    assert max(out["ks_affine_vs_mh"]) < 0.1, out["ks_affine_vs_mh"]
    dm = np.abs(np.array(out["affine_mean"]) - np.array(out["mh_mean"])) / sd
    assert np.all(dm < 0.25), dm
    assert 0.1 < out["affine_acceptance"] < 0.7

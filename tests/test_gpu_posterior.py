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


def test_ben21_posterior_matches_reference_smala_ghosts():
    """G5: the reference's own SMALA run on TEST_2-1_COMPACT.vels logged the RV curves of 45
    posterior samples (log_Ben-2-1 RDMGHOSTS).  Our posterior (device affine ensemble from the
    same start state) reproduces them: the ghosts' mean curve within 1.5 of our posterior sd at
    every one of the 1000 times (median < 0.5), and their spread within 30 % of ours (median ratio;
    45 samples estimate an sd to ~10 %).  Measured: max 0.79, median 0.24, ratio 0.90."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import posterior_ben21 as B

    out = B.main()
    z, r = out["mean_diff_in_our_sd"], out["sd_ratio_ref_over_ours"]
    assert z["max"] < 1.5 and z["median"] < 0.5, z
    assert 0.7 < r["median"] < 1.3, r

"""The reference's benchmark scripts' workloads (mcmc_benchmark_{mh,emcee,smala}.py) through the
reference-named API (scripts/reference_workloads.py), shortened: they run end to end on the GPU
and behave like samplers (acceptance in (0, 1], finite log-probabilities)."""
import os
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_reference_benchmark_workloads_run():
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    import reference_workloads as R

    out = {r["workload"]: r for r in R.main(["--scale", "0.01"])}
    mh, em, sm = (out[f"mcmc_benchmark_{k}.py"] for k in ("mh", "emcee", "smala"))
    for r in (mh, em, sm):
        assert 0.0 < r["acceptance_rate"] <= 1.0, r
        assert len(r["ac_times"]) == 10
    assert em["finite_lnprob"] and em["errors"] == 0
    assert sm["finite_logp"]

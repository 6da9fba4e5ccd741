"""Sanitizers on host code (GPU sanitizers are not available on this pool):
AddressSanitizer + UndefinedBehaviorSanitizer builds of (a) the CPU oracle with a driver over its
restatements (oracle/sanitize_driver.c) and (b) the C ABI's host side -- argument checks and
rvm_plan_create's schedule building (rvel-mcmc_amd/csrc/host_sanitize.cpp; the first HIP call
fails on a GPU-less host, an error return the driver expects).  CPU only."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


def _run(cmd, env=None):
    return subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=600)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_oracle_under_asan_ubsan():
    b = _run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"])
    assert b.returncode == 0, b.stderr
    r = _run([os.path.join(ROOT, "oracle", "_san", "oracle_san")])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr


@pytest.mark.skipif(shutil.which("hipcc") is None and not os.path.exists("/opt/rocm/bin/hipcc"),
                    reason="hipcc not available")
def test_abi_host_side_under_asan_ubsan():
    b = _run(["make", "-s", "-C", os.path.join(ROOT, "rvel-mcmc_amd"), "sanitize-host"])
    assert b.returncode == 0, b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0")  # the HIP runtime keeps its allocations
    r = _run([os.path.join(ROOT, "rvel-mcmc_amd", "build", "abi_san")], env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "0 failures" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr

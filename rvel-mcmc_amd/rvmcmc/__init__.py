"""rvmcmc -- MI355X-native radial-velocity MCMC (the rvel-mcmc hot path on gfx950).

Reference-compatible modules: state, observations, mcmc, driver.  Batched engine: engine,
ensemble, smala.  Native code: librvmcmc.so (HIP kernels + C ABI, include/rvmcmc.h).
"""
from . import _lib  # noqa: F401

__all__ = ["state", "observations", "mcmc", "driver", "engine", "ensemble", "smala"]

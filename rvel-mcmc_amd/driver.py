"""Reference import name `driver` (the notebooks and mcmc_benchmark_*.py do `import driver`)."""
from rvmcmc.driver import *  # noqa: F401,F403
from rvmcmc import driver as _m

globals().update({k: v for k, v in vars(_m).items() if not k.startswith("__")})

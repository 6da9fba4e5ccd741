"""Reference import name `observations` (the notebooks and mcmc_benchmark_*.py do `import observations`)."""
from rvmcmc.observations import *  # noqa: F401,F403
from rvmcmc import observations as _m

globals().update({k: v for k, v in vars(_m).items() if not k.startswith("__")})

"""Reference import name `mcmc` (the notebooks and mcmc_benchmark_*.py do `import mcmc`)."""
from rvmcmc.mcmc import *  # noqa: F401,F403
from rvmcmc import mcmc as _m

globals().update({k: v for k, v in vars(_m).items() if not k.startswith("__")})

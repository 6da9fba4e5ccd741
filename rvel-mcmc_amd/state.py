"""Reference import name `state` (the notebooks and mcmc_benchmark_*.py do `import state`)."""
from rvmcmc.state import *  # noqa: F401,F403
from rvmcmc import state as _m

globals().update({k: v for k, v in vars(_m).items() if not k.startswith("__")})

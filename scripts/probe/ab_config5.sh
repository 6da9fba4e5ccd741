for lib in scripts/probe/librvmcmc_old.so rvel-mcmc_amd/rvmcmc/librvmcmc.so; do
timeout -k 10 120 python -c "
import sys; sys.path[:0]=['scripts','rvel-mcmc_amd','oracle','tests']
from rvmcmc import _lib; _lib.LIB_PATH='$PWD/$lib'
import configs_bench as cb, json
print('$lib', json.dumps(cb.config5())[:200])
" 2>&1 | grep -v amdgpu.ids || exit 1; done

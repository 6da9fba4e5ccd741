#!/bin/bash
# (History: round 1's level-split layout with the last-arriver combine; the lib_*.so variants were
# built from commit 119fcdb with its RVM_EXP_* macros, which the current kernel no longer has.
# The current layout is measured with scripts/probe/prof_clock.py.)
# A/B of the level-split hand-off (plain 6144-walker launches, S2): product library, combine
# skipped, hand-off writes + combine skipped, type-B blocks first, LDS-coupled layout.
set -euo pipefail
export REPS=${REPS:-30}
for v in product nocombine nohandoff bfirst; do
  if [ $v = product ]; then lib=rvel-mcmc_amd/rvmcmc/librvmcmc.so; else lib=scripts/probe/lib_$v.so; fi
  echo "== $v"; RVM_LIB=$PWD/$lib timeout -k 10 120 python scripts/kbench.py ${WS:-6144 2048}
done
echo "== lds-coupled"; RVM_NO_LEVEL_SPLIT=1 timeout -k 10 120 python scripts/kbench.py ${WS:-6144}

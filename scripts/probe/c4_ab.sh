#!/bin/bash
# config 4 (SMALA FD) A/B over one library knob (AB_VAR / AB_VALS): configs_bench.py 4, and the
# steady-state step quantiles of scripts/probe/smala_tail_probe.py
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${T:-c4ab}
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${AB_VALS:-1 0}; do
    env $AB_VAR=$v timeout -k 10 300 python -u scripts/probe/smala_tail_probe.py 1000 ${STEPS:-400} 2>/dev/null \
      | grep ms_mean | sed "s|^{|{\"$AB_VAR\": \"$v\", |" >> gpurun_out/${T}_c4_tail.jsonl
  done
done
cat gpurun_out/${T}_c4_tail.jsonl

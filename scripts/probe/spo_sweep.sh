#!/bin/bash
# Steady-state rate of configs (CFGS) against the plan's base steps per shortest period (SPOS):
# scripts/configs_bench.py with RVM_CONFIGS_SPO.  Output: gpurun_out/${T}_spo_sweep.jsonl
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${T:-spo}
mkdir -p gpurun_out
for spo in ${SPOS:-8 12 16}; do
  RVM_CONFIGS_SPO=$spo timeout -k 10 300 python -u scripts/configs_bench.py ${CFGS:-3 2w} \
    | sed "s|^{|{\"spo\": $spo, |" >> gpurun_out/${T}_spo_sweep.jsonl
done
cut -c1-330 gpurun_out/${T}_spo_sweep.jsonl

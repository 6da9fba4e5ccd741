#!/bin/bash
# A/B (one box): past the cut guard, the bound chi2 - min(k d, 100 est) (RVM_CUT_GUARD_K = k) against
# the product's chi2 - 100 est (k = 0), interleaved twice; then the 2048-walker parity sweep at KS's
# last k.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${T:-r06zs}
mkdir -p gpurun_out
for rep in 1 2; do
  for k in ${KS:-0 10}; do
    export RVM_CUT_GUARD_K=$k
    timeout -k 10 300 python -u scripts/configs_bench.py ${CFGS:-3 2w 5} \
      | sed "s|^{|{\"cut_guard_k\": $k, |" >> gpurun_out/${T}_cut_k_ab.jsonl 2>> gpurun_out/${T}_cut_k_ab.err
    ITERS=300 timeout -k 10 200 python -u scripts/probe/steady_bench.py 4,5,6,7:5e-7 \
      | sed "s|^{|{\"cut_guard_k\": $k, |" >> gpurun_out/${T}_cut_k_ab.jsonl 2>> gpurun_out/${T}_cut_k_ab.err
  done
done
cut -c1-200 gpurun_out/${T}_cut_k_ab.jsonl
if [ -n "${SWEEP:-1}" ]; then
  timeout -k 10 500 python -u scripts/probe/parity_sweep.py 2048 3 > gpurun_out/${T}_parity_sweep_k.jsonl 2> gpurun_out/${T}_parity_sweep_k.err
  cut -c1-400 gpurun_out/${T}_parity_sweep_k.jsonl
fi

#!/bin/bash
# A/B (one box): the certain-reject cut's eccentricity guard on (default) and off (RVM_CUT_GUARD=0),
# interleaved twice: configs 3, 2w, 5 at their steady states and the bench chain's steady state.
# GUARDS: space-separated on[:factor] entries (RVM_CUT_GUARD, RVM_CUT_FACTOR), default "1 0".
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${T:-r06zm}
mkdir -p gpurun_out
for rep in 1 2; do
  for cg in ${GUARDS:-1 0}; do
    f=${cg#*:}; g=${cg%%:*}; [ "$f" = "$cg" ] && f=""
    export RVM_CUT_GUARD=$g
    if [ -n "$f" ]; then export RVM_CUT_FACTOR=$f; else unset RVM_CUT_FACTOR; fi
    timeout -k 10 300 python -u scripts/configs_bench.py ${CFGS:-3 2w 5} \
      | sed "s|^{|{\"cut_guard\": \"$cg\", |" >> gpurun_out/${T}_cut_guard_ab.jsonl 2>> gpurun_out/${T}_cut_guard_ab.err
    ITERS=300 timeout -k 10 200 python -u scripts/probe/steady_bench.py 4,5,6,7:5e-7 \
      | sed "s|^{|{\"cut_guard\": \"$cg\", |" >> gpurun_out/${T}_cut_guard_ab.jsonl 2>> gpurun_out/${T}_cut_guard_ab.err
  done
done
cut -c1-300 gpurun_out/${T}_cut_guard_ab.jsonl

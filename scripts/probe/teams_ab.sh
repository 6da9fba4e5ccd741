#!/bin/bash
# Refinement team ladder (round 6): the layouts' bit-identity tests, then the steady-state A/B of the
# team count on the bench chain (scripts/probe/steady_bench.py) and on configs CFGS at their steady
# state.  A variant "k" runs at most k teams with the depth hint, "kf" always k teams (RVM_TEAMS_HINT=0).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${T:-teams}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_resolve.py -k "layouts" -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
tail -2 gpurun_out/${T}_pytest.log
run() {  # variant, command...
  local k=$1; shift
  local hint=1
  [[ $k == *f ]] && hint=0
  RVM_TEAMS_HINT=$hint RVM_REFINE_TEAMS=${k%f} "$@"
}
for rep in 1 2; do
  for k in ${AB_VALS:-2 4 4f}; do
    run $k env ITERS=${AB_ITERS:-400} timeout -k 10 120 python -u scripts/probe/steady_bench.py 4,5,6,7:5e-7 \
      | sed "s|^{|{\"teams\": \"$k\", |" >> gpurun_out/${T}_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/${T}_ab.jsonl'):
    d=json.loads(l); print(d['teams'], round(d['ms_per_iteration'],4), round(d['logl_kernel_ms'],4), round(d['refine_kernel_ms'],4), [round(x,3) for x in d['refine_kernel_ms_quantiles']], d['faults']['refined'])
"
for k in ${CFG_TEAMS:-4 4f}; do
  run $k timeout -k 10 400 python -u scripts/configs_bench.py ${CFGS:-3 2w 5} \
    | sed "s|^{|{\"teams\": \"$k\", |" >> gpurun_out/${T}_configs.jsonl
done
python3 -c "
import json
for l in open('gpurun_out/${T}_configs.jsonl'):
    d=json.loads(l); print(d['teams'], d['config'][:40], round(d.get('ms_per_iteration', 0), 3), d.get('faults_in_window'))
"
# the paired 3-planet layout (RVM_CX_PAIRS) on config 5, when PAIRS_AB is set
if [ -n "${PAIRS_AB:-}" ]; then
  for rep in 1 2; do
    for v in 1 0; do
      RVM_CX_PAIRS=$v timeout -k 10 400 python -u scripts/configs_bench.py 5 \
        | sed "s|^{|{\"cx_pairs\": $v, |" >> gpurun_out/${T}_pairs.jsonl
    done
  done
  python3 -c "
import json
for l in open('gpurun_out/${T}_pairs.jsonl'):
    d=json.loads(l); print(d['cx_pairs'], round(d['ball_window']['ms_per_iteration'], 3), round(d['ms_per_iteration'], 3))
"
fi

#!/bin/bash
# Round-4 team refinement check: steady-state probe with teams on and off (A/B on one box), then
# the adaptive-resolution and IAS15 decision tests.  Test failures (pytest exit 1) are reported;
# any other failure stops the chain.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r04s}
timeout -k 10 200 python -u scripts/probe/steady_bench.py 4,5,6,7:5e-7 > gpurun_out/${T}_steady_teams.jsonl 2>&1 || { cat gpurun_out/${T}_steady_teams.jsonl; exit 1; }
cat gpurun_out/${T}_steady_teams.jsonl
RVM_REFINE_TEAMS=0 timeout -k 10 200 python -u scripts/probe/steady_bench.py 4,5,6,7:5e-7 > gpurun_out/${T}_steady_noteams.jsonl 2>&1 || { cat gpurun_out/${T}_steady_noteams.jsonl; exit 1; }
cat gpurun_out/${T}_steady_noteams.jsonl
rc=0
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_resolve.py \
    tests/test_gpu_ias15_decisions.py > gpurun_out/${T}_pytest_dec.log 2>&1 || rc=$?
grep -E "FAIL|ERROR" gpurun_out/${T}_pytest_dec.log | tail -20 || true
tail -2 gpurun_out/${T}_pytest_dec.log
exit $rc

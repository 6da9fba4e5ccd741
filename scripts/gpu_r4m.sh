#!/bin/bash
# Round-4: team B's merge loads in chunks -- the resolve and decision tests, then the steady state.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${T:-r04zl}
mkdir -p gpurun_out
rc=0
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_resolve.py \
    tests/test_gpu_ias15_decisions.py > gpurun_out/${T}_pytest.log 2>&1 || rc=$?
grep -E "FAIL|ERROR" gpurun_out/${T}_pytest.log | tail -20 || true
tail -1 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 200 python scripts/probe/steady_bench.py 4,5,6,7:5e-7 >> gpurun_out/${T}_steady.jsonl 2>> gpurun_out/${T}_steady.err || { tail -20 gpurun_out/${T}_steady.err; exit 1; }
done
cut -c1-200 gpurun_out/${T}_steady.jsonl

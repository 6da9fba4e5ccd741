#!/bin/bash
# Round-4 check after a rule change: the adaptive-resolution and IAS15 decision tests, the
# steady-state probe, and a kernel trace of the steady state (where its time goes).  Each GPU step
# has its own limit; the chain stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r04g}
# (pytest exit 1 = test failures: reported, the chain goes on; anything else stops it)
rc=0
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread ${TESTS:-tests/test_gpu_resolve.py \
    tests/test_gpu_ias15_decisions.py} > gpurun_out/${T}_pytest_dec.log 2>&1 || rc=$?
grep -E "FAIL|ERROR" gpurun_out/${T}_pytest_dec.log | tail -20 || true
tail -3 gpurun_out/${T}_pytest_dec.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u scripts/probe/steady_bench.py > gpurun_out/${T}_steady.jsonl 2>&1 || { cat gpurun_out/${T}_steady.jsonl; exit 1; }
cat gpurun_out/${T}_steady.jsonl
mkdir -p gpurun_out/${T}_prof_steady
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_steady" -o run --output-format csv -- \
    python3 "$R/scripts/probe/steady_bench.py" 4,5,6,7:5e-7 > "$R/gpurun_out/${T}_steady_under_rocprof.jsonl" 2>&1
echo done

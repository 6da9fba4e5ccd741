#!/bin/bash
# Round-4 eager halving passes: their tests and the adaptive-resolution / decision tests, then the
# small-launch configs (SMALA FD and exact, reference-API Mh) with eager passes on and off.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r04x}
rc=0
timeout -k 10 700 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_resolve.py \
    tests/test_gpu_ias15_decisions.py > gpurun_out/${T}_pytest_dec.log 2>&1 || rc=$?
grep -E "FAIL|ERROR" gpurun_out/${T}_pytest_dec.log | tail -20 || true
tail -2 gpurun_out/${T}_pytest_dec.log
[ $rc -le 1 ] || exit $rc
RVM_EAGER=1 timeout -k 10 300 python scripts/configs_bench.py 4 4x 1 > gpurun_out/${T}_configs_eager.jsonl 2> gpurun_out/${T}_configs_eager.err || { tail -20 gpurun_out/${T}_configs_eager.err; exit 1; }
RVM_EAGER=0 timeout -k 10 300 python scripts/configs_bench.py 4 4x 1 > gpurun_out/${T}_configs_noeager.jsonl 2> gpurun_out/${T}_configs_noeager.err || { tail -20 gpurun_out/${T}_configs_noeager.err; exit 1; }
cat gpurun_out/${T}_configs_eager.jsonl gpurun_out/${T}_configs_noeager.jsonl
exit $rc

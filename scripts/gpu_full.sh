#!/bin/bash
# Whole GPU test suite (one process), then smoke.  Each step time-limited; stops at the first failure.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3full}
RVM_PARITY_REPORT=gpurun_out/${TAG}_parity.jsonl timeout -k 10 ${TTEST:-900} python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; grep -E "passed|failed|FAILED|Error" gpurun_out/${TAG}_pytest.log | tail -15; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { cat gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log

#!/bin/bash
# Round-4: per-iteration likelihood-kernel profile at the steady state (timing build), the whole
# GPU test suite, then the default bench line.  Test failures (pytest exit 1) are reported and the
# chain goes on; any other failure stops it.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r04n}
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 200 python -u scripts/probe/steady_prof.py > gpurun_out/${T}_steady_prof.jsonl 2>&1 || { tail -20 gpurun_out/${T}_steady_prof.jsonl; exit 1; }
fi
rc=0
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_pytest_gpu.log 2>&1 || rc=$?
grep -E "FAIL|ERROR" gpurun_out/${T}_pytest_gpu.log | tail -20 || true
tail -2 gpurun_out/${T}_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json

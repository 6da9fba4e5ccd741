#!/bin/bash
# Round-4 check: adaptive-resolution GPU tests first (the refinement kernel), then the rest, the
# steady-state probe and a short bench.  Each GPU step has its own limit; the chain stops at the
# first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r04e}
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_resolve.py \
    > gpurun_out/${T}_pytest_resolve.log 2>&1 || { tail -60 gpurun_out/${T}_pytest_resolve.log; exit 1; }
tail -3 gpurun_out/${T}_pytest_resolve.log
timeout -k 10 200 python -u scripts/probe/steady_bench.py > gpurun_out/${T}_steady.jsonl 2>&1 || { cat gpurun_out/${T}_steady.jsonl; exit 1; }
cat gpurun_out/${T}_steady.jsonl
# A/B: both directions of a walker group in one workgroup (RVM_REFINE_SPLIT=0) against the split
RVM_REFINE_SPLIT=0 timeout -k 10 200 python -u scripts/probe/steady_bench.py 4,5,6,7:5e-7 > gpurun_out/${T}_steady_nosplit.jsonl 2>&1 || { cat gpurun_out/${T}_steady_nosplit.jsonl; exit 1; }
cat gpurun_out/${T}_steady_nosplit.jsonl
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests \
    --ignore=tests/test_gpu_resolve.py > gpurun_out/${T}_pytest_gpu.log 2>&1 || { grep -E "PASS|FAIL|ERROR" gpurun_out/${T}_pytest_gpu.log | tail -40; tail -80 gpurun_out/${T}_pytest_gpu.log; exit 1; }
tail -3 gpurun_out/${T}_pytest_gpu.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 3 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
cat gpurun_out/${T}_bench.json

#!/bin/bash
# Round-4: the eager replay's loads in chunks -- the eager and fused tests, then config 4 under
# rocprofv3 and plain (and the eager A/B).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
T=${T:-r04zj}
mkdir -p gpurun_out/${T}_prof_config4
rc=0
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_resolve.py \
    tests/test_gpu_fused_chains.py > gpurun_out/${T}_pytest.log 2>&1 || rc=$?
grep -E "FAIL|ERROR" gpurun_out/${T}_pytest.log | tail -20 || true
tail -1 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || exit $rc
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_config4" -o run --output-format csv -- \
    python3 "$R/scripts/configs_bench.py" 4 > "$R/gpurun_out/${T}_config4_under_rocprof.jsonl" 2> "$R/gpurun_out/${T}_config4_under_rocprof.err"
cd "$R"
timeout -k 10 200 python scripts/configs_bench.py 4 4 1 > gpurun_out/${T}_configs.jsonl 2> gpurun_out/${T}_configs.err || { tail -20 gpurun_out/${T}_configs.err; exit 1; }
RVM_EAGER=0 timeout -k 10 200 python scripts/configs_bench.py 4 > gpurun_out/${T}_configs_noeager.jsonl 2> gpurun_out/${T}_configs.err || { tail -20 gpurun_out/${T}_configs.err; exit 1; }
cat gpurun_out/${T}_config4_under_rocprof.jsonl gpurun_out/${T}_configs.jsonl gpurun_out/${T}_configs_noeager.jsonl | grep config | cut -c1-60,150-330

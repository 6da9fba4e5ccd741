#!/bin/bash
# GPU tests, then (if green) the default bench and a rocprofv3 kernel-stats run of a short bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --ess-iters 0 --no-cpu > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err" || exit 1
cd "$R"
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
cut -c1-200 gpurun_out/kernel_stats.csv | head -4

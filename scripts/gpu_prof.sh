#!/bin/bash
# kernel micro-bench + rocprofv3 kernel-trace of a short bench run
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python scripts/kbench.py 2048 4096 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kbench.log
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --ess-iters 0 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.err"
  cd "$GRAFT_REPO_ROOT"
  cat gpurun_out/prof_bench.json
  find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \;
fi

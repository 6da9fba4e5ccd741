#!/bin/bash
# One GPU-box session: GPU tests, smoke, short bench.  Each GPU step has its own time limit and
# the chain stops at the first failure (gpurun runs this under bash -o pipefail).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
STEPS=${STEPS:-10}
timeout -k 10 420 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 200 python scripts/kbench.py 2048 4096 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kbench.log
timeout -k 10 300 python bench.py --steps "$STEPS" --warmup 2 > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json

#!/bin/bash
# Quick kernel iteration on the GPU box: likelihood parity tests + kernel micro-bench.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_logl.py -q -x > gpurun_out/pytest_quick.log 2>&1 || { tail -40 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
timeout -k 10 200 python scripts/kbench.py ${KB_W:-2048 4096} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/kbench.log

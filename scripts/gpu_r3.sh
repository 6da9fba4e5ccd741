#!/bin/bash
# Round-3 GPU iteration: the named test files (default: adaptive resolution + likelihood + samplers),
# the kernel micro-bench and a short bench line.  Every GPU step has its own time limit; the chain
# stops at the first failure.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_resolve.py tests/test_gpu_logl.py tests/test_gpu_samplers.py}
TAG=${TAG:-r3}
timeout -k 10 ${TTEST:-500} python -u -m pytest $TESTS -x -v -s --timeout 150 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|W=" gpurun_out/${TAG}_pytest.log | tail -40; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python scripts/kbench.py 2048 6144 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_kbench.log || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --ess-iters 0 --no-cpu > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json

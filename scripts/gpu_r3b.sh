#!/bin/bash
# Round-3 GPU iteration 2: named tests, the refinement-cost probe on the bench's slots, a short bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TESTS=${TESTS:-tests/test_gpu_resolve.py}
TAG=${TAG:-r3b}
timeout -k 10 ${TTEST:-500} python -u -m pytest $TESTS -x -v -s --timeout 150 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|passed|failed|W=" gpurun_out/${TAG}_pytest.log | tail -30; [ $rc = 0 ] || exit $rc
timeout -k 10 200 python scripts/probe/resolve_cost.py scripts/probe/slots_it23.npz scripts/probe/slots_it2000.npz 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_cost.jsonl || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --ess-iters 0 --no-cpu > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 400 python scripts/probe/steady_bench.py ${STEADY:-} 2>&1 | grep -v amdgpu.ids | tee gpurun_out/${TAG}_steady.jsonl || exit 1
for spec in ${BENCH_VARIANTS:-}; do  # "LEVELS:TOL" variants of the bench line
  lv=${spec%%:*}; tol=${spec##*:}
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --ess-iters 0 --no-cpu --levels $lv --resolve-tol $tol > gpurun_out/${TAG}_bench_${lv}_${tol}.json 2>> gpurun_out/${TAG}_bench.err || exit 1
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1], round(d['value']/1e6,3), 'M', d['ms_per_step'], d['resolve'])" gpurun_out/${TAG}_bench_${lv}_${tol}.json
done

# quick GPU check of a library change: the steady-state probe twice and the refinement / contract tests
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${T:-r06x}
for rep in 1 2; do
  ITERS=400 timeout -k 10 120 python -u scripts/probe/steady_bench.py 4,5,6,7:5e-7 >> gpurun_out/${T}_steady.jsonl
done
python3 -c "
import json
for l in open('gpurun_out/${T}_steady.jsonl'):
    d=json.loads(l); print(round(d['ms_per_iteration'],4), round(d['logl_kernel_ms'],4), round(d['refine_kernel_ms'],4), [round(x,3) for x in d['refine_kernel_ms_quantiles']], d['faults'])
"
timeout -k 10 900 python -u -m pytest tests/test_gpu_resolve.py tests/test_gpu_contract.py ${EXTRA_TESTS:-} -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3

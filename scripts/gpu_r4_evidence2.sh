#!/bin/bash
# Round-4 evidence, part 2: every BASELINE config, the IAS15 decision tests with their JSON report,
# the 2-rank gloo rehearsal of the multi-GPU bench, and the default bench line (with
# profiles/pmc_latest.json measured on this kernel).  Test failures (pytest exit 1) are reported
# and the chain goes on; any other failure stops it.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
T=${T:-r04v}
mkdir -p gpurun_out
timeout -k 10 400 python scripts/configs_bench.py > gpurun_out/${T}_configs.jsonl 2> gpurun_out/${T}_configs.err || { tail -20 gpurun_out/${T}_configs.err; exit 1; }
cat gpurun_out/${T}_configs.jsonl
rc=0
RVM_PARITY_REPORT=gpurun_out/${T}_parity_ias15.jsonl timeout -k 10 500 python -u -m pytest -q --timeout 300 \
    --timeout-method thread tests/test_gpu_ias15_decisions.py > gpurun_out/${T}_pytest_dec.log 2>&1 || rc=$?
tail -2 gpurun_out/${T}_pytest_dec.log
[ $rc -le 1 ] || exit $rc
RVM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --ess-iters 40 \
  > gpurun_out/${T}_bench_n2_gloo.json 2> gpurun_out/${T}_bench_n2_gloo.err || { tail -30 gpurun_out/${T}_bench_n2_gloo.err; exit 1; }
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
echo evidence2 done

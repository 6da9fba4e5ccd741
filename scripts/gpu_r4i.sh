#!/bin/bash
# Round-4 eager passes: the eager bit-identity tests, then config 4 with eager passes 1, 2 and off
# (two rounds each, interleaved: one box's A/B).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r04zd}
timeout -k 10 300 python -u -m pytest -v --timeout 120 --timeout-method thread tests/test_gpu_resolve.py \
    -k "eager or layouts" > gpurun_out/${T}_pytest.log 2>&1 || { tail -20 gpurun_out/${T}_pytest.log; exit 1; }
tail -1 gpurun_out/${T}_pytest.log
for r in 1 2; do
  for m in p1 p2 off; do
    case $m in p1) e=1; p=1;; p2) e=1; p=2;; off) e=0; p=1;; esac
    echo -n "$m " >> gpurun_out/${T}_ab.txt
    RVM_EAGER=$e RVM_EAGER_PASSES=$p timeout -k 10 200 python scripts/configs_bench.py 4 >> gpurun_out/${T}_ab.txt 2> gpurun_out/${T}_ab.err || { tail -20 gpurun_out/${T}_ab.err; exit 1; }
  done
done
cut -c1-40,200-300 gpurun_out/${T}_ab.txt

set -euo pipefail
mkdir -p gpurun_out
export RVM_PARITY_REPORT=$PWD/gpurun_out/parity_ias15.jsonl
rm -f $RVM_PARITY_REPORT
timeout -k 10 600 python -u -m pytest tests/test_gpu_ias15_decisions.py -x -v -s --timeout 300 --timeout-method thread > gpurun_out/pytest_ias15.log 2>&1 || { tail -60 gpurun_out/pytest_ias15.log; exit 1; }
tail -15 gpurun_out/pytest_ias15.log
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json

#!/bin/bash
# Measure the T1 (kernel vs oracle, same algorithm) maxima of every T1 comparison in the GPU tests.
set -euo pipefail
mkdir -p gpurun_out
export RVM_T1_REPORT=$PWD/gpurun_out/t1_report.jsonl
rm -f $RVM_T1_REPORT
timeout -k 10 400 python -u -m pytest tests/test_gpu_logl.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_t1.log 2>&1 || { tail -40 gpurun_out/pytest_t1.log; exit 1; }
tail -3 gpurun_out/pytest_t1.log
cat $RVM_T1_REPORT

#!/bin/bash
# GPU tests (all, incl. the IAS15 decision parity report) + plain-launch kernel timings.
set -euo pipefail
mkdir -p gpurun_out
export RVM_PARITY_REPORT=$PWD/gpurun_out/parity_ias15.jsonl RVM_T1_REPORT=$PWD/gpurun_out/t1_report.jsonl
rm -f $RVM_PARITY_REPORT $RVM_T1_REPORT
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -60 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
REPS=30 timeout -k 10 120 python scripts/kbench.py ${WS:-6144 2048} 2>&1 | grep -v amdgpu.ids

#!/bin/bash
# Round evidence in one GPU call: GPU tests, smoke, the PMC passes over the bench's own launches
# (summary keyed to the kernel sources, copied to profiles/pmc_latest.json for bench.py), bench
# (N=1, with ESS and CPU baseline), rocprofv3 --kernel-trace --stats of a short bench run, every
# BASELINE config, and the 2-rank rehearsal of the sharded bench.  Each GPU step has its own time limit; the chain stops at the first failure.
# SKIP_TESTS=1 / SKIP_CONFIGS=1 / SKIP_PMC=1 leave those steps out.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  RVM_PARITY_REPORT=gpurun_out/parity_ias15.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { cat gpurun_out/smoke.log; exit 1; }
fi
if [ "${SKIP_PMC:-0}" != 1 ]; then
  bash scripts/pmc_profile.sh > gpurun_out/pmc_run.log 2>&1 || { tail -20 gpurun_out/pmc_run.log; exit 1; }
  grep -E "hbm_bytes_per_launch\"|fp64_flops_per_eval|kernel_signature" gpurun_out/pmc/summary.txt
  cp gpurun_out/pmc/pmc_latest.json profiles/pmc_latest.json
fi
timeout -k 10 300 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
# the N > 1 flow of bench.py (2 ranks on this one GPU over gloo: correctness, not scaling)
bash scripts/gpu_rehearse_dist.sh > /dev/null
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 10 --warmup 2 --ess-iters 0 --no-cpu --no-fixed-step-ref > "$R/gpurun_out/prof_bench.json" 2> "$R/gpurun_out/prof_bench.err"
cd "$R"
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} gpurun_out/kernel_stats.csv \;
cat gpurun_out/kernel_stats.csv | cut -c1-200
if [ "${SKIP_CONFIGS:-0}" != 1 ]; then
  timeout -k 10 400 python scripts/configs_bench.py 2>&1 | grep -v amdgpu.ids > gpurun_out/configs.jsonl
  cut -c1-220 gpurun_out/configs.jsonl
fi

#!/bin/bash
# Every BASELINE config (scripts/configs_bench.py), then rocprofv3 --kernel-trace --stats over the
# bench's own window (--steps 20 --warmup 3, as the default bench line): per-launch durations of the
# timed iterations.  Each GPU step has its own time limit; the chain stops at the first failure.
set -euo pipefail
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python scripts/configs_bench.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof20" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --ess-iters 0 --no-cpu --no-fixed-step-ref --kernel-iters 0 > "$R/gpurun_out/prof20_bench.json" 2> "$R/gpurun_out/prof20_bench.err"

#!/bin/bash
# Round-4: SMALA config 4 under rocprofv3 at HEAD (eager pass 1 on): kernel trace + stats.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
T=${T:-r04zg}
mkdir -p gpurun_out/${T}_prof_config4
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_config4" -o run --output-format csv -- \
    python3 "$R/scripts/configs_bench.py" 4 > "$R/gpurun_out/${T}_config4_under_rocprof.jsonl" 2> "$R/gpurun_out/${T}_config4_under_rocprof.err"
cd "$R"
timeout -k 10 200 python scripts/configs_bench.py 4 1b 2 > gpurun_out/${T}_configs.jsonl 2> gpurun_out/${T}_configs.err || { tail -20 gpurun_out/${T}_configs.err; exit 1; }
cat gpurun_out/${T}_config4_under_rocprof.jsonl gpurun_out/${T}_configs.jsonl | grep config
head -12 gpurun_out/${T}_prof_config4/run_kernel_stats.csv | cut -c1-220

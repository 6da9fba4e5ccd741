#!/bin/bash
# Round-4 evidence, part 1: smoke, rocprofv3 kernel traces + stats of the bench window and of the
# steady state, then the PMC passes over the bench's own launches (scripts/pmc_profile.sh ->
# gpurun_out/pmc/pmc_latest.json).  Each step has its own limit; the chain stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
T=${T:-r04u}
mkdir -p gpurun_out/${T}_prof_bench gpurun_out/${T}_prof_steady
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { cat gpurun_out/${T}_smoke.log; exit 1; }
tail -2 gpurun_out/${T}_smoke.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_bench" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 20 --warmup 3 --ess-iters 0 --no-cpu --no-fixed-step-ref \
    > "$R/gpurun_out/${T}_bench_under_rocprof.json" 2> "$R/gpurun_out/${T}_bench_under_rocprof.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_steady" -o run --output-format csv -- \
    python3 "$R/scripts/probe/steady_bench.py" 4,5,6,7:5e-7 > "$R/gpurun_out/${T}_steady_under_rocprof.jsonl" 2>&1
cd "$R"
timeout -k 10 900 bash scripts/pmc_profile.sh > gpurun_out/${T}_pmc.log 2>&1 || { tail -20 gpurun_out/${T}_pmc.log; exit 1; }
cp gpurun_out/pmc/pmc_latest.json gpurun_out/${T}_pmc_latest.json
tail -5 gpurun_out/${T}_pmc.log
echo evidence1 done

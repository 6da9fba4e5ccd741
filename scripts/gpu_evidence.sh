#!/bin/bash
# Bench evidence in one call (T = tag): the default bench line; the steady-state bench under
# rocprofv3 (kernel trace + stats, and the last dispatches' means beside that run's own line); the PMC
# passes over the steady-state launch sequence (scripts/pmc_profile.sh -> pmc_latest.json).  Each GPU
# step has its own time limit; the chain stops at the first failure.  STEPS selects what runs
# (default "bench prof pmc").
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
T=${T:-r05}
STEPS=${STEPS:-"bench prof pmc"}
mkdir -p gpurun_out
for step in $STEPS; do
  case $step in
    bench)
      timeout -k 10 500 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err \
        || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
      head -c 600 gpurun_out/${T}_bench.json; echo ;;
    prof)
      mkdir -p gpurun_out/${T}_prof_steady
      cd /tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_steady" -o run --output-format csv -- \
        python3 "$R/bench.py" --steps 20 --warmup 3 --ball-steps 0 --burn-in 3000 --ess-iters 0 --kernel-iters 64 \
        --no-cpu --no-fixed-step-ref > "$R/gpurun_out/${T}_bench_under_rocprof.json" 2> "$R/gpurun_out/${T}_bench_under_rocprof.err"
      cd "$R"
      tr=$(find gpurun_out/${T}_prof_steady -name "*kernel_trace.csv" | head -1)
      python3 scripts/trace_window.py "$tr" 84 > gpurun_out/${T}_rocprof_window.json
      cat gpurun_out/${T}_rocprof_window.json ;;
    pmc)
      timeout -k 10 900 bash scripts/pmc_profile.sh > gpurun_out/${T}_pmc.log 2>&1 || { tail -20 gpurun_out/${T}_pmc.log; exit 1; }
      cp gpurun_out/pmc/pmc_latest.json gpurun_out/${T}_pmc_latest.json
      tail -5 gpurun_out/pmc/summary.txt ;;
  esac
done
echo evidence done

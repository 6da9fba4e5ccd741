#!/bin/bash
# Round-4 final evidence in one call: the whole GPU suite, smoke, the PMC passes over the bench's
# own launches (-> profiles/pmc_latest.json on the box, copied back under gpurun_out/), the bench
# under rocprofv3 (kernel trace + stats with the bench line of the same run), the default bench
# line, the steady state under rocprofv3.  Test failures (pytest exit 1) are reported and the chain
# goes on; any other failure stops it.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
T=${T:-r04z}
mkdir -p gpurun_out/${T}_prof_bench gpurun_out/${T}_prof_steady
rc=0
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${T}_pytest_gpu.log 2>&1 || rc=$?
grep -E "FAIL|ERROR" gpurun_out/${T}_pytest_gpu.log | tail -20 || true
tail -2 gpurun_out/${T}_pytest_gpu.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { cat gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 700 bash scripts/pmc_profile.sh > gpurun_out/${T}_pmc.log 2>&1 || { tail -20 gpurun_out/${T}_pmc.log; exit 1; }
cp gpurun_out/pmc/pmc_latest.json gpurun_out/${T}_pmc_latest.json
cp gpurun_out/pmc/pmc_latest.json profiles/pmc_latest.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_bench" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 20 --warmup 3 --ess-iters 0 --no-cpu --no-fixed-step-ref \
    > "$R/gpurun_out/${T}_bench_under_rocprof.json" 2> "$R/gpurun_out/${T}_bench_under_rocprof.err"
cd "$R"
timeout -k 10 400 python -u bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { tail -30 gpurun_out/${T}_bench.err; exit 1; }
cd /tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_steady" -o run --output-format csv -- \
    python3 "$R/scripts/probe/steady_bench.py" 4,5,6,7:5e-7 > "$R/gpurun_out/${T}_steady_under_rocprof.jsonl" 2>&1
echo final done rc=$rc
exit $rc

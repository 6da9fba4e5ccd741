set -euo pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 > gpurun_out/r04a_bench.json 2> gpurun_out/r04a_bench.err
cat gpurun_out/r04a_bench.json
timeout -k 10 200 python -u scripts/probe/steady_bench.py > gpurun_out/r04a_steady.jsonl 2>&1
cat gpurun_out/r04a_steady.jsonl

#!/bin/bash
# A/B of the halving passes' segments on one box: B = the library in the tree (speculative halving
# segments), A = scripts/probe/librvmcmc_A.so (gated).  Resolve tests on B, then per library the
# steady-state probe and a short bench line; rocprofv3 per-launch trace of B's bench window.
set -euo pipefail
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_resolve.py -x -q --timeout 150 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -20 gpurun_out/ab_pytest.log; exit 1; }
tail -1 gpurun_out/ab_pytest.log
for v in B A; do
  if [ $v = A ]; then cp scripts/probe/librvmcmc_A.so rvel-mcmc_amd/rvmcmc/librvmcmc.so; fi
  timeout -k 10 300 python scripts/probe/steady_bench.py > gpurun_out/ab_steady_$v.jsonl 2> gpurun_out/ab_steady_$v.err
  timeout -k 10 200 python bench.py --steps 20 --warmup 3 --ess-iters 0 --no-cpu > gpurun_out/ab_bench_$v.json 2> gpurun_out/ab_bench_$v.err
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,3), d['ms_per_step'])" gpurun_out/ab_bench_$v.json $v
  cut -c1-160 gpurun_out/ab_steady_$v.jsonl
  if [ $v = B ]; then
    cd /tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/ab_prof" -o run --output-format csv -- python3 "$R/bench.py" --steps 20 --warmup 3 --ess-iters 0 --no-cpu --no-fixed-step-ref --kernel-iters 0 > "$R/gpurun_out/ab_prof_bench.json" 2> "$R/gpurun_out/ab_prof_bench.err"
    cd "$R"
  fi
done

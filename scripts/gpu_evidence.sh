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
STEPS=${STEPS:-"bench prof pmc"}   # also: tests segbench configs
mkdir -p gpurun_out
for step in $STEPS; do
  case $step in
    tests)
      RVM_PARITY_REPORT=gpurun_out/${T}_parity.jsonl timeout -k 10 900 python -u -m pytest tests -m gpu -x -q \
        --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1 \
        || { grep -E "FAIL|Error" gpurun_out/${T}_pytest.log | tail -20; tail -3 gpurun_out/${T}_pytest.log; exit 1; }
      tail -2 gpurun_out/${T}_pytest.log
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 \
        || { cat gpurun_out/${T}_smoke.log; exit 1; }
      tail -1 gpurun_out/${T}_smoke.log ;;
    segbench)
      timeout -k 10 120 ./scripts/probe/seg_bench ${SEG_ARGS:-0.22 32 0.22 112 0.40 112 0.40 224 0.55 112} \
        > gpurun_out/${T}_seg_bench.txt 2>&1 || { cat gpurun_out/${T}_seg_bench.txt; exit 1; }
      cat gpurun_out/${T}_seg_bench.txt ;;
    steadyab)
      # A/B at the bench chain's steady state: the default library against the variants in AB_LIBS
      # (built by make -C rvel-mcmc_amd variant-*), interleaved twice
      for rep in 1 2; do
        for lib in default ${AB_LIBS:-scripts/probe/librvmcmc_mg5.so}; do
          if [ "$lib" = default ]; then
            ITERS=${AB_ITERS:-300} timeout -k 10 200 python -u scripts/probe/steady_bench.py 4,5,6,7:5e-7 >> gpurun_out/${T}_steady_ab.jsonl 2>> gpurun_out/${T}_steady_ab.err || exit 1
          else
            RVM_LIB_PATH=$lib ITERS=${AB_ITERS:-300} timeout -k 10 200 python -u scripts/probe/steady_bench.py 4,5,6,7:5e-7 >> gpurun_out/${T}_steady_ab.jsonl 2>> gpurun_out/${T}_steady_ab.err || exit 1
          fi
        done
      done
      cut -c1-400 gpurun_out/${T}_steady_ab.jsonl ;;
    c4ab)
      # config 4 (SMALA FD: eager halving passes on the centres): the default library against AB_LIBS
      for rep in 1 2; do
        for lib in default ${AB_LIBS:-scripts/probe/librvmcmc_mg5.so}; do
          if [ "$lib" = default ]; then lp=""; else lp=$lib; fi
          RVM_LIB_PATH=$lp timeout -k 10 200 python -u scripts/configs_bench.py ${ABCFG:-4} \
            | sed "s|^{|{\"lib\": \"${lib}\", |" >> gpurun_out/${T}_c4ab.jsonl 2>> gpurun_out/${T}_c4ab.err || exit 1
        done
      done
      cut -c1-300 gpurun_out/${T}_c4ab.jsonl ;;
    rehearse2)
      # world-size-2 rehearsal of the bench on the box's one GPU (gloo: RCCL cannot put two ranks on
      # one device), timed at the chain's steady state like the N = 1 line
      RVM_DIST_BACKEND=gloo timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
        --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 20 --warmup 3 --ess-iters 2000 --no-cpu \
        > gpurun_out/${T}_bench_n2_gloo.json 2> gpurun_out/${T}_bench_n2_gloo.err \
        || { tail -30 gpurun_out/${T}_bench_n2_gloo.err; exit 1; }
      head -c 600 gpurun_out/${T}_bench_n2_gloo.json; echo ;;
    configs)
      timeout -k 10 600 python -u scripts/configs_bench.py ${CONFIGS:-} > gpurun_out/${T}_configs.jsonl 2> gpurun_out/${T}_configs.err \
        || { tail -20 gpurun_out/${T}_configs.err; exit 1; }
      cut -c1-300 gpurun_out/${T}_configs.jsonl ;;
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
    profcfg)
      # kernel trace of one configuration (PCFG) of scripts/configs_bench.py
      mkdir -p gpurun_out/${T}_prof_cfg${PCFG:-2}
      cd /tmp
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${T}_prof_cfg${PCFG:-2}" -o run --output-format csv -- \
        python3 "$R/scripts/configs_bench.py" ${PCFG:-2} > "$R/gpurun_out/${T}_cfg${PCFG:-2}_under_rocprof.jsonl" \
        2> "$R/gpurun_out/${T}_cfg${PCFG:-2}_under_rocprof.err"
      cd "$R"
      st=$(find gpurun_out/${T}_prof_cfg${PCFG:-2} -name "*kernel_stats.csv" | head -1)
      cut -c1-200 "$st" | head -12 ;;
    pmc)
      timeout -k 10 900 bash scripts/pmc_profile.sh > gpurun_out/${T}_pmc.log 2>&1 || { tail -20 gpurun_out/${T}_pmc.log; exit 1; }
      cp gpurun_out/pmc/pmc_latest.json gpurun_out/${T}_pmc_latest.json
      tail -5 gpurun_out/pmc/summary.txt ;;
  esac
done
echo evidence done

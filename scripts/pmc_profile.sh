#!/bin/bash
# PMC passes (counters only with --kernel-trace, one group per run) over the kernel micro-bench,
# then scripts/pmc_summary.py turns them into profiles/pmc_latest.json (per-launch HBM bytes,
# FP64 flops, issue efficiency).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
cd /tmp
i=0
PMC_GROUPS=${GROUPS_OVERRIDE:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP64_TRANS SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_LDS SQ_INSTS_SMEM|SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE SQ_ACTIVE_INST_SCA|SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_THREAD_CYCLES_VALU SQ_IFETCH SQ_INSTS_BRANCH SQ_INST_CYCLES_SALU|FETCH_SIZE|WRITE_SIZE"}
IFS='|' read -ra GRPS <<< "$PMC_GROUPS"
# PMC_TARGET=bench (default): the bench's own launch sequences at the chain's steady state (the last
# PMC_LAST iterations after a PMC_BURN-iteration burn-in: speculative stretch iterations of 3 x 2048
# walker slots, each a likelihood and a refinement launch); PMC_TARGET=kbench: plain likelihood
# launches of PMC_W walkers
TARGET=${PMC_TARGET:-bench}
for grp in "${GRPS[@]}"; do
  i=$((i+1))
  if [ "$TARGET" = "bench" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/pmc/p$i" -o run --output-format csv -- python3 "$R/bench.py" --steps ${PMC_LAST:-20} --warmup 1 --ball-steps 0 --burn-in ${PMC_BURN:-2000} --ess-iters 0 --kernel-iters 0 --no-cpu --no-fixed-step-ref > "$R/gpurun_out/pmc/p$i.log" 2>&1
  else
    timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d "$R/gpurun_out/pmc/p$i" -o run --output-format csv -- python3 "$R/scripts/kbench.py" ${PMC_W:-2048} > "$R/gpurun_out/pmc/p$i.log" 2>&1
  fi
done
cd "$R"
if [ "$TARGET" = "bench" ]; then
  python3 scripts/pmc_summary.py gpurun_out/pmc ${PMC_W:-6144} 0 "speculative stretch iteration at the steady state (bench.py --burn-in ${PMC_BURN:-2000})" ${PMC_LAST:-20} | tee gpurun_out/pmc/summary.txt
else
  python3 scripts/pmc_summary.py gpurun_out/pmc ${PMC_W:-2048} 0 "plain likelihood launch (kbench.py)" | tee gpurun_out/pmc/summary.txt
fi

#!/bin/bash
# 2-rank rehearsal of the multi-GPU bench on a 1-GPU box: both ranks share cuda:0 and talk over
# gloo (RCCL refuses two ranks on one device); exercises the sharded sampler, the complement
# all-gather and the max-over-ranks timing of bench.py.  The driver's real N>1 runs use RCCL.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
RVM_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 1 --ess-iters 40 \
  > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err || { tail -30 gpurun_out/bench_n2_gloo.err; exit 1; }
cat gpurun_out/bench_n2_gloo.json

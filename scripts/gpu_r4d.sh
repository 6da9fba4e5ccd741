#!/bin/bash
# Round-4 steady-state profile: per-wave timing (RVM_PROFILE build) of a plain launch of the
# steady-state slots (scripts/probe/slots_it2000.npz) with the fixed step and with the adaptive
# resolution, the plain-launch cost of both, then the resolve / decision tests.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-r04l}
SLOTS=scripts/probe/slots_it2000.npz RESOLVE=0 timeout -k 10 120 python -u scripts/probe/prof_kernel.py > gpurun_out/${T}_prof_fixed.json 2>&1 || { tail -20 gpurun_out/${T}_prof_fixed.json; exit 1; }
SLOTS=scripts/probe/slots_it2000.npz RESOLVE=1 timeout -k 10 120 python -u scripts/probe/prof_kernel.py > gpurun_out/${T}_prof_resolve.json 2>&1 || { tail -20 gpurun_out/${T}_prof_resolve.json; exit 1; }
timeout -k 10 200 python -u scripts/probe/resolve_cost.py scripts/probe/slots_it2000.npz > gpurun_out/${T}_resolve_cost.jsonl 2>&1 || { tail -20 gpurun_out/${T}_resolve_cost.jsonl; exit 1; }
cat gpurun_out/${T}_resolve_cost.jsonl
T=$T bash scripts/gpu_r4c.sh

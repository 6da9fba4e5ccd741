# A/B at the bench chain's steady state over one environment knob of the library:
#   AB_VAR=RVM_SPEC2_SPO AB_VALS="160 0" T=tag bash scripts/probe/ab_env.sh
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${T:-r06ab}
for rep in 1 2; do
  for v in $AB_VALS; do
    env $AB_VAR=$v ITERS=${AB_ITERS:-400} timeout -k 10 120 python -u scripts/probe/steady_bench.py 4,5,6,7:5e-7 \
      | sed "s|^{|{\"$AB_VAR\": \"$v\", |" >> gpurun_out/${T}_ab.jsonl
  done
done
python3 -c "
import json
for l in open('gpurun_out/${T}_ab.jsonl'):
    d=json.loads(l); print(d['$AB_VAR'], round(d['ms_per_iteration'],4), round(d['logl_kernel_ms'],4), round(d['refine_kernel_ms'],4), [round(x,3) for x in d['refine_kernel_ms_quantiles']], d['faults']['refined'])
"

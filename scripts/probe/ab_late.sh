set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 96 0; do
    RVM_LATE_SPO=$v ITERS=400 timeout -k 10 120 python -u scripts/probe/steady_bench.py 4,5,6,7:5e-7 | sed "s|^{|{\"late_spo\": $v, |" >> gpurun_out/r06b_steady_ab_late.jsonl
  done
done
cut -c1-330 gpurun_out/r06b_steady_ab_late.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_resolve.py -x -q --timeout 300 --timeout-method thread 2>&1 | tail -3

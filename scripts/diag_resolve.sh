set -uo pipefail
for tol in 0 5e-7; do
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --ess-iters 0 --no-cpu --kernel-iters 0 --resolve-tol $tol > gpurun_out/diag_$tol.json 2>gpurun_out/diag_$tol.err || { tail -5 gpurun_out/diag_$tol.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/diag_$tol.json'));print('$tol', d['value'], d['ms_per_step'], d['resolve'], d['roofline_hbm']['acceptance_timed'])"
done

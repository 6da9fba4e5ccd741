"""Summarise rocprofv3 PMC passes over the bench's launch sequence -> profiles/pmc_latest.json.

Per kernel (rvm::logl_kernel, rvm::refine_kernel) the mean over the LAST `last` dispatches of each
pass (the bench's steady-state window; `skip` drops leading likelihood dispatches instead when
last = 0), then per iteration (one likelihood and one refinement launch): fp64 flops as executed
(SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes) and HBM bytes.  HBM bytes follow MI355X_MICROARCH.md §HBM:
FETCH_SIZE / WRITE_SIZE are in KiB and FETCH_SIZE counts half of the bytes of a wide coalesced
stream on gfx950 (the x2 correction is applied and the raw value kept beside it).
usage: pmc_summary.py DIR WALKERS_PER_LAUNCH SKIP DESCRIPTION [LAST]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d, W = sys.argv[1], int(sys.argv[2])
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0
what = sys.argv[4] if len(sys.argv) > 4 else "likelihood launch"
last = int(sys.argv[5]) if len(sys.argv) > 5 else 0
KERNELS = {"logl": "logl_kernel", "refine": "refine_kernel"}
vals = {k: defaultdict(list) for k in KERNELS}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    allrows = list(csv.DictReader(open(f)))
    for k, name in KERNELS.items():
        rows = [r for r in allrows if name in r.get("Kernel_Name", "")]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        ids = ids[-last:] if last > 0 else (ids[skip:] if k == "logl" else ids)
        keep = set(ids)
        # sum the per-dimension rows of each (dispatch, counter), then collect per counter
        acc = defaultdict(float)
        for r in rows:
            if int(r["Dispatch_Id"]) in keep:
                acc[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
        for (_, cname), v in acc.items():
            vals[k][cname].append(v)
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_signature  # noqa: E402


def mean(k, c):
    v = vals[k].get(c)
    return sum(v) / len(v) if v else None


# keyed to the kernel sources it was measured on: bench.py refuses a summary of another kernel
out = {"walkers_per_launch": W, "kernels": "rvm::logl_kernel<2> + rvm::refine_kernel<2>", "launch": what,
       "window": f"last {last} dispatches of each kernel per pass" if last else f"logl dispatches after {skip}",
       "kernel_signature": kernel_signature(), "per_kernel": {}}
fi, hb = 0.0, 0.0
for k in KERNELS:
    pk = {"dispatches_per_pass": max((len(v) for v in vals[k].values()), default=0)}
    for c in vals[k]:
        pk["raw_" + c] = mean(k, c)
    fs, ws = mean(k, "FETCH_SIZE"), mean(k, "WRITE_SIZE")
    if fs is not None and ws is not None:
        pk["hbm_bytes_per_launch"] = (2.0 * fs + ws) * 1024.0
        pk["hbm_bytes_per_launch_uncorrected"] = (fs + ws) * 1024.0
        hb += pk["hbm_bytes_per_launch"]
    fl, flt = mean(k, "SQ_INSTS_VALU_FLOPS_FP64"), mean(k, "SQ_INSTS_VALU_FLOPS_FP64_TRANS")
    if fl is not None:
        # SQ_INSTS_VALU_FLOPS_FP64 counts per wave-instruction (FMA = 2), x 64 lanes = flops (every lane
        # counted, active or not: an upper bound where waves run partly empty)
        pk["fp64_flops_per_launch"] = 64.0 * (fl + (flt or 0.0))
        fi += pk["fp64_flops_per_launch"]
    out["per_kernel"][k] = pk
out["fp64_flops_per_iteration"] = fi or None
out["hbm_bytes_per_launch"] = hb or None  # (one likelihood + one refinement launch per iteration)
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(d, "pmc_latest.json"), "w"), indent=1)

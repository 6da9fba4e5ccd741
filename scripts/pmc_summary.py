"""Summarise rocprofv3 PMC passes for rvm::logl_kernel (per launch) -> profiles/pmc_latest.json.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB; FETCH_SIZE counts
half of the bytes of a wide coalesced stream on gfx950 (the x2 correction is applied and the raw
value kept beside it -- our loads are 8 B/lane, an uncalibrated width)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

d, W = sys.argv[1], int(sys.argv[2])
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0      # leading logl dispatches to drop per pass
what = sys.argv[4] if len(sys.argv) > 4 else "likelihood launch"
vals = defaultdict(list)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    rows = [r for r in csv.DictReader(open(f)) if "logl_kernel" in r.get("Kernel_Name", "")]
    ids = sorted({int(r["Dispatch_Id"]) for r in rows})[skip:]
    keep = set(ids)
    # sum the per-dimension rows of each (dispatch, counter), then collect per counter
    acc = defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) in keep:
            acc[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])
    for (_, name), v in acc.items():
        vals[name].append(v)
# each dispatch appears once per counter (values already summed over XCDs/SEs by rocprofv3 when
# the counter is a _sum; otherwise one row per dimension instance -> accumulate per dispatch)
per = {}
for k, v in vals.items():
    per[k] = v
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import kernel_signature  # noqa: E402

# keyed to the kernel sources it was measured on: bench.py refuses a summary of another kernel
out = {"walkers_per_launch": W, "kernel": "rvm::logl_kernel<2>", "launch": what,
       "kernel_signature": kernel_signature()}
def mean(k):
    v = per.get(k)
    return sum(v) / len(v) if v else None
for k in per:
    out["raw_" + k] = mean(k)
fs, ws = mean("FETCH_SIZE"), mean("WRITE_SIZE")
if fs is not None and ws is not None:
    out["hbm_bytes_per_launch"] = (2.0 * fs + ws) * 1024.0
    out["hbm_bytes_per_launch_uncorrected"] = (fs + ws) * 1024.0
fl, flt = mean("SQ_INSTS_VALU_FLOPS_FP64"), mean("SQ_INSTS_VALU_FLOPS_FP64_TRANS")
if fl is not None:
    # SQ_INSTS_VALU_FLOPS_FP64 counts per wave-instruction (FMA = 2; it equals 2*FMA_F64 + MUL_F64 +
    # ADD_F64 instruction counts), so x64 lanes gives fp64 flops (all lanes active in this kernel)
    out["fp64_flops_per_launch"] = 64.0 * (fl + (flt or 0.0))
    out["fp64_flops_per_eval"] = out["fp64_flops_per_launch"] / W
print(json.dumps(out, indent=1))

json.dump(out, open(os.path.join(d, "pmc_latest.json"), "w"), indent=1)

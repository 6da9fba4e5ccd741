"""Mean duration per kernel over the LAST n dispatches of a rocprofv3 kernel trace (the bench's
steady-state window: its timed iterations and the kernel-timing pass are the run's last ones), to set
beside the bench line's HIP-event kernel_ms.  usage: trace_window.py TRACE_CSV N [KERNEL_SUBSTR ...]"""
import csv
import json
import sys


def main():
    path, n = sys.argv[1], int(sys.argv[2])
    names = sys.argv[3:] or ["logl_kernel", "refine_kernel", "stretch_iteration_end_kernel"]
    rows = list(csv.DictReader(open(path)))
    out = {"trace": path, "window": f"last {n} dispatches per kernel"}
    for k in names:
        d = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows if k in r["Kernel_Name"]))
        d = d[-n:]
        if not d:
            continue
        dur = [(e - s) / 1e3 for s, e in d]
        dur_sorted = sorted(dur)
        out[k] = {"dispatches": len(dur), "mean_us": sum(dur) / len(dur), "min_us": dur_sorted[0],
                  "median_us": dur_sorted[len(dur) // 2], "max_us": dur_sorted[-1]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

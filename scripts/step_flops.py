"""Count the fp64 flops of one Wisdom-Holman step in the compiled gfx950 ISA (F_step
from the step loop's ISA, frozen in roofline.py).  Compiles scripts/probe/step_flops.hip with the
library's flags and counts, between the STEP_BEGIN / STEP_END markers of the ungated (speculative,
NT = 6) instantiation, the fp64 VALU instructions: FMA 2 flops, mul / add 1, v_rcp_f64 / v_rsq_f64 1
(one flop each: the refinement around them is counted as the FMAs it compiles to).  Prints JSON."""
import collections
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "scripts", "probe", "step_flops.hip")
FLOPS = {"v_fma_f64": 2, "v_fmac_f64": 2, "v_mul_f64": 1, "v_add_f64": 1, "v_rcp_f64": 1, "v_rsq_f64": 1}


def isa_counts(gated=False):
    with tempfile.TemporaryDirectory() as d:
        subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c",
                               "--save-temps", "-o", os.path.join(d, "s.o"), SRC], cwd=d,
                              stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        asm = [f for f in os.listdir(d) if f.endswith(".s") and "gfx950" in f]
        text = open(os.path.join(d, asm[0])).read()
    # the kernel body of the wanted instantiation (mangled: ..._Li6ELb0E.. / ..._Li6ELb1E..)
    key = "Li6ELb1E" if gated else "Li6ELb0E"
    start = text.index(f"{key}EvPdid:")
    body = text[start:text.index("s_endpgm", start)].splitlines()
    # the step loop: from the label of the loop header whose body holds the STEP_BEGIN marker to the
    # branch back to it (every block of the rotated loop lies in between; the markers alone do not
    # bound the step -- the scheduler moves arithmetic across them)
    k = next(i for i, ln in enumerate(body) if "STEP_BEGIN" in ln)
    h = max(i for i in range(k) if re.match(r"\.LBB\d+_\d+:.*Loop Header", body[i]))
    label = body[h].split(":")[0]
    e = next(i for i in range(k, len(body)) if re.match(rf"\s+s_(c)?branch\w*\s+{re.escape(label)}\b", body[i]))
    loop = [[None, None, body[h:e + 1]]]
    c = collections.Counter()
    for b in loop:
        for line in b[2]:
            m = re.match(r"\s+(v_[a-z0-9_]+)", line)
            if m:
                c[re.sub(r"_(e32|e64|dpp|sdwa)$", "", m.group(1))] += 1
    return c


def main():
    out = {}
    for gated in (False,):
        c = isa_counts(gated)
        flops = sum(FLOPS.get(k, 0) * v for k, v in c.items())
        valu = sum(v for k, v in c.items())
        f64 = sum(v for k, v in c.items() if k in FLOPS)
        out["gated" if gated else "speculative"] = {"fp64_flops_per_lane_step": flops, "valu_per_lane_step": valu,
                                                    "fp64_valu_per_lane_step": f64,
                                                    "counts": dict(sorted(c.items()))}
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()

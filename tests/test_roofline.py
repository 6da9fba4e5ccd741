"""The bench's frozen algorithmic flop count (roofline.py) is what the compiled step
loop executes: scripts/step_flops.py recompiles scripts/probe/step_flops.hip for gfx950 (hipcc
cross-compiles on the CPU) and counts the fp64 flops of one step."""
import json
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import roofline  # noqa: E402


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc") and shutil.which("hipcc") is None, reason="no hipcc")
def test_frozen_step_flops_match_the_isa():
    out = json.loads(subprocess.check_output([sys.executable, os.path.join(ROOT, "scripts", "step_flops.py")],
                                             timeout=600))
    assert out["speculative"]["fp64_flops_per_lane_step"] == roofline.F_STEP_LANE, out["speculative"]


def test_flops_per_eval_of_the_bench_plan():
    # S2 bench plan: levels 4..7, 112 + 120 base steps (bench line config.level1_steps)
    assert roofline.flops_per_eval((4, 5, 6, 7), 112, 120, 2) == roofline.F_STEP_LANE * 2 * 22 * 232

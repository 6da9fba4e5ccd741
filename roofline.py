"""The frozen algorithmic flop count of the likelihood and the MI355X peaks the bench
line's roofline uses.

F_step is the fp64 work of ONE Wisdom-Holman kick-drift-kick step of one planet lane, counted in
the compiled gfx950 ISA of the step loop (scripts/step_flops.py over scripts/probe/step_flops.hip:
the segment loop's ungated drift, kick_prep and kick_apply, Stumpff series of 6 terms -- the fine
levels' loop): FMA 2 flops, mul / add 1, v_rcp_f64 / v_rsq_f64 1.  It is frozen here so that the
bench's `frac` measures efficiency: work the kernel wastes (speculative variants not taken,
redone segments, the adaptive resolution's extension and halving passes, prologues) is not credited.
tests/test_roofline.py recompiles the probe and checks the constant.

F_eval (one walker-logL, the algorithm's minimum) = F_step x lanes per walker (2 for two planets) x
sum of the plan's level multipliers (4 + 5 + 6 + 7 = 22) x base steps over both directions (the
schedule's level-1 steps, 112 + 120 = 232 on the bench's S2 data): 1.84 MFLOP.
"""

F_STEP_LANE = 180  # fp64 flops per planet lane per WH step (gfx950 ISA, scripts/step_flops.py)

FP64_VALU_PEAK_TFLOPS = 78.6  # MI355X FP64 vector (the microarch guide lists no FP64 figure)
HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E peak 8.0 TB/s


def flops_per_eval(level_mult, steps_fwd, steps_bwd, n_planets=2):
    """Algorithmic fp64 flops of one walker-logL of a plan: the fixed-step Richardson levels only, one
    planet lane per planet (F_STEP_LANE is the 2-planet kick's step; other planet counts scale it)."""
    return float(F_STEP_LANE * min(n_planets, 4) * sum(int(m) for m in level_mult) * (int(steps_fwd) + int(steps_bwd)))


def describe(level_mult, steps_fwd, steps_bwd, n_planets=2):
    return (f"roofline.py: {F_STEP_LANE} fp64 flops per lane-step (gfx950 ISA of the step loop, "
            f"scripts/step_flops.py) x {min(n_planets, 4)} planet lanes x sum(level multipliers) "
            f"{sum(int(m) for m in level_mult)} x {int(steps_fwd) + int(steps_bwd)} base steps (both directions)")

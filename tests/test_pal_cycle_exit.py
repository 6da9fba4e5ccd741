"""The kernel's Pal Kepler solve (rvm_device.h pal_solve_F) leaves the reference's Newton loop early
when it settles into a roundoff 2-cycle, and must still return the iterate the 100-step loop ends
on (the reference's loop: REBOUND reb_tools_pal_to_particle as restated in oracle/rvoracle.c
pal_to_cart).  This checks the exit rule itself, restated in Python over float64 with the same
update, against the plain 100-step loop: identical results for every input, far fewer steps.
(The device's own sincos is not libm's, so the kernel cannot be compared bit for bit with a CPU
loop; the rule is what is tested here, the kernel's results through T1/T2 elsewhere.)"""
import math

import numpy as np


def _reference_loop(lam, k, h):
    F = lam
    n = 0
    for _ in range(100):
        s, c = math.sin(F), math.cos(F)
        step = (F - k * s + h * c - lam) / (1.0 - k * c - h * s)
        F = F - step
        n += 1
        if abs(step) <= 1e-16 * max(abs(F), 1.0):
            break
    return F, n


def _cycle_exit_loop(lam, k, h):
    F, Fp, n = lam, math.nan, 0
    for it in range(100):
        s, c = math.sin(F), math.cos(F)
        step = (F - k * s + h * c - lam) / (1.0 - k * c - h * s)
        Fn = F - step
        n += 1
        conv = not (abs(step) > 1e-16 * max(abs(Fn), 1.0))
        cyc = (not conv) and Fn == Fp
        Fc = Fn if ((99 - it) & 1) == 0 else F
        Fp, F = F, (Fc if cyc else Fn)
        if conv or cyc:
            break
    return F, n


def test_cycle_exit_returns_the_100_step_iterate():
    rng = np.random.default_rng(3)
    n_cases = 20000
    e = rng.uniform(0.0, 0.6, n_cases)
    w = rng.uniform(0.0, 2 * np.pi, n_cases)
    lam = rng.uniform(-20.0, 20.0, n_cases)
    full = steps_ref = steps_new = 0
    for i in range(n_cases):
        k, h = e[i] * math.cos(w[i]), e[i] * math.sin(w[i])
        a, na = _reference_loop(float(lam[i]), k, h)
        b, nb = _cycle_exit_loop(float(lam[i]), k, h)
        assert a == b or (math.isnan(a) and math.isnan(b)), (lam[i], k, h, a, b)
        full += na == 100
        steps_ref += na
        steps_new += nb
    # the 2-cycle is common (about one input in ten runs all 100 reference steps) ...
    assert full > n_cases // 50
    # ... and the exit removes most of the iterations
    assert steps_new < 0.5 * steps_ref

"""The C-ABI library loads on a CPU-only host and exports every symbol include/rvmcmc.h declares.

No compute calls here (no GPU); the GPU tests exercise the same entry points."""
import os
import re

from conftest import ROOT

from rvmcmc import _lib


def header_functions():
    src = open(os.path.join(ROOT, "include", "rvmcmc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rvm_[a-z_0-9]+)\s*\(", src)))


def test_header_declares_expected_surface():
    fns = header_functions()
    for f in ("rvm_plan_create", "rvm_logl_batch", "rvm_stretch_propose", "rvm_stretch_accept",
              "rvm_mh_propose", "rvm_mh_accept", "rvm_fd_params", "rvm_smala_derive", "rvm_smala_propose",
              "rvm_smala_accept", "rvm_smala_derive_sides", "rvm_smala_center_accept", "rvm_stretch_half_step", "rvm_stretch_iteration_begin",
              "rvm_stretch_iteration_end", "rvm_logl_derivs", "rvm_logl_derivs_workspace_bytes", "rvm_smala_metric",
              "rvm_last_error", "rvm_abi_version"):
        assert f in fns


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    for f in header_functions():
        assert hasattr(lib, f), f"librvmcmc.so lacks {f}"
    assert lib.rvm_abi_version() == _lib.ABI_VERSION == 12


def test_python_binding_matches_header():
    assert set(_lib.SIGNATURES) == set(header_functions())


def test_argument_errors_do_not_touch_the_device():
    import ctypes as C

    lib = _lib.load()
    cfg = _lib.RvmConfig(0, 0.1, 4, 100.0)  # n_planets = 0 -> rejected before any HIP call
    h = C.c_void_p()
    z = (C.c_double * 1)(0.0)
    rc = lib.rvm_plan_create(C.byref(cfg), z, z, z, 1, 64, C.byref(h))
    assert rc < 0 and b"n_planets" in lib.rvm_last_error()
    assert lib.rvm_logl_batch(None, 1, 0, 1.0, 0, 0, 0, 0) < 0
    m = _lib.ParamMapC()
    assert lib.rvm_stretch_half_step(None, C.byref(m), 10, 1, 0, 0, 0, 0, 1, 0, 2.0, 0, 0, 0, 1.0, 0, 0, 0, 0) < 0
    assert lib.rvm_stretch_iteration_begin(None, C.byref(m), 10, 1, 0, 8, 0, 0, 0, 0, 8, 0, 0, 2.0, 0, 0, 1.0, 0, 0, 0,
                                           0, 0) < 0
    # end: half 1's walker range must lie in the second half (s1_begin >= n_half)
    one = (C.c_double * 1)(0.0)
    ione = (C.c_int32 * 1)(0)
    assert lib.rvm_stretch_iteration_end(10, 1, 0, 0, one, 0, ione, ione, one, 0, one, 8, one, one, one, ione, 2.0,
                                         0, 0, 0, 0, 0, 0) < 0
    assert b"walker ranges" in lib.rvm_last_error()
    rows = (C.c_int32 * 2)(0, 1)
    assert lib.rvm_logl_derivs(None, 1, 0, 2, rows, 1.0, 0, 0, 0, 0, 0, 0) < 0
    # more epochs in one direction than the LDS-staged schedule holds: an argument error, caught
    # before any HIP call
    n = 1701
    t = (C.c_double * n)(*[0.01 * (i + 1) for i in range(n)])
    ones = (C.c_double * n)(*([1.0] * n))
    cfg2 = _lib.RvmConfig(2, 0.5, 4, 100.0)
    rc = lib.rvm_plan_create(C.byref(cfg2), t, ones, ones, n, 64, C.byref(h))
    assert rc < 0 and b"too many epochs" in lib.rvm_last_error()
    # adaptive resolution bounds, and the fault-counter / timeout entry points on a null plan
    cfg3 = _lib.RvmConfig(2, 0.5, 4, 100.0)
    cfg3.resolve_tol, cfg3.resolve_max = 5e-7, 13
    rc = lib.rvm_plan_create(C.byref(cfg3), z, z, z, 1, 64, C.byref(h))
    assert rc < 0 and b"resolve_max" in lib.rvm_last_error()
    assert lib.rvm_plan_faults(None, 0, None, None, None, None, None, 0) < 0
    assert lib.rvm_plan_set_handoff_timeout(None, 1.0) < 0
    assert lib.rvm_plan_extension(None, None) < 0
    assert lib.rvm_plan_set_verify_eccentricity(None, 0.3) < 0
    assert lib.rvm_plan_set_certain_reject(None, 0) < 0
    assert lib.rvm_plan_counters(None, 0, None, 0, None) < 0
    # workspace: per (chain, pair i >= j) and direction, 4 f64 partial sums and an int32 status
    assert lib.rvm_logl_derivs_workspace_bytes(256, 10) == 256 * 55 * 2 * (4 * 8 + 4)


def test_struct_layouts_match_header():
    """ctypes mirrors of rvm_config / rvm_smala_cache have the C layouts (x86-64 SysV)."""
    import ctypes as C

    # int32 n_planets | pad | f64 dt | int32 n_levels | pad | f64 npoints | int32 mult[6] | f64 hint
    # | int32 inclined | pad | f64 resolve_tol | int32 resolve_max | pad
    assert C.sizeof(_lib.RvmConfig) == 88 and _lib.RvmConfig.inclined.offset == 64
    assert _lib.RvmConfig.resolve_tol.offset == 72 and _lib.RvmConfig.resolve_max.offset == 80
    assert _lib.RvmConfig.level_mult.offset == 32 and _lib.RvmConfig.period_hint.offset == 56
    assert C.sizeof(_lib.SmalaCache) == 7 * 8


def test_struct_layouts_match_compiled_header(tmp_path):
    """The same layouts as gcc sees them when compiling include/rvmcmc.h."""
    import ctypes as C
    import shutil
    import subprocess

    import pytest

    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    src = tmp_path / "layout.c"
    src.write_text("""
#include <stddef.h>
#include <stdio.h>
#include "rvmcmc.h"
int main(void) {
    printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu\\n", sizeof(rvm_config), offsetof(rvm_config, level_mult),
           offsetof(rvm_config, inclined), sizeof(rvm_smala_cache), sizeof(rvm_param_map),
           offsetof(rvm_param_map, src), offsetof(rvm_param_map, base), offsetof(rvm_config, resolve_tol),
           offsetof(rvm_config, resolve_max));
    return 0;
}
""")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split()]
    assert got == [C.sizeof(_lib.RvmConfig), _lib.RvmConfig.level_mult.offset, _lib.RvmConfig.inclined.offset,
                   C.sizeof(_lib.SmalaCache), C.sizeof(_lib.ParamMapC), _lib.ParamMapC.src.offset,
                   _lib.ParamMapC.base.offset, _lib.RvmConfig.resolve_tol.offset, _lib.RvmConfig.resolve_max.offset]

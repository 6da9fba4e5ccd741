"""ctypes binding of librvmcmc.so (the C ABI declared in include/rvmcmc.h).

There is no fallback: if the library is missing or fails to load, every entry point raises.
The hot path is the HIP kernel or nothing.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# (RVM_LIB_PATH: another build of the same ABI, for A/B runs of compile-time variants -- scripts/probe)
LIB_PATH = os.environ.get("RVM_LIB_PATH") or os.path.join(_HERE, "librvmcmc.so")

RVM_STATUS_OK = 0
RVM_STATUS_PRIOR = 1
RVM_STATUS_ENCOUNTER = 2
RVM_STATUS_NONFINITE = 3
RVM_STATUS_UNRESOLVED = 4
RVM_STATUS_SKIPPED = 5  # rvm_stretch_iteration_begin status_spec only
RVM_MAX_PLANETS = 4
RVM_MAX_LEVELS = 6
RVM_N_COUNTERS = 7  # rvm_plan_counters
ABI_VERSION = 12  # include/rvmcmc.h RVM_ABI_VERSION


class RvmConfig(C.Structure):
    _fields_ = [
        ("n_planets", C.c_int32),
        ("dt", C.c_double),
        ("n_levels", C.c_int32),
        ("npoints_norm", C.c_double),
        ("level_mult", C.c_int32 * RVM_MAX_LEVELS),
        ("period_hint", C.c_double),
        ("inclined", C.c_int32),
        ("resolve_tol", C.c_double),
        ("resolve_max", C.c_int32),
    ]


RVM_SMALA_MAX_PARAMS = 20
RVM_MAX_PARAM_ROWS = 7 * RVM_MAX_PLANETS


class ParamMapC(C.Structure):  # include/rvmcmc.h: rvm_param_map
    _fields_ = [
        ("n_rows", C.c_int32),
        ("src", C.c_int32 * RVM_MAX_PARAM_ROWS),
        ("base", C.c_double * RVM_MAX_PARAM_ROWS),
    ]


class SmalaCache(C.Structure):  # include/rvmcmc.h: rvm_smala_cache (device pointers)
    _fields_ = [(k, C.c_void_p) for k in ("lp", "grad", "mu", "L", "G", "logdet", "ok")]


class RvmError(RuntimeError):
    pass


# exported symbol -> (restype, argtypes); mirrors include/rvmcmc.h exactly
_dp = C.c_void_p  # device pointers are passed as integers (torch.Tensor.data_ptr())
SIGNATURES = {
    "rvm_abi_version": (C.c_int, []),
    "rvm_smala_derive": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, _dp, C.c_double, _dp, _dp, _dp, _dp, _dp,
                                   C.c_double, C.c_double, C.c_double, C.POINTER(SmalaCache), _dp]),
    "rvm_smala_metric": (C.c_int, [C.c_int32, C.c_int32, _dp, _dp, _dp, _dp, _dp, C.c_double, C.c_double,
                                   C.POINTER(SmalaCache), _dp]),
    "rvm_smala_propose": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, _dp, C.POINTER(SmalaCache), C.c_double,
                                    C.c_uint64, C.c_uint64, _dp, _dp, _dp]),
    "rvm_smala_accept": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, _dp, C.POINTER(SmalaCache), _dp,
                                   C.POINTER(SmalaCache), C.c_double, C.c_uint64, C.c_uint64, _dp, _dp, _dp, _dp]),
    "rvm_smala_stencil_logl": (C.c_int, [C.c_void_p, C.POINTER(ParamMapC), C.c_int32, C.c_int32, _dp, C.c_double,
                                         _dp, C.c_double, _dp, _dp, _dp, _dp]),
    "rvm_smala_derive_accept": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, C.c_int32, _dp, _dp, C.c_double, _dp, _dp,
                                          _dp, _dp, _dp, C.c_double, C.c_double, C.c_double, C.POINTER(SmalaCache),
                                          C.POINTER(SmalaCache), C.c_uint64, C.c_uint64, _dp, _dp, _dp, _dp]),
    "rvm_smala_derive_sides": (C.c_int, [C.c_int32, C.c_int32, C.c_int32, _dp, C.c_double, _dp, _dp, _dp, _dp, _dp,
                                         C.c_double, C.c_double, C.c_double, C.POINTER(SmalaCache), _dp]),
    "rvm_smala_center_accept": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, _dp, _dp, _dp, _dp, C.POINTER(SmalaCache),
                                          C.POINTER(SmalaCache), C.c_double, C.c_uint64, C.c_uint64, _dp, _dp, _dp,
                                          _dp]),
    "rvm_smala_metric_accept": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, _dp, _dp, _dp, _dp, _dp, _dp, C.c_double,
                                          C.c_double, C.POINTER(SmalaCache), C.POINTER(SmalaCache), C.c_uint64,
                                          C.c_uint64, _dp, _dp, _dp, _dp]),
    "rvm_last_error": (C.c_char_p, []),
    "rvm_plan_create": (C.c_int, [C.POINTER(RvmConfig), C.POINTER(C.c_double), C.POINTER(C.c_double),
                                  C.POINTER(C.c_double), C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]),
    "rvm_plan_destroy": (None, [C.c_void_p]),
    "rvm_plan_faults": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_int64), C.POINTER(C.c_int64),
                                  C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_int64), _dp]),
    "rvm_plan_set_handoff_timeout": (C.c_int, [C.c_void_p, C.c_double]),
    "rvm_plan_time_kernels": (C.c_int, [C.c_void_p, C.c_int32]),
    "rvm_plan_kernel_times": (C.c_int, [C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_float), C.c_int32,
                                        C.POINTER(C.c_int32)]),
    "rvm_plan_extension": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    "rvm_plan_set_verify_eccentricity": (C.c_int, [C.c_void_p, C.c_double]),
    "rvm_plan_set_certain_reject": (C.c_int, [C.c_void_p, C.c_int32]),
    "rvm_plan_counters": (C.c_int, [C.c_void_p, C.c_int32, C.POINTER(C.c_int64), C.c_int32, C.c_void_p]),
    "rvm_plan_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                C.POINTER(C.c_int32)]),
    "rvm_logl_batch": (C.c_int, [C.c_void_p, C.c_int32, _dp, C.c_double, _dp, _dp, _dp, _dp]),
    "rvm_stretch_propose": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, _dp, C.c_int32, _dp, C.c_double, C.c_uint64,
                                      C.c_uint64, C.c_uint32, _dp, _dp, _dp, _dp]),
    "rvm_stretch_accept": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, _dp, _dp, _dp, _dp, _dp, C.c_uint64, C.c_uint64,
                                     C.c_uint32, _dp, _dp, _dp]),
    "rvm_stretch_half_step": (C.c_int, [C.c_void_p, C.POINTER(ParamMapC), C.c_int32, C.c_int32, C.c_int64, _dp, _dp,
                                        _dp, C.c_int32, _dp, C.c_double, C.c_uint64, C.c_uint64, C.c_uint32,
                                        C.c_double, _dp, _dp, _dp, _dp]),
    "rvm_stretch_iteration_begin": (C.c_int, [C.c_void_p, C.POINTER(ParamMapC), C.c_int32, C.c_int32, C.c_int64,
                                              C.c_int64, _dp, _dp, _dp, _dp, C.c_int32, _dp, _dp, C.c_double, C.c_uint64,
                                              C.c_uint64, C.c_double, _dp, _dp, _dp, _dp, _dp]),
    "rvm_stretch_iteration_end": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, C.c_int64, _dp, _dp, _dp, _dp, _dp,
                                            _dp, _dp, C.c_int32, _dp, _dp, _dp, _dp, C.c_double, C.c_uint64,
                                            C.c_uint64, _dp, _dp, _dp, _dp]),
    "rvm_mh_propose": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, _dp, _dp, C.c_double, C.c_uint64, C.c_uint64, _dp,
                                 _dp, _dp]),
    "rvm_mh_accept": (C.c_int, [C.c_int32, C.c_int32, C.c_int64, _dp, _dp, _dp, _dp, C.c_uint64, C.c_uint64, _dp, _dp,
                                _dp]),
    "rvm_mh_step": (C.c_int, [C.c_void_p, C.POINTER(ParamMapC), C.c_int32, C.c_int32, C.c_int64, _dp, _dp, _dp,
                              C.c_double, C.c_uint64, C.c_uint64, C.c_double, _dp, _dp, _dp, _dp]),
    "rvm_fd_params": (C.c_int, [C.c_int32, C.c_int32, _dp, C.c_double, _dp, _dp, _dp]),
    "rvm_logl_derivs_workspace_bytes": (C.c_size_t, [C.c_int32, C.c_int32]),
    "rvm_logl_derivs": (C.c_int, [C.c_void_p, C.c_int32, _dp, C.c_int32, C.POINTER(C.c_int32), C.c_double, _dp, _dp,
                                  _dp, _dp, _dp, _dp]),
}

_lib = None


def load():
    """Load librvmcmc.so (raises RvmError if it is absent or incomplete)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RvmError(
            f"librvmcmc.so not found at {LIB_PATH}: build it with `make -C rvel-mcmc_amd` "
            "(or __graft_entry__.build()); there is no CPU fallback")
    try:
        lib = C.CDLL(LIB_PATH)
    except OSError as e:
        raise RvmError(f"failed to load {LIB_PATH}: {e}") from e
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)  # AttributeError here means the .so lacks an ABI symbol
        fn.restype = res
        fn.argtypes = args
    if lib.rvm_abi_version() != ABI_VERSION:
        raise RvmError("librvmcmc.so ABI version mismatch")
    _lib = lib
    return lib


def check(rc: int, what: str):
    if rc != 0:
        msg = load().rvm_last_error()
        raise RvmError(f"{what} failed ({rc}): {msg.decode() if msg else ''}")


def stream_handle(stream=None) -> int:
    """hipStream_t of a torch stream (default: the current stream of the current device)."""
    import torch

    s = stream if stream is not None else torch.cuda.current_stream()
    return int(s.cuda_stream)

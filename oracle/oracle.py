"""oracle/oracle.py -- Python side of the CPU oracle.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker or the timed CPU baseline.  The product package (rvel-mcmc_amd/rvmcmc)
never imports it.

Contents
--------
* ctypes bindings of oracle/liboracle.so (rvoracle.c): the IAS15 restatement of the reference's
  likelihood path (reference-equivalent physics) and the WH restatement of the kernel algorithm.
* numpy restatements of the reference's observation constructors:
    - ``obs_from_file``   follows observations.py:53-69 (Observation_FromFile)
    - ``fake_obs``        follows observations.py:19-50 (FakeObservation), legacy global
                          MT19937 draw order
* ``pal_params``: dict-of-planets -> the oracle's [np][7] record (m, a, h, k, l, ix, iy).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None

ORACLE_OK, ORACLE_PRIOR, ORACLE_ENCOUNTER, ORACLE_NONFINITE = 0, 1, 2, 3


def build(force: bool = False) -> str:
    so = os.path.join(_HERE, "liboracle.so")
    src = os.path.join(_HERE, "rvoracle.c")
    if force or not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return so


def lib():
    global _LIB
    if _LIB is None:
        so = os.environ.get("RVO_LIB") or os.path.join(_HERE, "liboracle.so")  # (RVO_LIB: a study build)
        if not os.path.exists(so):
            build()
        L = C.CDLL(so)
        dp = C.POINTER(C.c_double)
        L.rvo_prior_hard.argtypes = [C.c_int, dp, C.c_int, C.c_int]
        L.rvo_prior_hard.restype = C.c_int
        L.rvo_setup_vectors.argtypes = [C.c_int, dp, dp, dp]
        L.rvo_get_rv_ias15.argtypes = [C.c_int, dp, C.c_double, dp, C.c_int, dp, C.POINTER(C.c_long)]
        L.rvo_get_rv_ias15.restype = C.c_int
        L.rvo_logl_ias15.argtypes = [C.c_int, dp, C.c_int, C.c_int, C.c_double, dp, dp, dp, C.c_int, dp, dp, dp,
                                     C.c_int, C.c_double, dp]
        L.rvo_logl_ias15.restype = C.c_int
        L.rvo_logl_ias15_batch.argtypes = [C.c_int, C.c_int, dp, C.c_int, C.c_int, C.c_double, dp, dp, dp, C.c_int,
                                           dp, dp, dp, C.c_int, C.c_double, dp, C.POINTER(C.c_int32)]
        L.rvo_wh_rv.argtypes = [C.c_int, dp, C.c_double, dp, C.c_int, C.c_double, C.c_int, dp]
        L.rvo_wh_rv.restype = C.c_int
        L.rvo_logl_wh.argtypes = [C.c_int, dp, C.c_int, C.c_int, C.c_double, dp, dp, dp, C.c_int, C.c_double,
                                  C.c_double, C.c_int, dp]
        L.rvo_logl_wh.restype = C.c_int
        L.rvo_richardson_weights.argtypes = [C.c_int, dp]
        L.rvo_whx_rv.argtypes = [C.c_int, dp, C.c_double, dp, C.c_int, C.c_double, C.c_int, dp]
        L.rvo_whx_rv.restype = C.c_int
        L.rvo_logl_whx_batch.argtypes = [C.c_int, C.c_int, dp, C.c_int, C.c_int, C.c_double, dp, dp, dp, C.c_int,
                                         C.c_double, C.c_double, C.c_int, dp, C.POINTER(C.c_int32)]
        ip = C.POINTER(C.c_int)
        L.rvo_richardson_weights_seq.argtypes = [C.c_int, ip, dp]
        L.rvo_whx_rv_seq.argtypes = [C.c_int, dp, C.c_double, dp, C.c_int, C.c_double, C.c_int, ip, dp]
        L.rvo_whx_rv_seq.restype = C.c_int
        L.rvo_logl_whx_seq_batch.argtypes = [C.c_int, C.c_int, dp, C.c_int, C.c_int, C.c_double, dp, dp, dp,
                                             C.c_int, C.c_double, C.c_double, C.c_int, ip, dp,
                                             C.POINTER(C.c_int32)]
        L.rvo_logl_whx_adapt_batch.argtypes = [C.c_int, C.c_int, dp, C.c_int, C.c_int, C.c_double, dp, dp, dp,
                                               C.c_int, C.c_double, C.c_double, C.c_int, ip, C.c_int, C.c_double, C.c_int,
                                               C.POINTER(C.c_int32), C.c_int, dp, dp, dp, C.c_double,
                                               dp, C.POINTER(C.c_int32), C.POINTER(C.c_int32), dp,
                                               C.POINTER(C.c_int32)]
        _LIB = L
    return _LIB


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


def _f64(a):
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64))


PAL_KEYS = ("m", "a", "h", "k", "l", "ix", "iy")


def pal_params(planets) -> np.ndarray:
    """list of planet dicts -> float64 [np][7] (missing h/k/l/ix/iy default to 0 as in REBOUND)."""
    out = np.zeros((len(planets), 7))
    for i, p in enumerate(planets):
        for j, k in enumerate(PAL_KEYS):
            out[i, j] = float(p.get(k, 0.0))
    return out


def _flags(planets):
    has_hk = int(any(("h" in p) or ("k" in p) for p in planets))
    has_inc = int(any(("ix" in p) or ("iy" in p) for p in planets))
    return has_hk, has_inc


def setup_vectors(planets):
    """(heliocentric, barycentric) [nbody][6] = x,y,z,vx,vy,vz (state.py:36-47; G1 fixture)."""
    pl = _f64(pal_params(planets))
    nb = len(planets) + 1
    helio = np.zeros((nb, 6))
    bary = np.zeros((nb, 6))
    lib().rvo_setup_vectors(len(planets), _p(pl), _p(helio), _p(bary))
    return helio, bary


def get_rv_ias15(planets, times, hill_factor=0.0):
    """state.py:61-73 with IAS15: returns (rv, status, nsteps)."""
    pl = _f64(pal_params(planets))
    t = _f64(times)
    rv = np.full(len(t), np.nan)
    ns = C.c_long(0)
    st = lib().rvo_get_rv_ias15(len(planets), _p(pl), float(hill_factor), _p(t), len(t), _p(rv), C.byref(ns))
    return rv, st, ns.value


def logl_ias15(planets, obs, hill_factor=1.0):
    """state.py:103-110 get_logp with the IAS15 restatement -> (logp, status)."""
    pl = _f64(pal_params(planets))
    has_hk, has_inc = _flags(planets)
    a = [_f64(x) for x in (obs.tf, obs.rvf, obs.errorf, obs.tb, obs.rvb, obs.errorb)]
    out = np.zeros(1)
    st = lib().rvo_logl_ias15(len(planets), _p(pl), has_hk, has_inc, float(hill_factor), _p(a[0]), _p(a[1]),
                              _p(a[2]), len(a[0]), _p(a[3]), _p(a[4]), _p(a[5]), len(a[3]), float(obs.Npoints),
                              _p(out))
    return float(out[0]), st


def logl_ias15_batch(params, np_, obs, hill_factor=1.0, has_hk=1, has_inc=0):
    """params: [W][np][7] float64 -> (logl[W], status[W])."""
    pl = _f64(params)
    W = pl.shape[0]
    a = [_f64(x) for x in (obs.tf, obs.rvf, obs.errorf, obs.tb, obs.rvb, obs.errorb)]
    out = np.zeros(W)
    st = np.zeros(W, dtype=np.int32)
    lib().rvo_logl_ias15_batch(W, np_, _p(pl), has_hk, has_inc, float(hill_factor), _p(a[0]), _p(a[1]), _p(a[2]),
                               len(a[0]), _p(a[3]), _p(a[4]), _p(a[5]), len(a[3]), float(obs.Npoints), _p(out),
                               st.ctypes.data_as(C.POINTER(C.c_int32)))
    return out, st


def wh_rv(planets, times, h_target, sub=1, hill_factor=0.0):
    pl = _f64(pal_params(planets))
    t = _f64(times)
    rv = np.full(len(t), np.nan)
    st = lib().rvo_wh_rv(len(planets), _p(pl), float(hill_factor), _p(t), len(t), float(h_target), int(sub), _p(rv))
    return rv, st


def logl_wh(planets, obs, h_target, sub=1, hill_factor=1.0):
    pl = _f64(pal_params(planets))
    has_hk, has_inc = _flags(planets)
    t = _f64(np.concatenate([obs.tf, obs.tb]))
    rv = _f64(np.concatenate([obs.rvf, obs.rvb]))
    er = _f64(np.concatenate([obs.errorf, obs.errorb]))
    out = np.zeros(1)
    st = lib().rvo_logl_wh(len(planets), _p(pl), has_hk, has_inc, float(hill_factor), _p(t), _p(rv), _p(er), len(t),
                           float(obs.Npoints), float(h_target), int(sub), _p(out))
    return float(out[0]), st


def richardson_weights(nl):
    if not isinstance(nl, (int, np.integer)):
        return richardson_weights_seq(nl)
    w = np.zeros(nl)
    lib().rvo_richardson_weights(int(nl), _p(w))
    return w


def whx_rv(planets, times, dt, n_levels, hill_factor=0.0):
    """Kernel-algorithm restatement: Richardson-extrapolated WH model RV at `times`."""
    pl = _f64(pal_params(planets))
    t = _f64(times)
    rv = np.full(len(t), np.nan)
    if not isinstance(n_levels, (int, np.integer)):
        m, mp = _mult(n_levels)
        st = lib().rvo_whx_rv_seq(len(planets), _p(pl), float(hill_factor), _p(t), len(t), float(dt), len(m), mp,
                                  _p(rv))
        return rv, st
    st = lib().rvo_whx_rv(len(planets), _p(pl), float(hill_factor), _p(t), len(t), float(dt), int(n_levels), _p(rv))
    return rv, st


def logl_whx_batch(params, np_, obs, dt, n_levels, hill_factor=1.0, has_hk=1, has_inc=0):
    """params [W][np][7] -> (logl[W], status[W]) with the kernel's algorithm (T1 reference).
    n_levels: int (harmonic levels 1..n) or a sequence of level multipliers."""
    if not isinstance(n_levels, (int, np.integer)):
        return logl_whx_seq_batch(params, np_, obs, dt, n_levels, hill_factor, has_hk, has_inc)
    pl = _f64(params)
    W = pl.shape[0]
    t = _f64(np.concatenate([obs.tf, obs.tb]))
    rv = _f64(np.concatenate([obs.rvf, obs.rvb]))
    er = _f64(np.concatenate([obs.errorf, obs.errorb]))
    out = np.zeros(W)
    st = np.zeros(W, dtype=np.int32)
    lib().rvo_logl_whx_batch(W, np_, _p(pl), has_hk, has_inc, float(hill_factor), _p(t), _p(rv), _p(er), len(t),
                             float(obs.Npoints), float(dt), int(n_levels), _p(out),
                             st.ctypes.data_as(C.POINTER(C.c_int32)))
    return out, st


def _mult(mult):
    m = np.ascontiguousarray(np.asarray(mult, dtype=np.int32))
    return m, m.ctypes.data_as(C.POINTER(C.c_int))


def richardson_weights_seq(mult):
    m, mp = _mult(mult)
    w = np.zeros(len(m))
    lib().rvo_richardson_weights_seq(len(m), mp, _p(w))
    return w


def logl_whx_seq_batch(params, np_, obs, dt, mult, hill_factor=1.0, has_hk=1, has_inc=0):
    """As logl_whx_batch with level k stepping dt/mult[k] (general extrapolation sequence)."""
    pl = _f64(params)
    W = pl.shape[0]
    t = _f64(np.concatenate([obs.tf, obs.tb]))
    rv = _f64(np.concatenate([obs.rvf, obs.rvb]))
    er = _f64(np.concatenate([obs.errorf, obs.errorb]))
    out = np.zeros(W)
    st = np.zeros(W, dtype=np.int32)
    m, mp = _mult(mult)
    lib().rvo_logl_whx_seq_batch(W, np_, _p(pl), has_hk, has_inc, float(hill_factor), _p(t), _p(rv), _p(er),
                                 len(t), float(obs.Npoints), float(dt), len(m), mp, _p(out),
                                 st.ctypes.data_as(C.POINTER(C.c_int32)))
    return out, st


ORACLE_UNRESOLVED = 4


def ext_multiplier(mult, rf_max):
    """The extension level's steps per base step (0: none): one more than the finest level, when
    the plan refines at all and has room for one more level (RVM_MAX_LEVELS = 6; rvm_abi.hip --
    a plan whose stored levels would not fit its memory cap has none: rvm_plan_extension)."""
    m = [int(x) for x in mult]
    return max(m) + 1 if rf_max > 0 and 2 <= len(m) < 6 else 0


def logl_whx_adapt_batch(params, np_, obs, dt, mult, tol, rf_max, hill_factor=1.0, has_hk=1, has_inc=0, ext=None,
                         ctx=None, ecc_guard=0.0):
    """The kernel's algorithm with adaptive resolution (rvm_config.resolve_tol / resolve_max):
    a direction whose extrapolation-error estimate exceeds tol / 2 gets the extension level (ext
    steps per base step; default ext_multiplier) and, if that does not settle it, passes with every
    step halved (rvoracle.c whx_direction_adapt).
    params [W][np][7] -> (logl[W], status[W], stages [W][2] (0 the plan's step, 1 the extension,
    1 + r r halvings; without the extension r), estimates [W][2], margins [W][2]); margin = the
    closest any decision came to its bound, min |x/bound - 1| (a decision at roundoff distance may
    go the other way in a second implementation).  tol = 0 is the plain rvo_whx algorithm.
    ctx = dict(mode [W] (0 none, 1 emcee stretch, 2 MH), dim, z [W], u [W], lnp0 [W]): the sampler's
    accept inputs of each walker, for the certain-reject cut; then a sixth result, cut [W][2].
    ecc_guard > 0: walkers with a planet of eccentricity above it always get the extension
    (rvm_plan_set_verify_eccentricity)."""
    pl = _f64(params)
    W = pl.shape[0]
    t = _f64(np.concatenate([obs.tf, obs.tb]))
    rv = _f64(np.concatenate([obs.rvf, obs.rvb]))
    er = _f64(np.concatenate([obs.errorf, obs.errorb]))
    out = np.zeros(W)
    st = np.zeros(W, dtype=np.int32)
    rf = np.zeros((W, 2), dtype=np.int32)
    cut = np.zeros((W, 2), dtype=np.int32)
    est = np.zeros((W, 4))
    m, mp = _mult(mult)
    tol_dir = 0.5 * float(tol) if tol > 0 else np.inf
    ext = ext_multiplier(mult, rf_max) if ext is None else int(ext)
    ip32 = C.POINTER(C.c_int32)
    if ctx is not None:
        mode = np.ascontiguousarray(np.asarray(ctx["mode"], dtype=np.int32))
        dz, du, dl = (_f64(np.broadcast_to(np.asarray(ctx[k], dtype=np.float64), (W,))) for k in ("z", "u", "lnp0"))
        cargs = (mode.ctypes.data_as(ip32), int(ctx["dim"]), _p(dz), _p(du), _p(dl))
    else:
        cargs = (None, 0, None, None, None)
    lib().rvo_logl_whx_adapt_batch(W, np_, _p(pl), has_hk, has_inc, float(hill_factor), _p(t), _p(rv), _p(er),
                                   len(t), float(obs.Npoints), float(dt), len(m), mp, ext, tol_dir, int(rf_max),
                                   *cargs, float(ecc_guard), _p(out), st.ctypes.data_as(ip32),
                                   rf.ctypes.data_as(ip32), _p(est),
                                   cut.ctypes.data_as(ip32))
    if ctx is not None:
        return out, st, rf, est[:, :2], est[:, 2:], cut
    return out, st, rf, est[:, :2], est[:, 2:]


def min_distance_ratio(params, np_, obs, dt, n_levels):
    """Closest pair approach / exit distance seen by the WH restatement (diagnostic)."""
    L = lib()
    L.rvo_debug_min_ratio.restype = C.c_double
    L.rvo_debug_min_ratio.argtypes = [C.c_int]
    L.rvo_debug_min_ratio(1)
    logl_whx_batch(params, np_, obs, dt, n_levels)
    return float(np.sqrt(L.rvo_debug_min_ratio(1)))


def kernel_params_to_oracle(K, n_planets):
    """kernel SoA [5*np][W] (m,a,h,k,l) -> oracle [W][np][7]."""
    K = np.asarray(K, dtype=np.float64)
    W = K.shape[1]
    out = np.zeros((W, n_planets, 7))
    for p in range(n_planets):
        out[:, p, :5] = K[5 * p:5 * p + 5].T
    return out


# ---------------------------------------------------------------------------------------------
# Observation constructors (numpy restatements)
# ---------------------------------------------------------------------------------------------
class OracleObs:
    """Plain container with the reference Observation attributes (observations.py:6-16)."""

    def __init__(self, **kw):
        for k in ("tf", "tb", "rvf", "rvb", "errorf", "errorb", "t", "rv", "err"):
            setattr(self, k, kw.get(k))
        self.Npoints = kw.get("Npoints", 0)


def obs_from_file(filename, Npoints=30):
    """observations.py:53-69 Observation_FromFile."""
    readtimes = np.genfromtxt(filename, usecols=(0), delimiter=" ", dtype="d")
    readrvs = np.genfromtxt(filename, usecols=(1), delimiter=" ", dtype="d")
    readerrors = np.genfromtxt(filename, usecols=(2), delimiter=" ", dtype="d")
    readb, readf = np.array_split(readtimes * 0.01720, 2)
    shift = readb[len(readb) - 1]
    tf = readf - shift
    tb = readb - shift
    rvb, rvf = np.array_split(readrvs * 3.355e-5, 2)
    errorb, errorf = np.array_split(readerrors * 3.355e-5, 2)
    return OracleObs(tf=tf, tb=tb, rvf=rvf, rvb=rvb, errorf=errorf, errorb=errorb, Npoints=Npoints,
                     t=np.concatenate((tb, tf)), rv=np.concatenate((rvb, rvf)),
                     err=np.concatenate((errorb, errorf)))


def fake_obs(planets, Npoints=30, error=0.0, errorVar=0.0, tmax=1.5, rv_fn=None):
    """observations.py:19-50 FakeObservation; global legacy numpy RNG in the reference's order.

    The simulation has no exit_min_distance (no Encounter) and integrates tf in order, then
    continues to tb in order.  `rv_fn(planets, times) -> rv` defaults to the IAS15 restatement.
    """
    half = int(Npoints / 2.0)
    tf = np.append([0], np.sort(np.random.uniform(0.0, tmax / 2.0, half)))
    tb = np.sort(np.random.uniform(0.0, -tmax / 2.0, half))
    if rv_fn is None:
        rv_all, st, _ = get_rv_ias15(planets, np.concatenate([tf, tb]), hill_factor=0.0)
        assert st == 0
    else:
        rv_all = rv_fn(planets, np.concatenate([tf, tb]))
    rvf = np.zeros(half + 1)
    rvb = np.zeros(half)
    errorf = np.zeros(half + 1)
    errorb = np.zeros(half)
    for i in range(len(tf)):
        errorf[i] = error + np.random.normal(0.0, errorVar)
        rvf[i] = rv_all[i] + np.random.normal(0.0, errorf[i])
    for i in range(len(tb)):
        errorb[i] = error + np.random.normal(0.0, errorVar)
        rvb[i] = rv_all[len(tf) + i] + np.random.normal(0.0, errorb[i])
    return OracleObs(tf=tf, tb=tb, rvf=rvf, rvb=rvb, errorf=errorf, errorb=errorb, Npoints=Npoints,
                     t=np.concatenate((tb, tf)), rv=np.concatenate((rvb, rvf)),
                     err=np.concatenate((errorb, errorf)))

"""Reference-physics decision parity: sampler decisions against the IAS15 oracle.

Test infrastructure only.  The reference samplers evaluate `State.get_logp` with REBOUND's IAS15
(state.py:36-73, 103-110); `oracle/rvoracle.c` restates IAS15 (pinned by G1-G4).  Here the
reference side of a sampler step is restated in numpy with the SAME draws the device used and the
IAS15 oracle as the likelihood:

  * emcee 2.2.1 stretch (mcmc.py:57-65): z, j, q = c_j - z (c_j - x),
    accept if (dim - 1) ln z + lnp(q) - lnp(x) > ln u3;
  * Mh.step (mcmc.py:107-121): q = x + step * scales * g, priorHard -> reject, accept if
    exp(lnp(q) - lnp(x)) > u, Encounter -> reject.

A device decision may differ from the IAS15-driven one only where the two likelihoods legitimately
differ: walkers whose margin |lnpdiff - ln u| is below MARGIN (the WH + Richardson vs IAS15
tolerance, T2 1e-6), proposals whose status differs (an encounter caught by one integrator and not
the other: the kernel tests the exit distance at every kick, REBOUND after each IAS15 step --
SURVEY H2), and chaotic proposals whose IAS15 logL itself moves by more than ROUNDOFF_REL (relative)
when an input moves by 1e-15 (ias15_roundoff: no second integrator can follow them).  All three are
counted and reported; every other decision must be identical, and every other OK proposal must
have |dlogL| <= MARGIN.
"""
import json
import os
from concurrent.futures import ThreadPoolExecutor

import numpy as np

import oracle as O

MARGIN = 1e-6  # walkers with |lnpdiff - ln U| < 1e-6 are exempt (counted)
ROUNDOFF_REL = 1e-9  # IAS15 logL response to a 1e-15 relative input nudge, relative to max(1, |logL|)
NUDGES = [(0, 4, 1), (-1, 4, -1), (0, 1, 1), (-1, 1, -1)]
ST_OK, ST_PRIOR, ST_ENC, ST_UNRESOLVED = 0, 1, 2, 4


def n_threads():
    """The CPUs this process may run on (the GPU box's share; os.cpu_count() is the whole machine)."""
    try:
        n = max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        n = max(1, os.cpu_count() or 1)
    # the GPU box exports its CPU share as OMP_NUM_THREADS (16 per GPU) while the affinity mask
    # covers the whole machine: the smaller of the two
    try:
        n = min(n, max(1, int(os.environ.get("OMP_NUM_THREADS", n))))
    except ValueError:
        pass
    return n


def ias15_logl(P, n_planets, obs, hill=1.0, has_inc=0):
    """IAS15 oracle logL of P [W][np][7] on all of the box's CPU share (ctypes drops the GIL)."""
    P = np.ascontiguousarray(P, dtype=np.float64)
    W = len(P)
    if W == 0:
        return np.zeros(0), np.zeros(0, dtype=np.int32)
    nt = min(n_threads(), W)
    chunks = np.array_split(np.arange(W), nt)
    with ThreadPoolExecutor(nt) as ex:
        parts = list(ex.map(lambda ix: O.logl_ias15_batch(P[ix], n_planets, obs, hill, 1, has_inc), chunks))
    return np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]).astype(np.int32)


def ias15_roundoff(P, n_planets, obs, ref, hill=1.0, has_inc=0):
    """Per-proposal roundoff sensitivity of the IAS15 logL: max over 1e-15 relative nudges of one
    input (l, a of the first / last planet) of |logL' - logL| / max(1, |logL|) (inf where a nudge
    flips the status).  Measured on the device-independent reference alone, so an exemption by it
    cannot be earned by the device's own error."""
    sens = np.zeros(len(P))
    if len(P) == 0:
        return sens
    st0 = None
    for pl, par, sgn in NUDGES:
        P2 = np.array(P, dtype=np.float64, copy=True)
        P2[:, pl, par] *= 1 + sgn * 1e-15
        r2, s2 = ias15_logl(P2, n_planets, obs, hill, has_inc)
        if st0 is None:
            st0 = ias15_logl(P, n_planets, obs, hill, has_inc)[1]
        both = (s2 == 0) & (st0 == 0)
        sens[both] = np.maximum(sens[both], np.abs(r2[both] - ref[both]) / np.maximum(1.0, np.abs(ref[both])))
        sens[s2 != st0] = np.inf
    return sens


def to_oracle(pm, X):
    """Free-parameter rows X [W][dim] of a State's ParamMap -> oracle layout [W][np][7]."""
    if len(X) == 0:
        return np.zeros((0, pm.n_planets, 7))
    K = np.stack([pm.vector_to_kernel_np(x) for x in np.asarray(X, dtype=np.float64)], 1)  # [rows][W]
    rows = 7 if pm.inclined else 5
    W = K.shape[1]
    out = np.zeros((W, pm.n_planets, 7))
    for p in range(pm.n_planets):
        out[:, p, :rows] = K[rows * p:rows * (p + 1)].T
    return out


def stretch_proposal(x, c, u1, u2, a=2.0):
    """emcee 2.2.1 _propose_stretch with given uniforms (plain IEEE, no FMA: bit-identical to
    rvm_stretch.h)."""
    zz = ((a - 1.) * u1 + 1) * ((a - 1.) * u1 + 1) / a
    j = np.floor(u2 * len(c)).astype(int)
    j = np.clip(j, 0, len(c) - 1)
    q = c[j] - zz[:, None] * (c[j] - x)
    return q, zz


class Tally:
    """Decision comparison counts of one sampler run."""

    def __init__(self, name):
        self.name = name
        self.n = 0
        self.agree = 0
        self.exempt_margin = 0
        self.exempt_status = 0
        self.disagree_exempt = 0
        self.mismatch = []
        self.status_pairs = {}
        self.accepted_ref = 0
        self.max_dlogl_ok = 0.0
        self.n_enc_ref = 0
        self.n_prior = 0
        self.exempt_roundoff = 0
        self.disagree_roundoff = 0
        self.n_beyond_margin_dlogl = 0
        self.beyond_margin_not_roundoff = 0
        self.n_unresolved = 0

    def add(self, acc_dev, acc_ref, margin, st_dev, st_ref, lnq_dev=None, lnq_ref=None, idx_offset=0,
            roundoff=None, current_differs=None):
        """margin: |lnpdiff_ias15 - ln u| per decision.  roundoff (optional): the IAS15 logL's own
        roundoff sensitivity per proposal (ias15_roundoff); proposals above ROUNDOFF_REL are
        exempt from the decision and T2 checks (counted separately).  current_differs (optional):
        walkers whose CURRENT position has a logL status the two chains disagree on (one finite,
        the other -inf: a status disagreement counted when that position was proposed or set),
        whose decision then compares against different lnp0."""
        acc_dev = np.asarray(acc_dev, bool)
        acc_ref = np.asarray(acc_ref, bool)
        st_dev = np.asarray(st_dev)
        st_ref = np.asarray(st_ref)
        near = margin < MARGIN
        # a status pair is exempt only where the two integrators legitimately differ (an encounter
        # caught by one and not the other); a walker the device left UNRESOLVED (4) has no
        # counterpart in the reference (IAS15 always integrates, mcmc.py:28-35 maps only exceptions
        # to -inf): its decision must match like any other
        sdiff = (st_dev != st_ref) & (st_dev != ST_UNRESOLVED)
        self.n_unresolved += int((st_dev == ST_UNRESOLVED).sum())
        exempt = near | sdiff
        if current_differs is not None:
            cd = np.asarray(current_differs, bool) & ~exempt
            self.exempt_current = getattr(self, "exempt_current", 0) + int(cd.sum())
            exempt = exempt | cd
        chaotic = np.zeros(len(acc_dev), bool)
        if roundoff is not None:
            chaotic = np.asarray(roundoff) > ROUNDOFF_REL
            ro = chaotic & ~exempt
            self.exempt_roundoff += int(ro.sum())
            self.disagree_roundoff += int(((acc_dev != acc_ref) & ro).sum())
            exempt = exempt | ro
        same = acc_dev == acc_ref
        self.n += len(acc_dev)
        self.agree += int(same.sum())
        self.exempt_margin += int(near.sum())
        self.exempt_status += int(sdiff.sum())
        self.disagree_exempt += int((~same & exempt).sum())
        self.accepted_ref += int(acc_ref.sum())
        self.n_enc_ref += int((st_ref == ST_ENC).sum())
        self.n_prior += int((st_ref == ST_PRIOR).sum())
        for a, b in zip(st_dev[st_dev != st_ref], st_ref[st_dev != st_ref]):
            k = f"{int(a)}/{int(b)}"
            self.status_pairs[k] = self.status_pairs.get(k, 0) + 1
        self.mismatch += [int(i) + idx_offset for i in np.nonzero(~same & ~exempt)[0]]
        if lnq_dev is not None:
            ok = (st_dev == ST_OK) & (st_ref == ST_OK)
            if ok.any():
                dl = np.abs(lnq_dev[ok] - lnq_ref[ok])
                self.max_dlogl_ok = max(self.max_dlogl_ok, float(np.max(dl)))
                self.n_beyond_margin_dlogl += int((dl > MARGIN).sum())
                self.beyond_margin_not_roundoff += int(((dl > MARGIN) & ~chaotic[ok]).sum())
                nc = ~chaotic[ok]
                if nc.any():
                    self.max_dlogl_ok_not_roundoff = max(getattr(self, "max_dlogl_ok_not_roundoff", 0.0),
                                                         float(np.max(dl[nc])))

    def report(self, **extra):
        d = {"test": self.name, "decisions": self.n, "identical": self.agree,
             "exempt_current_status_disagreement": getattr(self, "exempt_current", 0),
             "exempt_near_margin": self.exempt_margin, "exempt_status_disagreement": self.exempt_status,
             "status_pairs_device/ias15": self.status_pairs, "differing_but_exempt": self.disagree_exempt,
             "mismatches_not_exempt": len(self.mismatch), "accepted_ias15": self.accepted_ref,
             "encounters_ias15": self.n_enc_ref, "prior_rejections": self.n_prior,
             "max_abs_dlogl_ok_proposals": self.max_dlogl_ok, "ok_proposals_dlogl_above_margin":
             self.n_beyond_margin_dlogl, "exempt_ias15_roundoff_sensitive": self.exempt_roundoff,
             "differing_ias15_roundoff_sensitive": self.disagree_roundoff,
             "ok_proposals_dlogl_above_margin_not_roundoff": self.beyond_margin_not_roundoff,
             "max_abs_dlogl_ok_proposals_not_roundoff": getattr(self, "max_dlogl_ok_not_roundoff", 0.0),
             "unresolved_device": self.n_unresolved, "margin": MARGIN, "roundoff_rel": ROUNDOFF_REL}
        d.update(extra)
        line = json.dumps(d)
        print(line)
        path = os.environ.get("RVM_PARITY_REPORT")
        if path:
            with open(path, "a") as f:
                f.write(line + "\n")
        return d

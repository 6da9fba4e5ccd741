"""Observation containers (mirror of /root/reference/observations.py).

* Observation_FromFile (observations.py:53-69): 3-column .vels (days, m/s, m/s); days * 0.01720
  -> code time, m/s * 3.355e-5 -> code velocity; np.array_split(..., 2) gives (tb, tf) = (first
  half, second half); both shifted so that tb ends at t = 0.
* FakeObservation (observations.py:19-50): tf = [0] + sorted U(0, tmax/2) draws, tb = sorted
  U(0, -tmax/2) draws; per epoch sigma_i = error + N(0, errorVar) then rv_i = vx + N(0, sigma_i),
  all from numpy's legacy global RNG in the reference's order.  The model RV
  comes from the GPU kernel (no exit distance, as the reference's FakeObservation simulation has
  none).
"""
from __future__ import annotations

import numpy as np


class Observation:
    tf = None
    tb = None
    rvf = None
    rvb = None
    Npoints = 0
    errorf = None
    errorb = None
    t = None
    rv = None
    err = None


class FakeObservation(Observation):
    def __init__(self, state, Npoints=30, error=0., errorVar=0., tmax=1.5):
        self.Npoints = Npoints
        self.error = error
        self.errorVar = errorVar
        half = int(self.Npoints / 2.)
        self.tf = np.append([0], np.sort(np.random.uniform(0., tmax / 2., half)))
        self.tb = np.sort(np.random.uniform(0., -tmax / 2., half))
        rv_model = _model_rv(state, np.concatenate([self.tf, self.tb]))
        self.rvf = np.zeros(half + 1)
        self.rvb = np.zeros(half)
        self.errorf = np.zeros(half + 1)
        self.errorb = np.zeros(half)
        for i in range(len(self.tf)):
            self.errorf[i] = error + np.random.normal(0., self.errorVar)
            self.rvf[i] = rv_model[i] + np.random.normal(0., self.errorf[i])
        for i in range(len(self.tb)):
            self.errorb[i] = error + np.random.normal(0., self.errorVar)
            self.rvb[i] = rv_model[len(self.tf) + i] + np.random.normal(0., self.errorb[i])
        self.t = np.concatenate((self.tb, self.tf), axis=0)
        self.rv = np.concatenate((self.rvb, self.rvf), axis=0)
        self.err = np.concatenate((self.errorb, self.errorf), axis=0)


class Observation_FromFile(Observation):
    def __init__(self, filename='yourfile.txt', Npoints=30):
        readtimes = np.genfromtxt(filename, usecols=(0), delimiter=' ', dtype='d')
        readrvs = np.genfromtxt(filename, usecols=(1), delimiter=' ', dtype='d')
        readerrors = np.genfromtxt(filename, usecols=(2), delimiter=' ', dtype='d')
        readb, readf = np.array_split(readtimes * 0.01720, 2)
        shift = readb[len(readb) - 1]
        self.Npoints = Npoints
        self.tf = readf - shift
        self.tb = readb - shift
        self.rvb, self.rvf = np.array_split(readrvs * 3.355e-5, 2)
        self.errorb, self.errorf = np.array_split(readerrors * 3.355e-5, 2)
        self.t = np.concatenate((self.tb, self.tf), axis=0)
        self.rv = np.concatenate((self.rvb, self.rvf), axis=0)
        self.err = np.concatenate((self.errorb, self.errorf), axis=0)


def _model_rv(state, times):
    """Star barycentric vx at `times` with no encounter check (the FakeObservation simulation)."""
    saved = state.hillRadiusFactor
    try:
        state.hillRadiusFactor = 0.0
        return state.get_rv(times)
    finally:
        state.hillRadiusFactor = saved

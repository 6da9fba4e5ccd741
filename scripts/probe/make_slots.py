"""Build the probe input of scripts/probe/resolve_cost.py: the 6144 walker slots of one speculative
stretch iteration (half 0 against half 1; half 1 against half 0 both ways) formed from a dumped
bench ensemble (scripts/dump_bench_ensemble.py -> profiles/r03_bench_ensemble.npz), with the bench's
observation set.  Usage: python scripts/probe/make_slots.py KEY OUT.npz"""
import sys

import numpy as np


def main():
    key, out = sys.argv[1], sys.argv[2]
    d = np.load("profiles/r03_bench_ensemble.npz")
    X = d[key]
    n = len(X) // 2
    rng = np.random.default_rng(1)
    a = 2.0

    def stretch(x, c):
        z = ((a - 1.0) * rng.random(len(x)) + 1.0) ** 2 / a
        j = rng.integers(0, len(c), len(x))
        return c[j] - z[:, None] * (c[j] - x)

    q0 = stretch(X[:n], X[n:])
    q1a = stretch(X[n:], X[:n])
    q1b = stretch(X[n:], q0)
    K = np.concatenate([q0, q1a, q1b])
    np.savez(out, K=K, **{k: d[k] for k in ("tf", "tb", "rvf", "rvb", "errorf", "errorb")})
    print(out, K.shape)


if __name__ == "__main__":
    main()

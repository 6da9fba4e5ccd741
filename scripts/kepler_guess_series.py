"""Series reversion behind the Kepler drift's initial guess (rvm_device.h drift): in universal
variables u = dt / r0 = G1(X) + s G2(X) + g G3(X) (s = eta0 / r0, g = GM / r0, beta = 2 GM / r0 - v0^2),
X = u + a2 u^2 + a3 u^3 + ...; the kernel uses a2..a4 (T3 = a3, T4 = a4) and, with G5, a5 (T5).
Prints the coefficients (sympy) and checks the fifth-order guess numerically against the solved X."""
import sympy as sp
X,u,s,g,b = sp.symbols('X u s g beta')
# u = t/r0 as a function of X (universal variables), to X^6:
# G1 = X - b X^3/6 + b^2 X^5/120 ; G2 = X^2/2 - b X^4/24 + b^2 X^6/720 ; G3 = X^3/6 - b X^5/120
# t = r0 G1 + eta G2 + GM G3 -> u = G1 + s G2 + g G3   (s = eta/r0, g = GM/r0)
G1 = X - b*X**3/6 + b**2*X**5/120
G2 = X**2/2 - b*X**4/24 + b**2*X**6/720
G3 = X**3/6 - b*X**5/120
useries = sp.expand(G1 + s*G2 + g*G3)
# revert: X = u + a2 u^2 + ... + a5 u^5
a = sp.symbols('a2:7')
Xs = u + sum(a[i]*u**(i+2) for i in range(5))
expr = sp.expand(useries.subs(X, Xs)) - u
sol = {}
for k in range(2, 7):
    c = sp.expand(expr).coeff(u, k)
    c = c.subs(sol)
    ak = sp.solve(sp.Eq(c, 0), a[k-2])[0]
    sol[a[k-2]] = sp.simplify(ak)
    print(f"a{k} =", sp.factor(sp.expand(sol[a[k-2]])))


import math  # noqa: E402

import numpy as np  # noqa: E402


def check(n=2000, seed=1):
    """relative error of the 4th- and 5th-order guesses against Newton-solved X on random eccentric
    states and steps (median over the sample, per step-size bin)"""
    rng = np.random.default_rng(seed)

    def stumpff(z):
        c2 = sum((-z) ** j / math.factorial(2 * j + 2) for j in range(12))
        c3 = sum((-z) ** j / math.factorial(2 * j + 3) for j in range(12))
        return c2, c3

    out = []
    for _ in range(n):
        a, e, M = rng.uniform(0.5, 1.6), rng.uniform(0.0, 0.6), rng.uniform(0, 2 * np.pi)
        E = M
        for _ in range(50):
            E = E - (E - e * np.sin(E) - M) / (1 - e * np.cos(E))
        r0 = a * (1 - e * np.cos(E))
        eta = np.sqrt(a) * e * np.sin(E)   # r . v with GM = 1
        beta = 1.0 / a
        dt = rng.choice([1 / 32, 1 / 64, 1 / 112]) * 2 * np.pi * a ** 1.5
        uu, ss, gg = dt / r0, eta / r0, 1.0 / r0
        X = uu
        for _ in range(60):
            z = beta * X * X
            c2, c3 = stumpff(z)
            G1, G2, G3 = X * (1 - z * c3), X * X * c2, X ** 3 * c3
            f = r0 * G1 + eta * G2 + G3 - dt
            fp = r0 * (1 - z * c2) + eta * G1 + G2
            X -= f / fp
        T3 = ss * ss / 2 + (beta - gg) / 6
        T4 = -ss * (9 * beta - 10 * gg + 15 * ss ** 2) / 24
        T5 = (9 * beta ** 2 - 19 * beta * gg + 90 * beta * ss ** 2 + 10 * gg ** 2 - 105 * gg * ss ** 2 + 105 * ss ** 4) / 120
        x4 = uu * (1 + uu * (-ss / 2 + uu * (T3 + uu * T4)))
        x5 = uu * (1 + uu * (-ss / 2 + uu * (T3 + uu * (T4 + uu * T5))))
        out.append((abs(x4 - X) / X, abs(x5 - X) / X))
    o = np.array(out)
    for name, k in (("4th order", 0), ("5th order", 1)):
        print(f"{name}: median rel err {np.median(o[:, k]):.2e}, fraction > 9e-6 (the first Halley step's "
              f"acceptance): {np.mean(o[:, k] > 9e-6):.3f}")


check()

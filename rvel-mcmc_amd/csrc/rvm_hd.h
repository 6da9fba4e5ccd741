// rvm_hd.h -- hyper-dual fp64 arithmetic and the hyper-dual restatement of the integrator
// building blocks, for exact first and second derivatives of the walker log-likelihood.
//
// The reference differentiates its likelihood with REBOUND's first- and second-order variational
// equations (state.py:218-294: setup_sim_vars adds one order-1 variation per free parameter and
// one order-2 variation per pair, get_chi2_d_dd accumulates chi2, its gradient and its Hessian
// from the variational particles' star vx).  Here the same quantities are the exact derivatives
// of the plan's discrete integrator (Wisdom-Holman + Richardson, rvm_logl.hip), obtained by
// forward-mode differentiation: every real number x of the computation carries
//   (x, dx/dp_i, dx/dp_j, d2x/dp_i dp_j)
// for one parameter pair (i, j), the order-1 and order-2 variations of one pair of the reference's
// variational particles.  Control flow (Kepler solver branches, encounter test, prior) depends on
// the primal values only; iterative solves (Pal's eccentric anomaly, the universal Kepler
// equation) converge on the primal and then take two Newton steps in hyper-dual arithmetic from
// the converged root (implicit-function derivatives: the first step makes the first-order parts
// exact, the second the second-order part).
#pragma once
#include "rvm_device.h"

namespace rvm {

struct HD {
    double v, a, b, ab;  // value, d/dp_i, d/dp_j, d2/dp_i dp_j
};

__device__ __forceinline__ HD hd_c(double v) { return HD{v, 0.0, 0.0, 0.0}; }
__device__ __forceinline__ HD operator+(HD x, HD y) { return HD{x.v + y.v, x.a + y.a, x.b + y.b, x.ab + y.ab}; }
__device__ __forceinline__ HD operator-(HD x, HD y) { return HD{x.v - y.v, x.a - y.a, x.b - y.b, x.ab - y.ab}; }
__device__ __forceinline__ HD operator-(HD x) { return HD{-x.v, -x.a, -x.b, -x.ab}; }
__device__ __forceinline__ HD operator+(HD x, double s) { return HD{x.v + s, x.a, x.b, x.ab}; }
__device__ __forceinline__ HD operator+(double s, HD x) { return HD{x.v + s, x.a, x.b, x.ab}; }
__device__ __forceinline__ HD operator-(HD x, double s) { return HD{x.v - s, x.a, x.b, x.ab}; }
__device__ __forceinline__ HD operator-(double s, HD x) { return HD{s - x.v, -x.a, -x.b, -x.ab}; }
__device__ __forceinline__ HD operator*(double s, HD x) { return HD{s * x.v, s * x.a, s * x.b, s * x.ab}; }
__device__ __forceinline__ HD operator*(HD x, double s) { return s * x; }
__device__ __forceinline__ HD operator*(HD x, HD y) {
    return HD{x.v * y.v, fma(x.v, y.a, x.a * y.v), fma(x.v, y.b, x.b * y.v),
              fma(x.v, y.ab, fma(x.a, y.b, fma(x.b, y.a, x.ab * y.v)))};
}
// f(x) for a scalar function with f = f(x.v), f1 = f'(x.v), f2 = f''(x.v)
__device__ __forceinline__ HD hd_chain(double f, double f1, double f2, HD x) {
    return HD{f, f1 * x.a, f1 * x.b, fma(f1, x.ab, (f2 * x.a) * x.b)};
}
// reciprocals and square roots from v_rcp_f64 / v_rsq_f64 with one cubic refinement (rvm_device.h
// rcp_nr / rsq_nr: faithfully rounded, no IEEE division sequence)
__device__ __forceinline__ HD hd_inv(HD x) {
    const double f = rcp_nr(x.v);
    return hd_chain(f, -f * f, 2.0 * f * f * f, x);
}
__device__ __forceinline__ HD operator/(HD x, HD y) { return x * hd_inv(y); }
__device__ __forceinline__ HD operator/(HD x, double s) { return (1.0 / s) * x; }
__device__ __forceinline__ HD operator/(double s, HD x) { return s * hd_inv(x); }
__device__ __forceinline__ HD hd_sqrt(HD x) {
    const double y = rsq_nr(x.v), f = x.v * y;  // y = 1/sqrt(x)
    return hd_chain(f, 0.5 * y, (-0.25 * y) * (y * y), x);
}
__device__ __forceinline__ HD hd_sin(HD x) {
    double s, c;
    sincos(x.v, &s, &c);
    return hd_chain(s, c, -s, x);
}
__device__ __forceinline__ HD hd_cos(HD x) {
    double s, c;
    sincos(x.v, &s, &c);
    return hd_chain(c, -s, -c, x);
}

// ---- lane-group exchange (rvm_device.h grp_get) component by component ---------------------------
template <int L, int Q>
__device__ __forceinline__ HD grp_get_hd(HD x) {
    return HD{grp_get<L, Q>(x.v), grp_get<L, Q>(x.a), grp_get<L, Q>(x.b), grp_get<L, Q>(x.ab)};
}
template <int L>
__device__ __forceinline__ HD grp_get_hd(HD x, int q) {
    switch (q) {
        case 0:
            return grp_get_hd<L, 0>(x);
        case 1:
            return grp_get_hd<L, 1>(x);
        case 2:
            return grp_get_hd<L, 2>(x);
        default:
            return grp_get_hd<L, 3>(x);
    }
}

// ---- Stumpff functions of a hyper-dual argument (any z): quarter z until |z| <= 0.1, 8-term
// series, double back (the same identities as stumpff_full; they hold exactly, so their
// hyper-dual images carry the exact derivatives) -----------------------------------------------
__device__ __forceinline__ void stumpff_hd(HD z, HD& c0, HD& c1, HD& c2, HD& c3) {
    int n = 0;
    double sc = 1.0;
    while (fabs(z.v * sc) > 0.1 && n < 40) {
        sc *= 0.25;
        n++;
    }
    const HD zs = sc * z;
    HD a = hd_c(StumpffK::K2[7]), b = hd_c(StumpffK::K3[7]);
#pragma unroll
    for (int j = 6; j >= 0; j--) {
        a = a * zs + StumpffK::K2[j];
        b = b * zs + StumpffK::K3[j];
    }
    HD C2 = a, C3 = b;
    HD C1 = 1.0 - zs * C3;
    HD C0 = 1.0 - zs * C2;
    for (; n > 0; n--) {
        C3 = 0.25 * (C2 + C0 * C3);
        C2 = 0.5 * (C1 * C1);
        C1 = C0 * C1;
        C0 = 2.0 * (C0 * C0) - 1.0;
    }
    c0 = C0;
    c1 = C1;
    c2 = C2;
    c3 = C3;
}

// G-functions G_k(X, beta) = X^k c_k(beta X^2)
__device__ __forceinline__ void gfun_hd(HD X, HD beta, HD& G0, HD& G1, HD& G2, HD& G3) {
    const HD X2 = X * X;
    HD c0, c1, c2, c3;
    stumpff_hd(beta * X2, c0, c1, c2, c3);
    G0 = c0;
    G1 = X * c1;
    G2 = X2 * c2;
    G3 = X2 * X * c3;
}

// Primal universal-Kepler root for the hyper-dual drift, per lane: Halley steps from the
// fourth-order Taylor guess of rvm_device.h drift (8-term Stumpff series for |z| <= 0.3, the full
// evaluation beyond), stopped once a correction is below 1e-6 |X| -- Halley is cubic, so the
// remaining error is ~1e-18 |X|, and drift_hd's hyper-dual quadratic-model step refines the root
// once more -- with the bracketed solver for hard steps or no convergence.
__device__ __forceinline__ double kepler_primal(double r0, double eta, double zeta, double beta, double GM,
                                                double dt) {
    const double ir0 = rcp_nr(r0);
    const double u = dt * ir0, sg = eta * ir0, g = GM * ir0;
    const double hs = 0.5 * sg;
    const double T3 = fma(hs, sg, (beta - g) * (1.0 / 6.0));
    const double T4 = sg * fma(-0.625 * sg, sg, fma(5.0 / 12.0, g, -0.375 * beta));
    double X = u * fma(u, fma(u, fma(u, T4, T3), -hs), 1.0);
    bool done = false;
    if (fabs(beta) * (u * u) <= 0.5) {
        for (int it = 0; it < 12 && !done; it++) {
            const double X2 = X * X, z = beta * X2;
            double c0, c1, c2, c3;
            if (fabs(z) <= 0.3) {
                stumpff23<8>(z, c2, c3);
                c1 = fma(-z, c3, 1.0);
                c0 = fma(-z, c2, 1.0);
            } else {
                stumpff_full(z, c0, c1, c2, c3);
            }
            const double G1 = X * c1, G2 = X2 * c2, G3 = X2 * X * c3;
            const double f = fma(GM, G3, fma(eta, G2, fma(r0, G1, -dt)));
            const double fp = fma(GM, G2, fma(eta, G1, r0 * c0));
            const double fpp = fma(zeta, G1, eta * c0);
            const double dX = (f * fp) * rcp_nr(fma(-0.5 * f, fpp, fp * fp));
            X -= dX;
            done = !(fabs(dX) > 1e-6 * fabs(X)) || !isfinite(dX);
        }
    }
    if (!done || !isfinite(X)) {
        double G0, G1, G2, G3;
        kepler_safe(r0, eta, zeta, beta, GM, dt, X, G0, G1, G2, G3);
    }
    return X;
}

// One planet's Jacobi coordinate in hyper-dual form plus the walker constants every lane needs.
template <int NP>
struct LaneHD {
    HD rx, ry, rz, vx, vy, vz;
    HD GM;          // interior mass M_p of the own coordinate
    HD m[NP];       // planet masses
    HD iMi[NP + 1]; // 1 / interior masses (iMi[0] = 1)
    HD mu[NP];      // m_q / M_q
    HD kA, kB, kC;  // closed-form two-planet kick coefficients of the own lane (kick2_hd)
    HD c12;         // m_1 / M_1 (heliocentric x_2 = r'_2 + c12 r'_1)
    double dmin2;   // (hill_factor * max r_Hill)^2, primal (the encounter test is a primal decision)
    int p;
    uint64_t encm;
};

// Kepler drift of the own coordinate by dt (rvm_device.h drift, same physics).  The primal root X
// of F(X) = r0 G1 + eta G2 + GM G3 - dt comes from kepler_primal; the G-functions are evaluated
// ONCE, in hyper-dual arithmetic at that fixed X (their variations then carry only the
// dependence on beta), and the variations of the root follow from the quadratic model
//   F + F_X d + F_XX d^2 / 2 = 0,   d = X_hd - X:   d0 = -F / F_X,  d = -(F + F_XX d0^2 / 2) / F_X
// (exact to second order: d0^2 has only an order-2 part), with F_X = r, F_XX = eta G0 + zeta G1.
// G_k(X + d) = G_k + G_k' d + G_k'' d^2 / 2 with G_k' = G_(k-1), G_0' = -beta G1, G_0'' = -beta G0,
// G_1'' = -beta G1.
template <bool D3, int NP>
__device__ __forceinline__ void drift_hd(LaneHD<NP>& s, double dt) {
    HD r2 = s.rx * s.rx + s.ry * s.ry;
    HD v2 = s.vx * s.vx + s.vy * s.vy;
    HD eta = s.rx * s.vx + s.ry * s.vy;
    if constexpr (D3) {
        r2 = r2 + s.rz * s.rz;
        v2 = v2 + s.vz * s.vz;
        eta = eta + s.rz * s.vz;
    }
    const HD r0 = hd_sqrt(r2);
    const HD ir0 = hd_inv(r0);
    const HD beta = 2.0 * (s.GM * ir0) - v2;
    const HD zeta = s.GM - beta * r0;
    const double X = kepler_primal(r0.v, eta.v, zeta.v, beta.v, s.GM.v, dt);
    const double X2 = X * X;
    HD c0, c1, c2, c3;
    stumpff_hd(X2 * beta, c0, c1, c2, c3);
    HD G0 = c0, G1 = X * c1, G2 = X2 * c2, G3 = (X2 * X) * c3;
    const HD F = r0 * G1 + eta * G2 + s.GM * G3 - dt;
    const HD Fx = r0 * G0 + eta * G1 + s.GM * G2;
    const HD Fxx = eta * G0 + zeta * G1;
    const HD iFx = hd_inv(Fx);
    const HD d0 = -(F * iFx);
    const HD d = -((F + 0.5 * (Fxx * (d0 * d0))) * iFx);
    const HD hd2 = 0.5 * (d * d);
    const HD nbG1 = -(beta * G1);
    const HD H0 = G0 + nbG1 * d - (beta * G0) * hd2;
    const HD H1 = G1 + G0 * d + nbG1 * hd2;
    const HD H2 = G2 + G1 * d + G0 * hd2;
    const HD H3 = G3 + G2 * d + G1 * hd2;
    const HD rr = r0 * H0 + eta * H1 + s.GM * H2;
    const HD irr = hd_inv(rr);
    const HD gG2 = s.GM * H2;
    const HD f = 1.0 - gG2 * ir0;
    const HD g = dt - s.GM * H3;
    const HD fd = -((s.GM * H1) * (ir0 * irr));
    const HD gd = 1.0 - gG2 * irr;
    const HD rx = s.rx, ry = s.ry, vx = s.vx, vy = s.vy;
    s.rx = f * rx + g * vx;
    s.ry = f * ry + g * vy;
    s.vx = fd * rx + gd * vx;
    s.vy = fd * ry + gd * vy;
    if constexpr (D3) {
        const HD rz = s.rz, vz = s.vz;
        s.rz = f * rz + g * vz;
        s.vz = fd * rz + gd * vz;
    }
}

// x^(-3/2)
__device__ __forceinline__ HD hd_rcube(HD x) {
    const double y = rsq_nr(x.v), y2 = y * y;
    const double f = y2 * y;  // x^(-3/2); x^(-1) = y^2
    return hd_chain(f, -1.5 * f * y2, 3.75 * f * (y2 * y2), x);
}

// Two-planet kick in closed form (rvm_device.h kick2, same interaction), hyper-dual:
//   v' += dt [ A r'/|r'|^3 + B x2/r02^3 + C d12/r12^3 ]
// with the lane's (A, B, C) = (0, -m2, m2) for planet 1 and (M2, -M2/M1, -m1 M2/M1) for planet 2
// (LaneHD::kA/kB/kC, set by lane_finish_hd); the encounter bit of planet 1's lane is the one read.
template <int L, bool D3>
__device__ __forceinline__ void kick2_hd(LaneHD<2>& s, double dt) {
    const HD x1 = grp_get_hd<L, 0>(s.rx), y1 = grp_get_hd<L, 0>(s.ry);
    const HD R2x = grp_get_hd<L, 1>(s.rx), R2y = grp_get_hd<L, 1>(s.ry);
    const HD c = s.c12;
    const HD x2 = R2x + c * x1, y2 = R2y + c * y1;
    const HD dx = x2 - x1, dy = y2 - y1;
    HD r02 = x2 * x2 + y2 * y2, r12 = dx * dx + dy * dy, own = s.rx * s.rx + s.ry * s.ry;
    HD z2 = hd_c(0.0), dz = hd_c(0.0);
    if constexpr (D3) {
        const HD z1 = grp_get_hd<L, 0>(s.rz), R2z = grp_get_hd<L, 1>(s.rz);
        z2 = R2z + c * z1;
        dz = z2 - z1;
        r02 = r02 + z2 * z2;
        r12 = r12 + dz * dz;
        own = own + s.rz * s.rz;
    }
    s.encm |= ballot(r02.v < s.dmin2) | ballot(r12.v < s.dmin2) | ballot(own.v < s.dmin2);
    const HD A = s.kA * hd_rcube(own), B = s.kB * hd_rcube(r02), C = s.kC * hd_rcube(r12);
    s.vx = s.vx + dt * (A * s.rx + B * x2 + C * dx);
    s.vy = s.vy + dt * (A * s.ry + B * y2 + C * dy);
    if constexpr (D3) s.vz = s.vz + dt * (A * s.rz + B * z2 + C * dz);
}

// Interaction kick (rvm_device.h kick_generic, same physics, hyper-dual): heliocentric positions
// from the lane group, pairwise accelerations, the Jacobi acceleration of the own coordinate minus
// its Kepler part; the encounter test on every pair (primal).
template <int NP, int L, bool D3>
__device__ __forceinline__ void kick_hd(LaneHD<NP>& s, double dt) {
    constexpr int NB = NP + 1;
    HD x[NB], y[NB], z[NB], ax[NB], ay[NB], az[NB];
    x[0] = y[0] = z[0] = hd_c(0.0);
    HD cmx = hd_c(0.0), cmy = hd_c(0.0), cmz = hd_c(0.0);
#pragma unroll
    for (int i = 1; i < NB; i++) {
        const HD Rx = grp_get_hd<L>(s.rx, i - 1), Ry = grp_get_hd<L>(s.ry, i - 1);
        const HD Rz = D3 ? grp_get_hd<L>(s.rz, i - 1) : hd_c(0.0);
        x[i] = Rx + cmx * s.iMi[i - 1];
        y[i] = Ry + cmy * s.iMi[i - 1];
        z[i] = Rz + cmz * s.iMi[i - 1];
        cmx = cmx + s.m[i - 1] * x[i];
        cmy = cmy + s.m[i - 1] * y[i];
        if constexpr (D3) cmz = cmz + s.m[i - 1] * z[i];
    }
#pragma unroll
    for (int i = 0; i < NB; i++) ax[i] = ay[i] = az[i] = hd_c(0.0);
    uint64_t enc = 0;
#pragma unroll
    for (int i = 0; i < NB; i++) {
#pragma unroll
        for (int j = i + 1; j < NB; j++) {
            const HD dx = x[j] - x[i], dy = y[j] - y[i], dz = z[j] - z[i];
            HD r2 = dx * dx + dy * dy;
            if constexpr (D3) r2 = r2 + dz * dz;
            enc |= ballot(r2.v < s.dmin2);
            const HD ir = hd_inv(hd_sqrt(r2));
            const HD ir3 = ir * ir * ir;
            const HD mj = (j == 0) ? hd_c(1.0) : s.m[j - 1];
            const HD mi = (i == 0) ? hd_c(1.0) : s.m[i - 1];
            const HD fj = mj * ir3, fi = mi * ir3;
            ax[i] = ax[i] + fj * dx;
            ay[i] = ay[i] + fj * dy;
            ax[j] = ax[j] - fi * dx;
            ay[j] = ay[j] - fi * dy;
            if constexpr (D3) {
                az[i] = az[i] + fj * dz;
                az[j] = az[j] - fi * dz;
            }
        }
    }
    s.encm |= enc;
    HD max_ = ax[0], may_ = ay[0], maz_ = az[0];  // M_star = 1
    HD ajx = hd_c(0.0), ajy = hd_c(0.0), ajz = hd_c(0.0);
#pragma unroll
    for (int i = 1; i < NB; i++) {
        if (s.p == i - 1) {
            ajx = ax[i] - max_ * s.iMi[i - 1];
            ajy = ay[i] - may_ * s.iMi[i - 1];
            ajz = az[i] - maz_ * s.iMi[i - 1];
        }
        max_ = max_ + s.m[i - 1] * ax[i];
        may_ = may_ + s.m[i - 1] * ay[i];
        if constexpr (D3) maz_ = maz_ + s.m[i - 1] * az[i];
    }
    HD r2 = s.rx * s.rx + s.ry * s.ry;
    if constexpr (D3) r2 = r2 + s.rz * s.rz;
    const HD ir = hd_inv(hd_sqrt(r2));
    const HD kep = s.GM * (ir * ir * ir);
    s.vx = s.vx + dt * (ajx + kep * s.rx);
    s.vy = s.vy + dt * (ajy + kep * s.ry);
    if constexpr (D3) s.vz = s.vz + dt * (ajz + kep * s.rz);
}

template <int NP, int L, bool D3>
__device__ __forceinline__ void kick_hd_any(LaneHD<NP>& s, double dt) {
    if constexpr (NP == 2)
        kick2_hd<L, D3>(s, dt);
    else
        kick_hd<NP, L, D3>(s, dt);
}

// kick2_hd's per-lane coefficients (after p, GM, m, iMi are set)
template <int NP>
__device__ __forceinline__ void lane_finish_hd(LaneHD<NP>& s) {
    if constexpr (NP == 2) {
        const bool p1 = s.p == 0;
        const HD q = s.GM * s.iMi[1];
        s.kA = p1 ? hd_c(0.0) : s.GM;
        s.kB = p1 ? -s.m[1] : -q;
        s.kC = p1 ? s.m[1] : -(q * s.m[0]);
        s.c12 = s.m[0] * s.iMi[1];
    }
}

// star barycentric x-velocity v0 = -sum_q (m_q / M_q) v'_q
template <int NP, int L>
__device__ __forceinline__ HD star_vx_hd(const LaneHD<NP>& s) {
    HD v = hd_c(0.0);
#pragma unroll
    for (int q = 0; q < NP; q++) v = v - s.mu[q] * grp_get_hd<L>(s.vx, q);
    return v;
}

// Pal (2009) -> heliocentric Cartesian (rvm_device.h pal_to_cart) with hyper-dual elements: the
// eccentric-longitude equation F - k sin F + h cos F = lambda is solved on the primal, then two
// hyper-dual Newton steps give F's derivatives.
__device__ __forceinline__ void pal_to_cart_hd(HD mu, HD a, HD lam, HD k, HD h, HD& X, HD& Y, HD& VX, HD& VY) {
    HD F = hd_c(pal_solve_F(lam.v, k.v, h.v));
#pragma unroll
    for (int it = 0; it < 2; it++) {
        const HD sF = hd_sin(F), cF = hd_cos(F);
        F = F - (F - k * sF + h * cF - lam) / (1.0 - k * cF - h * sF);
    }
    const HD sF = hd_sin(F), cF = hd_cos(F);
    const HD beta = hd_inv(1.0 + hd_sqrt(1.0 - h * h - k * k));
    const HD n = hd_sqrt(mu / (a * a * a));
    const HD r = a * (1.0 - k * cF - h * sF);
    const HD hkb = h * k * beta;
    const HD ahh = 1.0 - h * h * beta, akk = 1.0 - k * k * beta;
    X = a * (ahh * cF + hkb * sF - k);
    Y = a * (akk * sF + hkb * cF - h);
    const HD fac = n * a * a / r;
    VX = fac * (hkb * cF - ahh * sF);
    VY = fac * (akk * cF - hkb * sF);
}

// REBOUND Pal inclination (rvm_device.h pal_incline), hyper-dual
__device__ __forceinline__ void pal_incline_hd(HD ix, HD iy, HD& X, HD& Y, HD& Z, HD& VX, HD& VY, HD& VZ) {
    HD w2 = 4.0 - ix * ix - iy * iy;
    if (w2.v < 0.0) w2 = -w2;  // fabs, as the primal
    const HD W = hd_sqrt(w2);
    const HD axx = 1.0 - 0.5 * (iy * iy), axy = 0.5 * (ix * iy), ayy = 1.0 - 0.5 * (ix * ix);
    const HD x = X, y = Y, vx = VX, vy = VY;
    X = axx * x + axy * y;
    Y = axy * x + ayy * y;
    Z = 0.5 * (W * (ix * y - iy * x));
    VX = axx * vx + axy * vy;
    VY = axy * vx + ayy * vy;
    VZ = 0.5 * (W * (ix * vy - iy * vx));
}

}  // namespace rvm

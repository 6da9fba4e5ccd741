// rvm_device.h -- device-side building blocks of the gfx950 RV likelihood kernel.
//
// Physics restated from the reference's hot path:
//   * Pal (2009) elements -> heliocentric Cartesian about the star (REBOUND
//     sim.add(primary=star, m, a, h, k, l); state.py:41), G = 1, M_star = 1.
//   * Heliocentric -> Jacobi coordinates; the reference's move_to_com (state.py:45) is implied
//     (Jacobi coordinates are translation invariant and the star's barycentric velocity is
//     v0 = -sum_i (m_i / M_i) v'_i with V_cm = 0).
//   * Wisdom-Holman drift-kick-drift: Kepler drift of each Jacobi coordinate about the interior
//     mass M_i in universal variables (Danby's Stumpff functions, Halley iterations), interaction
//     kick from the pairwise forces minus the Kepler part.
//   * The encounter test of REBOUND's exit_min_distance (state.py:46) on every pair at every kick.
//
// Everything is fp64; one lane = one (walker, direction, extrapolation level).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rvm {

// ---- Stumpff functions c0..c3 (Danby): series for |z| <= 1, quartering+doubling otherwise ------
__device__ __forceinline__ void stumpff(double z, double& c0, double& c1, double& c2, double& c3) {
    // c2 = sum_j (-z)^j / (2j+2)!,  c3 = sum_j (-z)^j / (2j+3)!  (10 terms: error < z^10/22! )
    int n = 0;
    while (fabs(z) > 1.0 && n < 40) {  // rare: only for large steps / hyperbolic orbits
        z *= 0.25;
        n++;
    }
    const double i2[10] = {1.0 / 2.0,
                           1.0 / 24.0,
                           1.0 / 720.0,
                           1.0 / 40320.0,
                           1.0 / 3628800.0,
                           1.0 / 479001600.0,
                           1.0 / 87178291200.0,
                           1.0 / 20922789888000.0,
                           1.0 / 6402373705728000.0,
                           1.0 / 2432902008176640000.0};
    const double i3[10] = {1.0 / 6.0,
                           1.0 / 120.0,
                           1.0 / 5040.0,
                           1.0 / 362880.0,
                           1.0 / 39916800.0,
                           1.0 / 6227020800.0,
                           1.0 / 1307674368000.0,
                           1.0 / 355687428096000.0,
                           1.0 / 121645100408832000.0,
                           1.0 / 51090942171709440000.0};
    double a2 = i2[9], a3 = i3[9];
#pragma unroll
    for (int j = 8; j >= 0; j--) {
        a2 = i2[j] - z * a2;
        a3 = i3[j] - z * a3;
    }
    double C2 = a2, C3 = a3;
    double C1 = 1.0 - z * C3;
    double C0 = 1.0 - z * C2;
    for (; n > 0; n--) {
        C3 = (C2 + C0 * C3) * 0.25;
        C2 = C1 * C1 * 0.5;
        C1 = C0 * C1;
        C0 = 2.0 * C0 * C0 - 1.0;
    }
    c0 = C0;
    c1 = C1;
    c2 = C2;
    c3 = C3;
}

// ---- Pal (2009) -> heliocentric Cartesian (coplanar); REBOUND reb_tools_pal_to_particle -------
__device__ __forceinline__ void pal_to_cart(double mu, double a, double lam, double k, double h, double& X,
                                            double& Y, double& VX, double& VY) {
    // Newton from F = lam; a lane stops updating at its own convergence (as a scalar loop would),
    // so the result never depends on the other lanes of the wave.
    double F = lam;
    bool done = false;
    for (int it = 0; it < 100; it++) {
        double sF, cF;
        sincos(F, &sF, &cF);
        const double fF = F - k * sF + h * cF - lam;
        const double dF = 1.0 - k * cF - h * sF;
        const double step = fF / dF;
        const double Fn = F - step;
        const bool conv = !(fabs(step) > 1e-16 * (fabs(Fn) > 1.0 ? fabs(Fn) : 1.0));
        F = done ? F : Fn;
        done = done || conv;
        if (__all(done)) break;
    }
    double sF, cF;
    sincos(F, &sF, &cF);
    const double beta = 1.0 / (1.0 + sqrt(1.0 - h * h - k * k));
    const double n = sqrt(mu / (a * a * a));
    const double r = a * (1.0 - k * cF - h * sF);
    X = a * ((1.0 - h * h * beta) * cF + h * k * beta * sF - k);
    Y = a * ((1.0 - k * k * beta) * sF + h * k * beta * cF - h);
    const double fac = n * a * a / r;
    VX = fac * (h * k * beta * cF - (1.0 - h * h * beta) * sF);
    VY = fac * ((1.0 - k * k * beta) * cF - h * k * beta * sF);
}

// ---- the Jacobi-coordinate state of one lane ---------------------------------------------------
template <int NP>
struct Sys {
    double rx[NP], ry[NP], vx[NP], vy[NP];  // Jacobi coordinates of planets 1..NP
    double m[NP];                           // planet masses
    double Mi[NP + 1];                      // interior masses, Mi[0] = M_star = 1
    double dmin2;                           // (hill_factor * max r_Hill)^2
    int enc;                                // encounter flag
};

// Kepler drift of every Jacobi coordinate by dt, jointly (independent chains -> ILP).
template <int NP>
__device__ __forceinline__ void drift(Sys<NP>& s, double dt) {
    double r0[NP], eta[NP], beta[NP], zeta[NP], X[NP], GM[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) {
        GM[p] = s.Mi[p + 1];
        const double rr = s.rx[p] * s.rx[p] + s.ry[p] * s.ry[p];
        r0[p] = sqrt(rr);
        const double v2 = s.vx[p] * s.vx[p] + s.vy[p] * s.vy[p];
        eta[p] = s.rx[p] * s.vx[p] + s.ry[p] * s.vy[p];
        beta[p] = 2.0 * GM[p] / r0[p] - v2;
        zeta[p] = GM[p] - beta[p] * r0[p];
        X[p] = dt / r0[p] - dt * dt * eta[p] / (2.0 * r0[p] * r0[p] * r0[p]);
    }
    // Halley iterations; each (lane, planet) freezes at its own convergence so that results are
    // independent of the wave's other lanes (bit-reproducible across batch compositions).
    bool done[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) done[p] = false;
    for (int it = 0; it < 50; it++) {
        bool all = true;
#pragma unroll
        for (int p = 0; p < NP; p++) {
            double c0, c1, c2, c3;
            stumpff(beta[p] * X[p] * X[p], c0, c1, c2, c3);
            const double x = X[p];
            const double G1 = x * c1, G2 = x * x * c2, G3 = x * x * x * c3;
            const double f = r0[p] * G1 + eta[p] * G2 + GM[p] * G3 - dt;
            const double fp = r0[p] * c0 + eta[p] * G1 + GM[p] * G2;
            const double fpp = eta[p] * c0 + zeta[p] * G1;
            const double dX = f * fp / (fp * fp - 0.5 * f * fpp);
            const double Xn = x - dX;
            const bool conv = !(fabs(dX) > 2e-16 * fabs(Xn));
            X[p] = done[p] ? x : Xn;
            done[p] = done[p] || conv;
            all = all && done[p];
        }
        if (__all(all)) break;
    }
#pragma unroll
    for (int p = 0; p < NP; p++) {
        double c0, c1, c2, c3;
        const double x = X[p];
        stumpff(beta[p] * x * x, c0, c1, c2, c3);
        const double G1 = x * c1, G2 = x * x * c2, G3 = x * x * x * c3;
        const double rr = r0[p] * c0 + eta[p] * G1 + GM[p] * G2;
        const double f = 1.0 - GM[p] * G2 / r0[p];
        const double g = dt - GM[p] * G3;
        const double fd = -GM[p] * G1 / (rr * r0[p]);
        const double gd = 1.0 - GM[p] * G2 / rr;
        const double nrx = f * s.rx[p] + g * s.vx[p];
        const double nry = f * s.ry[p] + g * s.vy[p];
        const double nvx = fd * s.rx[p] + gd * s.vx[p];
        const double nvy = fd * s.ry[p] + gd * s.vy[p];
        s.rx[p] = nrx;
        s.ry[p] = nry;
        s.vx[p] = nvx;
        s.vy[p] = nvy;
    }
}

// Interaction kick by dt (and the encounter test on every pair at the kick positions).
template <int NP>
__device__ __forceinline__ void kick(Sys<NP>& s, double dt) {
    constexpr int NB = NP + 1;
    double x[NB], y[NB], ax[NB], ay[NB];
    x[0] = 0.0;
    y[0] = 0.0;
    double cmx = 0.0, cmy = 0.0;
#pragma unroll
    for (int i = 1; i < NB; i++) {
        x[i] = s.rx[i - 1] + cmx / s.Mi[i - 1];
        y[i] = s.ry[i - 1] + cmy / s.Mi[i - 1];
        cmx += s.m[i - 1] * x[i];
        cmy += s.m[i - 1] * y[i];
    }
#pragma unroll
    for (int i = 0; i < NB; i++) {
        ax[i] = 0.0;
        ay[i] = 0.0;
    }
    int enc = 0;
#pragma unroll
    for (int i = 0; i < NB; i++) {
#pragma unroll
        for (int j = i + 1; j < NB; j++) {
            const double dx = x[j] - x[i], dy = y[j] - y[i];
            const double r2 = dx * dx + dy * dy;
            enc |= (r2 < s.dmin2);
            const double ir3 = 1.0 / (r2 * sqrt(r2));
            const double mj = (j == 0) ? 1.0 : s.m[j - 1];
            const double mi = (i == 0) ? 1.0 : s.m[i - 1];
            ax[i] += mj * ir3 * dx;
            ay[i] += mj * ir3 * dy;
            ax[j] -= mi * ir3 * dx;
            ay[j] -= mi * ir3 * dy;
        }
    }
    s.enc |= enc;
    double max_ = ax[0], may_ = ay[0];  // M_star = 1
#pragma unroll
    for (int i = 1; i < NB; i++) {
        const double rx = s.rx[i - 1], ry = s.ry[i - 1];
        const double rj2 = rx * rx + ry * ry;
        const double kep = s.Mi[i] / (rj2 * sqrt(rj2));
        const double ajx = ax[i] - max_ / s.Mi[i - 1];
        const double ajy = ay[i] - may_ / s.Mi[i - 1];
        s.vx[i - 1] += dt * (ajx + kep * rx);
        s.vy[i - 1] += dt * (ajy + kep * ry);
        max_ += s.m[i - 1] * ax[i];
        may_ += s.m[i - 1] * ay[i];
    }
}

template <int NP>
__device__ __forceinline__ double star_vx(const Sys<NP>& s) {
    double v = 0.0;
#pragma unroll
    for (int p = 0; p < NP; p++) v -= (s.m[p] / s.Mi[p + 1]) * s.vx[p];
    return v;
}

// ---- Philox4x32-10 counter-based RNG -------------------------------------------------------------
struct u32x4 {
    uint32_t x, y, z, w;
};

__device__ __forceinline__ u32x4 philox(u32x4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c = u32x4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return c;
}

// two uniforms in the open interval (0, 1), 53-bit resolution
__device__ __forceinline__ void uniform2(uint64_t seed, uint64_t item, uint64_t iteration, uint32_t stream, double& u0,
                                         double& u1) {
    const u32x4 c{(uint32_t)item, (uint32_t)(item >> 32), (uint32_t)iteration,
                  (uint32_t)((iteration >> 32) & 0xFFFFu) | (stream << 16)};
    const u32x4 r = philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const uint64_t a = ((uint64_t)(r.x >> 5) << 26) | (uint64_t)(r.y >> 6);
    const uint64_t b = ((uint64_t)(r.z >> 5) << 26) | (uint64_t)(r.w >> 6);
    u0 = ((double)a + 0.5) * (1.0 / 9007199254740992.0);
    u1 = ((double)b + 0.5) * (1.0 / 9007199254740992.0);
}

}  // namespace rvm

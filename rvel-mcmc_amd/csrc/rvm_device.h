// rvm_device.h -- device-side building blocks of the gfx950 RV likelihood kernel.
//
// Physics restated from the reference's hot path:
//   * Pal (2009) elements -> heliocentric Cartesian about the star (REBOUND
//     sim.add(primary=star, m, a, h, k, l); state.py:41), G = 1, M_star = 1.
//   * Heliocentric -> Jacobi coordinates; the reference's move_to_com (state.py:45) is implied
//     (Jacobi coordinates are translation invariant and the star's barycentric velocity is
//     v0 = -sum_i (m_i / M_i) v'_i with V_cm = 0).
//   * Wisdom-Holman kick-drift-kick: Kepler drift of each Jacobi coordinate about the interior
//     mass M_i in universal variables (Danby's Stumpff functions, Halley iterations), interaction
//     kick from the pairwise forces minus the Kepler part.
//   * The encounter test of REBOUND's exit_min_distance (state.py:46) on every pair at every kick.
//
// Everything is fp64; one lane = one (walker, planet, direction, extrapolation level).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rvm {

// ---- fp64 reciprocal / reciprocal-sqrt: hardware estimate + one cubic refinement ----------------
// The compiler's IEEE division / sqrt expansions are ~10 dependent instructions each; the hot loop
// only needs faithfully rounded results.  v_rcp_f64 / v_rsq_f64 are good to ~5e-8 relative
// (measured, scripts/probe/rcp_precision.hip); one third-order correction
//   1/a    = r (1 + e + e^2),             e = 1 - a r
//   1/sqrt = y (1 + e/2 + 3 e^2 / 8),     e = 1 - a y^2
// leaves an error ~e^3 ~ 1e-22, i.e. the result is limited by rounding only.
__device__ __forceinline__ double rcp_nr(double x) {
    const double r = __builtin_amdgcn_rcp(x);
    const double e = fma(-x, r, 1.0);
    return fma(r, fma(e, e, e), r);
}

__device__ __forceinline__ double rsq_nr(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    const double e = fma(-x * y, y, 1.0);
    return fma(y, e * fma(0.375, e, 0.5), y);
}

// Wave-wide vote straight from the compare mask (s_cmp on the ballot, no VGPR round trip as
// with __any, whose int argument is materialised with v_cndmask and compared again).
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }
__device__ __forceinline__ uint64_t ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// a*b + k with k wave-uniform (an SGPR pair): a three-address v_fma_f64.  Plain fma() with a
// constant addend is selected as the two-address v_fmac_f64 plus a copy of the constant into the
// destination on every use; the hot polynomials below avoid that copy.
__device__ __forceinline__ double fma_sk(double a, double b, double k) {
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
}

// A constant materialised once into a VGPR (opaque to the compiler, so it is not re-materialised
// with a v_mov inside the loops that use it as the second operand of fma_sk).
__device__ __forceinline__ double vconst(double k) {
    double r;
    asm volatile("v_mov_b64 %0, %1" : "=v"(r) : "s"(k));
    return r;
}

// Loop-invariant VGPR constants of the hot path (set once per segment, vconsts_for<NT>).
struct VConsts {
    double k2, k3;      // top Horner coefficients of c2, c3 for the level's series length
    double k2_8, k3_8;  // the same for the 8-term series (second Halley steps)
    double c1875;       // 15/8 of rcube_nr
};

// x^(-3/2) straight from v_rsq_f64: with y = rsq(x), e = 1 - x y^2,
//   x^(-3/2) = y^3 (1 - e)^(-3/2) = y^3 (1 + 3e/2 + 15e^2/8 + O(e^3))      (|e| ~ 5e-8)
__device__ __forceinline__ double rcube_nr(double x, double c1875) {
    const double y = __builtin_amdgcn_rsq(x);
    const double y2 = y * y;
    const double y3 = y2 * y;
    const double e = fma(-x, y2, 1.0);
    return fma(y3, e * fma_sk(e, c1875, 1.5), y3);
}

__device__ __forceinline__ double rcube_nr(double x) { return rcube_nr(x, 1.875); }

// ---- Stumpff functions (Danby) ------------------------------------------------------------------
// c2 = sum_j (-z)^j / (2j+2)!,  c3 = sum_j (-z)^j / (2j+3)!;  c1 = 1 - z c3,  c0 = 1 - z c2.
//
// Hot path: c2, c3 by Horner in z with NT terms (one fma per term with the coefficient in an
// SGPR: no constant copies).  The truncation error is at most ~2e-17 relative (0.2 ulp, below the
// Horner evaluation's own rounding) for |z| <= B(NT):
//   NT = 6: B = 0.1 (z^6/14! <= 1.2e-17)   NT = 7: B = 0.3 (z^7/16! <= 1.1e-17)   NT = 8: B = 0.3 (z^8/18! <= 1e-20)
// The term count is chosen per extrapolation level (wave-uniform, see logl_kernel), and lanes
// with |z| > B(NT) redo the evaluation with stumpff_full, so a walker's result depends only on
// its own (z, level), never on the other lanes of the wave.
template <int NT>
__device__ __forceinline__ constexpr double stumpff_bound() {
    return NT >= 7 ? 0.3 : 0.1;
}

struct StumpffK {
    static constexpr double K2[9] = {1.0 / 2.0,         -1.0 / 24.0,           1.0 / 720.0,
                                     -1.0 / 40320.0,    1.0 / 3628800.0,       -1.0 / 479001600.0,
                                     1.0 / 87178291200.0, -1.0 / 20922789888000.0, 1.0 / 6402373705728000.0};
    static constexpr double K3[9] = {1.0 / 6.0,           -1.0 / 120.0,           1.0 / 5040.0,
                                     -1.0 / 362880.0,     1.0 / 39916800.0,       -1.0 / 6227020800.0,
                                     1.0 / 1307674368000.0, -1.0 / 355687428096000.0, 1.0 / 121645100408832000.0};
};

template <int NT>
__device__ __forceinline__ VConsts vconsts_for() {
    return VConsts{vconst(StumpffK::K2[NT - 1]), vconst(StumpffK::K3[NT - 1]), vconst(StumpffK::K2[7]),
                   vconst(StumpffK::K3[7]), vconst(1.875)};
}

// with the top coefficients k2 = K2[NT-1], k3 = K3[NT-1] already in VGPRs (vconsts_for<NT>)
template <int NT>
__device__ __forceinline__ void stumpff23(double z, double& c2, double& c3, double k2, double k3) {
    double a = fma_sk(z, k2, StumpffK::K2[NT - 2]), b = fma_sk(z, k3, StumpffK::K3[NT - 2]);
#pragma unroll
    for (int j = NT - 3; j >= 0; j--) {
        a = fma_sk(a, z, StumpffK::K2[j]);
        b = fma_sk(b, z, StumpffK::K3[j]);
    }
    c2 = a;
    c3 = b;
}

template <int NT>
__device__ __forceinline__ void stumpff23(double z, double& c2, double& c3) {
    constexpr double K2[9] = {1.0 / 2.0,         -1.0 / 24.0,           1.0 / 720.0,
                              -1.0 / 40320.0,    1.0 / 3628800.0,       -1.0 / 479001600.0,
                              1.0 / 87178291200.0, -1.0 / 20922789888000.0, 1.0 / 6402373705728000.0};
    constexpr double K3[9] = {1.0 / 6.0,           -1.0 / 120.0,           1.0 / 5040.0,
                              -1.0 / 362880.0,     1.0 / 39916800.0,       -1.0 / 6227020800.0,
                              1.0 / 1307674368000.0, -1.0 / 355687428096000.0, 1.0 / 121645100408832000.0};
    double a = fma_sk(z, K2[NT - 1], K2[NT - 2]), b = fma_sk(z, K3[NT - 1], K3[NT - 2]);
#pragma unroll
    for (int j = NT - 3; j >= 0; j--) {
        a = fma_sk(a, z, K2[j]);
        b = fma_sk(b, z, K3[j]);
    }
    c2 = a;
    c3 = b;
}

// Any |z|: quarter z until |z| <= 0.3, 8-term series, then the double-angle recurrences.
__device__ __forceinline__ void stumpff_full(double z, double& c0, double& c1, double& c2, double& c3) {
    int n = 0;
    while (fabs(z) > 0.3 && n < 40) {  // rare: only for large steps / hyperbolic orbits
        z *= 0.25;
        n++;
    }
    double C2, C3;
    stumpff23<8>(z, C2, C3);
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
// Eccentric longitude F from lam = F - k sin F + h cos F: Newton from F = lam, at most 100 steps,
// stop once |step| <= 1e-16 max(|F|, 1) (the reference's loop).  A lane stops updating at its own
// convergence (as a scalar loop would), so the result never depends on the other lanes of the wave.
// Many walkers never meet that test: at roundoff the iteration settles into a 2-cycle between two
// neighbouring doubles whose steps both exceed the bound, and the scalar loop runs all 100
// iterations (~1000 cycles each; one such lane held its whole workgroup at the schedule barrier
// for up to 50 us, timing build).  The map is deterministic, so once F_{i+1} == F_{i-1} with
// neither step converged the sequence alternates for good, and the lane takes at once the iterate
// the 100-step loop ends on: the same bits, without the remaining iterations.
__device__ __forceinline__ double pal_solve_F(double lam, double k, double h) {
    double F = lam, Fp = __builtin_nan("");  // Fp: the iterate before F
    bool done = false;
    for (int it = 0; it < 100; it++) {
        double sF, cF;
        sincos(F, &sF, &cF);
        const double fF = F - k * sF + h * cF - lam;
        const double dF = 1.0 - k * cF - h * sF;
        const double step = fF / dF;
        const double Fn = F - step;
        const bool conv = !(fabs(step) > 1e-16 * (fabs(Fn) > 1.0 ? fabs(Fn) : 1.0));
        const bool cyc = !conv && Fn == Fp;
        const double Fc = ((99 - it) & 1) == 0 ? Fn : F;  // iterate 100 of the 2-cycle
        if (!done) {
            Fp = F;
            F = cyc ? Fc : Fn;
        }
        done = done || conv || cyc;
        if (__all(done)) break;
    }
    return F;
}

__device__ __forceinline__ void pal_to_cart(double mu, double a, double lam, double k, double h, double& X,
                                            double& Y, double& VX, double& VY) {
    const double F = pal_solve_F(lam, k, h);
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

// Inclined orbits (REBOUND's Pal coordinates ix, iy): rotate the orbital plane,
//   x' = (1 - iy^2/2) X + (ix iy/2) Y,  y' = (ix iy/2) X + (1 - ix^2/2) Y,
//   z' = (sqrt(4 - ix^2 - iy^2)/2) (ix Y - iy X)       (same for the velocity)
__device__ __forceinline__ void pal_incline(double ix, double iy, double& X, double& Y, double& Z, double& VX,
                                            double& VY, double& VZ) {
    const double W = sqrt(fabs(4.0 - ix * ix - iy * iy));
    const double axx = 1.0 - 0.5 * iy * iy, axy = 0.5 * ix * iy, ayy = 1.0 - 0.5 * ix * ix;
    const double x = X, y = Y, vx = VX, vy = VY;
    X = axx * x + axy * y;
    Y = axy * x + ayy * y;
    Z = 0.5 * W * (ix * y - iy * x);
    VX = axx * vx + axy * vy;
    VY = axy * vx + ayy * vy;
    VZ = 0.5 * W * (ix * vy - iy * vx);
}

// ---- lane layout: the planets of one walker live on L adjacent lanes ----------------------------
// L = lanes per walker (1, 2 or 4): planet p of a walker runs on lane (group base + p), so every
// Kepler drift runs on its own lane and the kick exchanges positions inside the lane group with
// DPP quad permutes (no LDS).  NP = 3 uses L = 4 with the 4th lane shadowing planet 3.
template <int NP>
struct LanesPerWalker {
    static constexpr int value = NP == 1 ? 1 : (NP == 2 ? 2 : 4);
};

// value of `v` held by lane Q of this lane's group (Q is a compile-time planet index)
template <int L, int Q>
__device__ __forceinline__ double grp_get(double v) {
    if constexpr (L == 1) {
        return v;
    } else {
        // quad_perm selects: L = 2 groups are lanes {0,1} and {2,3} of each quad, L = 4 the quad
        constexpr int q = Q % L;
        constexpr int ctrl = (L == 2) ? (q | (q << 2) | ((q + 2) << 4) | ((q + 2) << 6))
                                      : (q | (q << 2) | (q << 4) | (q << 6));
        const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), ctrl, 0xF, 0xF, false);
        const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), ctrl, 0xF, 0xF, false);
        return __hiloint2double(hi, lo);
    }
}

// runtime planet index (folds to a constant inside unrolled loops)
template <int L>
__device__ __forceinline__ double grp_get(double v, int q) {
    switch (q) {
        case 0:
            return grp_get<L, 0>(v);
        case 1:
            return grp_get<L, 1>(v);
        case 2:
            return grp_get<L, 2>(v);
        default:
            return grp_get<L, 3>(v);
    }
}

// Body pairs (a, b), a < b, of the closed-form kick for NP >= 3: all but (0, 1), whose term
// cancels the own Kepler term on planet 1's lane and vanishes on every other lane (kickN).
template <int NP>
struct KickPairs {
    static constexpr int n = NP >= 3 ? (NP + 1) * NP / 2 - 1 : 1;
};

// One lane: one planet's Jacobi coordinate plus the walker-wide constants every lane needs.
template <int NP>
struct Lane {
    double rx, ry, vx, vy;  // own Jacobi coordinate
    double rz, vz;          // out-of-plane components (inclined systems, D3 = true; else unused)
    double r, ir;           // |r'| and 1/|r'| at the current positions (carried from the drift)
    double GM, GM2;         // interior mass M_p (G = 1) of the own Jacobi coordinate, and 2 M_p
    double m[NP];           // planet masses
    double iMi[NP + 1];     // 1 / interior masses, iMi[0] = 1 (M_star = 1)
    double mu[NP];          // m_q / M_q: star barycentric velocity weights
    double dmin2, idmin2;   // (hill_factor * max r_Hill)^2 and its reciprocal
    double kA, kB, kC;      // closed-form 2-planet kick coefficients of the own lane (kick2)
    double kAh, kBh, kCh;   // the same times the current step (lane_set_step)
    double h;               // the current step (lane_set_step; kick_apply of NP != 2)
    double pair_s;          // kickN (3 planets): -0.0 / -1.0 selects the lane's round-0 pair
    double oA, oB;          // kick2: own pair vector o = oA r'_own + oB r'_other
    double kP1, kP2, kP3, kP4;      // kick2: own/other coefficients of the own velocity update
    double kP1h, kP2h, kP3h, kP4h;  // the same times the current step
    double kP[KickPairs<NP>::n];   // NP >= 3 (kickN): own-lane coefficient of every pair but (0,1)
    double kPh[KickPairs<NP>::n];  // the same times the current step
    int p;                  // own planet index (lane % L, clamped to NP-1)
    int q;                  // lane index within the walker's group (lane % L, not clamped)
    uint64_t encm;          // wave mask of lanes that saw a pair closer than the exit distance
                            // (SGPRs: the kick's compares go straight into it; identical bits on
                            // all lanes of a walker's group)
};

// Step-scaled kick coefficients: call whenever the step size changes (once per segment).
template <int NP>
__device__ __forceinline__ void lane_set_step(Lane<NP>& s, double h) {
    s.h = h;
    s.kAh = s.kA * h;
    s.kBh = s.kB * h;
    s.kCh = s.kC * h;
    if constexpr (NP == 2) {
        s.kP1h = s.kP1 * h;
        s.kP2h = s.kP2 * h;
        s.kP3h = s.kP3 * h;
        s.kP4h = s.kP4 * h;
    }
    if constexpr (NP >= 3) {
#pragma unroll
        for (int k = 0; k < KickPairs<NP>::n; k++) s.kPh[k] = s.kP[k] * h;
    }
}

// Derived per-lane constants (after p, GM, m, iMi, dmin2 are set).
template <int NP>
__device__ __forceinline__ void lane_finish(Lane<NP>& s) {
    s.GM2 = 2.0 * s.GM;
    s.idmin2 = 1.0 / s.dmin2;  // +inf for dmin2 = 0 (no exit distance)
    if constexpr (NP == 2) {
        // (kick2 tests |r'| < dmin, the star -- planet-1 distance, on planet 1's lanes only: +inf on
        // planet 2's makes the test false there without masking its ballot)
        if (s.p != 0) s.idmin2 = __builtin_inf();
        // kick2: lane of planet 1: (A, B, C) = (0, -m2, m2); planet 2: (M2, -M2/M1, -m1 M2/M1)
        const bool p1 = s.p == 0;
        const double q = s.GM * s.iMi[1];
        s.kA = p1 ? 0.0 : s.GM;
        s.kB = p1 ? -s.m[1] : -q;
        s.kC = p1 ? s.m[1] : -q * s.m[0];
        s.pair_s = p1 ? -0.0 : -1.0;
        // kick2 in own/other form: with c = m1/M1, x2 = r'_2 + c r'_1 and d12 = x2 - r'_1,
        //   planet 1's lane (own = r'_1): x2 = c own + oth,  d12 = (c - 1) own + oth, own pair x2
        //   planet 2's lane (own = r'_2): x2 = own + c oth,  d12 = own + (c - 1) oth, own pair d12
        // so v += A r' + B x2 / r02^3 + C d12 / r12^3 = (A + P1 ic_own + P2 ic_oth) own
        //                                              + (P3 ic_own + P4 ic_oth) oth
        const double c = s.m[0] * s.iMi[1], c1 = c - 1.0;
        s.oA = p1 ? c : 1.0;
        s.oB = p1 ? 1.0 : c1;
        s.kP1 = p1 ? s.kB * c : s.kC;
        s.kP2 = p1 ? s.kC * c1 : s.kB;
        s.kP3 = p1 ? s.kB : s.kC * c1;
        s.kP4 = p1 ? s.kC : s.kB * c;
    } else {
        // kickN, 3 planets: round-0 pair of group lane q is (q >> 1, 2 + (q & 1)) in body indices:
        // -0.0 for the star pairs (0,2), (0,3), -1.0 for (1,2), (1,3)
        s.pair_s = (NP == 3 && s.q >= 2) ? -1.0 : -0.0;
        s.kB = s.kC = 0.0;
        s.kA = 0.0;
#pragma unroll
        for (int k = 0; k < KickPairs<NP>::n; k++) s.kP[k] = 0.0;
        if constexpr (NP >= 3) {
            // kickN: Jacobi acceleration of coordinate i = p + 1 (bodies 0..NP, m_0 = M_star = 1)
            //   a'_i = sum_{j != i} m_j d_ij / r_ij^3 - (1/M_{i-1}) sum_{a < i <= b} m_a m_b d_ab / r_ab^3
            // so pair (a, b) enters with c_ab = [a = i] m_b - [b = i] m_a - [a < i <= b] m_a m_b / M_{i-1},
            // and the own Kepler term M_i r'_i / |r'_i|^3 is added back for i >= 2 (for i = 1 it
            // cancels c_01 exactly; c_01 = 0 on every other lane).
            const int i = s.p + 1;
            s.kA = i == 1 ? 0.0 : s.GM;
            double iMprev = 0.0;  // 1 / M_{i-1}, summed rather than indexed (no runtime array index)
#pragma unroll
            for (int q = 0; q < NP; q++) iMprev += s.p == q ? s.iMi[q] : 0.0;
            int k = 0;
#pragma unroll
            for (int a = 0; a <= NP; a++) {
#pragma unroll
                for (int b = a + 1; b <= NP; b++) {
                    if (a == 0 && b == 1) continue;
                    const double ma = a == 0 ? 1.0 : s.m[a - 1], mb = s.m[b - 1];
                    double c = 0.0;
                    if (a == i) c += mb;
                    if (b == i) c -= ma;
                    if (a < i && i <= b) c -= ma * mb * iMprev;
                    s.kP[k++] = c;
                }
            }
        }
    }
    lane_set_step(s, 0.0);
}

// Safeguarded universal-Kepler solve for the rare hard cases (a step spanning a large part of an
// orbit, a poor initial guess): f(X) = r0 G1 + eta0 G2 + GM G3 - dt is increasing in X (f' = r > 0)
// with f(0) = -dt, so the root is bracketed by doubling from dt/r0 and Halley steps that leave
// the bracket are replaced by bisection.  Returns the G-functions at the converged X.
__device__ __forceinline__ void kepler_safe(double r0, double eta, double zeta, double beta, double GM, double dt,
                                         double& Xo, double& G0, double& G1, double& G2, double& G3) {
    const double sgn = dt >= 0.0 ? 1.0 : -1.0;
    double lo = 0.0, hi = dt / r0;
    double c0, c1, c2, c3;
    for (int i = 0; i < 200; i++) {  // expand until sgn*f(hi) > 0
        stumpff_full(beta * hi * hi, c0, c1, c2, c3);
        const double f = r0 * hi * c1 + eta * hi * hi * c2 + GM * hi * hi * hi * c3 - dt;
        if (sgn * f > 0.0 || !(f == f)) break;
        lo = hi;
        hi *= 2.0;
    }
    double X = 0.5 * (lo + hi);
    for (int i = 0; i < 200; i++) {
        stumpff_full(beta * X * X, c0, c1, c2, c3);
        const double g1 = X * c1, g2 = X * X * c2, g3 = X * X * X * c3;
        const double f = r0 * g1 + eta * g2 + GM * g3 - dt;
        const double fp = r0 * c0 + eta * g1 + GM * g2;
        const double fpp = eta * c0 + zeta * g1;
        if (sgn * f > 0.0)
            hi = X;
        else
            lo = X;
        double Xn = X - f * fp / (fp * fp - 0.5 * f * fpp);
        if (!(sgn * (Xn - lo) > 0.0 && sgn * (hi - Xn) > 0.0)) Xn = 0.5 * (lo + hi);
        const bool conv = !(fabs(Xn - X) > 2e-16 * fabs(Xn)) || lo == hi;
        X = Xn;
        if (conv) break;
    }
    stumpff_full(beta * X * X, c0, c1, c2, c3);
    Xo = X;
    G0 = c0;
    G1 = X * c1;
    G2 = X * X * c2;
    G3 = X * X * X * c3;
}

// One Halley step for the universal Kepler equation f(X) = r0 G1 + eta0 G2 + GM G3 - dt at X = x
// with the NT-term Stumpff series: returns the G-functions at x, f'(x), f''(x), the correction q
// (X_new = x - q), z = beta x^2 and x^3.  Valid only for |z| <= stumpff_bound<NT>() (the caller
// sends other lanes to the general solver).
template <int NT>
__device__ __forceinline__ void halley(double x, double beta, double r0, double eta, double zeta, double GM,
                                       double dt, double& G0, double& G1, double& G2, double& G3, double& fp,
                                       double& fpp, double& q, double& z, double& x3, double k2v, double k3v,
                                       double& f) {
    const double x2 = x * x;
    z = beta * x2;
    x3 = x2 * x;
    double c2, c3;
    stumpff23<NT>(z, c2, c3, k2v, k3v);
    G3 = x3 * c3;
    G2 = x2 * c2;
    G1 = fma(-beta, G3, x);  // x c1 = x (1 - z c3)
    G0 = fma(-z, c2, 1.0);
    f = fma(GM, G3, fma(eta, G2, fma(r0, G1, -dt)));
    fp = fma(zeta, G2, fma(eta, G1, r0));  // r0 G0 + eta G1 + GM G2 with G0 = 1 - beta G2
    fpp = fma(zeta, G1, eta * G0);
    const double den = fma(-0.5 * f, fpp, fp * fp);
    const double num = f * fp;
    // num/den: v_rcp_f64 (~5e-8) + one residual correction (error ~2e-15 of the correction)
    const double rd = __builtin_amdgcn_rcp(den);
    const double q0 = num * rd;
    q = fma(rd, fma(-den, q0, num), q0);
}

// Acceptance of a Halley step with relative correction qt = q/x: the error left in X is
// ~ c z qt^3 (c << 1; Halley is cubic and its constant scales with z = beta x^2), and the Taylor
// update of the G-functions over the correction (drift_apply) truncates at ~ z qt^3 / 3 relative.
// With |z| <= B(NT) (checked separately) the cheap form used on the hot path, |q| <= tol |x| with
//   NT = 6: 9.0e-6   NT = 7: 6.2e-6   NT = 8: 4.6e-6,
// keeps |q^3 z| <= 7.3e-17 |x^3|: both truncations stay below ~2.5e-17 relative (a quarter ulp).
// At the default steps (P/32 .. P/56) and e <~ 0.25 the finest levels pass after one step.
template <int NT>
__device__ __forceinline__ constexpr double halley_tol() {
    return NT >= 8 ? 4.6e-6 : (NT == 7 ? 6.2e-6 : 9.0e-6);
}

template <int NT>
__device__ __forceinline__ bool halley_ok(double q, double x) {
    // (false for a NaN correction: a Halley step from a guess far outside the series' range can
    // give one, and the lane must then take the general solver -- found when a walker near a
    // parabolic pericentre came out NONFINITE where the oracle's solver reports the encounter)
    return fabs(q) <= halley_tol<NT>() * fabs(x);
}

// general form (any z) for the rare solver (false for NaN: the bracketed solve takes over)
__device__ __forceinline__ bool halley_done(double q, double z, double x3) {
    return fabs((q * q) * (q * z)) <= 3e-17 * fabs(x3);
}

// Universal-Kepler solve for the rare lanes: Halley with the full Stumpff evaluation (any z)
// from the best estimate, then the bracketed solve for large steps or no convergence.  Returns
// the G-functions, f', f'' at the last evaluation point and the final correction Q (X = x - Q).
__device__ __forceinline__ void kepler_rare(double r0, double eta, double zeta, double beta, double GM, double dt,
                                         double xi, bool hard, double& G0, double& G1, double& G2, double& G3,
                                         double& fp, double& fpp, double& Q) {
    bool done = false;
    double X = xi;
    if (!hard) {
        for (int it = 0; it < 8 && !done; it++) {
            double c0, c1, cc2, cc3;
            const double zi = beta * X * X;
            stumpff_full(zi, c0, c1, cc2, cc3);
            const double g1 = X * c1, g2 = X * X * cc2, g3 = X * X * X * cc3;
            const double ff = r0 * g1 + eta * g2 + GM * g3 - dt;
            const double ffp = r0 * c0 + eta * g1 + GM * g2;
            const double ffpp = eta * c0 + zeta * g1;
            const double dX = ff * ffp / (ffp * ffp - 0.5 * ff * ffpp);
            G0 = c0;
            G1 = g1;
            G2 = g2;
            G3 = g3;
            fp = ffp;
            fpp = ffpp;
            Q = dX;
            done = halley_done(dX, zi, X * X * X);
            X = X - dX;
        }
    }
    if (hard || !done) {
        kepler_safe(r0, eta, zeta, beta, GM, dt, X, G0, G1, G2, G3);
        fp = r0 * G0 + eta * G1 + GM * G2;
        fpp = eta * G0 + zeta * G1;
        Q = 0.0;
    }
}

// New position/velocity from the G-functions at the last evaluation point and the final Halley
// correction Q (Taylor update of G1..G3 and of r = f' from there to X = x - Q), Gauss f and g.
struct DriftOut {
    double rx, ry, vx, vy, rz, vz, r, ir;
};

template <bool D3, int NP>
__device__ __forceinline__ DriftOut drift_apply(const Lane<NP>& s, double dt, double beta, double eta, double zeta,
                                                double G0, double G1, double G2, double G3, double fp, double fpp,
                                                double Q) {
    const double GM = s.GM, ir0 = s.ir;
    const double d = -Q, d2 = (0.5 * Q) * Q;
    const double H1 = fma(d, G0, fma(-d2 * beta, G1, G1));
    const double H2 = fma(d2, G0, fma(d, G1, G2));
    const double H3 = fma(d2 * d * (1.0 / 3.0), G0, fma(d2, G1, fma(d, G2, G3)));
    const double f3 = fma(zeta, G0, -(beta * eta) * G1);  // third derivative of f
    const double rr = fma(d2, f3, fma(d, fpp, fp));
    const double irr = rcp_nr(rr);
    const double gG2 = GM * H2;
    const double f_ = fma(-gG2, ir0, 1.0);
    const double g_ = fma(-GM, H3, dt);
    const double fd = -((GM * ir0) * H1) * irr;  // GM ir0: shared with the drift's guess
    const double gd = fma(-gG2, irr, 1.0);
    DriftOut o;
    o.rx = fma(f_, s.rx, g_ * s.vx);
    o.ry = fma(f_, s.ry, g_ * s.vy);
    o.vx = fma(fd, s.rx, gd * s.vx);
    o.vy = fma(fd, s.ry, gd * s.vy);
    if constexpr (D3) {
        o.rz = fma(f_, s.rz, g_ * s.vz);
        o.vz = fma(fd, s.rz, gd * s.vz);
    }
    o.r = rr;
    o.ir = irr;
    return o;
}

#ifdef RVM_PROFILE
// timing build only (counted with -DRVM_PROFILE_FAILS): why first Halley steps fail, per series length (NT 6/7/8 -> rows 0/1/2):
// [drifts (lanes), |z| > B, z fine but Halley not accepted]; read with rvm_prof_fail_copy
// row 3: [wave-steps taking the second Halley step, wave-steps entering kepler_rare, lanes in it]
static __device__ unsigned long long rvm_fail[4][3];
__device__ __forceinline__ void rare_count(int k, uint64_t mask) {
    if ((threadIdx.x & 63) == (int)__builtin_ctzll(ballot(true)))
        atomicAdd(&rvm_fail[3][k], k == 2 ? (unsigned long long)__builtin_popcountll(mask) : 1ull);
}
__device__ __forceinline__ void drift_fail_count(int nt, bool zok, bool hok) {
    const uint64_t all = ballot(true), zb = ballot(!zok), hb = ballot(zok && !hok);
    if ((threadIdx.x & 63) == (int)__builtin_ctzll(all)) {
        const int row = nt <= 6 ? 0 : (nt == 7 ? 1 : 2);
        atomicAdd(&rvm_fail[row][0], (unsigned long long)__builtin_popcountll(all));
        if (zb) atomicAdd(&rvm_fail[row][1], (unsigned long long)__builtin_popcountll(zb));
        if (hb) atomicAdd(&rvm_fail[row][2], (unsigned long long)__builtin_popcountll(hb));
    }
}
#endif

// Kepler drift of the own Jacobi coordinate by dt in universal variables (Danby): solve
// r0 G1 + eta0 G2 + GM G3 = dt for X by Halley steps from the fourth-order Taylor guess
//   X = u (1 - u s/2 + u^2 T3 + u^3 T4),   u = dt/r0, s = eta0/r0, g = GM/r0,
//   T3 = s^2/2 + (beta - g)/6,  T4 = s (5g/12 - 3 beta/8 - 5 s^2/8)
// (series inversion of dt = r0 X + eta0 X^2/2 + zeta X^3/6 - beta eta0 X^4/24 + ...), accepted by
// halley_ok.  A lane's step is "good" when one Halley step with the NT-term series is accepted.
//
// GATED = true: the wave votes on the good flags and lanes that are not good redo the solve with
//   kepler_rare (a second short-series Halley step first on the coarse levels, NT >= 7).  Each
//   lane at its own convergence, so results never depend on the other lanes of the wave.
// GATED = false: no vote -- the vote is a VALU->SALU->branch round trip that costs ~100 cycles of
//   a ~660-cycle step on one wave -- the result is only valid for good lanes and `bad` collects
//   the others; the caller (segment<> in rvm_logl.hip) re-runs the whole segment gated when any
//   lane was not good.  Good lanes compute bit-identical states either way.
// No square root anywhere in the step.
// Whether the lane's walker has already seen a pair inside the exit distance (Lane::encm; the
// walker's bits relative to its first lane as kick_enc_bits): its result is ENCOUNTER whatever it
// integrates next -- the reference stops there (exit_min_distance raises, state.py:36-47) -- so its
// drifts no longer send the wave to the second Halley step or the general solver (an encountered
// crossing orbit took them at every pericentre to the end of the span: the steady state's slowest
// waves).  Only that lane's own, discarded values change.
template <int NP>
__device__ __forceinline__ bool lane_encountered(const Lane<NP>& s) {
    constexpr int L = LanesPerWalker<NP>::value;
    constexpr uint64_t bits = NP == 2 ? 3ull : (NP == 3 ? 0xFull : 1ull);  // kick_enc_bits
    const int base = (int)(threadIdx.x & 63) & ~(L - 1);
    return ((s.encm >> base) & bits) != 0;
}

// The same as a wave mask (scalar work on Lane::encm): every lane of a walker whose kick_enc_bits
// hold an encounter -- lane i is set exactly where lane_encountered is true on lane i
template <int NP>
__device__ __forceinline__ uint64_t encountered_lanes(uint64_t m) {
    constexpr int L = LanesPerWalker<NP>::value;
    if constexpr (L == 1) {
        return m;
    } else if constexpr (L == 2) {
        const uint64_t t = (m | (m >> 1)) & 0x5555555555555555ull;  // (bits 3: either lane of the pair)
        return t | (t << 1);
    } else {
        const uint64_t t = (NP == 3 ? (m | (m >> 1) | (m >> 2) | (m >> 3)) : m) & 0x1111111111111111ull;
        return t | (t << 1) | (t << 2) | (t << 3);
    }
}

// The wave's vote on the first Halley step (drift below) takes the failing lanes' mask and, only when
// it is not empty, removes the lanes of walkers that have met an encounter (their values are
// discarded, so their solves must not send the wave to the second step): ok1 = the lane is not in
// the result, exactly as ok1 = !bad1 || lane_encountered(s).  Round 6: the per-lane
// lane_encountered test took 3 VALU and 3 SALU of every gated step (~5 % of a lone wave's step).

// G5: one more term of the guess's series, X = u (1 - us/2 + u^2 T3 + u^3 T4 + u^4 T5),
//   T5 = (9 beta^2 - 19 beta g + 90 beta s^2 + 10 g^2 - 105 g s^2 + 105 s^4) / 120
// (series reversion of u = G1 + s G2 + g G3 to fifth order; scripts/kepler_guess_series.py): ~9 VALU
// more per drift, and the first Halley step is accepted far more often on eccentric orbits near
// pericentre, where the wave otherwise takes the second step (~250 cycles on a lone wave:
// scripts/probe/seg_bench.hip, profiles/r05g_seg_bench_g5.txt).  Off in every shipped kernel: the
// ~55 cycles it adds to every other step outweigh that at the steps the passes take
// (rvm_refine.hip RVM_REFINE_G5, rvm_logl.hip RVM_MAIN_G5).
// KG, the guess: 0 fourth order, 1 fifth order (G5).  (A per-lane choice -- G5 on a lane's step after
// one whose first Halley test failed -- cost more than either: 935 against 863 / 697 cycles per step
// at e = 0.55, 689 against 620 / 680 at e = 0.22; profiles/r05o_seg_bench.txt)
//
// ACC (gated drift only): what a lane whose first Halley step fails the cheap test gets.
//   0: a second Halley step with the 8-term series, then kepler_rare (rounds 1-5).
//   1: first the z-aware form of the acceptance the cheap test's constant derives from,
//      |q|^3 |z| <= 7.3e-17 |x|^3 (at the passes' fine steps z is far below the series bound, and
//      the constant tolerance rejects corrections the error bound accepts); then as 0.
//      Then a lane still failing with |q| <= 1e-4 |x| takes a Newton step at X1 = x - q from the
//      Taylor expansion of the Kepler function about x (f^(4) = -beta f'', so no new series), and
//      the third-order terms of the Taylor update fold into drift_apply's inputs; else as 0.
//   2: the same as 1.
//   3: ACC 0's solve with the vote after the update (the late vote): the same bits as 0.
//   4: ACC 1's solve with the late vote.
//   (steady-state walkers at a pass's finest step, P/112: 12 % of wave-steps fail the cheap test,
//   6.8 % the z-aware one, and 80 % of the lanes failing that pass the 1e-4 bound --
//   scripts/probe/kepler_accept_probe.hip, profiles/r06a_kepler_accept_probe.jsonl)
template <int NT, bool GATED, bool D3 = false, int NP, int KG = 0, int ACC = 0>
__device__ __forceinline__ void drift(Lane<NP>& s, double dt, bool& bad, const VConsts& vk) {
    const double GM = s.GM, r0 = s.r, ir0 = s.ir;
    double v2 = fma(s.vx, s.vx, s.vy * s.vy);
    double eta = fma(s.rx, s.vx, s.ry * s.vy);
    if constexpr (D3) {
        v2 = fma(s.vz, s.vz, v2);
        eta = fma(s.rz, s.vz, eta);
    }
    const double beta = fma(s.GM2, ir0, -v2);
    const double zeta = fma(-beta, r0, GM);
    const double u = dt * ir0, sg = eta * ir0, g = GM * ir0;
    const double hs = 0.5 * sg;
    const double T3 = fma(hs, sg, (beta - g) * (1.0 / 6.0));
    const double T4 = sg * fma(-0.625 * sg, sg, fma(5.0 / 12.0, g, -0.375 * beta));
    auto guess5 = [&]() {
        const double s2 = sg * sg;
        const double T5 = fma(beta, fma(9.0 / 120.0, beta, fma(-19.0 / 120.0, g, 0.75 * s2)),
                              fma(g, fma(1.0 / 12.0, g, -0.875 * s2), 0.875 * (s2 * s2)));
        return u * fma(u, fma(u, fma(u, fma(u, T5, T4), T3), -hs), 1.0);
    };
    double x;
    if constexpr (KG == 1) {
        x = guess5();
    } else {
        x = u * fma(u, fma(u, fma(u, T4, T3), -hs), 1.0);
    }
    double G0, G1, G2, G3, fp, fpp, Q, z, x3, f0;
    halley<NT>(x, beta, r0, eta, zeta, GM, dt, G0, G1, G2, G3, fp, fpp, Q, z, x3, vk.k2, vk.k3, f0);
    constexpr double B = stumpff_bound<NT>();
#ifdef RVM_PROFILE_FAILS
    drift_fail_count(NT, fabs(z) <= B, halley_ok<NT>(Q, x));
#endif
    // A step spanning a large part of an orbit (|beta| (dt/r0)^2 > 0.5) that passes these tests has
    // converged all the same; only kepler_rare treats such steps separately (bracketed solver).
    // The lanes whose first Halley step failed (ok1 false) get a better solve here; every lane of the
    // wave calls it (it votes).  ZT: first the z-aware acceptance and the Taylor second step (ACC 2).
    auto second_chance = [&](bool ok1, const bool ZT) __attribute__((always_inline)) {
        bool ok = ok1;
        if (ZT) {
            const bool zok = fabs(z) <= B;
            ok = ok || (zok && fabs((Q * Q) * (Q * z)) <= 7.3e-17 * fabs(x3));
            if (!ok && zok && fabs(Q) <= 1e-4 * fabs(x)) {
                // derivatives of f at x: f3 = zeta G0 - beta eta G1, f4 = -beta f'' (d/dX G0 = -beta G1)
                const double f3 = fma(zeta, G0, -(beta * eta) * G1);
                const double f4 = -beta * fpp;
                const double d = -Q;
                const double F = fma(d, fma(d, fma(d, fma(d, f4 * (1.0 / 24.0), f3 * (1.0 / 6.0)), 0.5 * fpp), fp), f0);
                const double F1 = fma(d, fma(d, fma(d, f4 * (1.0 / 6.0), 0.5 * f3), fpp), fp);
                const double q2 = F * rcp_nr(F1);
                if (fabs(q2) <= 1e-8 * fabs(x)) {
                    // X = x - Qt: the update's third-order terms folded into drift_apply's inputs
                    const double Qt = Q + q2;
                    const double c = ((Qt * Qt) * Qt) * (1.0 / 6.0) * beta;
                    const double g0 = G0, g1 = G1;
                    G1 = fma(c, g0, G1);
                    G2 = fma(c, g1, G2);
                    fp = fma(c, fpp, fp);
                    Q = Qt;
                    ok = true;
                }
            }
        }
        // a second Halley step with the 8-term series (|z| <= 0.3) for the lanes that need it:
        // pericentre passages on the coarse levels, and walkers whose periods are much shorter
        // than the plan's period hint on any level
        constexpr double B8 = stumpff_bound<8>();
        double xe = x;
        if (!ok) {
            const double X1 = x - Q;
            if (fabs(beta * X1 * X1) <= B8) {
                xe = X1;
                double fu;
                halley<8>(xe, beta, r0, eta, zeta, GM, dt, G0, G1, G2, G3, fp, fpp, Q, z, x3, vk.k2_8, vk.k3_8, fu);
                ok = fabs(z) <= B8 && halley_ok<8>(Q, xe);
            }
        }
        if (__builtin_expect(ballot(!ok) != 0, 0)) {
#ifdef RVM_PROFILE_FAILS
            rare_count(1, 0);
            rare_count(2, ballot(!ok));
#endif
            if (!ok) {
                const bool hard = fabs(beta) * (u * u) > 0.5;
                const double start = xe - Q;
                kepler_rare(r0, eta, zeta, beta, GM, dt, isfinite(start) && xe != x ? start : x, hard, G0, G1, G2,
                            G3, fp, fpp, Q);
            }
        }
    };
    DriftOut o;
    if constexpr (GATED && ACC >= 3) {
        // late vote: the update from the first Halley step for every lane, and the wave's vote only
        // after it -- the vote's compare then waits on nothing, and the branch is not taken on a
        // clean step (the early vote drained the lone wave's pipeline at the end of the Halley chain:
        // ~125 cycles per step).  A failing lane's update is recomputed.  ACC 3 gives exactly
        // ACC 0's bits.
        // (a ballot per compare: each is the compare's own mask, where the ballot of their OR was
        // materialised as a lane value and compared again -- two more instructions every step; and
        // opaque, so ok1 below is read from the mask rather than re-derived from the compares)
        uint64_t raw = ballot(!(fabs(z) <= B)) | ballot(!halley_ok<NT>(Q, x));
        asm volatile("" : "+s"(raw));
        o = drift_apply<D3>(s, dt, beta, eta, zeta, G0, G1, G2, G3, fp, fpp, Q);
        if (__builtin_expect(raw != 0, 0)) {
#ifdef RVM_PROFILE_FAILS
            rare_count(0, 0);
#endif
            // (the lanes of encountered walkers out: vote_fails; with none left every lane is ok)
            const uint64_t fm = raw & ~encountered_lanes<NP>(s.encm);
            const bool ok1 = ((fm >> (threadIdx.x & 63)) & 1) == 0;
            second_chance(ok1, ACC == 4);
            if (!ok1) o = drift_apply<D3>(s, dt, beta, eta, zeta, G0, G1, G2, G3, fp, fpp, Q);
        }
    } else {
        if constexpr (GATED) {
            // (the early vote keeps the per-lane encounter test: the likelihood kernel's gated levels
            // run it two waves to a SIMD, where the late vote's scalar form measured slower)
            const bool ok1 = (fabs(z) <= B && halley_ok<NT>(Q, x)) || lane_encountered(s);
            if (ballot(!ok1) != 0) {
#ifdef RVM_PROFILE_FAILS
                rare_count(0, 0);
#endif
                second_chance(ok1, ACC == 1 || ACC == 2);
            }
        } else {
            // (the wave's verdict, on every lane: the caller ballots it at the segment's end)
            bad = bad || ((!(fabs(z) <= B) || !halley_ok<NT>(Q, x)) && !lane_encountered(s));
        }
        o = drift_apply<D3>(s, dt, beta, eta, zeta, G0, G1, G2, G3, fp, fpp, Q);
    }
    s.rx = o.rx;
    s.ry = o.ry;
    s.vx = o.vx;
    s.vy = o.vy;
    if constexpr (D3) {
        s.rz = o.rz;
        s.vz = o.vz;
    }
    s.r = o.r;
    s.ir = o.ir;
}

// gated drift (no speculation)
template <int NT, int NP>
__device__ __forceinline__ void drift(Lane<NP>& s, double dt) {
    bool unused = false;
    drift<NT, true>(s, dt, unused, vconsts_for<NT>());
}

// Interaction kick of the own Jacobi velocity by dt (and the encounter test on every pair):
//   gather every planet's Jacobi position from the lane group, heliocentric positions
//   x_i = r'_i + (sum_{j<i} m_j x_j)/M_{i-1}, pairwise accelerations (1/r^3 from rsq), the Jacobi
//   acceleration a'_i = a_i - (sum_{j<i} m_j a_j)/M_{i-1}, and v'_i += dt (a'_i + M_i r'_i/|r'_i|^3)
//   (the Kepler part is removed because the drift integrates it exactly).
template <int NP, int L, bool D3 = false>
__device__ __forceinline__ void kick_generic(Lane<NP>& s, double dt) {
    constexpr int NB = NP + 1;
    double x[NB], y[NB], zz[NB], ax[NB], ay[NB], az[NB];
    x[0] = 0.0;
    y[0] = 0.0;
    zz[0] = 0.0;
    double cmx = 0.0, cmy = 0.0, cmz = 0.0;
#pragma unroll
    for (int i = 1; i < NB; i++) {
        double Rx, Ry, Rz = 0.0;
        if constexpr (NP == 1) {
            Rx = s.rx;
            Ry = s.ry;
            if constexpr (D3) Rz = s.rz;
        } else {
            Rx = grp_get<L>(s.rx, i - 1);
            Ry = grp_get<L>(s.ry, i - 1);
            if constexpr (D3) Rz = grp_get<L>(s.rz, i - 1);
        }
        x[i] = Rx + cmx * s.iMi[i - 1];
        y[i] = Ry + cmy * s.iMi[i - 1];
        zz[i] = D3 ? Rz + cmz * s.iMi[i - 1] : 0.0;
        cmx += s.m[i - 1] * x[i];
        cmy += s.m[i - 1] * y[i];
        if constexpr (D3) cmz += s.m[i - 1] * zz[i];
    }
#pragma unroll
    for (int i = 0; i < NB; i++) {
        ax[i] = 0.0;
        ay[i] = 0.0;
        az[i] = 0.0;
    }
    uint64_t enc = 0;
    // star -- planet 1 distance is |r'_1|, already known to planet 1's lane from its drift
    const double ir01 = (NP == 1) ? s.ir : grp_get<L>(s.ir, 0);
#pragma unroll
    for (int i = 0; i < NB; i++) {
#pragma unroll
        for (int j = i + 1; j < NB; j++) {
            const double dx = x[j] - x[i], dy = y[j] - y[i], dz = zz[j] - zz[i];
            double ir;
            if (i == 0 && j == 1) {
                ir = ir01;
                enc |= ballot(ir * ir > s.idmin2);
            } else {
                double r2 = dx * dx + dy * dy;
                if constexpr (D3) r2 += dz * dz;
                enc |= ballot(r2 < s.dmin2);
                ir = rsq_nr(r2);
            }
            const double ir3 = ir * ir * ir;
            const double mj = (j == 0) ? 1.0 : s.m[j - 1];
            const double mi = (i == 0) ? 1.0 : s.m[i - 1];
            ax[i] += mj * ir3 * dx;
            ay[i] += mj * ir3 * dy;
            ax[j] -= mi * ir3 * dx;
            ay[j] -= mi * ir3 * dy;
            if constexpr (D3) {
                az[i] += mj * ir3 * dz;
                az[j] -= mi * ir3 * dz;
            }
        }
    }
    s.encm |= enc;
    // Jacobi acceleration of the own coordinate (index i = p + 1)
    double max_ = ax[0], may_ = ay[0], maz_ = az[0];  // M_star = 1
    double ajx = 0.0, ajy = 0.0, ajz = 0.0;
#pragma unroll
    for (int i = 1; i < NB; i++) {
        const double tx = ax[i] - max_ * s.iMi[i - 1];
        const double ty = ay[i] - may_ * s.iMi[i - 1];
        const double tz = az[i] - maz_ * s.iMi[i - 1];
        if (s.p == i - 1) {
            ajx = tx;
            ajy = ty;
            ajz = tz;
        }
        max_ += s.m[i - 1] * ax[i];
        may_ += s.m[i - 1] * ay[i];
        if constexpr (D3) maz_ += s.m[i - 1] * az[i];
    }
    const double kep = s.GM * (s.ir * s.ir * s.ir);
    s.vx += dt * (ajx + kep * s.rx);
    s.vy += dt * (ajy + kep * s.ry);
    if constexpr (D3) s.vz += dt * (ajz + kep * s.rz);
}

// Two-planet kick in closed form (same interaction as the generic kick; G = M_star = 1):
//   dv'_1 = dt m_2 (d12/r12^3 - d02/r02^3)
//   dv'_2 = dt [ M_2 r'_2/|r'_2|^3 - (M_2/M_1)(d02/r02^3 + m_1 d12/r12^3) ]
// with heliocentric x_1 = r'_1, x_2 = r'_2 + (m_1/M_1) r'_1, d02 = x_2, d12 = x_2 - x_1.  The
// own |r'| (= star--planet-1 distance on planet 1's lane) is carried from the drift.
//
// Own/other form (lane_finish): each lane reads only the OTHER planet's Jacobi position and
// the other pair's inverse cube from its partner lane (one DPP swap per 32-bit half: 6 moves per
// kick instead of 12), forms its own pair vector o = oA own + oB oth (planet 1's lane: d02,
// planet 2's lane: d12; one v_rsq_f64 per lane and kick), and updates its velocity as
// v += (A + P1 ic_own + P2 ic_oth) own + (P3 ic_own + P4 ic_oth) oth (32 VALU per kick, was 40).
// The encounter bits of both lanes count (kick_enc_bits: the logl epilogue ORs a walker's pair).
template <int L>
__device__ __forceinline__ double pair_swap(double v) {
    static_assert(L == 2, "pair_swap exchanges the two lanes of a 2-planet walker");
    constexpr int ctrl = 1 | (0 << 2) | (3 << 4) | (2 << 6);  // quad_perm [1, 0, 3, 2]
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), ctrl, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), ctrl, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

template <int L, bool D3 = false>
__device__ __forceinline__ void kick2(Lane<2>& s, double c1875 = 1.875) {
    static_assert(L == 2, "kick2 pairs the two planets' lanes");
    const double ox_ = pair_swap<L>(s.rx), oy_ = pair_swap<L>(s.ry);  // the other planet's r'
    const double ox = fma(s.oA, s.rx, s.oB * ox_), oy = fma(s.oA, s.ry, s.oB * oy_);
    double rsq = fma(ox, ox, oy * oy);
    double oz_ = 0.0;
    if constexpr (D3) {
        oz_ = pair_swap<L>(s.rz);
        const double oz = fma(s.oA, s.rz, s.oB * oz_);
        rsq = fma(oz, oz, rsq);
    }
    // own pair on every lane; star--planet-1 from |r'_1| on planet 1's lanes only (|r'_2| is a
    // Jacobi distance, not a pair)
    const double ir2 = s.ir * s.ir;
    s.encm |= ballot(rsq < s.dmin2) | ballot(ir2 > s.idmin2);  // (idmin2 +inf on planet 2's lanes)
    const double ic = rcube_nr(rsq, c1875);
    const double ico = pair_swap<L>(ic);
    const double A = s.kAh * (s.ir * ir2);
    const double al = fma(s.kP2h, ico, fma(s.kP1h, ic, A));
    const double be = fma(s.kP4h, ico, s.kP3h * ic);
    s.vx = fma(al, s.rx, fma(be, ox_, s.vx));
    s.vy = fma(al, s.ry, fma(be, oy_, s.vy));
    if constexpr (D3) s.vz = fma(al, s.rz, fma(be, oz_, s.vz));
}

// Closed-form kick for NP >= 3 planets (the same interaction as kick_generic): every lane of
// the group forms the heliocentric positions and the inverse cubes of all pairs but (0, 1), and
// applies its own coefficients (lane_finish, step folded in by lane_set_step):
//   v'_i += h [ A_i r'_i / |r'_i|^3 + sum_ab c_ab(i) d_ab / r_ab^3 ],   d_ab = x_b - x_a.
// The star--planet-1 exit check uses |r'_1| = |x_1| on planet 1's lane, the only lane whose
// encounter bit is read.
template <int NP, int L, bool D3 = false>
__device__ __forceinline__ void kickN(Lane<NP>& s, double c1875) {
    constexpr int NB = NP + 1;
    double x[NB], y[NB], z[NB];
    x[0] = y[0] = z[0] = 0.0;
    double cmx = 0.0, cmy = 0.0, cmz = 0.0;
#pragma unroll
    for (int i = 1; i < NB; i++) {
        const double Rx = grp_get<L>(s.rx, i - 1), Ry = grp_get<L>(s.ry, i - 1);
        const double Rz = D3 ? grp_get<L>(s.rz, i - 1) : 0.0;
        x[i] = i == 1 ? Rx : fma(cmx, s.iMi[i - 1], Rx);
        y[i] = i == 1 ? Ry : fma(cmy, s.iMi[i - 1], Ry);
        z[i] = i == 1 ? Rz : fma(cmz, s.iMi[i - 1], Rz);
        if (i + 1 < NB) {
            cmx = fma(s.m[i - 1], x[i], cmx);
            cmy = fma(s.m[i - 1], y[i], cmy);
            if constexpr (D3) cmz = fma(s.m[i - 1], z[i], cmz);
        }
    }
    double vx = s.vx, vy = s.vy, vz = s.vz;
    if constexpr (NP == 3 && L == 4) {
        // The four pairs (0,2), (0,3), (1,2), (1,3) are split over the group's four lanes (lane q
        // takes pair k = q: b = 2 + (q & 1), a = 1 on lanes 2 and 3), one inverse cube each,
        // exchanged by DPP; (2,3) is formed on every lane.  The distances are the same expressions
        // as in the generic loop below (fma(-0, x1, xb) = xb, fma(-1, x1, xb) = xb - x1), so the
        // bits are the same: 2 v_rsq_f64 per lane and kick instead of 5.  Encounter bits: each
        // lane's own pair, (2,3) everywhere, star--planet-1 on the planets' first lanes only
        // (kick_enc_bits<3> reads all four lanes of a walker).
        const bool b3 = (s.q & 1) != 0;
        const double bx = b3 ? x[3] : x[2], by = b3 ? y[3] : y[2];
        const double ox = fma(s.pair_s, x[1], bx), oy = fma(s.pair_s, y[1], by);
        double ro = fma(ox, ox, oy * oy);
        if constexpr (D3) {
            const double bz = b3 ? z[3] : z[2];
            const double oz = fma(s.pair_s, z[1], bz);
            ro = fma(oz, oz, ro);
        }
        const double dx = x[3] - x[2], dy = y[3] - y[2], dz = z[3] - z[2];
        double r23 = fma(dx, dx, dy * dy);
        if constexpr (D3) r23 = fma(dz, dz, r23);
        s.encm |= (ballot(s.ir * s.ir > s.idmin2) & 0x1111111111111111ull) | ballot(ro < s.dmin2) |
                  ballot(r23 < s.dmin2);
        const double io = rcube_nr(ro, c1875);
        const double i23 = rcube_nr(r23, c1875);
        const double ic[4] = {grp_get<L, 0>(io), grp_get<L, 1>(io), grp_get<L, 2>(io), grp_get<L, 3>(io)};
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int a = k >> 1, b = 2 + (k & 1);
            const double cf = s.kPh[k] * ic[k];
            vx = fma(cf, x[b] - x[a], vx);
            vy = fma(cf, y[b] - y[a], vy);
            if constexpr (D3) vz = fma(cf, z[b] - z[a], vz);
        }
        const double cf = s.kPh[4] * i23;
        vx = fma(cf, dx, vx);
        vy = fma(cf, dy, vy);
        if constexpr (D3) vz = fma(cf, dz, vz);
        const double A = s.kAh * (s.ir * (s.ir * s.ir));
        s.vx = fma(A, s.rx, vx);
        s.vy = fma(A, s.ry, vy);
        if constexpr (D3) s.vz = fma(A, s.rz, vz);
        return;
    }
    uint64_t enc = ballot(s.ir * s.ir > s.idmin2);
    int k = 0;
#pragma unroll
    for (int a = 0; a < NB; a++) {
#pragma unroll
        for (int b = a + 1; b < NB; b++) {
            if (a == 0 && b == 1) continue;
            const double dx = x[b] - x[a], dy = y[b] - y[a], dz = z[b] - z[a];
            double r2 = fma(dx, dx, dy * dy);
            if constexpr (D3) r2 = fma(dz, dz, r2);
            enc |= ballot(r2 < s.dmin2);
            const double cf = s.kPh[k++] * rcube_nr(r2, c1875);
            vx = fma(cf, dx, vx);
            vy = fma(cf, dy, vy);
            if constexpr (D3) vz = fma(cf, dz, vz);
        }
    }
    s.encm |= enc;
    const double A = s.kAh * (s.ir * (s.ir * s.ir));
    s.vx = fma(A, s.rx, vx);
    s.vy = fma(A, s.ry, vy);
    if constexpr (D3) s.vz = fma(A, s.rz, vz);
}

template <int NP, int L, bool D3 = false>
__device__ __forceinline__ void kick(Lane<NP>& s, double dt, double c1875 = 1.875) {
    // NP >= 2: the step is folded into the lane's coefficients (lane_set_step(s, dt) beforehand)
    if constexpr (NP == 2)
        kick2<L, D3>(s, c1875);
    else if constexpr (NP >= 3)
        kickN<NP, L, D3>(s, c1875);
    else
        kick_generic<NP, L, D3>(s, dt);
}

// ---- kick split for kick-drift-kick segments (rvm_logl.hip segment_steps) -------------------------
// A segment of ns steps runs K(h/2) [D(h) K(h)]^(ns-1) D(h) K(h/2): ns Kepler drifts instead of the
// ns + 1 of drift-kick-drift, at the same accuracy (Richardson-extrapolated, against the IAS15
// restatement: S2 1.5e-9 vs 1.4e-9, HD155358 1.4e-9 vs 1.8e-9).  The interaction depends on the
// positions only, so the closing half kick of a segment and the opening half kick of the next
// (same positions, the epoch in between) share one evaluation: kick_prep evaluates it (and runs
// the encounter test) once per position, kick_apply adds it to the velocity with the segment's
// step (HALF: half of it, an exact scaling by 0.5).  What is carried between the two: NP = 2 the
// other planet's r', both pair inverse cubes and |r'|^-3 (the step-scaled coefficients of the
// closed-form kick change with the segment's step); other NP the unscaled acceleration.
template <int NP>
struct KickPrep {
    double ax, ay, az;
};
template <>
struct KickPrep<2> {
    double ox_, oy_, oz_, ic, ico, ir3;
};

template <int NP, int L, bool D3 = false>
__device__ __forceinline__ KickPrep<NP> kick_prep(Lane<NP>& s, double c1875) {
    KickPrep<NP> k;
    if constexpr (NP == 2) {
        k.ox_ = pair_swap<L>(s.rx);
        k.oy_ = pair_swap<L>(s.ry);
        const double ox = fma(s.oA, s.rx, s.oB * k.ox_), oy = fma(s.oA, s.ry, s.oB * k.oy_);
        double rsq = fma(ox, ox, oy * oy);
        k.oz_ = 0.0;
        if constexpr (D3) {
            k.oz_ = pair_swap<L>(s.rz);
            const double oz = fma(s.oA, s.rz, s.oB * k.oz_);
            rsq = fma(oz, oz, rsq);
        }
        const double ir2 = s.ir * s.ir;
        s.encm |= ballot(rsq < s.dmin2) | ballot(ir2 > s.idmin2);  // (idmin2 +inf on planet 2's lanes)
        k.ic = rcube_nr(rsq, c1875);
        k.ico = pair_swap<L>(k.ic);
        k.ir3 = s.ir * ir2;
    } else {
        // the kick of the unit step from zero velocity: the acceleration itself
        Lane<NP> t = s;
        t.vx = t.vy = t.vz = 0.0;
        if constexpr (NP >= 3) {
            t.kAh = t.kA;  // unscaled coefficients: the unit step
#pragma unroll
            for (int q = 0; q < KickPairs<NP>::n; q++) t.kPh[q] = t.kP[q];
            kickN<NP, L, D3>(t, c1875);
        } else {
            kick_generic<NP, L, D3>(t, 1.0);
        }
        s.encm = t.encm;
        k.ax = t.vx;
        k.ay = t.vy;
        k.az = t.vz;
    }
    return k;
}

template <int NP, bool HALF, bool D3 = false>
__device__ __forceinline__ void kick_apply(Lane<NP>& s, const KickPrep<NP>& k) {
    if constexpr (NP == 2) {
        const double A = s.kAh * k.ir3;
        double al = fma(s.kP2h, k.ico, fma(s.kP1h, k.ic, A));
        double be = fma(s.kP4h, k.ico, s.kP3h * k.ic);
        if constexpr (HALF) {
            al *= 0.5;
            be *= 0.5;
        }
        s.vx = fma(al, s.rx, fma(be, k.ox_, s.vx));
        s.vy = fma(al, s.ry, fma(be, k.oy_, s.vy));
        if constexpr (D3) s.vz = fma(al, s.rz, fma(be, k.oz_, s.vz));
    } else {
        const double hk = HALF ? 0.5 * s.h : s.h;
        s.vx = fma(hk, k.ax, s.vx);
        s.vy = fma(hk, k.ay, s.vy);
        if constexpr (D3) s.vz = fma(hk, k.az, s.vz);
    }
}

// Encounter bits of a walker in Lane::encm relative to its first lane: kick2 and the 3-planet
// kickN split the pair tests over the walker's lanes, kickN (4 planets) / kick_generic put all of
// them on every lane.
template <int NP>
__device__ __forceinline__ constexpr uint64_t kick_enc_bits() {
    return NP == 2 ? 3ull : (NP == 3 ? 0xFull : 1ull);
}

// star barycentric x-velocity: v0 = -sum_q (m_q / M_q) v'_q (gathered over the lane group)
template <int NP, int L>
__device__ __forceinline__ double star_vx(const Lane<NP>& s) {
    double v = 0.0;
#pragma unroll
    for (int q = 0; q < NP; q++) {
        const double vq = (NP == 1) ? s.vx : grp_get<L>(s.vx, q);
        v -= s.mu[q] * vq;
    }
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

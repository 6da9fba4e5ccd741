/*
 * oracle/rvoracle.c -- CPU restatement of the reference's log-likelihood path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (rvel-mcmc_amd/) links, loads or calls
 * this file; only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg do, and
 * only as the checker / the timed CPU baseline.
 *
 * What it restates (reference = /root/reference, Python 2 + REBOUND):
 *   - state.py:36-47   State.setup_sim   star m=1, planets added with primary=star through
 *                                         REBOUND's Pal (2009) elements, Hill radii, move_to_com,
 *                                         exit_min_distance = hillRadiusFactor * max r_Hill
 *   - state.py:61-73   State.get_rv      fresh simulation, integrate(t) for t in ARRAY ORDER,
 *                                         record particles[0].vx
 *   - state.py:89-98   State.get_chi2    sum (rv-obs)^2/sigma^2 over tf then tb, / obs.Npoints
 *   - state.py:103-110 State.get_logp    priorHard -> -inf, else -chi2
 *   - state.py:299-315 State.priorHard   a<=0.02, m<=5e-6, h^2+k^2>=1, ix^2+iy^2>=4
 *   - REBOUND (third-party C, not vendored; ~v3.x, early 2017):
 *       reb_tools_pal_to_particle (Pal 2009 -> Cartesian), reb_move_to_com,
 *       the IAS15 integrator (Rein & Spiegel 2015, MNRAS 446, 1424) with REBOUND defaults
 *       epsilon=1e-9, safety_factor=0.25, min_dt=0, epsilon_global=1, initial dt=0.001,
 *       reb_integrate(tmax) with exact_finish_time=1, and the exit_min_distance encounter
 *       check run after every step (raises rebound.Encounter).
 *     The IAS15 constants are DERIVED (oracle/gen_ias15_consts.py), not transcribed.
 *   Parity of this restatement is pinned by the reference's stored outputs:
 *   G1 (Pal + COM vectors), G2 (logp of HD155358 `sol`), G3 (1000-point RV curve), G4.
 *
 * It also holds `rvo_wh_*`: a plain-C restatement of the SAME Wisdom-Holman algorithm the HIP
 * kernel runs (Jacobi coordinates, KDK, epoch-aligned segments), used for the T1 parity tier
 * (GPU vs CPU, same algorithm) and as the "port" CPU baseline.  It is written independently of
 * the kernel source (no shared headers).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "ias15_consts.h"

#define RVO_MAXP 7
#define RVO_MAXB (RVO_MAXP + 1)
#define RVO_N3 (3 * RVO_MAXB)

enum { RVO_OK = 0, RVO_PRIOR = 1, RVO_ENCOUNTER = 2, RVO_NONFINITE = 3 };

/* ------------------------------------------------------------------------------------------ */
/* Pal (2009) elements -> Cartesian, REBOUND `sim.add(primary=..., m, a, h, k, l[, ix, iy])`.  */
/* k = e cos(varpi), h = e sin(varpi), l = mean longitude, (ix,iy) = 2 sin(i/2)(cos O, sin O) */
/* SURVEY.md App. A.2 (pinned bit-level by G1).                                                */
/* ------------------------------------------------------------------------------------------ */
static void pal_to_cart(double mu, double a, double lam, double k, double h, double ix, double iy,
                        double* pos, double* vel) {
    /* Kepler's equation in eccentric longitude: lam = F - k sin F + h cos F (Newton from F=lam) */
    double F = lam;
    for (int it = 0; it < 100; it++) {
        const double sF = sin(F), cF = cos(F);
        const double fF = F - k * sF + h * cF - lam;
        const double dF = 1.0 - k * cF - h * sF;
        const double step = fF / dF;
        F -= step;
        if (fabs(step) <= 1e-16 * (fabs(F) > 1.0 ? fabs(F) : 1.0)) break;
    }
    const double sF = sin(F), cF = cos(F);
    const double beta = 1.0 / (1.0 + sqrt(1.0 - h * h - k * k));
    const double n = sqrt(mu / (a * a * a));
    const double r = a * (1.0 - k * cF - h * sF);
    const double X = a * ((1.0 - h * h * beta) * cF + h * k * beta * sF - k);
    const double Y = a * ((1.0 - k * k * beta) * sF + h * k * beta * cF - h);
    const double fac = n * a * a / r;
    const double VX = fac * (h * k * beta * cF - (1.0 - h * h * beta) * sF);
    const double VY = fac * ((1.0 - k * k * beta) * cF - h * k * beta * sF);
    if (ix == 0.0 && iy == 0.0) {
        pos[0] = X; pos[1] = Y; pos[2] = 0.0;
        vel[0] = VX; vel[1] = VY; vel[2] = 0.0;
        return;
    }
    /* rotate the orbital plane about the node line by i (Rodrigues), expressed in (ix, iy) */
    const double W = sqrt(fabs(4.0 - ix * ix - iy * iy));
    const double axx = 1.0 - 0.5 * iy * iy, axy = 0.5 * ix * iy;
    const double ayy = 1.0 - 0.5 * ix * ix;
    pos[0] = axx * X + axy * Y;
    pos[1] = axy * X + ayy * Y;
    pos[2] = 0.5 * W * (ix * Y - iy * X);
    vel[0] = axx * VX + axy * VY;
    vel[1] = axy * VX + ayy * VY;
    vel[2] = 0.5 * W * (ix * VY - iy * VX);
}

/* planet parameter record used across the oracle ABI: m, a, h, k, l, ix, iy */
#define RVO_PSTRIDE 7

/* state.py:299-315 -- first failing condition wins, planets in order. */
int rvo_prior_hard(int np, const double* pl, int has_hk, int has_inc) {
    for (int i = 0; i < np; i++) {
        const double* p = pl + RVO_PSTRIDE * i;
        if (p[1] <= 0.02) return 1;
        if (p[0] <= 5e-6) return 1;
        if (has_hk && (p[2] * p[2] + p[3] * p[3] >= 1.0)) return 1;
        if (has_inc && (p[5] * p[5] + p[6] * p[6] >= 4.0)) return 1;
    }
    return 0;
}

/* state.py:36-47: bodies (star first), barycentric after move_to_com; returns max Hill radius */
static double setup_bodies(int np, const double* pl, double* m, double* x, double* v) {
    double hill = 0.0;
    m[0] = 1.0;
    x[0] = x[1] = x[2] = 0.0;
    v[0] = v[1] = v[2] = 0.0;
    for (int i = 0; i < np; i++) {
        const double* p = pl + RVO_PSTRIDE * i;
        const int b = i + 1;
        m[b] = p[0];
        /* G = 1; primary = the star particle (m = 1, at rest at the origin) */
        pal_to_cart(1.0 * (m[0] + p[0]), p[1], p[4], p[3], p[2], p[5], p[6], x + 3 * b, v + 3 * b);
        const double rh = p[1] * pow(p[0] / (3.0 * m[0]), 1.0 / 3.0);
        if (rh > hill) hill = rh;
    }
    /* reb_move_to_com */
    const int nb = np + 1;
    double M = 0, cx[3] = {0, 0, 0}, cv[3] = {0, 0, 0};
    for (int b = 0; b < nb; b++) {
        M += m[b];
        for (int c = 0; c < 3; c++) {
            cx[c] += m[b] * x[3 * b + c];
            cv[c] += m[b] * v[3 * b + c];
        }
    }
    for (int c = 0; c < 3; c++) { cx[c] /= M; cv[c] /= M; }
    for (int b = 0; b < nb; b++)
        for (int c = 0; c < 3; c++) {
            x[3 * b + c] -= cx[c];
            v[3 * b + c] -= cv[c];
        }
    return hill;
}

/* Expose setup for the G1 fixture: heliocentric (before COM) and barycentric (after) vectors. */
void rvo_setup_vectors(int np, const double* pl, double* helio_xv, double* bary_xv) {
    double m[RVO_MAXB], x[RVO_N3], v[RVO_N3];
    for (int i = 0; i < np; i++) {
        const double* p = pl + RVO_PSTRIDE * i;
        double px[3], pv[3];
        pal_to_cart(1.0 + p[0], p[1], p[4], p[3], p[2], p[5], p[6], px, pv);
        for (int c = 0; c < 3; c++) {
            helio_xv[6 * (i + 1) + c] = px[c];
            helio_xv[6 * (i + 1) + 3 + c] = pv[c];
        }
    }
    for (int c = 0; c < 6; c++) helio_xv[c] = 0.0;
    setup_bodies(np, pl, m, x, v);
    for (int b = 0; b <= np; b++)
        for (int c = 0; c < 3; c++) {
            bary_xv[6 * b + c] = x[3 * b + c];
            bary_xv[6 * b + 3 + c] = v[3 * b + c];
        }
}

/* ------------------------------------------------------------------------------------------ */
/* IAS15 (REBOUND default integrator), restated.                                               */
/* ------------------------------------------------------------------------------------------ */
typedef struct {
    int N;                  /* bodies */
    double t, dt, dt_last_done, dt_last_success;
    double m[RVO_MAXB];
    double x[RVO_N3], v[RVO_N3], a[RVO_N3];
    double x0[RVO_N3], v0[RVO_N3], a0[RVO_N3], at[RVO_N3];
    double csx[RVO_N3], csv[RVO_N3];
    double g[7][RVO_N3], b[7][RVO_N3], e[7][RVO_N3], br[7][RVO_N3], er[7][RVO_N3];
    double exit_min_distance;
    double epsilon, safety_factor, min_dt;
    long nsteps, nrejected;
} ias_sim;

static void gravity(const ias_sim* s, const double* x, double* acc) {
    const int N = s->N;
    for (int k = 0; k < 3 * N; k++) acc[k] = 0.0;
    for (int i = 0; i < N; i++) {
        for (int j = i + 1; j < N; j++) {
            const double dx = x[3 * i] - x[3 * j];
            const double dy = x[3 * i + 1] - x[3 * j + 1];
            const double dz = x[3 * i + 2] - x[3 * j + 2];
            const double r2 = dx * dx + dy * dy + dz * dz;
            const double r = sqrt(r2);
            const double pf = 1.0 / (r2 * r); /* G = 1 */
            const double pfj = -pf * s->m[j];
            const double pfi = pf * s->m[i];
            acc[3 * i] += pfj * dx;
            acc[3 * i + 1] += pfj * dy;
            acc[3 * i + 2] += pfj * dz;
            acc[3 * j] += pfi * dx;
            acc[3 * j + 1] += pfi * dy;
            acc[3 * j + 2] += pfi * dz;
        }
    }
}

static inline void add_cs(double* p, double* csp, double inp) {
    const double y = inp - *csp;
    const double t = *p + y;
    *csp = (t - *p) - y;
    *p = t;
}

static void ias_predict_next_step(double ratio, int N3, double (*e_in)[RVO_N3], double (*b_in)[RVO_N3],
                                  double (*e)[RVO_N3], double (*b)[RVO_N3]) {
    if (ratio > 20.0) {
        for (int j = 0; j < 7; j++)
            for (int k = 0; k < N3; k++) { e[j][k] = 0.0; b[j][k] = 0.0; }
        return;
    }
    const double q1 = ratio, q2 = q1 * q1, q3 = q1 * q2, q4 = q2 * q2, q5 = q2 * q3, q6 = q3 * q3,
                 q7 = q3 * q4;
    for (int k = 0; k < N3; k++) {
        double be[7];
        for (int j = 0; j < 7; j++) be[j] = b_in[j][k] - e_in[j][k];
        const double B0 = b_in[0][k], B1 = b_in[1][k], B2 = b_in[2][k], B3 = b_in[3][k], B4 = b_in[4][k],
                     B5 = b_in[5][k], B6 = b_in[6][k];
        e[0][k] = q1 * (B6 * 7.0 + B5 * 6.0 + B4 * 5.0 + B3 * 4.0 + B2 * 3.0 + B1 * 2.0 + B0);
        e[1][k] = q2 * (B6 * 21.0 + B5 * 15.0 + B4 * 10.0 + B3 * 6.0 + B2 * 3.0 + B1);
        e[2][k] = q3 * (B6 * 35.0 + B5 * 20.0 + B4 * 10.0 + B3 * 4.0 + B2);
        e[3][k] = q4 * (B6 * 35.0 + B5 * 15.0 + B4 * 5.0 + B3);
        e[4][k] = q5 * (B6 * 21.0 + B5 * 6.0 + B4);
        e[5][k] = q6 * (B6 * 7.0 + B5);
        e[6][k] = q7 * B6;
        for (int j = 0; j < 7; j++) b[j][k] = e[j][k] + be[j];
    }
}

/* one IAS15 step attempt; returns 1 if accepted, 0 if rejected (dt shrunk, state restored) */
static int ias_step_try(ias_sim* s) {
    const int N3 = 3 * s->N;
    const double* h = IAS15_H;
    const double* rr = IAS15_RR;
    const double* c = IAS15_C;
    const double* d = IAS15_D;
    double (*g)[RVO_N3] = s->g;
    double (*b)[RVO_N3] = s->b;

    for (int k = 0; k < N3; k++) {
        s->x0[k] = s->x[k];
        s->v0[k] = s->v[k];
        s->a0[k] = s->a[k];
    }
    for (int k = 0; k < N3; k++) {
        g[0][k] = b[6][k] * d[15] + b[5][k] * d[10] + b[4][k] * d[6] + b[3][k] * d[3] + b[2][k] * d[1] +
                  b[1][k] * d[0] + b[0][k];
        g[1][k] = b[6][k] * d[16] + b[5][k] * d[11] + b[4][k] * d[7] + b[3][k] * d[4] + b[2][k] * d[2] + b[1][k];
        g[2][k] = b[6][k] * d[17] + b[5][k] * d[12] + b[4][k] * d[8] + b[3][k] * d[5] + b[2][k];
        g[3][k] = b[6][k] * d[18] + b[5][k] * d[13] + b[4][k] * d[9] + b[3][k];
        g[4][k] = b[6][k] * d[19] + b[5][k] * d[14] + b[4][k];
        g[5][k] = b[6][k] * d[20] + b[5][k];
        g[6][k] = b[6][k];
    }
    const double dt = s->dt;
    double pc_err = 1e300, pc_err_last = 2.0;
    int iterations = 0;
    double xp[RVO_N3];
    while (1) {
        if (pc_err < 1e-16) break;
        if (iterations > 2 && pc_err_last <= pc_err) break;
        if (iterations >= 12) break; /* REBOUND warns: predictor-corrector did not converge */
        pc_err_last = pc_err;
        pc_err = 0.0;
        iterations++;
        for (int n = 1; n < 8; n++) {
            double sx[9];
            sx[0] = dt * h[n];
            sx[1] = sx[0] * sx[0] / 2.0;
            sx[2] = sx[1] * h[n] / 3.0;
            sx[3] = sx[2] * h[n] / 2.0;
            sx[4] = 3.0 * sx[3] * h[n] / 5.0;
            sx[5] = 2.0 * sx[4] * h[n] / 3.0;
            sx[6] = 5.0 * sx[5] * h[n] / 7.0;
            sx[7] = 3.0 * sx[6] * h[n] / 4.0;
            sx[8] = 7.0 * sx[7] * h[n] / 9.0;
            for (int k = 0; k < N3; k++) {
                xp[k] = -s->csx[k] + ((sx[8] * b[6][k] + sx[7] * b[5][k] + sx[6] * b[4][k] + sx[5] * b[3][k] +
                                       sx[4] * b[2][k] + sx[3] * b[1][k] + sx[2] * b[0][k] + sx[1] * s->a0[k] +
                                       sx[0] * s->v0[k]) +
                                      s->x0[k]);
            }
            gravity(s, xp, s->at);
            double maxak = 0.0, maxb6ktmp = 0.0;
            for (int k = 0; k < N3; k++) {
                const double gk = s->at[k] - s->a0[k];
                double tmp;
                switch (n) {
                    case 1:
                        tmp = g[0][k];
                        g[0][k] = gk / rr[0];
                        b[0][k] += g[0][k] - tmp;
                        break;
                    case 2:
                        tmp = g[1][k];
                        g[1][k] = (gk / rr[1] - g[0][k]) / rr[2];
                        tmp = g[1][k] - tmp;
                        b[0][k] += tmp * c[0];
                        b[1][k] += tmp;
                        break;
                    case 3:
                        tmp = g[2][k];
                        g[2][k] = ((gk / rr[3] - g[0][k]) / rr[4] - g[1][k]) / rr[5];
                        tmp = g[2][k] - tmp;
                        b[0][k] += tmp * c[1];
                        b[1][k] += tmp * c[2];
                        b[2][k] += tmp;
                        break;
                    case 4:
                        tmp = g[3][k];
                        g[3][k] = (((gk / rr[6] - g[0][k]) / rr[7] - g[1][k]) / rr[8] - g[2][k]) / rr[9];
                        tmp = g[3][k] - tmp;
                        b[0][k] += tmp * c[3];
                        b[1][k] += tmp * c[4];
                        b[2][k] += tmp * c[5];
                        b[3][k] += tmp;
                        break;
                    case 5:
                        tmp = g[4][k];
                        g[4][k] = ((((gk / rr[10] - g[0][k]) / rr[11] - g[1][k]) / rr[12] - g[2][k]) / rr[13] -
                                   g[3][k]) /
                                  rr[14];
                        tmp = g[4][k] - tmp;
                        b[0][k] += tmp * c[6];
                        b[1][k] += tmp * c[7];
                        b[2][k] += tmp * c[8];
                        b[3][k] += tmp * c[9];
                        b[4][k] += tmp;
                        break;
                    case 6:
                        tmp = g[5][k];
                        g[5][k] = (((((gk / rr[15] - g[0][k]) / rr[16] - g[1][k]) / rr[17] - g[2][k]) / rr[18] -
                                    g[3][k]) /
                                       rr[19] -
                                   g[4][k]) /
                                  rr[20];
                        tmp = g[5][k] - tmp;
                        b[0][k] += tmp * c[10];
                        b[1][k] += tmp * c[11];
                        b[2][k] += tmp * c[12];
                        b[3][k] += tmp * c[13];
                        b[4][k] += tmp * c[14];
                        b[5][k] += tmp;
                        break;
                    case 7: {
                        tmp = g[6][k];
                        g[6][k] = ((((((gk / rr[21] - g[0][k]) / rr[22] - g[1][k]) / rr[23] - g[2][k]) / rr[24] -
                                     g[3][k]) /
                                        rr[25] -
                                    g[4][k]) /
                                       rr[26] -
                                   g[5][k]) /
                                  rr[27];
                        tmp = g[6][k] - tmp;
                        b[0][k] += tmp * c[15];
                        b[1][k] += tmp * c[16];
                        b[2][k] += tmp * c[17];
                        b[3][k] += tmp * c[18];
                        b[4][k] += tmp * c[19];
                        b[5][k] += tmp * c[20];
                        b[6][k] += tmp;
                        const double ak = fabs(s->at[k]);
                        if (isnormal(ak) && ak > maxak) maxak = ak;
                        const double b6ktmp = fabs(tmp);
                        if (isnormal(b6ktmp) && b6ktmp > maxb6ktmp) maxb6ktmp = b6ktmp;
                    } break;
                }
            }
            if (n == 7) pc_err = maxb6ktmp / maxak;
        }
    }

    /* new timestep (epsilon_global = 1) */
    const double dt_done = dt;
    if (s->epsilon > 0.0) {
        double maxak = 0.0, maxb6k = 0.0;
        for (int k = 0; k < N3; k++) {
            const double ak = fabs(s->at[k]);
            if (isnormal(ak) && ak > maxak) maxak = ak;
            const double b6k = fabs(b[6][k]);
            if (isnormal(b6k) && b6k > maxb6k) maxb6k = b6k;
        }
        const double integrator_error = maxb6k / maxak;
        double dt_new;
        if (isnormal(integrator_error)) {
            dt_new = pow(s->epsilon / integrator_error, 1.0 / 7.0) * dt_done;
        } else {
            dt_new = dt_done / s->safety_factor;
        }
        if (fabs(dt_new) < s->min_dt) dt_new = copysign(s->min_dt, dt_new);
        if (fabs(dt_new / dt_done) < s->safety_factor) {
            for (int k = 0; k < N3; k++) {
                s->x[k] = s->x0[k];
                s->v[k] = s->v0[k];
            }
            s->dt = dt_new;
            if (s->dt_last_success != 0.0) {
                const double ratio = s->dt / s->dt_last_success;
                ias_predict_next_step(ratio, N3, s->er, s->br, s->e, s->b);
            }
            s->nrejected++;
            return 0;
        }
        if (fabs(dt_new / dt_done) > 1.0 / s->safety_factor) dt_new = dt_done / s->safety_factor;
        s->dt = dt_new;
    }

    /* advance to the end of the step (compensated summation) */
    for (int k = 0; k < N3; k++) {
        const double dx = ((((((((b[6][k] * 7.0 / 9.0 + b[5][k]) * 3.0 / 4.0 + b[4][k]) * 5.0 / 7.0 + b[3][k]) *
                                   2.0 / 3.0 +
                               b[2][k]) *
                                  3.0 / 5.0 +
                              b[1][k]) /
                                 2.0 +
                             b[0][k]) /
                                3.0 +
                            s->a0[k]) *
                               dt_done / 2.0 +
                           s->v0[k]) *
                          dt_done;
        add_cs(&s->x0[k], &s->csx[k], dx);
        const double dv = (((((((b[6][k] * 7.0 / 8.0 + b[5][k]) * 6.0 / 7.0 + b[4][k]) * 5.0 / 6.0 + b[3][k]) *
                                  4.0 / 5.0 +
                              b[2][k]) *
                                 3.0 / 4.0 +
                             b[1][k]) *
                                2.0 / 3.0 +
                            b[0][k]) /
                               2.0 +
                           s->a0[k]) *
                          dt_done;
        add_cs(&s->v0[k], &s->csv[k], dv);
        s->x[k] = s->x0[k];
        s->v[k] = s->v0[k];
    }
    s->t += dt_done;
    s->dt_last_done = dt_done;
    s->dt_last_success = dt_done;
    for (int j = 0; j < 7; j++)
        for (int k = 0; k < N3; k++) {
            s->er[j][k] = s->e[j][k];
            s->br[j][k] = s->b[j][k];
        }
    const double ratio = s->dt / dt_done;
    ias_predict_next_step(ratio, N3, s->e, s->b, s->e, s->b);
    s->nsteps++;
    return 1;
}

static void ias_step(ias_sim* s) {
    gravity(s, s->x, s->a); /* reb_update_acceleration before integrator part2 */
    while (!ias_step_try(s)) {
    }
}

static int encounter(const ias_sim* s) {
    if (!(s->exit_min_distance > 0.0)) return 0;
    const double min2 = s->exit_min_distance * s->exit_min_distance;
    for (int i = 0; i < s->N; i++)
        for (int j = 0; j < i; j++) {
            const double dx = s->x[3 * i] - s->x[3 * j];
            const double dy = s->x[3 * i + 1] - s->x[3 * j + 1];
            const double dz = s->x[3 * i + 2] - s->x[3 * j + 2];
            if (dx * dx + dy * dy + dz * dz < min2) return 1;
        }
    return 0;
}

/* reb_integrate(tmax) with exact_finish_time = 1. Returns 0 or RVO_ENCOUNTER. */
static int ias_integrate(ias_sim* s, double tmax) {
    if (encounter(s)) return RVO_ENCOUNTER;
    if (s->t == tmax) return 0;
    if (s->dt * (tmax - s->t) < 0.0) s->dt = -s->dt;
    const double dtsign = s->dt >= 0.0 ? 1.0 : -1.0;
    double last_full_dt = s->dt;
    s->dt_last_done = 0.0;
    while (1) {
        int last = 0;
        if ((s->t + s->dt) * dtsign >= tmax * dtsign) {
            if (s->t == tmax) break;
            last = 1;
            if (s->dt_last_done != 0.0) last_full_dt = s->dt_last_done;
            s->dt = tmax - s->t;
        }
        const double want = s->dt;
        ias_step(s);
        if (encounter(s)) {
            s->dt = last_full_dt;
            return RVO_ENCOUNTER;
        }
        if (last && s->dt_last_done == want) {
            s->t = tmax;
            break;
        }
        if (!isfinite(s->t)) return RVO_NONFINITE;
    }
    s->dt = last_full_dt;
    return 0;
}

static void ias_init(ias_sim* s, int np, const double* pl, double hill_factor) {
    memset(s, 0, sizeof(*s));
    s->N = np + 1;
    const double hill = setup_bodies(np, pl, s->m, s->x, s->v);
    s->exit_min_distance = hill_factor * hill;
    s->dt = 0.001;
    s->epsilon = 1e-9;
    s->safety_factor = 0.25;
    s->min_dt = 0.0;
}

/* state.py:61-73 -- one fresh simulation, integrate to each time IN ARRAY ORDER, star vx. */
int rvo_get_rv_ias15(int np, const double* pl, double hill_factor, const double* times, int n, double* rv,
                     long* nsteps) {
    ias_sim* s = (ias_sim*)malloc(sizeof(ias_sim));
    ias_init(s, np, pl, hill_factor);
    int st = 0;
    for (int i = 0; i < n; i++) {
        st = ias_integrate(s, times[i]);
        if (st) break;
        rv[i] = s->v[0];
    }
    if (nsteps) *nsteps = s->nsteps;
    free(s);
    return st;
}

/* state.py:89-110 + priorHard.  Returns status; *logl = -chi2/npoints or -inf. */
int rvo_logl_ias15(int np, const double* pl, int has_hk, int has_inc, double hill_factor, const double* tf,
                   const double* rvf, const double* ef, int nf, const double* tb, const double* rvb,
                   const double* eb, int nb, double npoints, double* logl) {
    if (rvo_prior_hard(np, pl, has_hk, has_inc)) {
        *logl = -INFINITY;
        return RVO_PRIOR;
    }
    double* rv = (double*)malloc(sizeof(double) * (size_t)(nf > nb ? nf : nb) + 8);
    double chi2f = 0.0, chi2b = 0.0;
    int st = rvo_get_rv_ias15(np, pl, hill_factor, tf, nf, rv, NULL);
    if (!st) {
        for (int i = 0; i < nf; i++) chi2f += ((rv[i] - rvf[i]) * (rv[i] - rvf[i])) / (ef[i] * ef[i]);
        st = rvo_get_rv_ias15(np, pl, hill_factor, tb, nb, rv, NULL);
    }
    if (!st) {
        for (int i = 0; i < nb; i++) chi2b += ((rv[i] - rvb[i]) * (rv[i] - rvb[i])) / (eb[i] * eb[i]);
    }
    free(rv);
    if (st) {
        *logl = -INFINITY;
        return st;
    }
    const double lp = -((chi2b + chi2f) / npoints);
    if (!isfinite(lp)) {
        *logl = -INFINITY;
        return RVO_NONFINITE;
    }
    *logl = lp;
    return RVO_OK;
}

/* batch helper: W walkers, params [W][np][7] */
void rvo_logl_ias15_batch(int W, int np, const double* pl, int has_hk, int has_inc, double hill_factor,
                          const double* tf, const double* rvf, const double* ef, int nf, const double* tb,
                          const double* rvb, const double* eb, int nb, double npoints, double* logl, int32_t* status) {
    for (int w = 0; w < W; w++) {
        status[w] = rvo_logl_ias15(np, pl + (size_t)w * np * RVO_PSTRIDE, has_hk, has_inc, hill_factor, tf, rvf, ef,
                                   nf, tb, rvb, eb, nb, npoints, logl + w);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* Wisdom-Holman (WHFast-style) restatement of the HIP kernel's algorithm (T1 tier).           */
/*   Jacobi coordinates, Kepler drift (universal variables, Danby Stumpff functions),          */
/*   interaction kick, KDK, epoch-aligned segments: the segment between consecutive epochs     */
/*   (outward from t=0) of length D is cut into n = max(1, ceil(D/h - 1e-9)) equal steps,     */
/*   each step K(h/2) D(h) K(h/2) with interior half-kicks merged (the kernel evaluates the    */
/*   interaction at a segment's last positions once for the closing and the next segment's      */
/*   opening half kick; here both are evaluated: the same positions give the same values).      */
/*   Epochs with t>=0 are visited ascending from 0, t<0 descending from 0.                     */
/* ------------------------------------------------------------------------------------------ */
static void stumpff(double z, double* c0, double* c1, double* c2, double* c3) {
    int n = 0;
    while (fabs(z) > 0.1) {
        z *= 0.25;
        n++;
    }
    /* c2 = 1/2! - z/4! + z^2/6! ..., c3 = 1/3! - z/5! + ... */
    double s2 = 0.0, s3 = 0.0;
    {
        /* Horner from high order */
        const double f2[9] = {1.0 / 2, 1.0 / 24, 1.0 / 720, 1.0 / 40320, 1.0 / 3628800, 1.0 / 479001600,
                              1.0 / 87178291200.0, 1.0 / 20922789888000.0, 1.0 / 6402373705728000.0};
        const double f3[9] = {1.0 / 6, 1.0 / 120, 1.0 / 5040, 1.0 / 362880, 1.0 / 39916800, 1.0 / 6227020800.0,
                              1.0 / 1307674368000.0, 1.0 / 355687428096000.0, 1.0 / 121645100408832000.0};
        for (int j = 8; j >= 0; j--) {
            s2 = f2[j] - z * s2;
            s3 = f3[j] - z * s3;
        }
    }
    double C2 = s2, C3 = s3;
    double C1 = 1.0 - z * C3;
    double C0 = 1.0 - z * C2;
    for (; n > 0; n--) {
        z *= 4.0;
        C3 = (C2 + C0 * C3) * 0.25;
        C2 = C1 * C1 * 0.5;
        C1 = C0 * C1;
        C0 = 2.0 * C0 * C0 - 1.0;
    }
    *c0 = C0;
    *c1 = C1;
    *c2 = C2;
    *c3 = C3;
}

/* Bracketed universal-Kepler solve (the kernel's rare-case path): f(X) = r0 G1 + eta0 G2 + GM G3 - dt
 * increases with X and f(0) = -dt; double from dt/r0 until the sign changes, then Halley steps,
 * replaced by bisection when they leave the bracket, to full convergence. */
static double kepler_safe(double r0, double eta0, double zeta0, double beta, double GM, double dt) {
    const double sgn = dt >= 0.0 ? 1.0 : -1.0;
    double lo = 0.0, hi = dt / r0, c0, c1, c2, c3;
    for (int i = 0; i < 200; i++) {
        stumpff(beta * hi * hi, &c0, &c1, &c2, &c3);
        const double f = r0 * hi * c1 + eta0 * hi * hi * c2 + GM * hi * hi * hi * c3 - dt;
        if (sgn * f > 0.0 || f != f) break;
        lo = hi;
        hi *= 2.0;
    }
    double X = 0.5 * (lo + hi);
    for (int i = 0; i < 200; i++) {
        stumpff(beta * X * X, &c0, &c1, &c2, &c3);
        const double G1 = X * c1, G2 = X * X * c2, G3 = X * X * X * c3;
        const double f = r0 * G1 + eta0 * G2 + GM * G3 - dt;
        const double fp = r0 * c0 + eta0 * G1 + GM * G2;
        const double fpp = eta0 * c0 + zeta0 * G1;
        if (sgn * f > 0.0)
            hi = X;
        else
            lo = X;
        double Xn = X - f * fp / (fp * fp - 0.5 * f * fpp);
        if (!(sgn * (Xn - lo) > 0.0 && sgn * (hi - Xn) > 0.0)) Xn = 0.5 * (lo + hi);
        const int conv = !(fabs(Xn - X) > 2e-16 * fabs(Xn)) || lo == hi;
        X = Xn;
        if (conv) break;
    }
    return X;
}

/* universal-variable Kepler drift of (r, v) about mass GM by dt; returns 0 ok, 1 no convergence.
 * Small steps (|beta| (dt/r0)^2 <= 0.5): Halley from a Taylor guess; otherwise (or without
 * convergence in 8 iterations) the bracketed solve. */
static int kepler_drift(double GM, double* r, double* v, double dt) {
    const double r0 = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    const double v2 = v[0] * v[0] + v[1] * v[1] + v[2] * v[2];
    const double eta0 = r[0] * v[0] + r[1] * v[1] + r[2] * v[2];
    const double beta = 2.0 * GM / r0 - v2;
    const double zeta0 = GM - beta * r0;
    double X = dt / r0 - dt * dt * eta0 / (2.0 * r0 * r0 * r0);
    double c0, c1, c2, c3, G1 = 0, G2 = 0, G3 = 0, rr = r0;
    int ok = 0;
    const int small = fabs(beta) * (dt / r0) * (dt / r0) <= 0.5;
    if (small) {
        for (int it = 0; it < 8; it++) {
            stumpff(beta * X * X, &c0, &c1, &c2, &c3);
            G1 = X * c1;
            G2 = X * X * c2;
            G3 = X * X * X * c3;
            const double G0 = c0;
            const double f = r0 * G1 + eta0 * G2 + GM * G3 - dt;
            rr = r0 * G0 + eta0 * G1 + GM * G2;
            const double fpp = eta0 * G0 + zeta0 * G1;
            /* Halley */
            const double dX = f * rr / (rr * rr - 0.5 * f * fpp);
            X -= dX;
            if (fabs(dX) <= 2e-16 * fabs(X) || dX == 0.0) {
                ok = 1;
                break;
            }
        }
    }
    if (!ok) X = kepler_safe(r0, eta0, zeta0, beta, GM, dt);
    stumpff(beta * X * X, &c0, &c1, &c2, &c3);
    G1 = X * c1;
    G2 = X * X * c2;
    G3 = X * X * X * c3;
    rr = r0 * c0 + eta0 * G1 + GM * G2;
    const double f = 1.0 - GM * G2 / r0;
    const double g = dt - GM * G3;
    const double fd = -GM * G1 / (rr * r0);
    const double gd = 1.0 - GM * G2 / rr;
    for (int c = 0; c < 3; c++) {
        const double rn = f * r[c] + g * v[c];
        const double vn = fd * r[c] + gd * v[c];
        r[c] = rn;
        v[c] = vn;
    }
    return 0;
}

typedef struct {
    int np;
    double m[RVO_MAXB];  /* m[0] = star */
    double Mi[RVO_MAXB]; /* interior masses M_i = sum_{j<=i} m_j */
    double r[RVO_MAXB][3], v[RVO_MAXB][3]; /* Jacobi coordinates, index 1..np */
    double dmin2;
    int enc;
} wh_state;

static void wh_init(wh_state* s, int np, const double* pl, double hill_factor) {
    memset(s, 0, sizeof(*s));
    s->np = np;
    s->m[0] = 1.0;
    s->Mi[0] = 1.0;
    double helio_x[RVO_MAXB][3], helio_v[RVO_MAXB][3];
    double hill = 0.0;
    for (int i = 1; i <= np; i++) {
        const double* p = pl + RVO_PSTRIDE * (i - 1);
        s->m[i] = p[0];
        s->Mi[i] = s->Mi[i - 1] + p[0];
        pal_to_cart(1.0 + p[0], p[1], p[4], p[3], p[2], p[5], p[6], helio_x[i], helio_v[i]);
        const double rh = p[1] * pow(p[0] / 3.0, 1.0 / 3.0);
        if (rh > hill) hill = rh;
    }
    s->dmin2 = (hill_factor * hill) * (hill_factor * hill);
    /* heliocentric -> Jacobi: r'_i = x_i - (sum_{1<=j<i} m_j x_j)/M_{i-1}  (star at origin) */
    double sx[3] = {0, 0, 0}, sv[3] = {0, 0, 0};
    for (int i = 1; i <= np; i++) {
        for (int c = 0; c < 3; c++) {
            s->r[i][c] = helio_x[i][c] - sx[c] / s->Mi[i - 1];
            s->v[i][c] = helio_v[i][c] - sv[c] / s->Mi[i - 1];
        }
        for (int c = 0; c < 3; c++) {
            sx[c] += s->m[i] * helio_x[i][c];
            sv[c] += s->m[i] * helio_v[i][c];
        }
    }
}

static double wh_star_vx(const wh_state* s) {
    double vx = 0.0;
    for (int i = 1; i <= s->np; i++) vx -= (s->m[i] / s->Mi[i]) * s->v[i][0];
    return vx;
}

static int wh_drift(wh_state* s, double h) {
    int bad = 0;
    for (int i = 1; i <= s->np; i++) bad |= kepler_drift(s->Mi[i], s->r[i], s->v[i], h);
    return bad;
}

/* diagnostics: smallest pair-distance^2 / exit-distance^2 seen by wh_kick since the last reset */
static _Thread_local double g_min_ratio = 1e300; /* diagnostic, per calling thread */
double rvo_debug_min_ratio(int reset) {
    const double v = g_min_ratio;
    if (reset) g_min_ratio = 1e300;
    return v;
}

static void wh_kick(wh_state* s, double h) {
    const int np = s->np;
    double x[RVO_MAXB][3]; /* heliocentric positions, star at origin */
    double acc[RVO_MAXB][3];
    double cm[3] = {0, 0, 0};
    x[0][0] = x[0][1] = x[0][2] = 0.0;
    for (int i = 1; i <= np; i++) {
        for (int c = 0; c < 3; c++) x[i][c] = s->r[i][c] + cm[c] / s->Mi[i - 1];
        for (int c = 0; c < 3; c++) cm[c] += s->m[i] * x[i][c];
    }
    for (int i = 0; i <= np; i++) acc[i][0] = acc[i][1] = acc[i][2] = 0.0;
    for (int i = 0; i <= np; i++)
        for (int j = i + 1; j <= np; j++) {
            const double dx = x[j][0] - x[i][0], dy = x[j][1] - x[i][1], dz = x[j][2] - x[i][2];
            const double r2 = dx * dx + dy * dy + dz * dz;
            if (r2 < s->dmin2) s->enc = 1;
            if (s->dmin2 > 0.0 && r2 / s->dmin2 < g_min_ratio) g_min_ratio = r2 / s->dmin2;
            const double ir3 = 1.0 / (r2 * sqrt(r2));
            acc[i][0] += s->m[j] * ir3 * dx;
            acc[i][1] += s->m[j] * ir3 * dy;
            acc[i][2] += s->m[j] * ir3 * dz;
            acc[j][0] -= s->m[i] * ir3 * dx;
            acc[j][1] -= s->m[i] * ir3 * dy;
            acc[j][2] -= s->m[i] * ir3 * dz;
        }
    double ma[3] = {s->m[0] * acc[0][0], s->m[0] * acc[0][1], s->m[0] * acc[0][2]};
    for (int i = 1; i <= np; i++) {
        const double* r = s->r[i];
        const double rj2 = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
        const double kep = s->Mi[i] / (rj2 * sqrt(rj2));
        for (int c = 0; c < 3; c++) {
            const double aj = acc[i][c] - ma[c] / s->Mi[i - 1];
            s->v[i][c] += h * (aj + kep * r[c]);
        }
        for (int c = 0; c < 3; c++) ma[c] += s->m[i] * acc[i][c];
    }
}

/* Integrate one direction.  eps_abs[]: |t| of the epochs, ascending; sign = +1 or -1.
 * h_target > 0: nominal step.  Writes rv[i].  Returns status. */
static int wh_direction(int np, const double* pl, double hill_factor, const double* abs_t, int n, double sign,
                        double h_target, int sub, double* rv) {
    wh_state s;
    wh_init(&s, np, pl, hill_factor);
    {
        /* initial encounter check (REBOUND heartbeat before the first step) */
        wh_state tmp = s;
        wh_kick(&tmp, 0.0);
        if (tmp.enc) return RVO_ENCOUNTER;
    }
    double tprev = 0.0;
    for (int i = 0; i < n; i++) {
        const double D = abs_t[i] - tprev;
        tprev = abs_t[i];
        int n1 = (D > 0.0) ? (int)ceil(D / h_target - 1e-9) : 0;
        if (D > 0.0 && n1 < 1) n1 = 1;
        const int ns = n1 * sub;
        if (ns > 0) {
            /* the segment's base step, then the level's: (sign D / n1) * (1/sub) */
            const double h = (sign * D / n1) * (1.0 / sub);
            wh_kick(&s, 0.5 * h);
            for (int j = 0; j < ns; j++) {
                wh_drift(&s, h);
                wh_kick(&s, (j == ns - 1) ? 0.5 * h : h);
            }
        }
        if (s.enc) return RVO_ENCOUNTER;
        rv[i] = wh_star_vx(&s);
        if (!isfinite(rv[i])) return RVO_NONFINITE;
    }
    return RVO_OK;
}

/* RV at arbitrary epochs (any order/sign) with the WH algorithm; `sub` multiplies step counts.
 * order: scratch int[n].  Returns status. */
int rvo_wh_rv(int np, const double* pl, double hill_factor, const double* t, int n, double h_target, int sub,
              double* rv) {
    /* split by sign, sort by |t| */
    int* idx = (int*)malloc(sizeof(int) * (size_t)(n + 1));
    double* at = (double*)malloc(sizeof(double) * (size_t)(n + 1));
    double* out = (double*)malloc(sizeof(double) * (size_t)(n + 1));
    int st = RVO_OK;
    for (int dir = 0; dir < 2 && st == RVO_OK; dir++) {
        int cnt = 0;
        for (int i = 0; i < n; i++) {
            const int fwd = t[i] >= 0.0;
            if ((dir == 0) == fwd) idx[cnt++] = i;
        }
        /* insertion sort by |t| (stable) */
        for (int a = 1; a < cnt; a++) {
            const int key = idx[a];
            int b = a - 1;
            while (b >= 0 && fabs(t[idx[b]]) > fabs(t[key])) {
                idx[b + 1] = idx[b];
                b--;
            }
            idx[b + 1] = key;
        }
        for (int a = 0; a < cnt; a++) at[a] = fabs(t[idx[a]]);
        if (cnt) st = wh_direction(np, pl, hill_factor, at, cnt, dir == 0 ? 1.0 : -1.0, h_target, sub, out);
        for (int a = 0; a < cnt && st == RVO_OK; a++) rv[idx[a]] = out[a];
    }
    free(idx);
    free(at);
    free(out);
    return st;
}

int rvo_logl_wh(int np, const double* pl, int has_hk, int has_inc, double hill_factor, const double* t,
                const double* rvobs, const double* err, int n, double npoints, double h_target, int sub,
                double* logl) {
    if (rvo_prior_hard(np, pl, has_hk, has_inc)) {
        *logl = -INFINITY;
        return RVO_PRIOR;
    }
    double* rv = (double*)malloc(sizeof(double) * (size_t)(n + 1));
    int st = rvo_wh_rv(np, pl, hill_factor, t, n, h_target, sub, rv);
    double chi2 = 0.0;
    if (st == RVO_OK)
        for (int i = 0; i < n; i++) chi2 += (rv[i] - rvobs[i]) * (rv[i] - rvobs[i]) / (err[i] * err[i]);
    free(rv);
    if (st != RVO_OK) {
        *logl = -INFINITY;
        return st;
    }
    *logl = -(chi2 / npoints);
    if (!isfinite(*logl)) {
        *logl = -INFINITY;
        return RVO_NONFINITE;
    }
    return RVO_OK;
}

/* ------------------------------------------------------------------------------------------ */
/* Richardson-extrapolated WH, the kernel's full algorithm ("port" of rvm_logl_batch):          */
/*   level L (0-based) integrates with (L+1)x the level-1 steps; the model RV at each epoch is  */
/*   sum_L w_L rv_L with w the Lagrange-at-zero weights in x = 1/(L+1)^2; an encounter seen by   */
/*   any level marks the walker.                                                                */
/* ------------------------------------------------------------------------------------------ */
/* Lagrange-at-zero weights for an arbitrary multiplier sequence: level k steps dt/mult[k],
 * x_k = 1/mult[k]^2 (the harmonic default is mult = 1, 2, ..., nl). */
void rvo_richardson_weights_seq(int nl, const int* mult, double* w) {
    for (int k = 0; k < nl; k++) {
        const double xk = 1.0 / ((double)mult[k] * mult[k]);
        double wk = 1.0;
        for (int j = 0; j < nl; j++) {
            if (j == k) continue;
            const double xj = 1.0 / ((double)mult[j] * mult[j]);
            wk *= xj / (xj - xk);
        }
        w[k] = wk;
    }
}

void rvo_richardson_weights(int nl, double* w) {
    int mult[8];
    for (int k = 0; k < nl && k < 8; k++) mult[k] = k + 1;
    rvo_richardson_weights_seq(nl, mult, w);
}

int rvo_whx_rv_seq(int np, const double* pl, double hill_factor, const double* t, int n, double dt, int nl,
                   const int* mult, double* rv) {
    double w[8];
    rvo_richardson_weights_seq(nl, mult, w);
    double* tmp = (double*)malloc(sizeof(double) * (size_t)(n + 1));
    for (int i = 0; i < n; i++) rv[i] = 0.0;
    int st = RVO_OK;
    for (int k = 0; k < nl; k++) {
        const int s = rvo_wh_rv(np, pl, hill_factor, t, n, dt, mult[k], tmp);
        if (s != RVO_OK) {
            if (st == RVO_OK || s == RVO_ENCOUNTER) st = s;
            continue;
        }
        for (int i = 0; i < n; i++) rv[i] += w[k] * tmp[i];
    }
    free(tmp);
    return st;
}

int rvo_whx_rv(int np, const double* pl, double hill_factor, const double* t, int n, double dt, int nl,
               double* rv) {
    int mult[8];
    for (int k = 0; k < nl && k < 8; k++) mult[k] = k + 1;
    return rvo_whx_rv_seq(np, pl, hill_factor, t, n, dt, nl, mult, rv);
}

int rvo_logl_whx_seq(int np, const double* pl, int has_hk, int has_inc, double hill_factor, const double* t,
                     const double* rvobs, const double* err, int n, double npoints, double dt, int nl, const int* mult,
                     double* logl) {
    if (rvo_prior_hard(np, pl, has_hk, has_inc)) {
        *logl = -INFINITY;
        return RVO_PRIOR;
    }
    double* rv = (double*)malloc(sizeof(double) * (size_t)(n + 1));
    int st = rvo_whx_rv_seq(np, pl, hill_factor, t, n, dt, nl, mult, rv);
    double chi2 = 0.0;
    if (st == RVO_OK)
        for (int i = 0; i < n; i++) chi2 += ((rv[i] - rvobs[i]) * (rv[i] - rvobs[i])) / (err[i] * err[i]);
    free(rv);
    if (st != RVO_OK) {
        *logl = -INFINITY;
        return st;
    }
    *logl = -(chi2 / npoints);
    if (!isfinite(*logl)) {
        *logl = -INFINITY;
        return RVO_NONFINITE;
    }
    return RVO_OK;
}

int rvo_logl_whx(int np, const double* pl, int has_hk, int has_inc, double hill_factor, const double* t,
                 const double* rvobs, const double* err, int n, double npoints, double dt, int nl, double* logl) {
    int mult[8];
    for (int k = 0; k < nl && k < 8; k++) mult[k] = k + 1;
    return rvo_logl_whx_seq(np, pl, has_hk, has_inc, hill_factor, t, rvobs, err, n, npoints, dt, nl, mult, logl);
}

/* batch over walkers: params [W][np][7]; threads: OpenMP-free (callers parallelise if they wish) */
void rvo_logl_whx_batch(int W, int np, const double* pl, int has_hk, int has_inc, double hill_factor,
                        const double* t, const double* rvobs, const double* err, int n, double npoints, double dt,
                        int nl, double* logl, int32_t* status) {
    for (int w = 0; w < W; w++)
        status[w] = rvo_logl_whx(np, pl + (size_t)w * np * RVO_PSTRIDE, has_hk, has_inc, hill_factor, t, rvobs, err,
                                 n, npoints, dt, nl, logl + w);
}

void rvo_logl_whx_seq_batch(int W, int np, const double* pl, int has_hk, int has_inc, double hill_factor,
                            const double* t, const double* rvobs, const double* err, int n, double npoints, double dt,
                            int nl, const int* mult, double* logl, int32_t* status) {
    for (int w = 0; w < W; w++)
        status[w] = rvo_logl_whx_seq(np, pl + (size_t)w * np * RVO_PSTRIDE, has_hk, has_inc, hill_factor, t, rvobs,
                                     err, n, npoints, dt, nl, mult, logl + w);
}

/* ------------------------------------------------------------------------------------------ */
/* Adaptive resolution: restatement of the kernel's per-walker refinement (rvm_logl.hip         */
/* main pass + extension, rvm_refine.hip halving passes).  Each direction is      */
/* integrated with the plan's step; its extrapolation error is estimated by the change of chi2   */
/* when the coarsest level is dropped,                                                          */
/*   est = sum_i |(r_i - o_i)^2 - (r3_i - o_i)^2| / sigma_i^2 / npoints,                        */
/* r = all levels' Richardson RV, r3 = the finer nl - 1 levels' (their own Lagrange weights).   */
/* A direction above the bound (est > tol_dir, a non-finite pass, or past the eccentricity      */
/* guard) is OPEN:                                                                              */
/*  stage 1, the extension (ext_mult > 0): one more level, ext_mult steps per base step, joins  */
/*   the stored levels: r5 = Richardson over all nl + 1 levels.  Settled (chi2 from r5) when     */
/*     dd = sum |(r5 - o)^2 - (r - o)^2| / s2 <= EXT_ACCEPT * tol_dir * npoints                   */
/*   -- the change of chi2 the extension brought, an estimate of the main pass's own error (and  */
/*   a conservative one of r5's: measured, r5's error stays below 0.43 tol_dir wherever this     */
/*   holds at EXT_ACCEPT = 1 (2.6 tol_dir at 2, round 3));                          */
/*  stages 2..: passes with every step halved (level k: mult 2^rf steps per base step, rf = 1..  */
/*   rf_max) over every direction still open, until est <= tol_dir, or until the estimate stops   */
/*   falling (from rf = 2 on, est >= half the previous pass's: the roundoff floor of the finer     */
/*   steps) with the best pass's est <= FLOOR_BOUND * tol_dir -- the direction then keeps its best */
/*   pass (the smallest est); still open after rf_max: RVO_UNRESOLVED.                            */
/* The walker's two directions advance through the stages together (round 4): an encounter in   */
/* either ends the walker (ENCOUNTER), and the certain-reject test (a sampler's accept inputs    */
/* given: dmode 1 emcee stretch, 2 MH) runs on the WALKER after the extension stage and after    */
/* each halving stage while a direction is open: with each direction's lower bound on its chi2   */
/*   lb = max(0, chi2 - min(d, CUT_EST_FACTOR est_raw))                                          */
/* of an OPEN direction (chi2 of its last stage; d = the change that stage brought: the          */
/* extension's dd, a halving pass's step-doubling change from the previous pass's RV, none for   */
/* the main pass; est_raw = that stage's estimate -- the main pass's for the extension; lb = 0    */
/* after a non-finite pass) and lb = chi2 of a settled one, the walker stops when               */
/* its accept test fails even at lp_hi = -(lb_f + lb_b) / npoints and reports lp_hi (each        */
/* direction's chi2 := its lb): rejected whatever further passes would give.                    */
/* ecc_guard > 0: a walker with a planet of e > ecc_guard counts as open after the main pass     */
/* whatever its estimate (it gets the extension; the estimate under-reads there).               */
/* A non-finite main pass or extension (the fixed step blowing up on an extreme orbit) counts as   */
/* open (lb 0); a non-finite halving pass ends the walker NONFINITE (round 5).                    */
/* ------------------------------------------------------------------------------------------ */
enum { RVO_UNRESOLVED = 4 };
#ifndef EXT_ACCEPT /* (overridable for studies of the rule: -DEXT_ACCEPT=...) */
#define EXT_ACCEPT 1.0
#endif
#ifndef CUT_EST_FACTOR
#define CUT_EST_FACTOR 100.0
#endif
#ifndef FLOOR_BOUND
#define FLOOR_BOUND 4.0
#endif
/* (round 6) a walker whose pericentre passage is quicker still than the eccentricity guard's --    */
/* (1 - e) below CUT_ECC_FACTOR x (1 - ecc_guard) -- keeps the main pass's bound after the extension: */
/* the extension's change does not bound its error there (rvm_internal.h RVM_CUT_ECC_FACTOR)         */
#ifndef CUT_ECC_FACTOR
#define CUT_ECC_FACTOR 0.6712
#endif


static double margin_of(double x, double bound) {
    return bound > 0.0 ? fabs(x / bound - 1.0) : INFINITY;
}

typedef struct {
    int mode; /* 0 none, 1 emcee stretch, 2 MH */
    int dim;
    double z, u, lnp0;
} rvo_decide;

/* the sampler's accept test at lp (rvm_stretch.h stretch_accepts / mh_accepts) */
static int decide_accepts(const rvo_decide* dc, double lp) {
    if (dc->mode == 1) return (double)(dc->dim - 1) * log(dc->z) + lp - dc->lnp0 > log(dc->u);
    return exp(lp - dc->lnp0) > dc->u;
}

/* the plan shared by both directions of a walker */
typedef struct {
    int np;
    const double* pl;
    double hill_factor, dt, tol_dir, npoints, ecc_guard, e2_cut;
    int nl, ext_mult, rf_max, adaptive, ext;
    const int* mult;
    double w[8], w3[8], w5[9];
} rvo_plan_ctx;

/* one direction's inputs, scratch and refinement state */
typedef struct {
    const double *at, *ob, *s2;
    int cnt;
    double sign;
    double *lv0, *lv, *prev; /* main pass's levels (+ the extension), a halving pass's, the last RV */
    int st, open, bad, stage, cut, floor, pend;
    double chi2, lb, est, est_raw, margin;
    double pest, best, bchi; /* the previous halving pass's est, the smallest est and its chi2 */
    double dext;             /* the extension's change dd / npoints (0: none) */
} rvo_dir;

/* (study, scripts/probe/encounter_confirm_study.py; 0 = the product rule): 1 = an encounter the main
 * pass's finest level sees does not end the walker either, 2 = besides, a halving pass's encounter
 * ends it only when the stage before it saw one too (a finer pass confirms), 3 = rule 1 and the
 * extension's encounter refines on too (halving passes end it), 4 = rule 3 and a halving pass's
 * encounter ends it only when the halving pass before it saw one too */
static int enc_confirm = 0;
void rvo_study_set_enc_confirm(int r) { enc_confirm = r; }
/* (study, scripts/probe/cut_guard_study.py: the cut guard's factor; < 0 = CUT_ECC_FACTOR, 0 = no guard) */
static double study_cut_factor = -1.0;
void rvo_study_set_cut_factor(double f) { study_cut_factor = f; }
/* past the cut guard the bound after the extension is chi2 - min(CUT_GUARD_K d, 100 est) (rvm_internal.h
 * RVM_CUT_GUARD_K): the three wrong cuts of tests/test_cut_guard.py had d a third of the error; the study
 * setter overrides it (0 = chi2 - 100 est, the first form of the guard) */
#ifndef CUT_GUARD_K
#define CUT_GUARD_K 10.0
#endif
static double study_guard_k = CUT_GUARD_K;
void rvo_study_set_guard_k(double k) { study_guard_k = k; }
/* (study: past the guard, pass 1's change d2 measured against the extension's RV, not the main pass's) */
static int study_prev_ext = 0;
void rvo_study_set_prev_ext(int on) { study_prev_ext = on; }

static double lb_of(double chi2, double d, double est_raw) {
    const double b = chi2 - fmin(d, CUT_EST_FACTOR * est_raw);
    return b > 0.0 ? b : 0.0;
}

/* stage 0: the plan's step */
static void dir_main(const rvo_plan_ctx* X, rvo_dir* D) {
    int st = RVO_OK, coarse = 0;
    int kf = 0; /* the finest level (largest multiplier) */
    for (int k = 1; k < X->nl; k++)
        if (X->mult[k] > X->mult[kf]) kf = k;
    for (int k = 0; k < X->nl; k++) {
        const int s = wh_direction(X->np, X->pl, X->hill_factor, D->at, D->cnt, D->sign, X->dt, X->mult[k],
                                   D->lv0 + (size_t)k * D->cnt);
        /* (round 5) adaptive: an encounter only a coarser level sees does not end the walker -- the
         * coarse levels' positions near a close approach are the least accurate -- the direction is
         * refined instead, its main pass treated like a non-finite one (rvm_logl.hip `cenc`) */
        if (s == RVO_ENCOUNTER && X->adaptive && (k != kf || enc_confirm)) {
            coarse = 1;
            D->pend = 1;
            continue;
        }
        if (s != RVO_OK && (st == RVO_OK || s == RVO_ENCOUNTER)) st = s;
    }
    if (st == RVO_ENCOUNTER || (st != RVO_OK && !X->adaptive)) {
        D->st = st;
        return;
    }
    D->bad = st != RVO_OK || coarse;
    if (D->bad) {
        D->chi2 = D->est = D->est_raw = NAN;
        D->lb = 0.0;
        for (int i = 0; i < D->cnt; i++) D->prev[i] = NAN;
        D->open = 1;
        return;
    }
    double chi2 = 0.0, est = 0.0;
    for (int i = 0; i < D->cnt; i++) {
        double r = 0.0, r3 = 0.0;
        for (int k = 0; k < X->nl; k++) r += X->w[k] * D->lv0[(size_t)k * D->cnt + i];
        for (int k = 1; k < X->nl; k++) r3 += X->w3[k] * D->lv0[(size_t)k * D->cnt + i];
        chi2 += (r - D->ob[i]) * (r - D->ob[i]) / D->s2[i];
        est += fabs((r - r3) * ((r - D->ob[i]) + (r3 - D->ob[i]))) / D->s2[i];
        D->prev[i] = r;
    }
    D->chi2 = chi2;
    D->est_raw = est;
    D->est = est / X->npoints;
    D->lb = chi2;
    if (!X->adaptive) return;
    if (margin_of(D->est, X->tol_dir) < D->margin) D->margin = margin_of(D->est, X->tol_dir);
    /* the eccentricity guard: an orbit whose pericentre passage is much quicker than the plan's
     * reference orbit always gets the extension (the estimate can miss there) */
    int eflag = 0;
    if (X->ext && X->ecc_guard > 0.0) {
        double e2 = 0.0;
        for (int p = 0; p < X->np; p++) {
            const double h = X->pl[p * RVO_PSTRIDE + 2], k = X->pl[p * RVO_PSTRIDE + 3];
            if (h * h + k * k > e2) e2 = h * h + k * k;
        }
        eflag = e2 > X->ecc_guard * X->ecc_guard;
        const double mg = margin_of(e2, X->ecc_guard * X->ecc_guard);
        if (mg < D->margin) D->margin = mg;
    }
    D->open = D->est > X->tol_dir || eflag;
    if (D->open) D->lb = lb_of(chi2, INFINITY, est);
}

/* stage 1: the extension level joined to the main pass's levels */
static void dir_extend(const rvo_plan_ctx* X, rvo_dir* D) {
    D->stage = 1;
    double* lx = D->lv0 + (size_t)X->nl * D->cnt;
    const int sx = wh_direction(X->np, X->pl, X->hill_factor, D->at, D->cnt, D->sign, X->dt, X->ext_mult, lx);
    if (sx == RVO_ENCOUNTER && enc_confirm >= 3) {
        D->pend = 1; /* (study) */
        return;
    }
    if (sx == RVO_ENCOUNTER) {
        D->st = sx;
        D->open = 0;
        return;
    }
    if (sx != RVO_OK || D->bad) return; /* (refines on; lb as the main pass left it) */
    double c5 = 0.0, dd = 0.0;
    for (int i = 0; i < D->cnt; i++) {
        double r = 0.0, r5 = 0.0;
        for (int k = 0; k < X->nl; k++) r += X->w[k] * D->lv0[(size_t)k * D->cnt + i];
        for (int k = 0; k < X->nl; k++) r5 += X->w5[k] * D->lv0[(size_t)k * D->cnt + i];
        r5 += X->w5[X->nl] * lx[i];
        const double q = r5 - D->ob[i];
        c5 += (q * q) / D->s2[i];
        dd += fabs((r5 - r) * (q + (r - D->ob[i]))) / D->s2[i];
    }
    if (!isfinite(c5) || !isfinite(dd)) return; /* (refines on; lb as the main pass left it) */
    const double bx = EXT_ACCEPT * X->tol_dir * X->npoints;
    if (margin_of(dd, bx) < D->margin) D->margin = margin_of(dd, bx);
    D->chi2 = c5;
    D->dext = dd / X->npoints;
    if (dd <= bx) {
        D->est = dd / X->npoints;
        D->open = 0;
        D->lb = c5;
    } else if (X->e2_cut < INFINITY) {
        /* (past the cut guard the bound stays the main pass's) */
        double e2 = 0.0;
        for (int p = 0; p < X->np; p++) {
            const double h = X->pl[p * RVO_PSTRIDE + 2], k = X->pl[p * RVO_PSTRIDE + 3];
            if (h * h + k * k > e2) e2 = h * h + k * k;
        }
        if (margin_of(e2, X->e2_cut) < D->margin) D->margin = margin_of(e2, X->e2_cut);
        if (e2 <= X->e2_cut) D->lb = lb_of(c5, dd, D->est_raw);
        else if (study_guard_k > 0.0) D->lb = lb_of(c5, study_guard_k * dd, D->est_raw); /* (CUT_GUARD_K) */
        if (e2 > X->e2_cut && study_prev_ext) /* (study: pass 1's change measured against the extension) */
            for (int i = 0; i < D->cnt; i++) {
                double r5 = X->w5[X->nl] * lx[i];
                for (int k = 0; k < X->nl; k++) r5 += X->w5[k] * D->lv0[(size_t)k * D->cnt + i];
                D->prev[i] = r5;
            }
    } else {
        D->lb = lb_of(c5, dd, D->est_raw);
    }
}

/* stage 1 + rf: every step halved rf times */
static void dir_halve(const rvo_plan_ctx* X, rvo_dir* D, int rf) {
    D->stage = (X->ext ? 1 : 0) + rf;
    int st = RVO_OK;
    for (int k = 0; k < X->nl; k++) {
        const int s = wh_direction(X->np, X->pl, X->hill_factor, D->at, D->cnt, D->sign, X->dt, X->mult[k] << rf,
                                   D->lv + (size_t)k * D->cnt);
        if (s != RVO_OK && (st == RVO_OK || s == RVO_ENCOUNTER)) st = s;
    }
    if (st == RVO_ENCOUNTER && rf < X->rf_max &&
        ((enc_confirm == 2 && !D->pend) || (enc_confirm == 4 && D->pend != 2))) {
        D->pend = 2; /* (study: a finer pass must confirm it) */
        D->chi2 = D->est = D->est_raw = NAN;
        D->lb = 0.0;
        D->pest = INFINITY;
        for (int i = 0; i < D->cnt; i++) D->prev[i] = NAN;
        return;
    }
    if (st == RVO_ENCOUNTER) {
        D->st = st;
        D->open = 0;
        return;
    }
    D->pend = 0;
    if (st != RVO_OK) { /* a non-finite halving pass ends the walker (round 5, ADVICE r4: refining on */
        D->st = RVO_NONFINITE; /* would run the last pass at 2^rf_max x the base steps) */
        D->open = 0;
        return;
    }
    double c2 = 0.0, e2 = 0.0, d2 = 0.0;
    for (int i = 0; i < D->cnt; i++) {
        double r = 0.0, r3 = 0.0;
        for (int k = 0; k < X->nl; k++) r += X->w[k] * D->lv[(size_t)k * D->cnt + i];
        for (int k = 1; k < X->nl; k++) r3 += X->w3[k] * D->lv[(size_t)k * D->cnt + i];
        c2 += (r - D->ob[i]) * (r - D->ob[i]) / D->s2[i];
        e2 += fabs((r - r3) * ((r - D->ob[i]) + (r3 - D->ob[i]))) / D->s2[i];
        d2 += fabs((r - D->prev[i]) * ((r - D->ob[i]) + (D->prev[i] - D->ob[i]))) / D->s2[i];
        D->prev[i] = r;
    }
    D->chi2 = c2;
    D->est_raw = e2;
    D->est = e2 / X->npoints;
    const int fin = isfinite(c2) && isfinite(e2);
    if (!fin) { /* (finite RVs whose sums overflow: non-finite all the same) */
        D->st = RVO_NONFINITE;
        D->open = 0;
        return;
    }
    if (margin_of(D->est, X->tol_dir) < D->margin) D->margin = margin_of(D->est, X->tol_dir);
    const int stall = fin && rf >= 2 && !(D->est < 0.5 * D->pest);
    if (fin && rf >= 2 && D->best <= FLOOR_BOUND * X->tol_dir && D->est > X->tol_dir &&
        margin_of(D->est, 0.5 * D->pest) < D->margin)
        D->margin = margin_of(D->est, 0.5 * D->pest); /* (the floor decision, when it could matter) */
    if (fin && D->est < D->best) {
        D->best = D->est;
        D->bchi = c2;
    }
    D->pest = fin ? D->est : INFINITY;
    if (!(D->est > X->tol_dir)) {
        D->open = 0;
        D->lb = c2;
    } else if (stall && D->best <= FLOOR_BOUND * X->tol_dir) { /* the roundoff floor: the best pass */
        D->open = 0;
        D->floor = 1;
        D->chi2 = D->lb = D->bchi;
        D->est = D->best;
    } else {
        D->lb = lb_of(c2, d2, e2); /* (d2 NaN after a non-finite pass: fmin takes the estimate) */
    }
}

/* the walker's certain-reject test; returns 1 (and stops every direction) on a cut */
static int walker_cut(const rvo_plan_ctx* X, rvo_dir* D, const rvo_decide* dc) {
    if (dc == NULL || dc->mode == 0 || X->ext_mult <= 0) return 0;
    const double lp_hi = -((D[0].lb + D[1].lb) / X->npoints);
    if (!isfinite(lp_hi)) return 0;
    const double lnpdiff = dc->mode == 1 ? (double)(dc->dim - 1) * log(dc->z) + lp_hi - dc->lnp0 : lp_hi - dc->lnp0;
    const double lu = log(dc->u);
    const double mg = fabs(lnpdiff - lu) / (1.0 + fabs(lu));
    for (int d = 0; d < 2; d++)
        if (mg < D[d].margin) D[d].margin = mg;
    if (decide_accepts(dc, lp_hi)) return 0;
    for (int d = 0; d < 2; d++) {
        D[d].cut = D[d].open;
        D[d].open = 0;
        D[d].chi2 = D[d].lb;
    }
    return 1;
}

static int any_enc(const rvo_dir* D) { return D[0].st == RVO_ENCOUNTER || D[1].st == RVO_ENCOUNTER; }
/* a direction whose halving pass ended the walker: an encounter or a non-finite pass */
static int any_end(const rvo_dir* D) {
    return any_enc(D) || D[0].st == RVO_NONFINITE || D[1].st == RVO_NONFINITE;
}
static int any_open(const rvo_dir* D) { return D[0].open || D[1].open; }

/* logp with adaptive resolution: rf_used[2] / est[2] (fwd, bwd) report the stage reached (0 the
 * plan's step, 1 the extension, 2.. halvings; without the extension 1.. halvings) and
 * the final estimates.  Status: PRIOR, else the forward direction's non-OK status, else the
 * backward one's (the kernel's direction meeting).  est[4]: the final estimates (fwd, bwd) and the
 * closest any decision came to its bound, min |x / bound - 1| (fwd, bwd): a decision a second
 * implementation may take the other way when that is at roundoff level.  cut[2]: the directions
 * a certain reject stopped. */
int rvo_logl_whx_adapt(int np, const double* pl, int has_hk, int has_inc, double hill_factor, const double* t,
                       const double* rvobs, const double* err, int n, double npoints, double dt, int nl,
                       const int* mult, int ext_mult, double tol_dir, int rf_max, const rvo_decide* dc,
                       double ecc_guard, double* logl, int32_t* rf_used, double* est, int32_t* cut) {
    rf_used[0] = rf_used[1] = 0;
    cut[0] = cut[1] = 0;
    est[0] = est[1] = 0.0;
    est[2] = est[3] = INFINITY;
    if (rvo_prior_hard(np, pl, has_hk, has_inc)) {
        *logl = -INFINITY;
        return RVO_PRIOR;
    }
    rvo_plan_ctx X;
    memset(&X, 0, sizeof X);
    X.np = np;
    X.pl = pl;
    X.hill_factor = hill_factor;
    X.dt = dt;
    X.tol_dir = tol_dir;
    X.npoints = npoints;
    X.ecc_guard = ecc_guard;
    {
        const double ec = 1.0 - (1.0 - ecc_guard) * (study_cut_factor >= 0.0 ? study_cut_factor : CUT_ECC_FACTOR);
        X.e2_cut = ecc_guard > 0.0 ? ec * ec : INFINITY;
    }
    X.nl = nl;
    X.mult = mult;
    X.rf_max = rf_max;
    X.adaptive = nl >= 2 && tol_dir < INFINITY;
    X.ext = ext_mult > 0 && rf_max > 0 && nl >= 2 && nl < 8;
    X.ext_mult = X.ext ? ext_mult : 0;
    rvo_richardson_weights_seq(nl, mult, X.w);
    if (nl >= 2) rvo_richardson_weights_seq(nl - 1, mult + 1, X.w3 + 1);
    if (X.ext) {
        int m5[9];
        for (int k = 0; k < nl; k++) m5[k] = mult[k];
        m5[nl] = ext_mult;
        rvo_richardson_weights_seq(nl + 1, m5, X.w5);
    }
    int* idx = (int*)malloc(sizeof(int) * (size_t)(n + 1));
#ifdef JUMP_T
    int jumped = 0;
#endif
    rvo_dir D[2];
    memset(D, 0, sizeof D);
    double* buf[2];
    for (int dir = 0; dir < 2; dir++) {
        int cnt = 0;
        for (int i = 0; i < n; i++)
            if ((dir == 0) == (t[i] >= 0.0)) idx[cnt++] = i;
        for (int a = 1; a < cnt; a++) { /* stable insertion sort by |t| */
            const int key = idx[a];
            int b = a - 1;
            while (b >= 0 && fabs(t[idx[b]]) > fabs(t[key])) {
                idx[b + 1] = idx[b];
                b--;
            }
            idx[b + 1] = key;
        }
        /* |t|, observed RV, sigma^2; the main pass's levels (+ the extension), a halving pass's
         * levels, the last pass's RV */
        buf[dir] = (double*)malloc(sizeof(double) * (size_t)((4 + 2 * nl + 1) * cnt + 1));
        double* A = buf[dir];
        double* ob = A + cnt;
        double* s2 = ob + cnt;
        for (int a = 0; a < cnt; a++) {
            A[a] = fabs(t[idx[a]]);
            ob[a] = rvobs[idx[a]];
            s2[a] = err[idx[a]] * err[idx[a]];
        }
        rvo_dir* d = &D[dir];
        d->at = A;
        d->ob = ob;
        d->s2 = s2;
        d->cnt = cnt;
        d->sign = dir == 0 ? 1.0 : -1.0;
        d->lv0 = s2 + cnt;
        d->lv = d->lv0 + (size_t)(nl + 1) * cnt;
        d->prev = d->lv + (size_t)nl * cnt;
        d->st = RVO_OK;
        d->margin = INFINITY;
        d->pest = d->best = INFINITY;
    }
    for (int dir = 0; dir < 2; dir++)
        if (D[dir].cnt) dir_main(&X, &D[dir]);
    if (!any_enc(D) && X.ext) {
        for (int dir = 0; dir < 2 && !any_enc(D); dir++)
            if (D[dir].open) dir_extend(&X, &D[dir]);
    }
    if (!any_enc(D) && X.adaptive) {
        int rf = 0;
#ifdef JUMP_T /* (study build: a walker whose extension changed an open direction by more than
                 JUMP_T x tol_dir starts its halving passes at rf = 2) */
        for (int dir = 0; dir < 2; dir++)
            if (D[dir].open && D[dir].dext > JUMP_T * X.tol_dir) rf = 1;
        jumped = rf;
#endif
        while (any_open(D) && !walker_cut(&X, D, dc)) {
            if (rf == rf_max) {
                for (int dir = 0; dir < 2; dir++)
                    if (D[dir].open) D[dir].st = RVO_UNRESOLVED;
                break;
            }
            rf++;
            for (int dir = 0; dir < 2 && !any_end(D); dir++)
                if (D[dir].open) dir_halve(&X, &D[dir], rf);
            if (any_end(D)) break;
        }
    }
    for (int dir = 0; dir < 2; dir++) {
        cut[dir] = D[dir].cut;
#ifdef JUMP_T
        if (jumped) cut[dir] |= 2; /* (study build: the walker started at rf = 2) */
#endif
        rf_used[dir] = D[dir].stage;
        est[dir] = D[dir].est;
        est[2 + dir] = D[dir].margin;
    }
    free(idx);
    free(buf[0]);
    free(buf[1]);
    int st = D[0].st != RVO_OK ? D[0].st : D[1].st;
    const double lp = -((D[1].chi2 + D[0].chi2) / npoints);
    if (st == RVO_OK && !isfinite(lp)) st = RVO_NONFINITE;
    *logl = st == RVO_OK ? lp : -INFINITY;
    return st;
}

void rvo_logl_whx_adapt_batch(int W, int np, const double* pl, int has_hk, int has_inc, double hill_factor,
                              const double* t, const double* rvobs, const double* err, int n, double npoints,
                              double dt, int nl, const int* mult, int ext_mult, double tol_dir, int rf_max,
                              const int32_t* dmode, int dim, const double* dz, const double* du, const double* dlnp0,
                              double ecc_guard, double* logl, int32_t* status, int32_t* rf_used, double* est,
                              int32_t* cut) {
    for (int w = 0; w < W; w++) {
        rvo_decide dc = {dmode ? dmode[w] : 0, dim, dz ? dz[w] : 1.0, du ? du[w] : 0.5, dlnp0 ? dlnp0[w] : 0.0};
        status[w] = rvo_logl_whx_adapt(np, pl + (size_t)w * np * RVO_PSTRIDE, has_hk, has_inc, hill_factor, t, rvobs,
                                       err, n, npoints, dt, nl, mult, ext_mult, tol_dir, rf_max, &dc, ecc_guard, logl + w,
                                       rf_used + 2 * w, est + 4 * w, cut + 2 * w);
    }
}

/* Sanitizer driver for the CPU oracle (test infrastructure): exercises the restatements on a
 * few walkers (S2-like two-planet states, a prior-rejected state, a close pair, an inclined state)
 * under AddressSanitizer + UndefinedBehaviorSanitizer.  Built by `make -C oracle sanitize`, run by
 * tests/test_sanitizers.py (sanitizers on the host-side code). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>

int rvo_prior_hard(int np, const double* pl, int has_hk, int has_inc);
void rvo_setup_vectors(int np, const double* pl, double* helio_xv, double* bary_xv);
void rvo_logl_ias15_batch(int W, int np, const double* pl, int has_hk, int has_inc, double hill_factor,
                          const double* tf, const double* rvf, const double* ef, int nf, const double* tb,
                          const double* rvb, const double* eb, int nb, double npoints, double* logl, int32_t* status);
void rvo_logl_whx_seq_batch(int W, int np, const double* pl, int has_hk, int has_inc, double hill_factor,
                            const double* t, const double* rvobs, const double* err, int n, double npoints, double dt,
                            int nl, const int* mult, double* logl, int32_t* status);

#define NF 6
#define NB 5
int main(void) {
    /* [W][np][7]: m a h k l ix iy */
    double pl[4][2][7] = {
        {{1.2e-3, 0.88, 0.218, 0.015, 0.3, 0, 0}, {2.1e-3, 1.55, 0.16, 0.02, 2.2, 0, 0}},
        {{1.2e-3, 0.01, 0.218, 0.015, 0.3, 0, 0}, {2.1e-3, 1.55, 0.16, 0.02, 2.2, 0, 0}}, /* prior: a <= 0.02 */
        {{1.2e-3, 0.88, 0.0, 0.0, 0.3, 0, 0}, {2.1e-3, 0.89, 0.0, 0.0, 0.3, 0, 0}},       /* encounter */
        {{1.2e-3, 0.88, 0.218, 0.015, 0.3, 0.05, -0.03}, {2.1e-3, 1.55, 0.16, 0.02, 2.2, 0.06, -0.03}}};
    double tf[NF] = {0.0, 0.7, 1.9, 3.1, 4.0, 6.2}, tb[NB] = {-0.5, -1.4, -2.2, -3.9, -5.0};
    double rvf[NF], rvb[NB], ef[NF], eb[NB], t[NF + NB], rv[NF + NB], er[NF + NB];
    for (int i = 0; i < NF; i++) rvf[i] = 1e-4 * sin(i), ef[i] = 1.5e-4, t[i] = tf[i], rv[i] = rvf[i], er[i] = ef[i];
    for (int i = 0; i < NB; i++)
        rvb[i] = -1e-4 * cos(i), eb[i] = 1.6e-4, t[NF + i] = tb[i], rv[NF + i] = rvb[i], er[NF + i] = eb[i];
    double helio[3 * 6], bary[3 * 6], logl[4];
    int32_t st[4];
    rvo_setup_vectors(2, &pl[0][0][0], helio, bary);
    int bad = rvo_prior_hard(2, &pl[1][0][0], 1, 0) == 0;
    rvo_logl_ias15_batch(4, 2, &pl[0][0][0], 1, 1, 1.0, tf, rvf, ef, NF, tb, rvb, eb, NB, 100.0, logl, st);
    bad |= st[0] != 0 || st[1] != 1 || st[2] != 2 || st[3] != 0 || !isfinite(logl[0]);
    const int mult[4] = {4, 5, 6, 7};
    double logl2[4];
    int32_t st2[4];
    rvo_logl_whx_seq_batch(4, 2, &pl[0][0][0], 1, 1, 1.0, t, rv, er, NF + NB, 100.0, 0.65, 4, mult, logl2, st2);
    bad |= st2[0] != 0 || st2[1] != 1 || st2[2] != 2 || fabs(logl2[0] - logl[0]) > 1e-6;
    printf("ias15 %.12g %.12g | whx %.12g %.12g | status %d %d %d %d\n", logl[0], logl[3], logl2[0], logl2[3], st[0],
           st[1], st[2], st[3]);
    return bad;
}

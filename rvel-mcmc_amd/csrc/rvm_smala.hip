// rvm_smala.hip -- device SMALA (simplified manifold MALA, SoftAbs metric), mcmc.py:126-187.
//
// Per step and chain the reference (mcmc.py:144-187) needs logp, its gradient and Hessian, the
// SoftAbs metric G = Q diag(lambda coth(alpha lambda)) Q^T of eig(-H) (mcmc.py:135-139), its
// inverse and the Cholesky factor of the inverse (the proposal's covariance eps^2 G^-1), the drift
// mu = x + eps^2/2 G^-1 grad, and the Gaussian q-ratio of the proposal.  Derivatives come from one
// likelihood launch over the central-difference stencil (rvm_fd_params): the gradient from the
// stencil's logp, the Gauss-Newton Hessian H = -(2/N) J^T diag(1/sigma^2) J from its per-epoch
// model RVs (rv_out).  Everything after the launch happens here; the per-chain math runs one
// wave per chain with the chain's P x P matrices in LDS:
//
//   smala_derive_kernel   stencil -> lp, grad, mu, chol(G^-1), G, log det G^-1, ok
//                         (cyclic Jacobi eigen-solver for the symmetric P x P -H, rows on lanes)
//   smala_propose_kernel  x* = mu + eps chol(G^-1) z          (z: Philox Box-Muller or injected)
//   smala_accept_kernel   q-ratio, accept, copy the proposal's cached derivatives on accept
//
// Compiled without FMA contraction like the other sampler kernels.
#include <hip/hip_runtime.h>
#include <math.h>

#include "rvm_device.h"
#include "rvm_internal.h"

#pragma clang fp contract(off)

namespace rvm {

enum : uint32_t {
    RNG_SMALA_PROPOSE = 5,
    RNG_SMALA_ACCEPT = 6,
};

// butterfly sum over the wave: every lane ends with the same bits (each step adds the same pair)
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// From A = -H (P x P in LDS), the gradient gr and the point xv: SoftAbs metric of A by the
// cyclic Jacobi eigen-solver, G, G^-1, the drift, the Cholesky factor of G^-1 and log det G^-1
// into the chain's cache (mcmc.py:135-150).  One wave per chain; the arrays are the caller's LDS.
__device__ __forceinline__ void smala_metric_stage(int P, int C, int c, int lane, double* A, double* Qm, double* gr,
                                                   double* xv, double* lt, double* inv, double* ra, double* rb,
                                                   double* dn, int* rp, int& okflag, double lp_c, double alpha,
                                                   double eps, const SmalaCache& out) {
    constexpr int PM = RVM_SMALA_MAX_PARAMS;
    const int ntri = P * (P + 1) / 2;
    for (int i = lane; i < P * P; i += 64) Qm[i] = (i / P == i % P) ? 1.0 : 0.0;
    __syncthreads();
    // Jacobi eigen-solver, parallel (round-robin) ordering: A -> diag(lambda), Q -> eigenvectors
    // (A = Q diag(lambda) Q^T).  A sweep is N2-1 rounds (N2 = P rounded up to even); each round
    // applies N2/2 disjoint rotations at once (pair (p, q) zeroes A_pq as in the classic cyclic
    // method), so a sweep costs N2-1 barrier rounds instead of P(P-1)/2 sequential rotations.
    // Lanes own matrix entries: A' = J^T A J and Q' = Q J entry by entry, column i of J being
    // ra[i] e_i + rb[i] e_rp[i].
    {
        constexpr int EPL = (PM * PM + 63) / 64;  // matrix entries per lane
        const int N2 = (P + 1) & ~1;
        const int PP = P * P;
        for (int sweep = 0; sweep < 60; sweep++) {
            double off = 0.0, dia = 0.0;
            for (int idx = lane; idx < PP; idx += 64) {
                const int i = idx / P, j = idx - (idx / P) * P;
                const double v = A[idx];
                if (i == j) dia += v * v;
                else if (i < j) off += v * v;
            }
            off = wave_sum(off);
            dia = wave_sum(dia);
            if (!(off > 1e-32 * dia)) break;  // converged (or NaN: caught by the SoftAbs check)
            for (int r = 0; r < N2 - 1; r++) {
                if (lane < N2 / 2) {
                    int a, b;
                    if (lane == 0) {
                        a = r;
                        b = N2 - 1;
                    } else {
                        a = (r + lane) % (N2 - 1);
                        b = (r - lane + N2 - 1) % (N2 - 1);
                    }
                    const int p = a < b ? a : b, q = a < b ? b : a;
                    if (q < P) {
                        const double apq = A[p * P + q], app = A[p * P + p], aqq = A[q * P + q];
                        double cs = 1.0, sn = 0.0, tt = 0.0;
                        if (apq != 0.0) {
                            const double theta = (aqq - app) / (2.0 * apq);
                            tt = 1.0 / (fabs(theta) + sqrt(theta * theta + 1.0));
                            if (theta < 0.0) tt = -tt;
                            cs = 1.0 / sqrt(tt * tt + 1.0);
                            sn = tt * cs;
                        }
                        ra[p] = cs;
                        rb[p] = -sn;
                        rp[p] = q;
                        ra[q] = cs;
                        rb[q] = sn;
                        rp[q] = p;
                        dn[p] = app - tt * apq;
                        dn[q] = aqq + tt * apq;
                    } else if (p < P) {  // paired with the padding index: untouched this round
                        ra[p] = 1.0;
                        rb[p] = 0.0;
                        rp[p] = p;
                        dn[p] = A[p * P + p];
                    }
                }
                __syncthreads();
                double na[EPL], nq[EPL];
#pragma unroll
                for (int k = 0; k < EPL; k++) {
                    const int idx = lane + 64 * k;
                    if (idx < PP) {
                        const int i = idx / P, j = idx - (idx / P) * P;
                        const int ip = rp[i], jp = rp[j];
                        const double ai = ra[i], bi = rb[i], aj = ra[j], bj = rb[j];
                        if (i == j)
                            na[k] = dn[i];
                        else if (ip == j)
                            na[k] = 0.0;  // the pair this round zeroes
                        else
                            na[k] = ((ai * aj) * A[i * P + j] + (ai * bj) * A[i * P + jp]) +
                                    ((bi * aj) * A[ip * P + j] + (bi * bj) * A[ip * P + jp]);
                        nq[k] = aj * Qm[i * P + j] + bj * Qm[i * P + jp];
                    }
                }
                __syncthreads();
#pragma unroll
                for (int k = 0; k < EPL; k++) {
                    const int idx = lane + 64 * k;
                    if (idx < PP) {
                        A[idx] = na[k];
                        Qm[idx] = nq[k];
                    }
                }
                __syncthreads();
            }
        }
    }
    // SoftAbs (mcmc.py:135-139): lambda~ = lambda coth(alpha lambda), 1/alpha where |alpha lambda| < 1e-8
    if (lane < P) {
        const double lam = A[lane * P + lane];
        const double al = alpha * lam;
        const double l = fabs(al) < 1e-8 ? 1.0 / alpha : lam / tanh(al);
        lt[lane] = l;
        inv[lane] = 1.0 / l;
        if (!(isfinite(l) && l > 0.0)) okflag = 0;
    }
    __syncthreads();
    // G = Q diag(lambda~) Q^T (out) and G^-1 = Q diag(1/lambda~) Q^T (into A)
    for (int idx = lane; idx < ntri; idx += 64) {
        int p = 0, rem = idx;
        while (rem >= P - p) {
            rem -= P - p;
            p++;
        }
        const int q = p + rem;
        double g = 0.0, gi = 0.0;
        for (int k = 0; k < P; k++) {
            const double qpk = Qm[p * P + k], qqk = Qm[q * P + k];
            g += (qpk * lt[k]) * qqk;
            gi += (qpk * inv[k]) * qqk;
        }
        out.G[(size_t)(p * P + q) * C + c] = g;
        out.G[(size_t)(q * P + p) * C + c] = g;
        A[p * P + q] = gi;
        A[q * P + p] = gi;
    }
    __syncthreads();
    // drift mu = x + eps^2/2 G^-1 grad   (mcmc.py:150)
    if (lane < P) {
        double sgi = 0.0;
        for (int q = 0; q < P; q++) sgi += A[lane * P + q] * gr[q];
        out.mu[(size_t)lane * C + c] = xv[lane] + (0.5 * eps * eps) * sgi;
    }
    __syncthreads();
    // Cholesky of G^-1 (lower, in place; mcmc.py:149): column j, rows i > j in parallel
    for (int j = 0; j < P; j++) {
        double d = A[j * P + j];
        for (int k = 0; k < j; k++) d -= A[j * P + k] * A[j * P + k];
        const double ljj = sqrt(d > 0.0 ? d : 1.0);
        double lij = 0.0;
        const int i = lane;
        if (i > j && i < P) {
            double s = A[i * P + j];
            for (int k = 0; k < j; k++) s -= A[i * P + k] * A[j * P + k];
            lij = s / ljj;
        }
        __syncthreads();
        if (lane == 0) {
            A[j * P + j] = ljj;
            if (!(d > 0.0)) okflag = 0;
        }
        if (i > j && i < P) A[i * P + j] = lij;
        __syncthreads();
    }
    for (int idx = lane; idx < P * P; idx += 64) {
        const int i = idx / P, j = idx % P;
        out.L[(size_t)idx * C + c] = j <= i ? A[idx] : 0.0;
    }
    if (lane == 0) {
        double logdet = 0.0;  // log det G^-1
        for (int k = 0; k < P; k++) logdet += log(inv[k]);
        out.lp[c] = lp_c;
        out.logdet[c] = logdet;
        out.ok[c] = okflag;
    }
}

// One wave per chain: the P x P matrices live in LDS, lanes own matrix rows / entries, and the
// sequential parts (Jacobi rotations, Cholesky columns) run lock-step across the wave.
__device__ __forceinline__ void smala_derive_chain(int P, int C, int E, const double* __restrict__ x, double rel,
                                                   const double* __restrict__ fl, const double* __restrict__ lp_st,
                                                   const int32_t* __restrict__ st_st, const double* __restrict__ rv,
                                                   const double* __restrict__ w, double npoints, double alpha,
                                                   double eps, const SmalaCache& out, bool sides = false) {
    constexpr int PM = RVM_SMALA_MAX_PARAMS;
    constexpr int NTRI = PM * (PM + 1) / 2;        // upper-triangle entries
    constexpr int PER_LANE = (NTRI + 63) / 64;     // accumulators per lane
    __shared__ double A[PM * PM], Qm[PM * PM];
    __shared__ double den[PM], gr[PM], lt[PM], inv[PM], xv[PM];
    __shared__ double ra[PM], rb[PM], dn[PM];
    __shared__ int rp[PM];
    constexpr int JCH = 64;                        // epochs per J chunk
    __shared__ double Jc[JCH * PM], wc[JCH];
    __shared__ int okflag;
    const int c = blockIdx.x;
    const int lane = threadIdx.x;
    const int S = 2 * P + 1;
    const size_t SC = (size_t)S * C;
    const int ntri = P * (P + 1) / 2;
    if (lane == 0) okflag = 1;
    __syncthreads();
    // (sides: the centre row's status and logp are not read -- rvm_smala_center_accept brings the
    // centre's own, the only things of the cache that depend on them)
    for (int s = lane + (sides ? 1 : 0); s < S; s += 64)
        if (st_st[(size_t)s * C + c] != 0) okflag = 0;
    // realised steps exactly as rvm_fd_params formed the stencil; gradient
    if (lane < P) {
        const double xp = x[(size_t)lane * C + c];
        const double ax = fabs(xp) > fl[lane] ? fabs(xp) : fl[lane];
        const double e = rel * ax;
        const double d = (xp + e) - (xp - e);
        const double g = (lp_st[(size_t)(1 + 2 * lane) * C + c] - lp_st[(size_t)(2 + 2 * lane) * C + c]) / d;
        den[lane] = d;
        gr[lane] = g;
        xv[lane] = xp;
        out.grad[(size_t)lane * C + c] = g;
    }
    __syncthreads();
    // -H = (2/N) sum_e J_e^T (1/sigma_e^2) J_e, J_e[p] = (rv_e(x+e_p) - rv_e(x-e_p)) / den_p:
    // K = 64/P epochs of J per chunk in LDS, each lane accumulates its upper-triangle entries
    int tp[PER_LANE], tq[PER_LANE];
    double acc[PER_LANE];
#pragma unroll
    for (int j = 0; j < PER_LANE; j++) {
        const int idx = lane + 64 * j;
        int p = 0, rem = idx;
        while (p < P && rem >= P - p) {
            rem -= P - p;
            p++;
        }
        tp[j] = p;
        tq[j] = p + rem;
        acc[j] = 0.0;
    }
    // J in chunks of JCH epochs: every lane issues its loads of the chunk at once (the chunk's
    // latency is paid once, not once per epoch), then the triangle accumulates from LDS
    for (int e0 = 0; e0 < E; e0 += JCH) {
        const int kmax = E - e0 < JCH ? E - e0 : JCH;
        const int n = kmax * P;
#pragma unroll 4
        for (int idx = lane; idx < n; idx += 64) {
            const int k = idx / P, p = idx - (idx / P) * P;
            const double* re = rv + (size_t)(e0 + k) * SC;
            Jc[idx] = (re[(size_t)(1 + 2 * p) * C + c] - re[(size_t)(2 + 2 * p) * C + c]) / den[p];
        }
        if (lane < kmax) wc[lane] = w[e0 + lane];
        __syncthreads();
#pragma unroll
        for (int j = 0; j < PER_LANE; j++) {
            if (lane + 64 * j < ntri) {
                double a = acc[j];
                for (int k = 0; k < kmax; k++) a += (Jc[k * P + tp[j]] * wc[k]) * Jc[k * P + tq[j]];
                acc[j] = a;
            }
        }
        __syncthreads();
    }
    const double fac = 2.0 / npoints;
#pragma unroll
    for (int j = 0; j < PER_LANE; j++) {
        if (lane + 64 * j < ntri) {
            const double a = fac * acc[j];
            A[tp[j] * P + tq[j]] = a;
            A[tq[j] * P + tp[j]] = a;
        }
    }
    smala_metric_stage(P, C, c, lane, A, Qm, gr, xv, lt, inv, ra, rb, dn, rp, okflag, sides ? 0.0 : lp_st[c], alpha,
                       eps, out);
}

__global__ __launch_bounds__(64) void smala_derive_kernel(int P, int C, int E, const double* __restrict__ x,
                                                          double rel, const double* __restrict__ fl,
                                                          const double* __restrict__ lp_st,
                                                          const int32_t* __restrict__ st_st,
                                                          const double* __restrict__ rv,
                                                          const double* __restrict__ w, double npoints,
                                                          double alpha, double eps, SmalaCache out, int sides) {
    smala_derive_chain(P, C, E, x, rel, fl, lp_st, st_st, rv, w, npoints, alpha, eps, out, sides != 0);
}

// rvm_smala_metric: the same metric pipeline from exact derivatives (rvm_logl_derivs)
__device__ __forceinline__ void smala_metric_chain(int P, int C, const double* __restrict__ x,
                                                   const double* __restrict__ lp, const int32_t* __restrict__ status,
                                                   const double* __restrict__ grad, const double* __restrict__ hess,
                                                   double alpha, double eps, const SmalaCache& out) {
    constexpr int PM = RVM_SMALA_MAX_PARAMS;
    __shared__ double A[PM * PM], Qm[PM * PM];
    __shared__ double gr[PM], lt[PM], inv[PM], xv[PM];
    __shared__ double ra[PM], rb[PM], dn[PM];
    __shared__ int rp[PM];
    __shared__ int okflag;
    const int c = blockIdx.x;
    const int lane = threadIdx.x;
    if (lane == 0) okflag = status[c] == RVM_STATUS_OK && isfinite(lp[c]) ? 1 : 0;
    __syncthreads();
    if (lane < P) {
        const double g = grad[(size_t)lane * C + c];
        gr[lane] = g;
        xv[lane] = x[(size_t)lane * C + c];
        out.grad[(size_t)lane * C + c] = g;
        if (!isfinite(g)) okflag = 0;
    }
    for (int i = lane; i < P * P; i += 64) {
        const int r = i / P, q = i - (i / P) * P;
        // symmetric by construction (rvm_logl_derivs writes both triangles from one pair)
        const double h = hess[(size_t)i * C + c];
        A[r * P + q] = -h;
        if (!isfinite(h)) okflag = 0;
    }
    __syncthreads();
    if (!okflag) {  // keep the eigen-solver on finite numbers; the cache is marked not ok
        for (int i = lane; i < P * P; i += 64) A[i] = (i / P == i % P) ? 1.0 : 0.0;
        if (lane < P) gr[lane] = 0.0;
    }
    __syncthreads();
    const int ok0 = okflag;
    smala_metric_stage(P, C, c, lane, A, Qm, gr, xv, lt, inv, ra, rb, dn, rp, okflag, lp[c], alpha, eps, out);
    if (lane == 0 && !ok0) out.ok[c] = 0;
}

__global__ __launch_bounds__(64) void smala_metric_kernel(int P, int C, const double* __restrict__ x,
                                                          const double* __restrict__ lp,
                                                          const int32_t* __restrict__ status,
                                                          const double* __restrict__ grad,
                                                          const double* __restrict__ hess, double alpha, double eps,
                                                          SmalaCache out) {
    smala_metric_chain(P, C, x, lp, status, grad, hess, alpha, eps, out);
}

__device__ __forceinline__ double box_muller_s(double u0, double u1) {
    return sqrt(-2.0 * log(u0)) * cospi(2.0 * u1);
}

// One wave per chain: lane p draws z_p, then x*_p = mu_p + eps sum_{q<=p} L_pq z_q (mcmc.py:151).
__global__ __launch_bounds__(64) void smala_propose_kernel(int P, int C, int64_t begin, const double* __restrict__ x,
                                                           SmalaCache cur, double eps, uint64_t seed,
                                                           uint64_t iteration, const double* __restrict__ draws,
                                                           double* __restrict__ xs) {
    const int c = blockIdx.x;
    const int lane = threadIdx.x;
    __shared__ double zs[RVM_SMALA_MAX_PARAMS];
    if (!cur.ok[c]) {  // no usable metric at x: stay (the proposal is then rejected)
        if (lane < P) xs[(size_t)lane * C + c] = x[(size_t)lane * C + c];
        return;
    }
    if (lane < P) {
        double z;
        if (draws) {
            z = draws[(size_t)lane * C + c];
        } else {
            double u0, u1;
            uniform2(seed, (uint64_t)(begin + c), iteration, RNG_SMALA_PROPOSE | ((uint32_t)lane << 8), u0, u1);
            z = box_muller_s(u0, u1);
        }
        zs[lane] = z;
    }
    __syncthreads();
    if (lane < P) {
        double s = 0.0;
        for (int q = 0; q <= lane; q++) s += cur.L[(size_t)(lane * P + q) * C + c] * zs[q];
        xs[(size_t)lane * C + c] = cur.mu[(size_t)lane * C + c] + eps * s;
    }
}

// log N(y; mu, eps^2 G^-1) = -1/2 [ (y-mu)^T G (y-mu) / eps^2 + P log eps^2 + log det G^-1 + P log 2 pi ]
// given maha = (y-mu)^T G (y-mu)
__device__ __forceinline__ double mvn_logpdf(int P, double maha, double logdet, double eps) {
    return -0.5 * (maha / (eps * eps) + (double)P * log(eps * eps) + logdet + (double)P * log(2.0 * M_PI));
}

// One wave per chain: both Mahalanobis forms with the matrix entries spread over the lanes, then
// the accept (mcmc.py:167-187) and, on accept, the proposal's cached derivatives copied in parallel.
__device__ __forceinline__ void smala_accept_chain(int P, int C, int64_t begin, double* __restrict__ x,
                                                   const SmalaCache& cur, const double* __restrict__ xs,
                                                   const SmalaCache& prop, double eps, uint64_t seed,
                                                   uint64_t iteration, const double* __restrict__ draws,
                                                   int32_t* __restrict__ accepted, int32_t* __restrict__ failures) {
    const int c = blockIdx.x;
    const int lane = threadIdx.x;
    __shared__ double d1[RVM_SMALA_MAX_PARAMS], d2[RVM_SMALA_MAX_PARAMS];
    double u, unused;
    if (draws) {
        u = draws[c];
    } else {
        uniform2(seed, (uint64_t)(begin + c), iteration, RNG_SMALA_ACCEPT, u, unused);
    }
    const bool okc = cur.ok[c] != 0, okp = prop.ok[c] != 0;
    const double lpp = prop.lp[c];
    if (lane == 0 && failures && !okp && isfinite(lpp)) failures[c] += 1;  // metric failure, finite logp
    if (!(okc && okp && isfinite(lpp))) return;
    if (lane < P) {
        d1[lane] = xs[(size_t)lane * C + c] - cur.mu[(size_t)lane * C + c];  // x* under q(.|x)
        d2[lane] = x[(size_t)lane * C + c] - prop.mu[(size_t)lane * C + c];  // x under q(.|x*)
    }
    __syncthreads();
    double m1 = 0.0, m2 = 0.0;
    for (int idx = lane; idx < P * P; idx += 64) {
        const int p = idx / P, q = idx - (idx / P) * P;
        m1 += d1[p] * (cur.G[(size_t)idx * C + c] * d1[q]);
        m2 += d2[p] * (prop.G[(size_t)idx * C + c] * d2[q]);
    }
    m1 = wave_sum(m1);
    m2 = wave_sum(m2);
    // mcmc.py:176-181: ratio = exp(logp* - logp + log q(x|x*) - log q(x*|x)) > uniform
    const double q_ts_t = mvn_logpdf(P, m1, cur.logdet[c], eps);
    const double q_t_ts = mvn_logpdf(P, m2, prop.logdet[c], eps);
    const double ratio = exp(lpp - cur.lp[c] + q_t_ts - q_ts_t);
    if (!(ratio > u)) return;
    __syncthreads();  // every lane has read cur.* before it is overwritten
    if (lane < P) {
        x[(size_t)lane * C + c] = xs[(size_t)lane * C + c];
        cur.mu[(size_t)lane * C + c] = prop.mu[(size_t)lane * C + c];
        cur.grad[(size_t)lane * C + c] = prop.grad[(size_t)lane * C + c];
    }
    for (int i = lane; i < P * P; i += 64) {
        cur.L[(size_t)i * C + c] = prop.L[(size_t)i * C + c];
        cur.G[(size_t)i * C + c] = prop.G[(size_t)i * C + c];
    }
    if (lane == 0) {
        cur.lp[c] = lpp;
        cur.logdet[c] = prop.logdet[c];
        cur.ok[c] = 1;
        if (accepted) accepted[c] += 1;
    }
}

__global__ __launch_bounds__(64) void smala_accept_kernel(int P, int C, int64_t begin, double* __restrict__ x,
                                                          SmalaCache cur, const double* __restrict__ xs,
                                                          SmalaCache prop, double eps, uint64_t seed,
                                                          uint64_t iteration, const double* __restrict__ draws,
                                                          int32_t* __restrict__ accepted,
                                                          int32_t* __restrict__ failures) {
    smala_accept_chain(P, C, begin, x, cur, xs, prop, eps, seed, iteration, draws, accepted, failures);
}

// Fused second half of a SMALA step (rvm_smala_derive_accept / rvm_smala_metric_accept): the
// proposal's cache from its stencil (or exact derivatives), then, in the same wave, the accept.
// The barrier makes the cache entries this block just wrote visible to every lane of it.
__global__ __launch_bounds__(64) void smala_derive_accept_kernel(
    int P, int C, int E, const double* __restrict__ xs, double rel, const double* __restrict__ fl,
    const double* __restrict__ lp_st, const int32_t* __restrict__ st_st, const double* __restrict__ rv,
    const double* __restrict__ w, double npoints, double alpha, double eps, SmalaCache prop, int64_t begin,
    double* __restrict__ x, SmalaCache cur, uint64_t seed, uint64_t iteration, const double* __restrict__ draws,
    int32_t* __restrict__ accepted, int32_t* __restrict__ failures) {
    smala_derive_chain(P, C, E, xs, rel, fl, lp_st, st_st, rv, w, npoints, alpha, eps, prop);
    __syncthreads();
    smala_accept_chain(P, C, begin, x, cur, xs, prop, eps, seed, iteration, draws, accepted, failures);
}

// The accept after rvm_smala_derive_sides (rvm_smala_center_accept): the centre's own logp and status
// (the adaptive plan's, on its side stream) complete the proposal's cache -- its logp, and ok only if
// the centre's status is -- then the accept, as smala_derive_accept_kernel after the whole stencil.
__global__ __launch_bounds__(64) void smala_center_accept_kernel(int P, int C, int64_t begin, double* __restrict__ x,
                                                                 SmalaCache cur, const double* __restrict__ xs,
                                                                 SmalaCache prop, const double* __restrict__ lpc,
                                                                 const int32_t* __restrict__ stc, double eps,
                                                                 uint64_t seed, uint64_t iteration,
                                                                 const double* __restrict__ draws,
                                                                 int32_t* __restrict__ accepted,
                                                                 int32_t* __restrict__ failures) {
    const int c = blockIdx.x;
    if (threadIdx.x == 0) {
        prop.lp[c] = lpc[c];
        if (stc[c] != 0) prop.ok[c] = 0;
    }
    __syncthreads();
    smala_accept_chain(P, C, begin, x, cur, xs, prop, eps, seed, iteration, draws, accepted, failures);
}

__global__ __launch_bounds__(64) void smala_metric_accept_kernel(
    int P, int C, const double* __restrict__ xs, const double* __restrict__ lp, const int32_t* __restrict__ status,
    const double* __restrict__ grad, const double* __restrict__ hess, double alpha, double eps, SmalaCache prop,
    int64_t begin, double* __restrict__ x, SmalaCache cur, uint64_t seed, uint64_t iteration,
    const double* __restrict__ draws, int32_t* __restrict__ accepted, int32_t* __restrict__ failures) {
    smala_metric_chain(P, C, xs, lp, status, grad, hess, alpha, eps, prop);
    __syncthreads();
    smala_accept_chain(P, C, begin, x, cur, xs, prop, eps, seed, iteration, draws, accepted, failures);
}

hipError_t launch_smala_derive_accept(int P, int C, int E, const double* xs, double rel, const double* fl,
                                      const double* lp_st, const int32_t* st_st, const double* rv, const double* w,
                                      double npoints, double alpha, double eps, const SmalaCache& prop,
                                      int64_t begin, double* x, const SmalaCache& cur, uint64_t seed, uint64_t it,
                                      const double* draws, int32_t* accepted, int32_t* failures, hipStream_t st) {
    smala_derive_accept_kernel<<<C, 64, 0, st>>>(P, C, E, xs, rel, fl, lp_st, st_st, rv, w, npoints, alpha, eps, prop,
                                                 begin, x, cur, seed, it, draws, accepted, failures);
    return hipGetLastError();
}

hipError_t launch_smala_metric_accept(int P, int C, const double* xs, const double* lp, const int32_t* status,
                                      const double* grad, const double* hess, double alpha, double eps,
                                      const SmalaCache& prop, int64_t begin, double* x, const SmalaCache& cur,
                                      uint64_t seed, uint64_t it, const double* draws, int32_t* accepted,
                                      int32_t* failures, hipStream_t st) {
    smala_metric_accept_kernel<<<C, 64, 0, st>>>(P, C, xs, lp, status, grad, hess, alpha, eps, prop, begin, x, cur,
                                                 seed, it, draws, accepted, failures);
    return hipGetLastError();
}

hipError_t launch_smala_metric(int P, int C, const double* x, const double* lp, const int32_t* status,
                               const double* grad, const double* hess, double alpha, double eps, const SmalaCache& out,
                               hipStream_t st) {
    smala_metric_kernel<<<C, 64, 0, st>>>(P, C, x, lp, status, grad, hess, alpha, eps, out);
    return hipGetLastError();
}

hipError_t launch_smala_derive(int P, int C, int E, const double* x, double rel, const double* fl,
                               const double* lp_st, const int32_t* st_st, const double* rv, const double* w,
                               double npoints, double alpha, double eps, const SmalaCache& out, int sides,
                               hipStream_t st) {
    smala_derive_kernel<<<C, 64, 0, st>>>(P, C, E, x, rel, fl, lp_st, st_st, rv, w, npoints, alpha, eps, out, sides);
    return hipGetLastError();
}

hipError_t launch_smala_center_accept(int P, int C, int64_t begin, double* x, const SmalaCache& cur, const double* xs,
                                      const SmalaCache& prop, const double* lpc, const int32_t* stc, double eps,
                                      uint64_t seed, uint64_t it, const double* draws, int32_t* accepted,
                                      int32_t* failures, hipStream_t st) {
    smala_center_accept_kernel<<<C, 64, 0, st>>>(P, C, begin, x, cur, xs, prop, lpc, stc, eps, seed, it, draws, accepted,
                                                 failures);
    return hipGetLastError();
}

hipError_t launch_smala_propose(int P, int C, int64_t begin, const double* x, const SmalaCache& cur, double eps,
                                uint64_t seed, uint64_t it, const double* draws, double* xs, hipStream_t st) {
    smala_propose_kernel<<<C, 64, 0, st>>>(P, C, begin, x, cur, eps, seed, it, draws, xs);
    return hipGetLastError();
}

hipError_t launch_smala_accept(int P, int C, int64_t begin, double* x, const SmalaCache& cur, const double* xs,
                               const SmalaCache& prop, double eps, uint64_t seed, uint64_t it, const double* draws,
                               int32_t* accepted, int32_t* failures, hipStream_t st) {
    smala_accept_kernel<<<C, 64, 0, st>>>(P, C, begin, x, cur, xs, prop, eps, seed, it, draws, accepted, failures);
    return hipGetLastError();
}

}  // namespace rvm

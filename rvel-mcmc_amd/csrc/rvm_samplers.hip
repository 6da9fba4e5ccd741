// rvm_samplers.hip -- device-side proposal / accept steps of the reference samplers.
//
//   * emcee 2.2.1 EnsembleSampler stretch move (mcmc.py:40-65 drives it; the algorithm is emcee's
//     _propose_stretch + the two-half split of sample()).
//   * Gaussian random-walk Metropolis-Hastings (mcmc.py:89-121).
//   * The finite-difference stencil that feeds SMALA's gradient/metric (mcmc.py:144-187 with the
//     north-star's FD replacement of state.py:253-294).
// All positions are SoA [n_params][n] float64.  Random numbers come from Philox4x32-10 keyed by the
// GLOBAL walker index, so a sharded ensemble draws exactly what an unsharded one does.
#include <hip/hip_runtime.h>
#include <math.h>

#include "rvm_device.h"
#include "rvm_internal.h"
#include "rvm_stretch.h"

// No FMA contraction in the sampler arithmetic: proposals and accept tests are then bit-identical
// to a plain IEEE restatement (numpy) fed the same random numbers.
#pragma clang fp contract(off)

namespace rvm {

__global__ void stretch_propose_kernel(int P, int n0, int64_t s0_begin, const double* __restrict__ x, int n1,
                                       const double* __restrict__ c, double a, uint64_t seed, uint64_t iteration,
                                       uint32_t half, const double* __restrict__ draws, double* __restrict__ q,
                                       double* __restrict__ zout) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n0) return;
    double z;
    int j;
    if (draws)
        stretch_zj(draws[i], draws[n0 + i], a, n1, z, j);
    else
        stretch_draw(seed, (uint64_t)(s0_begin + i), iteration, half, a, n1, z, j);
    for (int p = 0; p < P; p++) q[(size_t)p * n0 + i] = stretch_q(c[(size_t)p * n1 + j], z, x[(size_t)p * n0 + i]);
    zout[i] = z;
}

__global__ void stretch_accept_kernel(int P, int n0, int64_t s0_begin, double* __restrict__ x,
                                      double* __restrict__ lnp, const double* __restrict__ q,
                                      const double* __restrict__ lnp_new, const double* __restrict__ z,
                                      uint64_t seed, uint64_t iteration, uint32_t half,
                                      const double* __restrict__ draws, int32_t* __restrict__ accepted) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n0) return;
    const double u3 = draws ? draws[i] : stretch_u3(seed, (uint64_t)(s0_begin + i), iteration, half);
    if (stretch_accepts(P, z[i], lnp_new[i], lnp[i], u3)) {
        for (int p = 0; p < P; p++) x[(size_t)p * n0 + i] = q[(size_t)p * n0 + i];
        lnp[i] = lnp_new[i];
        if (accepted) accepted[i] += 1;
    }
}

// Second half-step of a speculative iteration (rvm_stretch_iteration_end): threads [0, n) accept
// or reject half 1's walkers with the logl of the variant their partner's decision selects;
// threads [n, 2n) refresh half 0's walker-major mirror rows that the first half-step changed.
// A partner on this rank is read from x0 (already updated); any other is rebuilt from the
// iteration's starting positions and its own draws -- the same bits either way.
// MAXD > 0 (dim <= MAXD): every load a walker may need -- both variants' logl, the partner rows
// (x0, or c0 and c1 for both outcomes), its own row -- is issued before any of them is used, so a
// thread waits for one round of memory latency instead of one per dependent load and dimension
// (the kernel is latency-bound: n threads, a few loads each).  MAXD = 0: any dim.
template <int MAXD>
__global__ void stretch_iteration_end_kernel(const IterEndArgs g) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    const int n = g.n, P = g.dim;
    if (t < n) {
        const int k = t;
        double z;
        int j;
        stretch_draw(g.seed, (uint64_t)(g.s1_begin + k), g.iteration, 1u, g.a, g.n_half, z, j);
        const int64_t jl = (int64_t)j - g.s0_begin;
        const bool local = jl >= 0 && jl < n;
        if constexpr (MAXD > 0) {
            double zp = 0.0;
            int jp = 0;
            if (!local) stretch_draw(g.seed, (uint64_t)j, g.iteration, 0u, g.a, g.n_half, zp, jp);
            const int dv = g.dec_all[j];
            const double l1 = g.lnp_spec[(size_t)n + k], l2 = g.lnp_spec[(size_t)2 * n + k];
            const int32_t s1 = g.st_spec[(size_t)n + k], s2 = g.st_spec[(size_t)2 * n + k];
            const double lnp_old = g.lnp1[k];
            double xv[MAXD], cv[MAXD], cq[MAXD];
#pragma unroll
            for (int p = 0; p < MAXD; p++) {
                if (p < P) {
                    xv[p] = g.x1[(size_t)p * n + k];
                    if (local) {
                        cv[p] = g.x0[(size_t)p * n + jl];
                        cq[p] = 0.0;
                    } else {
                        cv[p] = g.c0[(size_t)j * P + p];
                        cq[p] = g.c1[(size_t)jp * P + p];
                    }
                }
            }
            const int v = dv != 0 ? 1 : 0;
            const double lnew = v ? l2 : l1;
            if (g.lnp_new_out) g.lnp_new_out[k] = lnew;
            if (g.status_new_out) g.status_new_out[k] = v ? s2 : s1;
            const double u3 = stretch_u3(g.seed, (uint64_t)(g.s1_begin + k), g.iteration, 1u);
            if (stretch_accepts(P, z, lnew, lnp_old, u3)) {
#pragma unroll
                for (int p = 0; p < MAXD; p++) {
                    if (p < P) {
                        double c = cv[p];
                        if (!local && v) c = stretch_q(cq[p], zp, c);
                        const double q = stretch_q(c, z, xv[p]);
                        g.x1[(size_t)p * n + k] = q;
                        if (g.x1_aos) g.x1_aos[(size_t)k * P + p] = q;
                    }
                }
                g.lnp1[k] = lnew;
                if (g.accepted1) g.accepted1[k] += 1;
            }
        } else {
            const int v = g.dec_all[j] != 0 ? 1 : 0;
            const double lnew = g.lnp_spec[(size_t)(1 + v) * n + k];
            if (g.lnp_new_out) g.lnp_new_out[k] = lnew;
            if (g.status_new_out) g.status_new_out[k] = g.st_spec[(size_t)(1 + v) * n + k];
            const double u3 = stretch_u3(g.seed, (uint64_t)(g.s1_begin + k), g.iteration, 1u);
            if (stretch_accepts(P, z, lnew, g.lnp1[k], u3)) {
                double zp = 0.0;
                int jp = 0;
                if (!local && v) stretch_draw(g.seed, (uint64_t)j, g.iteration, 0u, g.a, g.n_half, zp, jp);
                for (int p = 0; p < P; p++) {
                    double c;
                    if (local) {
                        c = g.x0[(size_t)p * n + jl];
                    } else {
                        c = g.c0[(size_t)j * P + p];
                        if (v) c = stretch_q(g.c1[(size_t)jp * P + p], zp, c);
                    }
                    const double q = stretch_q(c, z, g.x1[(size_t)p * n + k]);
                    g.x1[(size_t)p * n + k] = q;
                    if (g.x1_aos) g.x1_aos[(size_t)k * P + p] = q;
                }
                g.lnp1[k] = lnew;
                if (g.accepted1) g.accepted1[k] += 1;
            }
        }
    } else if (t < 2 * n) {
        const int i = t - n;
        if (g.x0_aos && g.dec_local[i])
            for (int p = 0; p < P; p++) g.x0_aos[(size_t)i * P + p] = g.x0[(size_t)p * n + i];
    }
}

__global__ void mh_propose_kernel(int P, int n, int64_t begin, const double* __restrict__ x,
                                  const double* __restrict__ scales, double step, uint64_t seed, uint64_t iteration,
                                  const double* __restrict__ draws, double* __restrict__ q) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    for (int p = 0; p < P; p++) {
        const double g = draws ? draws[(size_t)p * n + i] : mh_normal(seed, (uint64_t)(begin + i), iteration, p);
        q[(size_t)p * n + i] = mh_q(x[(size_t)p * n + i], step, scales[p], g);
    }
}

__global__ void mh_accept_kernel(int P, int n, int64_t begin, double* __restrict__ x, double* __restrict__ lnp,
                                 const double* __restrict__ q, const double* __restrict__ lnp_new, uint64_t seed,
                                 uint64_t iteration, const double* __restrict__ draws,
                                 int32_t* __restrict__ accepted) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double u = draws ? draws[i] : mh_u(seed, (uint64_t)(begin + i), iteration);
    if (mh_accepts(lnp_new[i], lnp[i], u)) {
        for (int p = 0; p < P; p++) x[(size_t)p * n + i] = q[(size_t)p * n + i];
        lnp[i] = lnp_new[i];
        if (accepted) accepted[i] += 1;
    }
}

// out: SoA [n_params][(2P+1) * n] with walker index s*n + c  (s = 0: x; s = 1+2p: +eps_p; 2+2p: -eps_p)
__global__ void fd_params_kernel(int P, int n, const double* __restrict__ x, double rel, const double* __restrict__ fl,
                                 double* __restrict__ out) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= n) return;
    const int S = 2 * P + 1;
    const size_t WW = (size_t)S * n;
    for (int p = 0; p < P; p++)
        for (int s = 0; s < S; s++) out[(size_t)p * WW + (size_t)s * n + c] = fd_point(x, fl, rel, n, p, s * n + c);
}

static inline dim3 grid1(int n) { return dim3((n + 255) / 256); }

hipError_t launch_stretch_propose(int P, int n0, int64_t s0b, const double* x, int n1, const double* c, double a,
                                  uint64_t seed, uint64_t it, uint32_t half, const double* draws, double* q,
                                  double* z, hipStream_t st) {
    stretch_propose_kernel<<<grid1(n0), 256, 0, st>>>(P, n0, s0b, x, n1, c, a, seed, it, half, draws, q, z);
    return hipGetLastError();
}
hipError_t launch_stretch_accept(int P, int n0, int64_t s0b, double* x, double* lnp, const double* q,
                                 const double* lnp_new, const double* z, uint64_t seed, uint64_t it, uint32_t half,
                                 const double* draws, int32_t* acc, hipStream_t st) {
    stretch_accept_kernel<<<grid1(n0), 256, 0, st>>>(P, n0, s0b, x, lnp, q, lnp_new, z, seed, it, half, draws, acc);
    return hipGetLastError();
}
hipError_t launch_stretch_iteration_end(const IterEndArgs& g, hipStream_t st) {
    if (g.dim <= 16)
        stretch_iteration_end_kernel<16><<<grid1(2 * g.n), 256, 0, st>>>(g);
    else
        stretch_iteration_end_kernel<0><<<grid1(2 * g.n), 256, 0, st>>>(g);
    return hipGetLastError();
}
hipError_t launch_mh_propose(int P, int n, int64_t b, const double* x, const double* scales, double step,
                             uint64_t seed, uint64_t it, const double* draws, double* q, hipStream_t st) {
    mh_propose_kernel<<<grid1(n), 256, 0, st>>>(P, n, b, x, scales, step, seed, it, draws, q);
    return hipGetLastError();
}
hipError_t launch_mh_accept(int P, int n, int64_t b, double* x, double* lnp, const double* q, const double* lnp_new,
                            uint64_t seed, uint64_t it, const double* draws, int32_t* acc, hipStream_t st) {
    mh_accept_kernel<<<grid1(n), 256, 0, st>>>(P, n, b, x, lnp, q, lnp_new, seed, it, draws, acc);
    return hipGetLastError();
}
hipError_t launch_fd_params(int P, int n, const double* x, double rel, const double* fl, double* out, hipStream_t st) {
    fd_params_kernel<<<grid1(n), 256, 0, st>>>(P, n, x, rel, fl, out);
    return hipGetLastError();
}

}  // namespace rvm

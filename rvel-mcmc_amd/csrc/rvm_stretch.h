// rvm_stretch.h -- emcee 2.2.1 stretch-move arithmetic shared by the separate propose / accept
// kernels (rvm_samplers.hip) and the fused half-step in the likelihood kernel (rvm_logl.hip), so
// both paths are bit-identical.  No FMA contraction here: the proposal and the accept test then
// also match a plain IEEE restatement (numpy) fed the same uniforms.
#pragma once
#include "rvm_device.h"

namespace rvm {

enum : uint32_t {
    RNG_STRETCH_PROPOSE = 1,
    RNG_STRETCH_ACCEPT = 2,
    RNG_MH_PROPOSE = 3,
    RNG_MH_ACCEPT = 4,
};

// z = ((a - 1) u1 + 1)^2 / a  and  j = floor(u2 n1) (emcee _propose_stretch)
__device__ __forceinline__ void stretch_zj(double u1, double u2, double a, int n1, double& z, int& j) {
#pragma clang fp contract(off)
    z = ((a - 1.0) * u1 + 1.0) * ((a - 1.0) * u1 + 1.0) / a;
    j = (int)floor(u2 * (double)n1);
    j = j < 0 ? 0 : (j >= n1 ? n1 - 1 : j);
}

// Philox draws of walker `gidx` (global index) for this iteration and half
__device__ __forceinline__ void stretch_draw(uint64_t seed, uint64_t gidx, uint64_t iteration, uint32_t half,
                                             double a, int n1, double& z, int& j) {
    double u1, u2;
    uniform2(seed, gidx, iteration, RNG_STRETCH_PROPOSE | (half << 8), u1, u2);
    stretch_zj(u1, u2, a, n1, z, j);
}

__device__ __forceinline__ double stretch_u3(uint64_t seed, uint64_t gidx, uint64_t iteration, uint32_t half) {
    double u3, unused;
    uniform2(seed, gidx, iteration, RNG_STRETCH_ACCEPT | (half << 8), u3, unused);
    return u3;
}

// q = c_j - z (c_j - x)
__device__ __forceinline__ double stretch_q(double cj, double z, double x) {
#pragma clang fp contract(off)
    return cj - z * (cj - x);
}

// emcee 2.2.1: lnpdiff = (dim - 1) * log(zz) + newlnprob - lnprob0 ; accept = lnpdiff > log(rand)
__device__ __forceinline__ bool stretch_accepts(int dim, double z, double lnp_new, double lnp_old, double u3) {
#pragma clang fp contract(off)
    const double lnpdiff = (double)(dim - 1) * log(z) + lnp_new - lnp_old;
    return lnpdiff > log(u3);
}

// ---- Gaussian random-walk MH (mcmc.py:89-121), shared by rvm_mh_propose / rvm_mh_accept and the
// fused rvm_mh_step (the likelihood kernel forms the proposal in its prologue, accepts at the end)

__device__ __forceinline__ double box_muller(double u0, double u1) {
#pragma clang fp contract(off)
    return sqrt(-2.0 * log(u0)) * cospi(2.0 * u1);
}

// N(0,1) draw of free parameter p of chain `gidx` (global index)
__device__ __forceinline__ double mh_normal(uint64_t seed, uint64_t gidx, uint64_t iteration, int p) {
    double u0, u1;
    uniform2(seed, gidx, iteration, RNG_MH_PROPOSE | ((uint32_t)p << 8), u0, u1);
    return box_muller(u0, u1);
}

// mcmc.py:91-92: shift = step_size * scales * N(0,1); prop.shift_params(shift)
__device__ __forceinline__ double mh_q(double x, double step, double scale, double g) {
#pragma clang fp contract(off)
    return x + (step * scale) * g;
}

__device__ __forceinline__ double mh_u(uint64_t seed, uint64_t gidx, uint64_t iteration) {
    double u, unused;
    uniform2(seed, gidx, iteration, RNG_MH_ACCEPT, u, unused);
    return u;
}

// mcmc.py:115: if np.exp(logp_proposal - logp) > np.random.uniform(): accept
__device__ __forceinline__ bool mh_accepts(double lnp_new, double lnp_old, double u) {
#pragma clang fp contract(off)
    return exp(lnp_new - lnp_old) > u;
}

// ---- SMALA's central-difference stencil (rvm_fd_params and the fused rvm_smala_stencil_logl):
// parameter p of stencil walker w = s * n + c around x [P][n]:  s = 1 + 2p: x_p + eps_p,
// s = 2 + 2p: x_p - eps_p, otherwise x_p; eps_p = rel * max(|x_p|, floor_p)
__device__ __forceinline__ double fd_point(const double* __restrict__ x, const double* __restrict__ fl, double rel,
                                           int n, int p, int w) {
#pragma clang fp contract(off)
    const int s = w / n, c = w - s * n;
    const double xp = x[(size_t)p * n + c];
    if (s != 1 + 2 * p && s != 2 + 2 * p) return xp;
    const double ax = fabs(xp) > fl[p] ? fabs(xp) : fl[p];
    const double eps = rel * ax;
    return s == 1 + 2 * p ? xp + eps : xp - eps;
}

}  // namespace rvm

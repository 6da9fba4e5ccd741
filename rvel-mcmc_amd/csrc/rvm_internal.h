// rvm_internal.h -- host/device shared launch descriptors of librvmcmc.so (not part of the ABI).
#pragma once
#include <stdint.h>

#include "../../include/rvmcmc.h"

namespace rvm {

// Epoch schedule of one integration direction (t >= 0 ascending from 0, or t < 0 descending).
struct DirSched {
    int32_t n_epochs;
    const int32_t* seg_n;     // level-1 steps in the segment ending at this epoch (0: same time)
    const double* seg_h1;     // signed base step of the segment: length / seg_n (0 if seg_n = 0)
    const double* obs_rv;     // observed RV
    const double* obs_s2;     // sigma^2
    const int32_t* obs_idx;   // index of the epoch in the plan's input order (rv_out rows)
};

// Everything a logl launch needs, passed by value as the kernel argument.
struct DevPlan {
    int32_t n_planets;
    int32_t n_levels;
    int32_t mult[RVM_MAX_LEVELS];  // level step multipliers (steps per base step)
    int32_t nt[RVM_MAX_LEVELS];    // Stumpff series terms per level (6, 7 or 8)
    int32_t spec[RVM_MAX_LEVELS];  // 1: speculative segments on this level (rvm_logl.hip)
    double inv_mult[RVM_MAX_LEVELS];  // 1 / mult: level step = seg_h1 * inv_mult
    double lw[RVM_MAX_LEVELS];     // Richardson (Lagrange-at-zero in h^2) weights
    double npoints;
    int32_t n_obs;
    int32_t inclined;  // 1: 7 parameter rows per planet (ix, iy), 3-D integration
    int32_t n_cu;      // compute units of the plan's device (launch shape, launch_logl)
    DirSched fwd, bwd;
};

// Fused stretch half-step (rvm_stretch_half_step) by value as a kernel argument; c == nullptr
// for a plain likelihood launch.
struct StretchArgs {
    const double* c;    // complement half, walker-major [n1][dim] (one contiguous row per c_j)
    double* x;          // this half's free parameters [dim][W] (accepted proposals written back)
    double* x_aos;      // walker-major mirror of x [W][dim] kept in step on accept (nullable)
    double* lnp;        // their log-probabilities [W]
    int32_t* accepted;  // accept counters [W] (nullable)
    int64_t s0_begin;   // global index of walker 0 of x (Philox key)
    uint64_t seed, iteration;
    double a;
    int32_t n1, dim;
    uint32_t half;
    int32_t src[RVM_MAX_PARAM_ROWS];  // rvm_param_map
    double base[RVM_MAX_PARAM_ROWS];
};

// rvm_smala_cache by value as a kernel argument (same layout)
struct SmalaCache {
    double* lp;
    double* grad;
    double* mu;
    double* L;
    double* G;
    double* logdet;
    int32_t* ok;
};

}  // namespace rvm

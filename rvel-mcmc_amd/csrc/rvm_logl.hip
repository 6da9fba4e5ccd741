// rvm_logl.hip -- the walker log-likelihood kernel for gfx950 (MI355X).
//
// Replaces, for a whole batch of walkers at once, the reference's
//   State.get_logp (state.py:103-110) -> priorHard (:299-315) -> get_chi2 (:89-98)
//   -> get_rv x2 (:61-73) -> setup_sim (:36-47) + REBOUND IAS15 integrate + Encounter.
//
// Work decomposition:
//   workgroup = 64 walkers x one direction (blockIdx.y: 0 = epochs t >= 0, 1 = t < 0)
//               x n_levels waves; wave L integrates the same 64 walkers with (L+1)x the steps
//               (Wisdom-Holman DKD, epoch-aligned segments).  At every epoch each wave drops its
//               64 model RVs into LDS, one barrier, and wave 0 forms the Richardson-extrapolated
//               RV (sum_L w_L rv_L, the h^2 -> 0 limit) and accumulates chi2 in registers.
//   lane      = one walker; Kepler solver state in registers; the epoch schedule is wave-uniform
//               (scalar loads), walker parameters are read once, coalesced, from SoA
//               [n_params][n_walkers].
// A second tiny kernel (finalize) combines the two directions: logl = -(chi2_b + chi2_f)/Npoints.
#include <hip/hip_runtime.h>
#include <math.h>

#include "rvm_device.h"
#include "rvm_internal.h"

namespace rvm {

template <int NP>
__global__ __launch_bounds__(64 * RVM_MAX_LEVELS) void logl_kernel(const DevPlan P, const int W,
                                                                   const double* __restrict__ params,
                                                                   const double hill_factor,
                                                                   double* __restrict__ chi2_part,
                                                                   int32_t* __restrict__ status_part,
                                                                   double* __restrict__ rv_out) {
    const int lvl = threadIdx.x >> 6;  // wave-uniform
    const int lane = threadIdx.x & 63;
    const int d = blockIdx.y;
    const int w = blockIdx.x * 64 + lane;
    const bool valid = w < W;
    const int wl = valid ? w : (W - 1);
    const int nl = P.n_levels;

    __shared__ double s_rv[2][RVM_MAX_LEVELS][64];
    __shared__ int s_enc[RVM_MAX_LEVELS][64];

    const DirSched S = d ? P.bwd : P.fwd;
    const int mult = P.mult[lvl];

    // ---- walker parameters (m, a, h, k, l per planet), prior (state.py:299-315) ----------------
    Sys<NP> s;
    double pa[NP], ph[NP], pk[NP], pl[NP];
    int status = RVM_STATUS_OK;
#pragma unroll
    for (int p = 0; p < NP; p++) {
        s.m[p] = params[(size_t)(5 * p + 0) * W + wl];
        pa[p] = params[(size_t)(5 * p + 1) * W + wl];
        ph[p] = params[(size_t)(5 * p + 2) * W + wl];
        pk[p] = params[(size_t)(5 * p + 3) * W + wl];
        pl[p] = params[(size_t)(5 * p + 4) * W + wl];
        const bool bad = !(pa[p] > 0.02) || !(s.m[p] > 5e-6) || !(ph[p] * ph[p] + pk[p] * pk[p] < 1.0) ||
                         !isfinite(pl[p]);
        if (bad) status = RVM_STATUS_PRIOR;
    }
    if (status != RVM_STATUS_OK) {  // keep the lane numerically benign; its result is discarded
#pragma unroll
        for (int p = 0; p < NP; p++) {
            s.m[p] = 1e-3;
            pa[p] = 1.0 + p;
            ph[p] = 0.0;
            pk[p] = 0.0;
            pl[p] = 0.0;
        }
    }

    // ---- setup_sim: Pal -> heliocentric -> Jacobi; Hill-radius exit distance -------------------
    s.Mi[0] = 1.0;
    double hill = 0.0;
    double sx = 0.0, sy = 0.0, svx = 0.0, svy = 0.0;
#pragma unroll
    for (int p = 0; p < NP; p++) {
        s.Mi[p + 1] = s.Mi[p] + s.m[p];
        double X, Y, VX, VY;
        pal_to_cart(1.0 + s.m[p], pa[p], pl[p], pk[p], ph[p], X, Y, VX, VY);
        s.rx[p] = X - sx / s.Mi[p];
        s.ry[p] = Y - sy / s.Mi[p];
        s.vx[p] = VX - svx / s.Mi[p];
        s.vy[p] = VY - svy / s.Mi[p];
        sx += s.m[p] * X;
        sy += s.m[p] * Y;
        svx += s.m[p] * VX;
        svy += s.m[p] * VY;
        const double rh = pa[p] * cbrt(s.m[p] / 3.0);
        hill = rh > hill ? rh : hill;
    }
    s.dmin2 = (hill_factor * hill) * (hill_factor * hill);
    s.enc = 0;
    {
        Sys<NP> t0 = s;  // REBOUND checks exit_min_distance before the first step too
        kick(t0, 0.0);
        s.enc = t0.enc;
    }

    // ---- integrate outward from t = 0 through this direction's epochs -------------------------
    double chi2 = 0.0;
    for (int e = 0; e < S.n_epochs; e++) {
        const int n1 = S.seg_n[e];
        const int ns = n1 * mult;
        if (ns > 0) {
            const double h = S.seg_len[e] / (double)ns;
            drift(s, 0.5 * h);
            for (int j = 0; j < ns - 1; j++) {
                kick(s, h);
                drift(s, h);
            }
            kick(s, h);
            drift(s, 0.5 * h);
        }
        s_rv[e & 1][lvl][lane] = star_vx(s);
        __syncthreads();
        if (lvl == 0) {
            double rvx = 0.0;
            for (int k = 0; k < nl; k++) rvx += P.lw[k] * s_rv[e & 1][k][lane];
            const double r = rvx - S.obs_rv[e];
            chi2 += (r * r) / S.obs_s2[e];
            if (rv_out != nullptr && valid) rv_out[(size_t)S.obs_idx[e] * W + w] = rvx;
        }
    }
    s_enc[lvl][lane] = s.enc;
    __syncthreads();
    if (lvl == 0 && valid) {
        int enc = 0;
        for (int k = 0; k < nl; k++) enc |= s_enc[k][lane];
        if (status == RVM_STATUS_OK && enc) status = RVM_STATUS_ENCOUNTER;
        if (status == RVM_STATUS_OK && !isfinite(chi2)) status = RVM_STATUS_NONFINITE;
        chi2_part[(size_t)d * W + w] = chi2;
        status_part[(size_t)d * W + w] = status;
    }
}

__global__ void finalize_kernel(const int W, const double npoints, const double* __restrict__ chi2_part,
                                const int32_t* __restrict__ status_part, double* __restrict__ logl,
                                int32_t* __restrict__ status) {
    const int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= W) return;
    const int sf = status_part[w], sb = status_part[W + w];
    int st = sf != RVM_STATUS_OK ? sf : sb;
    double lp = -((chi2_part[W + w] + chi2_part[w]) / npoints);  // state.py:98, 109
    if (st == RVM_STATUS_OK && !isfinite(lp)) st = RVM_STATUS_NONFINITE;
    logl[w] = st == RVM_STATUS_OK ? lp : -INFINITY;
    status[w] = st;
}

hipError_t launch_logl(const DevPlan& P, int W, const double* params, double hill_factor, double* chi2_part,
                       int32_t* status_part, double* logl, int32_t* status, double* rv_out, hipStream_t stream) {
    const dim3 grid((W + 63) / 64, 2);
    const dim3 block(64 * P.n_levels);
    switch (P.n_planets) {
        case 1:
            logl_kernel<1><<<grid, block, 0, stream>>>(P, W, params, hill_factor, chi2_part, status_part, rv_out);
            break;
        case 2:
            logl_kernel<2><<<grid, block, 0, stream>>>(P, W, params, hill_factor, chi2_part, status_part, rv_out);
            break;
        case 3:
            logl_kernel<3><<<grid, block, 0, stream>>>(P, W, params, hill_factor, chi2_part, status_part, rv_out);
            break;
        case 4:
            logl_kernel<4><<<grid, block, 0, stream>>>(P, W, params, hill_factor, chi2_part, status_part, rv_out);
            break;
        default:
            return hipErrorInvalidValue;
    }
    hipError_t err = hipGetLastError();
    if (err != hipSuccess) return err;
    finalize_kernel<<<(W + 255) / 256, 256, 0, stream>>>(W, P.npoints, chi2_part, status_part, logl, status);
    return hipGetLastError();
}

}  // namespace rvm

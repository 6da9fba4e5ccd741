// rvm_derivs.hip -- exact gradient and Hessian of the walker log-likelihood (rvm_logl_derivs).
//
// Replaces state.py:218-294 (setup_sim_vars: one order-1 REBOUND variation per free parameter
// and one order-2 variation per parameter pair; get_chi2_d_dd: chi2, its gradient and its
// Hessian accumulated from the variational particles' star vx at every epoch, ÷ obs.Npoints;
// get_logp_d_dd: the negatives) for a batch of chains at once.  The derivatives are those of the
// plan's own discrete integrator (the Wisdom-Holman + Richardson scheme of rvm_logl.hip, same
// schedule, same levels), computed in hyper-dual arithmetic (rvm_hd.h): a lane group integrates
// one chain for one parameter pair (i, j), i >= j, and carries the order-1 variations along p_i
// and p_j and the order-2 variation along (p_i, p_j) -- the reference's variational particles for
// that pair.  Per epoch the Richardson-combined star velocity rv (with rv_i, rv_j, rv_ij) adds
//   chi2 += r^2/s^2,  dchi2_i += 2 r rv_i/s^2,  d2chi2_ij += 2 (rv_i rv_j + r rv_ij)/s^2
// (state.py:264-268), r = rv - rv_obs.  Work layout as the likelihood kernel: workgroup = 64/L
// items x one direction (blockIdx.y) x one wave per Richardson level; the two directions are
// summed by a small finalize kernel (the reference integrates tf and reversed(tb) separately too,
// state.py:259-286).
#include <hip/hip_runtime.h>
#include <math.h>

#include "rvm_hd.h"
#include "rvm_internal.h"

namespace rvm {

struct DerivArgs {
    int32_t n_chains, n_dirs, n_pairs;
    int32_t dir_row[RVM_MAX_PARAM_ROWS];  // kernel parameter row of each differentiation direction
};

// pair index p = i (i + 1) / 2 + j, j <= i  ->  (i, j)
__device__ __forceinline__ void pair_of(int p, int& i, int& j) {
    int a = 0, rem = p;
    while (rem > a) {
        a++;
        rem -= a;
    }
    i = a;
    j = rem;
}

// MAXT: threads per block the kernel is compiled for (64 per Richardson level): 256 for plans of up
// to 4 levels (one wave per SIMD: the whole 512-VGPR budget, no spills), 384 for 5-6 levels
template <int NP, bool D3, int MAXT>
__global__ __launch_bounds__(MAXT) void derivs_kernel(const DevPlan P, const DerivArgs A,
                                                                    const double* __restrict__ params,
                                                                    const double hill_factor,
                                                                    double* __restrict__ ws,
                                                                    int32_t* __restrict__ wst) {
    constexpr int L = LanesPerWalker<NP>::value;
    constexpr int WPB = 64 / L;
    constexpr int PR = D3 ? 7 : 5;
    const int nl = P.n_levels;
    const int lvl = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int slot = lane / L, pl_idx = lane % L;
    const int d = blockIdx.y;
    const int n_items = A.n_chains * A.n_pairs;
    const int item = blockIdx.x * WPB + slot;
    const int it = item < n_items ? item : n_items - 1;
    const int c = it / A.n_pairs;
    int di, dj;
    pair_of(it - c * A.n_pairs, di, dj);
    const int row_i = A.dir_row[di], row_j = A.dir_row[dj];

    __shared__ HD s_rv[2][RVM_MAX_LEVELS][64];
    __shared__ int s_enc[RVM_MAX_LEVELS][64];

    const DirSched S = d ? P.bwd : P.fwd;
    const int lvl_u = __builtin_amdgcn_readfirstlane(lvl);
    const int mult = P.mult[lvl_u];
    const double inv_mult = P.inv_mult[lvl_u];

    // ---- parameters with their variations seeded, prior (state.py:299-315, primal) -------------
    auto prm = [&](int r) {
        return HD{params[(size_t)r * A.n_chains + c], r == row_i ? 1.0 : 0.0, r == row_j ? 1.0 : 0.0, 0.0};
    };
    LaneHD<NP> s;
    HD pa[NP], ph[NP], pk[NP], pl[NP], pix[NP], piy[NP];
    int status = RVM_STATUS_OK;
#pragma unroll
    for (int p = 0; p < NP; p++) {
        s.m[p] = prm(PR * p + 0);
        pa[p] = prm(PR * p + 1);
        ph[p] = prm(PR * p + 2);
        pk[p] = prm(PR * p + 3);
        pl[p] = prm(PR * p + 4);
        pix[p] = D3 ? prm(PR * p + 5) : hd_c(0.0);
        piy[p] = D3 ? prm(PR * p + 6) : hd_c(0.0);
        bool bad = !(pa[p].v > 0.02) || !(s.m[p].v > 5e-6) || !(ph[p].v * ph[p].v + pk[p].v * pk[p].v < 1.0) ||
                   !isfinite(pl[p].v);
        if constexpr (D3) bad = bad || !(pix[p].v * pix[p].v + piy[p].v * piy[p].v < 4.0);
        if (bad) status = RVM_STATUS_PRIOR;
    }
    if (status != RVM_STATUS_OK) {  // numerically benign stand-in; the result is discarded
#pragma unroll
        for (int p = 0; p < NP; p++) {
            s.m[p] = hd_c(1e-3);
            pa[p] = hd_c(1.0 + p);
            ph[p] = pk[p] = pl[p] = pix[p] = piy[p] = hd_c(0.0);
        }
    }

    // ---- setup_sim (state.py:36-47): Pal -> heliocentric -> Jacobi, exit distance ------------------
    s.p = pl_idx < NP ? pl_idx : NP - 1;
    HD Mi[NP + 1];
    Mi[0] = hd_c(1.0);
    double hill = 0.0;
#pragma unroll
    for (int p = 0; p < NP; p++) {
        Mi[p + 1] = Mi[p] + s.m[p];
        const double rh = pa[p].v * cbrt(s.m[p].v / 3.0);
        hill = rh > hill ? rh : hill;
    }
    s.iMi[0] = hd_c(1.0);
#pragma unroll
    for (int p = 1; p <= NP; p++) s.iMi[p] = hd_inv(Mi[p]);
#pragma unroll
    for (int p = 0; p < NP; p++) s.mu[p] = s.m[p] * s.iMi[p + 1];
    s.dmin2 = (hill_factor * hill) * (hill_factor * hill);
    HD own_m = s.m[0], own_a = pa[0], own_h = ph[0], own_k = pk[0], own_l = pl[0], own_M = Mi[1];
    HD own_ix = pix[0], own_iy = piy[0];
#pragma unroll
    for (int p = 1; p < NP; p++) {
        if (s.p == p) {
            own_m = s.m[p];
            own_a = pa[p];
            own_h = ph[p];
            own_k = pk[p];
            own_l = pl[p];
            own_M = Mi[p + 1];
            own_ix = pix[p];
            own_iy = piy[p];
        }
    }
    s.GM = own_M;
    HD X, Y, VX, VY, Z = hd_c(0.0), VZ = hd_c(0.0);
    pal_to_cart_hd(1.0 + own_m, own_a, own_l, own_k, own_h, X, Y, VX, VY);
    if constexpr (D3) pal_incline_hd(own_ix, own_iy, X, Y, Z, VX, VY, VZ);
    {
        HD sx = hd_c(0.0), sy = hd_c(0.0), sz = hd_c(0.0), svx = hd_c(0.0), svy = hd_c(0.0), svz = hd_c(0.0);
        HD jx = X, jy = Y, jz = Z, jvx = VX, jvy = VY, jvz = VZ;
#pragma unroll
        for (int q = 0; q < NP - 1; q++) {
            sx = sx + s.m[q] * grp_get_hd<L>(X, q);
            sy = sy + s.m[q] * grp_get_hd<L>(Y, q);
            svx = svx + s.m[q] * grp_get_hd<L>(VX, q);
            svy = svy + s.m[q] * grp_get_hd<L>(VY, q);
            if constexpr (D3) {
                sz = sz + s.m[q] * grp_get_hd<L>(Z, q);
                svz = svz + s.m[q] * grp_get_hd<L>(VZ, q);
            }
            if (s.p == q + 1) {
                jx = X - sx * s.iMi[q + 1];
                jy = Y - sy * s.iMi[q + 1];
                jvx = VX - svx * s.iMi[q + 1];
                jvy = VY - svy * s.iMi[q + 1];
                jz = Z - sz * s.iMi[q + 1];
                jvz = VZ - svz * s.iMi[q + 1];
            }
        }
        s.rx = jx;
        s.ry = jy;
        s.vx = jvx;
        s.vy = jvy;
        s.rz = jz;
        s.vz = jvz;
    }
    s.encm = 0;
    lane_finish_hd(s);
    if (S.n_epochs > 0) {  // REBOUND checks exit_min_distance before the first step too (when the
        LaneHD<NP> t0 = s; // direction has any epoch: state.py:61-73 integrates nothing otherwise)
        kick_hd_any<NP, L, D3>(t0, 0.0);
        s.encm = t0.encm;
    }

    // ---- epochs outward from t = 0: KDK segments, Richardson-combined rv and its variations -----
    double chi2 = 0.0, gi = 0.0, gj = 0.0, hij = 0.0;
    const int E = S.n_epochs;
    for (int e = 0; e < E; e++) {
        const int ns = S.seg_n[e] * mult;
        if (ns > 0) {
            const double h = S.seg_h1[e] * inv_mult;
            // kick-drift-kick (the likelihood kernel's segments, rvm_logl.hip segment_steps)
            kick_hd_any<NP, L, D3>(s, 0.5 * h);
            for (int j = 0; j < ns; j++) {
                drift_hd<D3>(s, h);
                kick_hd_any<NP, L, D3>(s, j == ns - 1 ? 0.5 * h : h);
            }
        }
        const HD v0 = star_vx_hd<NP, L>(s);
        if (pl_idx == 0) s_rv[e & 1][lvl][slot] = v0;
        __syncthreads();
        if (lvl == 0 && lane < WPB) {
            HD rv = hd_c(0.0);
            for (int k = 0; k < nl; k++) rv = rv + P.lw[k] * s_rv[e & 1][k][lane];
            const double r = rv.v - S.obs_rv[e], is2 = 1.0 / S.obs_s2[e];
            chi2 += (r * r) * is2;
            gi += (2.0 * r * rv.a) * is2;
            gj += (2.0 * r * rv.b) * is2;
            hij += (2.0 * fma(rv.a, rv.b, r * rv.ab)) * is2;
        }
    }
    if (pl_idx == 0) s_enc[lvl][slot] = (int)((s.encm >> lane) & 1) | (status == RVM_STATUS_PRIOR ? 2 : 0);
    __syncthreads();
    const int item_w = blockIdx.x * WPB + lane;  // lane `lane` of wave 0 owns item slot `lane`
    if (lvl == 0 && lane < WPB && item_w < n_items) {
        int enc = 0;
        for (int k = 0; k < nl; k++) enc |= s_enc[k][lane];
        int st = (enc & 2) ? RVM_STATUS_PRIOR : RVM_STATUS_OK;
        if (st == RVM_STATUS_OK && (enc & 1)) st = RVM_STATUS_ENCOUNTER;
        if (st == RVM_STATUS_OK && !(isfinite(chi2) && isfinite(gi) && isfinite(gj) && isfinite(hij)))
            st = RVM_STATUS_NONFINITE;
        const size_t o = (size_t)d * n_items + item_w;
        ws[4 * o + 0] = chi2;
        ws[4 * o + 1] = gi;
        ws[4 * o + 2] = gj;
        ws[4 * o + 3] = hij;
        wst[o] = st;
    }
}

// directions summed; logl, gradient (diagonal pairs) and the symmetric Hessian written out
__global__ __launch_bounds__(256) void derivs_finalize_kernel(int C, int NDIR, int npairs, double npoints,
                                                              const double* __restrict__ ws,
                                                              const int32_t* __restrict__ wst, double* logl,
                                                              double* grad, double* hess, int32_t* status) {
    const int n_items = C * npairs;
    const int idx = blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= n_items) return;
    const int c = idx / npairs;
    int i, j;
    pair_of(idx - c * npairs, i, j);
    const double* f = ws + 4 * (size_t)idx;
    const double* b = ws + 4 * ((size_t)n_items + idx);
    const int sf = wst[idx], sb = wst[n_items + idx];
    int st = sf != RVM_STATUS_OK ? sf : sb;
    const double lp0 = -((b[0] + f[0]) / npoints);  // state.py:286-294: logp = -(chi2b + chi2f)
    if (st == RVM_STATUS_OK && !isfinite(lp0)) st = RVM_STATUS_NONFINITE;
    const bool ok = st == RVM_STATUS_OK;
    const double hv = ok ? -((b[3] + f[3]) / npoints) : NAN;
    hess[((size_t)i * NDIR + j) * C + c] = hv;
    hess[((size_t)j * NDIR + i) * C + c] = hv;
    if (i == j) grad[(size_t)i * C + c] = ok ? -((b[1] + f[1]) / npoints) : NAN;
    if (i == 0 && j == 0) {
        if (logl) logl[c] = ok ? lp0 : -INFINITY;
        if (status) status[c] = st;
    }
}

hipError_t launch_derivs(const DevPlan& P, int C, const double* params, int n_dirs, const int32_t* dir_rows,
                         double hill_factor, double* ws, int32_t* wst, double* logl, double* grad, double* hess,
                         int32_t* status, hipStream_t stream) {
    DerivArgs A{};
    A.n_chains = C;
    A.n_dirs = n_dirs;
    A.n_pairs = n_dirs * (n_dirs + 1) / 2;
    for (int k = 0; k < RVM_MAX_PARAM_ROWS; k++) A.dir_row[k] = k < n_dirs ? dir_rows[k] : -1;
    const int lpw = P.n_planets == 1 ? 1 : (P.n_planets == 2 ? 2 : 4);
    const int wpb = 64 / lpw;
    const int n_items = C * A.n_pairs;
    const dim3 grid((n_items + wpb - 1) / wpb, 2);
    const dim3 block(64 * P.n_levels);
#define RVM_LAUNCH(NPV, D3V)                                                                     \
    do {                                                                                         \
        if (P.n_levels <= 4)                                                                     \
            derivs_kernel<NPV, D3V, 256><<<grid, block, 0, stream>>>(P, A, params, hill_factor, ws, wst); \
        else                                                                                     \
            derivs_kernel<NPV, D3V, 64 * RVM_MAX_LEVELS><<<grid, block, 0, stream>>>(P, A, params, hill_factor, ws, wst); \
    } while (0)
    const bool inc = P.inclined != 0;
    switch (P.n_planets) {
        case 1:
            if (inc) RVM_LAUNCH(1, true); else RVM_LAUNCH(1, false);
            break;
        case 2:
            if (inc) RVM_LAUNCH(2, true); else RVM_LAUNCH(2, false);
            break;
        case 3:
            if (inc) RVM_LAUNCH(3, true); else RVM_LAUNCH(3, false);
            break;
        case 4:
            if (inc) RVM_LAUNCH(4, true); else RVM_LAUNCH(4, false);
            break;
        default:
            return hipErrorInvalidValue;
    }
#undef RVM_LAUNCH
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    derivs_finalize_kernel<<<(n_items + 255) / 256, 256, 0, stream>>>(C, n_dirs, A.n_pairs, P.npoints, ws, wst, logl,
                                                                      grad, hess, status);
    return hipGetLastError();
}

}  // namespace rvm

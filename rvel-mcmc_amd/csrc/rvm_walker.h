// rvm_walker.h -- per-walker pieces shared by the likelihood kernel (rvm_logl.hip: main pass and
// extension) and the refinement kernel (rvm_refine.hip: halving passes): the segment loop, the
// walker's parameters and Wisdom-Holman lane state at t = 0, the sampler's accept inputs, the
// direction-meeting encoding and the walker's final writes.  Both translation units compile with
// `#pragma clang fp contract(on)` before including it, so a walker's bits are the same in both.
#pragma once
#include "rvm_device.h"
#include "rvm_internal.h"
#include "rvm_stretch.h"

// the gated drift's second chance for a lane whose first Halley step fails (rvm_device.h drift ACC)
#ifndef RVM_DRIFT_ACC
#define RVM_DRIFT_ACC 0
#endif

namespace rvm {

// One epoch-to-epoch segment of ns Wisdom-Holman kick-drift-kick steps of size h (ns >= 1,
// wave-uniform): K(h/2) [D(h) K(h)]^(ns-1) D(h) K(h/2).  kp holds the interaction at the current
// positions (rvm_device.h kick_prep): evaluated at the end of the previous segment, it serves this
// segment's opening half kick, and leaves holding the one at the next epoch.  (The step loop is
// unrolled by hand: the compiler will not unroll a runtime trip count around the convergent DPP /
// ballot operations.)
template <int NT, bool GATED, bool D3, int NP, int L, int KG = 0, int ACC = RVM_DRIFT_ACC>
__device__ __forceinline__ void segment_steps(Lane<NP>& s, KickPrep<NP>& kp, double h, int ns, bool& bad) {
    lane_set_step(s, h);
    const VConsts vk = vconsts_for<NT>();  // loop-invariant VGPR constants
    kick_apply<NP, true, D3>(s, kp);
    int j = 0;
    for (; j + 2 <= ns - 1; j += 2) {
        drift<NT, GATED, D3, NP, KG, ACC>(s, h, bad, vk);
        kp = kick_prep<NP, L, D3>(s, vk.c1875);
        kick_apply<NP, false, D3>(s, kp);
        drift<NT, GATED, D3, NP, KG, ACC>(s, h, bad, vk);
        kp = kick_prep<NP, L, D3>(s, vk.c1875);
        kick_apply<NP, false, D3>(s, kp);
    }
    if (j < ns - 1) {
        drift<NT, GATED, D3, NP, KG, ACC>(s, h, bad, vk);
        kp = kick_prep<NP, L, D3>(s, vk.c1875);
        kick_apply<NP, false, D3>(s, kp);
    }
    drift<NT, GATED, D3, NP, KG, ACC>(s, h, bad, vk);
    kp = kick_prep<NP, L, D3>(s, vk.c1875);
    kick_apply<NP, true, D3>(s, kp);
}

// SPEC: run the segment with ungated drifts (rvm_device.h) and vote once at its end; if any lane
// of the wave had a step that needs the general solver, restore the segment's initial state and
// redo it gated.  Used on the fine levels, where such steps are rare.  Returns whether the
// segment was redone (wave-uniform).  Either way every lane ends bit-identical to a gated run.
template <int NT, bool SPEC, bool D3, int NP, int L, int KG = 0, int ACC = RVM_DRIFT_ACC>
__device__ __forceinline__ bool segment(Lane<NP>& s, KickPrep<NP>& kp, double h, int ns, int& redo) {
    bool bad = false;
    if constexpr (SPEC) {
        const double rx = s.rx, ry = s.ry, vx = s.vx, vy = s.vy, r = s.r, ir = s.ir;
        const double rz = s.rz, vz = s.vz;
        const uint64_t encm = s.encm;
        const KickPrep<NP> kp0 = kp;
        segment_steps<NT, false, D3, NP, L, KG, ACC>(s, kp, h, ns, bad);
        if (__builtin_expect(ballot(bad) != 0, 0)) {
#ifdef RVM_PROFILE
            redo++;
#endif
            s.rx = rx;
            s.ry = ry;
            s.vx = vx;
            s.vy = vy;
            s.rz = rz;
            s.vz = vz;
            s.r = r;
            s.ir = ir;
            s.encm = encm;
            kp = kp0;
            segment_steps<NT, true, D3, NP, L, KG, ACC>(s, kp, h, ns, bad);
            return true;
        }
    } else {
        segment_steps<NT, true, D3, NP, L, KG, ACC>(s, kp, h, ns, bad);
    }
    (void)redo;
    return false;
}

// a gated segment with the Stumpff series length of the level (nt: 6, 7 or 8); KG: the Kepler guess
// (rvm_device.h drift: 0 fourth order, 1 fifth)
// (late: the gated drift's late vote, rvm_device.h drift ACC 3 -- the same bits, faster where few
// lanes fail their first Halley step: the refinement passes' fine levels)
template <bool D3, int NP, int L, int KG = 0, int ACC = RVM_DRIFT_ACC>
__device__ __forceinline__ void segment_gated(Lane<NP>& s, KickPrep<NP>& kp, double h, int ns, int nt,
                                              bool late = false) {
    int unused = 0;
    if (late) {
        if (nt <= 6)
            segment<6, false, D3, NP, L, KG, 3>(s, kp, h, ns, unused);
        else if (nt == 7)
            segment<7, false, D3, NP, L, KG, 3>(s, kp, h, ns, unused);
        else
            segment<8, false, D3, NP, L, KG, 3>(s, kp, h, ns, unused);
        return;
    }
    if (nt <= 6)
        segment<6, false, D3, NP, L, KG, ACC>(s, kp, h, ns, unused);
    else if (nt == 7)
        segment<7, false, D3, NP, L, KG, ACC>(s, kp, h, ns, unused);
    else
        segment<8, false, D3, NP, L, KG, ACC>(s, kp, h, ns, unused);
}

// kernel parameter row r of walker w: from the SoA input, or (fused sampler step) the row's fixed
// value or the walker's proposal of the free parameter feeding it: MH (sa.mh_scale), or stretch
// (kind 1 / 2: half 1's walker of a speculative iteration against its partner's rejected /
// accepted position, StretchArgs)
__device__ __forceinline__ double walker_param(bool mapped, const double* __restrict__ params, int W, int w,
                                               const StretchArgs& sa, int r, double z, int j, int kind, double zp,
                                               int jp) {
    if (!mapped) return params[(size_t)r * W + w];
    const int k = sa.src[r];
    if (k < 0) return sa.base[r];
    if (sa.fd_x) return fd_point(sa.fd_x, sa.fd_floor, sa.fd_rel, sa.fd_n, k, w);
    if (sa.mh_scale)
        return mh_q(sa.x[(size_t)k * sa.xstride + w], sa.mh_step, sa.mh_scale[k],
                    mh_normal(sa.seed, (uint64_t)(sa.s0_begin + w), sa.iteration, k));
    if (kind == 0) return stretch_q(sa.c[(size_t)j * sa.dim + k], z, sa.x[(size_t)k * sa.xstride + w]);
    double c = sa.c0[(size_t)j * sa.dim + k];
    if (kind == 2) c = stretch_q(sa.c[(size_t)jp * sa.dim + k], zp, c);  // q0(j): bit-identical to slot j's
    return stretch_q(c, z, sa.x1[(size_t)k * sa.n_spec + w]);
}

// a fused launch's walker slot: its kind (0 = half-step / half 0, 1 / 2 = half 1 against its
// partner's rejected / accepted position), walker index within its half, its stretch draws and
// (kind 2) the partner's
__device__ __forceinline__ void stretch_slot(const StretchArgs& sa, int wl, int& kind, int& wk, double& z, int& j,
                                             double& zp, int& jp) {
    const int nsp = sa.n_spec;
    kind = nsp > 0 ? (wl < nsp ? 0 : (wl < 2 * nsp ? 1 : 2)) : 0;
    wk = wl - kind * nsp;
    // (one call for the slot's own draw, each result in a local of its own: two calls writing z, j
    // from both branches were merged into one through a select of their addresses, which put z, j
    // in scratch -- 56 B per lane in the likelihood kernel)
    const uint64_t key = kind == 0 ? (uint64_t)(sa.s0_begin + wk) : (uint64_t)(sa.s1_begin + wk);
    double z0;
    int j0;
    stretch_draw(sa.seed, key, sa.iteration, kind == 0 ? sa.half : 1u, sa.a, sa.n1, z0, j0);
    z = z0;
    j = j0;
    double z1 = 0.0;
    int j1 = 0;
    // the partner's own draws (half 0's keys are its global indices 0 .. n1-1)
    if (kind == 2) stretch_draw(sa.seed, (uint64_t)j0, sa.iteration, 0u, sa.a, sa.n1, z1, j1);
    zp = z1;
    jp = j1;
}

// ---- setup_sim (state.py:36-47): prior, Pal -> heliocentric (own planet) -> Jacobi, Hill exit ----
// rowv: the walker's kernel parameter rows (m, a, h, k, l [, ix, iy] per planet).  Sets the lane's
// state at t = 0 (lane pl_idx of the walker's L lanes), `status` (RVM_STATUS_PRIOR, else
// unchanged) and e2w, the walker's largest e^2 (the eccentricity guard).
template <int NP, bool D3, int L>
__device__ __forceinline__ void walker_setup(const double* rowv, const int pl_idx, const double hill_factor,
                                             Lane<NP>& s, int& status, double& e2w) {
    constexpr int PR = D3 ? 7 : 5;  // parameter rows per planet
    double pa[NP], ph[NP], pk[NP], pl[NP], pix[NP], piy[NP];
#pragma unroll
    for (int p = 0; p < NP; p++) {
        s.m[p] = rowv[PR * p + 0];
        pa[p] = rowv[PR * p + 1];
        ph[p] = rowv[PR * p + 2];
        pk[p] = rowv[PR * p + 3];
        pl[p] = rowv[PR * p + 4];
        pix[p] = D3 ? rowv[PR * p + 5] : 0.0;
        piy[p] = D3 ? rowv[PR * p + 6] : 0.0;
        bool bad = !(pa[p] > 0.02) || !(s.m[p] > 5e-6) || !(ph[p] * ph[p] + pk[p] * pk[p] < 1.0) ||
                   !isfinite(pl[p]);
        if constexpr (D3) bad = bad || !(pix[p] * pix[p] + piy[p] * piy[p] < 4.0);  // state.py:311-313
        if (bad) status = RVM_STATUS_PRIOR;
    }
    e2w = 0.0;
#pragma unroll
    for (int p = 0; p < NP; p++) e2w = fmax(e2w, ph[p] * ph[p] + pk[p] * pk[p]);
    if (status != RVM_STATUS_OK) {  // keep the lane numerically benign; its result is discarded
#pragma unroll
        for (int p = 0; p < NP; p++) {
            s.m[p] = 1e-3;
            pa[p] = 1.0 + p;
            ph[p] = 0.0;
            pk[p] = 0.0;
            pl[p] = 0.0;
            pix[p] = 0.0;
            piy[p] = 0.0;
        }
    }
    s.p = pl_idx < NP ? pl_idx : NP - 1;
    s.q = pl_idx;
    double Mi[NP + 1];
    Mi[0] = 1.0;
    double hill = 0.0;
#pragma unroll
    for (int p = 0; p < NP; p++) {
        Mi[p + 1] = Mi[p] + s.m[p];
        const double rh = pa[p] * cbrt(s.m[p] / 3.0);
        hill = rh > hill ? rh : hill;
    }
#pragma unroll
    for (int p = 0; p <= NP; p++) s.iMi[p] = 1.0 / Mi[p];
#pragma unroll
    for (int p = 0; p < NP; p++) s.mu[p] = s.m[p] / Mi[p + 1];
    s.dmin2 = (hill_factor * hill) * (hill_factor * hill);
    double own_m = s.m[0], own_a = pa[0], own_h = ph[0], own_k = pk[0], own_l = pl[0], own_M = Mi[1];
    double own_ix = pix[0], own_iy = piy[0];
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
    double X, Y, VX, VY, Z = 0.0, VZ = 0.0;
    pal_to_cart(1.0 + own_m, own_a, own_l, own_k, own_h, X, Y, VX, VY);
    if constexpr (D3) {
        if (own_ix != 0.0 || own_iy != 0.0) pal_incline(own_ix, own_iy, X, Y, Z, VX, VY, VZ);
    }
    {
        // r'_p = x_p - (sum_{q<p} m_q x_q) / M_{p-1}   (heliocentric -> Jacobi)
        double sx = 0.0, sy = 0.0, sz = 0.0, svx = 0.0, svy = 0.0, svz = 0.0;
        double jx = X, jy = Y, jz = Z, jvx = VX, jvy = VY, jvz = VZ;
#pragma unroll
        for (int q = 0; q < NP - 1; q++) {
            const double xq = grp_get<L>(X, q), yq = grp_get<L>(Y, q);
            const double vxq = grp_get<L>(VX, q), vyq = grp_get<L>(VY, q);
            sx += s.m[q] * xq;
            sy += s.m[q] * yq;
            svx += s.m[q] * vxq;
            svy += s.m[q] * vyq;
            if constexpr (D3) {
                sz += s.m[q] * grp_get<L>(Z, q);
                svz += s.m[q] * grp_get<L>(VZ, q);
            }
            if (s.p == q + 1) {
                jx = X - sx * s.iMi[q + 1];
                jy = Y - sy * s.iMi[q + 1];
                jvx = VX - svx * s.iMi[q + 1];
                jvy = VY - svy * s.iMi[q + 1];
                if constexpr (D3) {
                    jz = Z - sz * s.iMi[q + 1];
                    jvz = VZ - svz * s.iMi[q + 1];
                }
            }
        }
        s.rx = jx;
        s.ry = jy;
        s.vx = jvx;
        s.vy = jvy;
        s.rz = D3 ? jz : 0.0;
        s.vz = D3 ? jvz : 0.0;
    }
    s.r = D3 ? sqrt(s.rx * s.rx + s.ry * s.ry + s.rz * s.rz) : sqrt(s.rx * s.rx + s.ry * s.ry);
    s.ir = 1.0 / s.r;
    s.encm = 0;
    lane_finish(s);
}

// global-address-space views for agent-scope atomics (cdna_hip_programming.md §6 Guideline 16)
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) int gi32;
// Bounded waits: a cross-workgroup wait gives up after P.spin_ticks of the 100 MHz real-time counter
// WITHOUT PROGRESS (restarted whenever the awaited side advances), counts the give-up in the plan's
// fault counter (rvm_plan_faults) and reports its walkers NONFINITE instead of hanging the GPU.
struct SpinClock {
    unsigned long long last;
    __device__ __forceinline__ void restart() { last = __builtin_amdgcn_s_memrealtime(); }
    __device__ __forceinline__ bool expired(unsigned long long ticks) const {
        return __builtin_amdgcn_s_memrealtime() - last > ticks;
    }
};

// A gated segment (segment_gated) that a partner can stop part-way: the work a team B or an eager
// block does speculatively (rvm_refine.hip) is cancelled through a word that reaches `tag`.  Polled
// at the epochs alone, a cancel waited for the rest of the segment -- up to ~100 us on the passes'
// long segments, which kept the refinement launch open after team A had finished every walker
// (scripts/probe/refine_prof.py).  The words (c1 may be null) are loaded every CH steps, each load
// tested after the CH steps that follow it (no wait on the step chain).  Returns false when cancelled:
// the lanes' state is then partial, and the caller discards it.  A segment that runs to its end
// computes exactly segment_gated's bits.
template <int NT, bool D3, int NP, int L, int KG, int CH = 64, int ACC = RVM_DRIFT_ACC>
__device__ __forceinline__ bool segment_steps_c(Lane<NP>& s, KickPrep<NP>& kp, double h, int ns, const gu64* c0,
                                                const gu64* c1, unsigned long long tag) {
    bool bad = false;
    lane_set_step(s, h);
    const VConsts vk = vconsts_for<NT>();
    kick_apply<NP, true, D3>(s, kp);
    // (unconditional loads: a load under a branch is waited for where the branches join; c1 null
    // reads c0 twice)
    const gu64* w1 = c1 ? c1 : c0;
    auto load = [](const gu64* c) { return __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
    // the ns - 1 drift-kick pairs in chunks of CH steps, each chunk's loop the plain segment_steps
    // loop; the words are loaded before a chunk and compared after it.  A compare before the chunk
    // made the wave wait for the load there, a test inside the step loop cost ~60 cycles per step, and
    // chunks of 16 (32) steps still ~17 (~3) -- the agent-scope load outlasting the chunk; 64 steps
    // cost nothing measurable and bound a cancel's latency at ~17 us (scripts/probe/seg_bench.hip,
    // profiles/r05q_seg_bench_cancel_chunks.txt)
    int left = ns - 1;
    while (left >= 2) {
        const unsigned long long a = load(c0), b = load(w1);
        const int c = left < CH ? (left & ~1) : CH;
        for (int j = 0; j < c; j += 2) {
            drift<NT, true, D3, NP, KG, ACC>(s, h, bad, vk);
            kp = kick_prep<NP, L, D3>(s, vk.c1875);
            kick_apply<NP, false, D3>(s, kp);
            drift<NT, true, D3, NP, KG, ACC>(s, h, bad, vk);
            kp = kick_prep<NP, L, D3>(s, vk.c1875);
            kick_apply<NP, false, D3>(s, kp);
        }
        left -= c;
        if (__builtin_amdgcn_readfirstlane((int)((a == tag) | (b == tag)))) return false;
    }
    if (left == 1) {
        drift<NT, true, D3, NP, KG, ACC>(s, h, bad, vk);
        kp = kick_prep<NP, L, D3>(s, vk.c1875);
        kick_apply<NP, false, D3>(s, kp);
    }
    drift<NT, true, D3, NP, KG, ACC>(s, h, bad, vk);
    kp = kick_prep<NP, L, D3>(s, vk.c1875);
    kick_apply<NP, true, D3>(s, kp);
    return true;
}

template <bool D3, int NP, int L, int KG = 0, int ACC = RVM_DRIFT_ACC>
__device__ __forceinline__ bool segment_gated_c(Lane<NP>& s, KickPrep<NP>& kp, double h, int ns, int nt,
                                                const gu64* c0, const gu64* c1, unsigned long long tag,
                                                bool late = false) {
    if (late) {
        if (nt <= 6) return segment_steps_c<6, D3, NP, L, KG, 64, 3>(s, kp, h, ns, c0, c1, tag);
        if (nt == 7) return segment_steps_c<7, D3, NP, L, KG, 64, 3>(s, kp, h, ns, c0, c1, tag);
        return segment_steps_c<8, D3, NP, L, KG, 64, 3>(s, kp, h, ns, c0, c1, tag);
    }
    if (nt <= 6) return segment_steps_c<6, D3, NP, L, KG, 64, ACC>(s, kp, h, ns, c0, c1, tag);
    if (nt == 7) return segment_steps_c<7, D3, NP, L, KG, 64, ACC>(s, kp, h, ns, c0, c1, tag);
    return segment_steps_c<8, D3, NP, L, KG, 64, ACC>(s, kp, h, ns, c0, c1, tag);
}

// ---- the two directions of a walker meet (rvm_logl.hip finish) -------------------------------
// One 64-bit slot per walker (plan workspace, RVM_SLOT_EMPTY between launches).  The direction that
// arrives first leaves its result there, the second takes it with one agent-scope exchange:
//   settled  chi2 >= 0 (sign bit clear, finite)
//   open     -lb (sign bit set, finite; -0.0 for lb = 0): the adaptive resolution's lower bound on
//            the direction's chi2 (rvm_refine.hip, oracle/rvoracle.c walker_cut)
//   status   a negative quiet NaN whose low byte is the status (PRIOR, ENCOUNTER, NONFINITE, ...)
#define RVM_SLOT_EMPTY 0x7FF4DEADBEEF0001ULL  // a NaN pattern no direction result can take
#define RVM_SLOT_STATUS 0xFFF8000000000000ULL
__device__ __forceinline__ unsigned long long slot_status(int st) {
    return RVM_SLOT_STATUS | (unsigned long long)(unsigned)st;
}
__device__ __forceinline__ bool slot_is_status(unsigned long long b) { return (b & 0xFFFFFFFFFFFFFF00ULL) == RVM_SLOT_STATUS; }

// per-direction flag bits of a walker (encflag / enc): 1 encounter, 2 prior, 4 unresolved after
// the last refinement, 8 a hand-off of this launch gave up (the values are not trustworthy)
#define RVM_ENC_UNRESOLVED 4
#define RVM_ENC_FAULT 8

// a direction's status from its flag bits and chi2 (prior > encounter > fault > unresolved;
// a settled direction's non-finite chi2 is NONFINITE)
__device__ __forceinline__ int dir_status(int enc, bool open, double chi2) {
    int st = (enc & 2) ? RVM_STATUS_PRIOR : RVM_STATUS_OK;
    if (st == RVM_STATUS_OK && (enc & 1)) st = RVM_STATUS_ENCOUNTER;
    if (st == RVM_STATUS_OK && (enc & RVM_ENC_FAULT)) st = RVM_STATUS_NONFINITE;
    if (st == RVM_STATUS_OK && (enc & RVM_ENC_UNRESOLVED)) st = RVM_STATUS_UNRESOLVED;
    if (st == RVM_STATUS_OK && !open && !isfinite(chi2)) st = RVM_STATUS_NONFINITE;
    return st;
}

// lower bound on an open direction's chi2 after a stage (oracle/rvoracle.c lb_of): chi2 less the
// change the stage brought (d; +inf if none) or a large multiple of its estimate, 0 if non-finite
__device__ __forceinline__ double open_lb(double chi2, double d, double est_raw) {
    const double b = chi2 - fmin(d, RVM_CUT_EST_FACTOR * est_raw);
    return b > 0.0 ? b : 0.0;  // (NaN -> 0)
}

// The sampler's accept inputs of walker slot wo of a fused launch (the certain-reject test):
// dmode 0 none, 1 emcee stretch, 2 MH; z, u and the current lnp.  Half 1's slots of a speculative
// iteration accept later (rvm_stretch_iteration_end) but their inputs are known (sa.lnp1).
__device__ __forceinline__ void accept_inputs(const StretchArgs& sa, int wo, int& dmode, double& dz, double& du,
                                              double& dl) {
    dmode = 0;
    dz = du = dl = 0.0;
    if (sa.c != nullptr) {
        int k2, wk2, j2, jp2;
        double z2, zp2;
        stretch_slot(sa, wo, k2, wk2, z2, j2, zp2, jp2);
        if (k2 == 0) {
            dmode = 1;
            du = stretch_u3(sa.seed, (uint64_t)(sa.s0_begin + wo), sa.iteration, sa.half);
            dl = sa.lnp[wo];
        } else if (sa.lnp1 != nullptr) {
            dmode = 1;
            du = stretch_u3(sa.seed, (uint64_t)(sa.s1_begin + wk2), sa.iteration, 1u);
            dl = sa.lnp1[wk2];
        }
        dz = z2;
    } else if (sa.mh_scale != nullptr) {
        dmode = 2;
        du = mh_u(sa.seed, (uint64_t)(sa.s0_begin + wo), sa.iteration);
        dl = sa.lnp[wo];
    }
}

__device__ __forceinline__ bool accepts_at(const StretchArgs& sa, int dmode, double dz, double du, double dl,
                                           double lp) {
    return dmode == 1 ? stretch_accepts(sa.dim, dz, lp, dl, du) : mh_accepts(lp, dl, du);
}

// The walker's final writes: logl / status, the fault counters, and (fused sampler launches) the
// accept with the proposal's rows row(r) written back on acceptance.
template <int R, typename Row>
__device__ __forceinline__ void walker_out(const DevPlan& P, const StretchArgs& sa, const int wo, const int stw,
                                           const double lp, double* __restrict__ logl_out,
                                           int32_t* __restrict__ status_out, Row&& row, const double z, const double u3,
                                           const double lnp0) {
    if (logl_out) logl_out[wo] = lp;
    if (status_out) status_out[wo] = stw;
    // (rare: counted for rvm_plan_faults -- never a silent rejection)
    if (stw == RVM_STATUS_NONFINITE || stw == RVM_STATUS_UNRESOLVED)
        __hip_atomic_fetch_add(P.counters + (stw == RVM_STATUS_NONFINITE ? 1 : 2), 1ull, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    const bool mh = sa.mh_scale != nullptr;
    const bool fused = sa.c != nullptr || mh;
    if (fused && (sa.n_spec == 0 || wo < sa.n_spec)) {
        // emcee / MH accept (half 1's slots of a speculative iteration only deliver their logl:
        // rvm_stretch_iteration_end)
        const bool acc = mh ? mh_accepts(lp, lnp0, u3) : stretch_accepts(sa.dim, z, lp, lnp0, u3);
        if (acc) {
#pragma unroll
            for (int r = 0; r < R; r++) {
                if (sa.src[r] >= 0) {
                    const double v = row(r);
                    sa.x[(size_t)sa.src[r] * sa.xstride + wo] = v;
                    if (sa.x_aos) sa.x_aos[(size_t)wo * sa.dim + sa.src[r]] = v;
                }
            }
            sa.lnp[wo] = lp;
            if (sa.accepted) sa.accepted[wo] += 1;
        }
        if (sa.dec) sa.dec[wo] = acc ? 1 : 0;
    }
}

}  // namespace rvm

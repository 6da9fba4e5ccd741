// rvm_logl.hip -- the walker log-likelihood kernel for gfx950 (MI355X).
//
// Replaces, for a whole batch of walkers at once, the reference's
//   State.get_logp (state.py:103-110) -> priorHard (:299-315) -> get_chi2 (:89-98)
//   -> get_rv x2 (:61-73) -> setup_sim (:36-47) + REBOUND IAS15 integrate + Encounter.
//
// Work decomposition:
//   workgroup = 64/L walkers x one direction (blockIdx.y: 0 = epochs t >= 0, 1 = t < 0)
//               x n_levels waves; wave L integrates the same walkers with mult[L]x the base steps
//               (Wisdom-Holman KDK, epoch-aligned segments).  At every epoch each wave drops its
//               64 model RVs into LDS, one barrier, and wave 0 forms the Richardson-extrapolated
//               RV (sum_L w_L rv_L, the h^2 -> 0 limit) and accumulates chi2 in registers.
//   lanes     = the planets of one walker sit on L = 1/2/4 adjacent lanes (one Kepler drift per
//               lane, positions exchanged by DPP quad permutes for the kick); solver state in
//               registers; the epoch schedule is staged once into LDS and read wave-uniformly;
//               walker parameters are read once from SoA [n_params][n_walkers].
// A walker's two directions meet in one 8-byte slot per walker (agent-scope atomic exchange): the
// lane that gets the other direction's result back finishes the walker, logl =
// -(chi2_b + chi2_f)/Npoints.  With StretchArgs the same launch is a whole emcee stretch
// half-step: the walkers' parameters are their proposals (formed in the prologue from the
// walker-major complement), and the finishing lane runs the accept (rvm_stretch.h).
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>

// FMA contraction only within one source expression (explicit fma() everywhere it matters): the
// same step code then rounds identically in every loop it is inlined into (speculative and gated
// segments, both launch layouts), so a walker's bits never depend on its wave-mates or the layout.
// (The default -ffp-contract=fast fuses across statements depending on the surrounding code.)
#pragma clang fp contract(on)

#include "rvm_walker.h"

// the main pass's drifts with the fifth-order Kepler guess (rvm_device.h drift G5; A/B knob, off:
// the main pass's waves share SIMDs, where the extra VALU cost more than the second Halley steps save
// at the bench window -- DESIGN.md §10)
#ifndef RVM_MAIN_G5
#define RVM_MAIN_G5 0
#endif

namespace rvm {

#ifdef RVM_PROFILE
// Timing build (make profile -> scripts/probe/librvmcmc_prof.so): per wave, s_memtime at kernel
// start, after the prologue, accumulated inside segments, accumulated in epoch handling (incl.
// the barrier), and at the end.  Read with rvm_prof_copy (scripts/probe/prof_kernel.py).
#define RVM_PROF_SLOTS 18
#define RVM_PROF_MAX_WAVES 4096
__device__ unsigned long long rvm_prof[RVM_PROF_MAX_WAVES * RVM_PROF_SLOTS];
#define PROF_T(v) const unsigned long long v = __builtin_readcyclecounter()
#define PROF_COUNT(var) (var)++
#else
#define PROF_T(v)
#define PROF_COUNT(var)
#endif


// Level-split hand-off of level 1 (type-B block -> the unit's combiner): the star vx of walker w at
// epoch e of direction d sits in P.lv_rv[(d lv_emax + e) lv_stride + w]; all-ones (a NaN no
// computed value takes: v0 is canonicalised) marks an empty slot.  The producer's agent-scope
// relaxed store is write-through (sc1), the consumer polls with agent-scope relaxed loads (L1
// bypassed) and puts the sentinel back: the value is the flag (cdna_hip_programming.md §6
// Guideline 16, R2), no fence on either side.  Encounter / prior flags likewise in P.lv_enc (-1).
#define RVM_LV_EMPTY 0xFFFFFFFFFFFFFFFFULL
// Bounded waits: a hand-off wait gives up after P.spin_ticks of the 100 MHz real-time counter
// WITHOUT PROGRESS (the clock restarts at every epoch that arrives, so a long launch never times
// out while it advances), counts the give-up in the plan's fault counter (rvm_plan_faults) and
// reports its walkers NONFINITE instead of hanging the GPU.  Blocks are all resident by
// construction: launch_logl uses the layout only when its grid fits the CUs.

// D3: inclined systems (7 parameter rows per planet, m a h k l ix iy; 3-D positions/velocities)
// (the 3-planet LDS-coupled instantiation within 168 VGPRs: three waves per SIMD, so that two blocks of
// the paired layout -- one group and its extension wave, five waves each -- share a CU, launch_logl_t;
// at 170 the second block waited for the first: two rounds)
template <int NP, bool D3, bool DEC>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(NP == 3 && !D3 && !DEC ? 3 : 1)))
void logl_kernel(const DevPlan P, const int W,
                                                                   const double* __restrict__ params,
                                                                   const double hill_factor,
                                                                   unsigned long long* __restrict__ slots,
                                                                   double* __restrict__ rv_out,
                                                                   double* __restrict__ logl_out,
                                                                   int32_t* __restrict__ status_out,
                                                                   const StretchArgs sa, const int nA, const int lsm) {
    constexpr int L = LanesPerWalker<NP>::value;  // lanes per walker (one per planet)
    constexpr int WPB = 64 / L;                    // walkers per block (= per wave)
    PROF_T(t_start);
#ifdef RVM_PROFILE
    const unsigned long long rt_start = __builtin_amdgcn_s_memrealtime();
#endif
    // A block holds G = 1 or 2 walker groups (launch_logl), each one wave per level.  Group 1
    // runs the levels in mirrored order: consecutive waves of a block land on consecutive SIMDs,
    // so wave i of group 1 shares a SIMD with wave i of group 0 and every SIMD carries
    // mult[i] + mult[nl-1-i] steps per base step instead of up to 2 mult[nl-1].
    //
    // Level-split layout (nA > 0; four levels m0 < m1 < m2 < m3, 1-D grid of 8-wave blocks, one
    // per CU, wave i on SIMD i % 4): a unit = (walker group, direction), u = 2 group + direction.
    // Type-A blocks (b < nA) carry levels 3, 2, 0 of units 2b, 2b + 1 and their combiners, type-B
    // blocks level 1 (the roles below).  Levels 3, 2, 0 of
    // a unit hand their star velocities to the combiner through an LDS ring (with per-level epoch
    // counters), level 1 -- in a type-B block on another CU, usually another XCD -- through HBM, one
    // agent-scope 8-byte store per walker and epoch whose arrival is the value itself (the slot holds
    // a NaN sentinel in between).  The combiner forms the Richardson RVs and chi^2 (same arithmetic
    // as the LDS-coupled path) epoch by epoch while the levels still integrate, then finishes the
    // walkers: when the last level ends, only its last epoch is left to combine.
    const int nl = P.n_levels;
    const int wv = threadIdx.x >> 6;
    constexpr bool dec = DEC;  // (nA > 0)
    int grp, lvl, G, d, w0;
    bool idle = false;
    // (recomputed where needed, not kept live through the integration)
    // the type-B blocks (level 1 of eight units, every SIMD critical) are dispatched first: the
    // last blocks of a grid start several us after the first (measured: 450 -> 439 us per
    // 6144-walker launch, scripts/probe/handoff_ab.sh)
    const int nB = (int)gridDim.x - nA;
    const int bid = (int)blockIdx.x < nB ? nA + (int)blockIdx.x : (int)blockIdx.x - nB;
    // level-split roles (8-wave blocks, wave i on SIMD i % 4; part: 0 whole level, 1 / 2 the head /
    // tail of a level split at an epoch, the state handed over through LDS in slot hs):
    //   type A, units 2b + (wv & 1): waves 0, 1 level 3; 2, 3 level 2; and either (splitA) 6, 7 the
    //     heads of level 0 (epochs [0, split0)), then the units' combiners, with 4, 5 its tails on
    //     SIMDs 0, 1 -- SIMD loads m3 + m0 (1 - f), m2 + m0 f with f = split0's share of the steps
    //     (rvm_plan_create: 0.735 at 4..7, 0.11 above the 8.5 / 8.5 balance because the tail's SIMD
    //     runs level 3 alone until the head ends); or 6, 7 level 0 whole and 4, 5 the combiners
    //     from the start (10, 7) when a direction has more epochs than the ring holds
    //   type B, tB = 8 units of level 1 per block: waves 0..7 one each (2 m1 per SIMD); or tB = 6
    //     (all CUs in use): waves 0..3 whole, 4 / 5 head / tail of unit 4, 6 / 7 of unit 5 (1.5 m1)
    //   with the extension level (lsx, an adaptive plan whose directions fit the ring): type A, units
    //     2b + (wv & 1), waves 0, 1 the extension (plan slot nl = 4, P.ext_mult steps per base step),
    //     2, 3 level 3, 4, 5 level 0 -- then the units' combiners --, 6, 7 level 1: SIMD loads
    //     m_x + m0 and m3 + m1; type B level 2 of tB = 8 units (2 m2), handed over through HBM
    const int tB = lsm & 0xFF;
    const bool splitA = ((lsm >> 8) & 1) != 0;  // (needs the whole direction in the ring: E <= RVM_LS_RING)
    const bool lsx = dec && ((lsm >> 9) & 1) != 0;
    const int hl = lsx ? 2 : 1;   // the level handed over through HBM (type-B blocks)
    const int NK = lsx ? 4 : 3;   // levels per unit in the type-A ring
    const int tsk = wv < 4 || tB == 8 ? wv : (wv < 6 ? 4 : 5);  // type-B task of this wave
    auto unit_of = [&]() { return bid < nA ? 2 * bid + (wv & 1) : tB * (bid - nA) + tsk; };
    int part = 0, hs = 0;
    if (dec) {
        const int b = bid;
        const int unit = __builtin_amdgcn_readfirstlane(unit_of());  // wave-uniform (SGPRs)
        lvl = __builtin_amdgcn_readfirstlane(
            b < nA ? (lsx ? (wv < 2 ? nl : (wv < 4 ? 3 : (wv < 6 ? 0 : 1))) : (wv < 2 ? 3 : (wv < 4 ? 2 : 0))) : hl);
        idle = b < nA && !splitA && !lsx && (wv == 4 || wv == 5);  // the combiners (no integration)
        if (b < nA) {
            part = splitA ? (wv >= 6 ? 1 : (wv >= 4 ? 2 : 0)) : 0;
            hs = wv & 1;
        } else {
            part = tB == 8 || wv < 4 ? 0 : ((wv & 1) ? 2 : 1);
            hs = (wv - 4) >> 1;
        }
        // wave-uniform in the compiler's eyes (SGPRs): branches on them stay scalar and the state
        // they select (the encounter mask) stays in SGPRs
        part = __builtin_amdgcn_readfirstlane(part);
        hs = __builtin_amdgcn_readfirstlane(hs);
        idle = __builtin_amdgcn_readfirstlane((int)idle) != 0;
        grp = 0;
        G = 1;
        d = unit & 1;
        w0 = (unit >> 1) * WPB;
    } else {
        // (cx: one group per block plus a wave for the extension level, nl + 1 waves)
        const bool cxw = (int)(blockDim.x >> 6) == nl + 1;
        grp = !cxw && wv >= nl ? 1 : 0;
        // wave-uniform extrapolation level (nl: the extension).  cx with four levels: waves 0..4 take
        // levels 1, 3, 2, the extension, 0 -- wave i runs on SIMD i % 4, so the fifth wave's SIMD
        // carries levels 0 + 1 (9 steps per base step) and the extension (8) has a SIMD of its own,
        // instead of extension + level 0 = 12 beside level 3 alone
        lvl = grp ? 2 * nl - 1 - wv : (cxw && nl == 4 ? (0x04231 >> (4 * wv)) & 15 : wv);
        G = cxw ? 1 : (blockDim.x >> 6) / nl;
        d = blockIdx.y;
        w0 = (blockIdx.x * G + grp) * WPB;  // first walker of the group
    }
    // Concurrent extension (LDS-coupled layout with one group per block, launch_logl): when the
    // blocks leave SIMDs with room (at most one block per CU), the adaptive resolution's extension
    // level (P.ext_mult steps per base step, plan slot nl) runs as an extra wave of the main pass
    // from t = 0 -- on a SIMD of its own, levels 0 and 1 sharing one -- instead of after it.  The combiner
    // forms r5 and its acceptance sums at every epoch; the flagged walkers then take the
    // extension's verdict at once (the same bits as extend_pass: the same integration, the same
    // sums), and only the halving passes remain.
    const bool cx = !dec && (int)(blockDim.x >> 6) == nl + 1;
    const bool live = w0 < W && !idle;  // level-split: waves past the last unit only help stage the schedule
    const bool comb = dec && idle;       // level-split: this unit's combiner from the start
    const int lane = threadIdx.x & 63;
    const int slot = lane / L;                     // walker slot within the group
    const int pl_idx = lane % L;
    const int w = w0 + slot;
    const bool valid = w < W;
    const int wl = valid ? w : (W - 1);

    // level-split hand-off inside a type-A block (unit ul = wv & 1; local level slot ks = 0, 1, 2
    // for levels 3, 2, 0): epochs published per level, epochs consumed by the combiner, the levels'
    // encounter / prior flags; the RVs themselves sit in the ring after the schedule (s_sched)
    __shared__ int s_lvp[2][4];
    __shared__ int s_cprog[2];
    // LDS-coupled layouts (round 5): each group's levels publish their star vx per epoch in a ring of
    // RVM_LC_RING epochs after the stretch staging and the lanes' t = 0 state (dynamic LDS,
    // [group][epoch % ring][level (nl + 1: the extension)][WPB]) and their progress here; the group's combiner (level 0's
    // wave) combines epoch e once every level has published it and publishes its own progress
    __shared__ int s_lcp[2][RVM_MAX_LEVELS + 1];
    __shared__ int s_lcc[2];
    __shared__ int s_encl[2][4][64];
    // head -> tail hand-off of a split level (slot hs): the lanes' dynamic state, the wave's
    // encounter mask and speculation state, and the ready flag
    __shared__ double s_hos[2][8][64];
    __shared__ unsigned long long s_hoe[2];
    __shared__ int s_hosp[2], s_hof[2];
    __shared__ int s_enc_all[2][RVM_MAX_LEVELS][64];
    // adaptive resolution: walker slots of each group (LDS-coupled) / unit (level-split) still above
    // the estimate bound; the level-split combiners' verdicts (0 pending, 1 finished, 2 refine) and
    // their results for the refinement team
    __shared__ unsigned long long s_need[2];
    __shared__ double s_fchi[2][64];
    __shared__ int s_fenc[2][64];
    // (the early certain-reject test of the refinement team: the main pass's estimate and the
    // concurrent extension's chi2 and change, per unit and walker slot)
    __shared__ double s_fx[1][2][64];
    int(*s_enc)[64] = s_enc_all[grp];
    // this direction's epoch schedule, staged once into LDS (wave-uniform broadcast reads later)
    extern __shared__ double s_sched[];  // [E] seg_h1 | [E] obs_rv | [E] obs_s2 | [E] (seg_n, obs_idx)
                                         // then, for a fused stretch half-step, [rows+3][G*WPB]

    const DirSched S = d ? P.bwd : P.fwd;
    // wave-uniform copies (SGPRs): the level's step divisor and Stumpff series length (rvm_device.h)
    const int lvl_u = __builtin_amdgcn_readfirstlane(lvl);
    const int mult = P.mult[lvl_u];
    const int nt = P.nt[lvl_u];
    const bool spec = P.spec[lvl_u] != 0 && nt <= 6;
    const double inv_mult = P.inv_mult[lvl_u];
    const int E = S.n_epochs;
    const int emax2 = P.fwd.n_epochs > P.bwd.n_epochs ? P.fwd.n_epochs : P.bwd.n_epochs;
    double* l_dir = dec ? s_sched + (size_t)d * 4 * emax2 : s_sched;  // level-split: both directions staged
    double* l_len = l_dir;
    double* l_rv = l_dir + E;
    double* l_s2 = l_dir + 2 * E;
    int* l_n = reinterpret_cast<int*>(l_dir + 3 * E);
    int* l_idx = l_n + E;
    // fused stretch half-step: the proposal rows, z, u3 and the current lnp of every walker of the
    // block, for the lane that finishes the walker (end of the kernel)
    const int GW = G * WPB;
    const int gi = grp * WPB + slot;  // walker slot within the block
    double* l_q = s_sched + 4 * E;    // [rows][GW], then z | u3 | lnp0
    // first chunk of the schedule: loads issued now, stored to LDS after the setup below so their
    // latency hides behind the Pal conversion
    const int i0 = threadIdx.x;
    double st_h = 0.0, st_rv = 0.0, st_s2 = 0.0;
    int st_n = 0, st_idx = 0;
    if (!dec && i0 < E) {
        st_h = S.seg_h1[i0];
        st_rv = S.obs_rv[i0];
        st_s2 = S.obs_s2[i0];
        st_n = S.seg_n[i0];
        st_idx = S.obs_idx[i0];
    }

    // ---- walker parameters (m, a, h, k, l [, ix, iy] per planet), prior (state.py:299-315) -----
    // Fused stretch half-step (sa.c != nullptr): the walker's parameters are its proposal
    // q = c_j - z (c_j - x) mapped onto the kernel rows (rvm_stretch.h, rvm_param_map).
    constexpr int PR = D3 ? 7 : 5;  // parameter rows per planet
    const bool stretch = sa.c != nullptr;
    const bool mh = sa.mh_scale != nullptr;  // fused MH step (rvm_mh_step)
    const bool fused = stretch || mh;        // accepts at the end
    const bool mapped = fused || sa.fd_x != nullptr;  // parameters formed from StretchArgs
    double zst = 0.0, zp = 0.0;
    int jst = 0, jp = 0, kind = 0, wk = wl;
    // slot kind (speculative iteration, StretchArgs): see stretch_slot
    if (stretch) stretch_slot(sa, wl, kind, wk, zst, jst, zp, jp);
    // one lane per walker stages the accept inputs; only kind-0 slots accept in this launch, and
    // sa.lnp holds just their n_spec (or W) entries -- half 1's slots must not read it
    const bool stager = !dec && fused && lvl == 0 && pl_idx == 0 && kind == 0;
    if (stager) {
        constexpr int R = PR * NP;
        l_q[R * GW + gi] = zst;
        l_q[(R + 1) * GW + gi] = mh ? mh_u(sa.seed, (uint64_t)(sa.s0_begin + wl), sa.iteration)
                                    : stretch_u3(sa.seed, (uint64_t)(sa.s0_begin + wl), sa.iteration, sa.half);
        l_q[(R + 2) * GW + gi] = sa.lnp[wl];
    }
    // the walker's parameter rows; a fused MH step spreads its Box-Muller proposals over the
    // walker's planet lanes (lane q forms rows q, q + L, ...; DPP broadcast within the group), so
    // each lane draws ceil(R / L) normals instead of R -- same bits, a shorter prologue
    constexpr int R = PR * NP;
    double rowv[R];
    if (L > 1 && mh) {
        constexpr int NI = (R + L - 1) / L;
#pragma unroll
        for (int i = 0; i < NI; i++) {
            // (the row's map entries selected with compile-time indices: a lane-dependent index into
            // the kernel argument would make the compiler copy StretchArgs to scratch)
            int k = -1;
            double bs = 0.0;
#pragma unroll
            for (int q = 0; q < L; q++) {
                const int rr = L * i + q < R ? L * i + q : R - 1;
                if (pl_idx == q) {
                    k = sa.src[rr];
                    bs = sa.base[rr];
                }
            }
            const double v = k < 0 ? bs
                                   : mh_q(sa.x[(size_t)k * sa.xstride + wk], sa.mh_step, sa.mh_scale[k],
                                          mh_normal(sa.seed, (uint64_t)(sa.s0_begin + wk), sa.iteration, k));
#pragma unroll
            for (int q = 0; q < L; q++)
                if (L * i + q < R) rowv[L * i + q] = grp_get<L>(v, q);
        }
    } else {
#pragma unroll
        for (int r = 0; r < R; r++) rowv[r] = walker_param(mapped, params, W, wk, sa, r, zst, jst, kind, zp, jp);
    }
    if (stager) {
#pragma unroll
        for (int r = 0; r < R; r++) l_q[r * GW + gi] = rowv[r];
    }
    // ---- setup_sim: prior, Pal -> heliocentric (own planet) -> Jacobi; Hill exit (rvm_walker.h) ----
    Lane<NP> s;
    int status = RVM_STATUS_OK;
    double e2w;  // the adaptive resolution's eccentricity guard (P.e2_guard): the walker's largest e^2
    walker_setup<NP, D3, L>(rowv, pl_idx, hill_factor, s, status, e2w);
    PROF_T(t_p1);
    PROF_T(t_p2);  // parameters read, prior checked, Pal -> Jacobi done
    // adaptive resolution: the lanes' state at t = 0 for refinement passes, in LDS after the
    // schedule and the stretch staging (LDS-coupled: [group][8][64]) or after the level-split ring
    // ([unit][8][64]; the unit's level-3 wave keeps it)
    const int ring_sz = emax2 < RVM_LS_RING ? emax2 : RVM_LS_RING;
    double* l_init = dec ? s_sched + (size_t)8 * emax2 + (size_t)2 * NK * ring_sz * WPB
                         : s_sched + (size_t)4 * emax2 + (fused ? (size_t)(R + 3) * GW : 0);
    if (P.rmax > 0 && (dec ? (bid < nA && wv < 2) : lvl == 0)) {
        double* o = l_init + (size_t)(dec ? wv : grp) * RVM_INIT_DOUBLES + lane;
        o[0] = s.rx;
        o[64] = s.ry;
        o[128] = s.vx;
        o[192] = s.vy;
        o[256] = s.rz;
        o[320] = s.vz;
        o[384] = s.r;
        o[448] = s.ir;
    }
    // the interaction at t = 0 (the first segment's opening half kick) and REBOUND's check of
    // exit_min_distance before the first step -- when it integrates at all: get_rv of an empty
    // epoch list never does
    KickPrep<NP> kp{};
    if (S.n_epochs > 0) kp = kick_prep<NP, L, D3>(s, 1.875);

    PROF_T(t_p3);  // lane constants, encounter check at t = 0
    if (!dec) {
        if (threadIdx.x < 2 * (RVM_MAX_LEVELS + 1)) (&s_lcp[0][0])[threadIdx.x] = 0;
        if (threadIdx.x < 2) s_lcc[threadIdx.x] = 0;
        if (i0 < E) {
            l_len[i0] = st_h;
            l_rv[i0] = st_rv;
            l_s2[i0] = st_s2;
            l_n[i0] = st_n;
            l_idx[i0] = st_idx;
        }
        for (int i = i0 + blockDim.x; i < E; i += blockDim.x) {
            l_len[i] = S.seg_h1[i];
            l_rv[i] = S.obs_rv[i];
            l_s2[i] = S.obs_s2[i];
            l_n[i] = S.seg_n[i];
            l_idx[i] = S.obs_idx[i];
        }
    } else {
        if (threadIdx.x < 8) (&s_lvp[0][0])[threadIdx.x] = 0;
        if (threadIdx.x < 2) s_cprog[threadIdx.x] = 0;
        if (threadIdx.x < 2) s_hof[threadIdx.x] = 0;
        for (int dd = 0; dd < 2; dd++) {
            const DirSched& SD = dd ? P.bwd : P.fwd;
            double* b = s_sched + (size_t)dd * 4 * emax2;
            const int ED = SD.n_epochs;
            int* bn = reinterpret_cast<int*>(b + 3 * ED);
            for (int i = i0; i < ED; i += blockDim.x) {
                b[i] = SD.seg_h1[i];
                b[ED + i] = SD.obs_rv[i];
                b[2 * ED + i] = SD.obs_s2[i];
                bn[i] = SD.seg_n[i];
                bn[ED + i] = SD.obs_idx[i];
            }
        }
    }

    // Level-split layout: waves wv and wv ^ 4 share a SIMD and run free (no epoch barrier couples
    // them).  Equal-priority waves issue oldest first, so one ran at its lone-wave rate and
    // the others crawled until it was done (the SIMD's instruction streams overlapped for a fraction
    // of the time only).  Each wave publishes its remaining work (steps weighted by the level's
    // step cost) in LDS at
    // every epoch and takes the higher issue priority while it has more left than its SIMD partner:
    // the pair finishes together, overlapped throughout.  A head and its partner instead keep equal
    // pace (weighted steps done): the head ends about when its tail can best share the other SIMD
    // (measured: head-first priority serialised its SIMD, remaining-work priority started the
    // tail too late).
    PROF_T(t_p4);  // schedule staged (before the barrier)
    __shared__ int s_rem[8], s_done[8];
    const int wcost = spec ? 10 : 12;  // gated steps (ballot per drift) cost ~20 % more (timing build)
    const int esplit = lvl == 0 ? S.split0 : S.split1;  // head / tail boundary of a split level
    // (readfirstlane: wave-uniform in the compiler's eyes too -- a per-lane epoch range turns the
    // step loops into exec-masked loops with a VGPR trip counter)
    const int e_lo = __builtin_amdgcn_readfirstlane(part == 2 ? esplit : 0);
    const int e_hi = __builtin_amdgcn_readfirstlane(part == 1 ? esplit : E);
    int rem = live ? mult * (S.n_steps - (part == 2 ? (lvl == 0 ? S.pre0 : S.pre1) : 0)) * wcost : 0;
    // a head runs first (its tail, on another SIMD, cannot start before it ends): it publishes more
    // remaining work than any whole level has
    int done = 0;
    // (LDS-coupled layouts, round 5: waves wv and wv ^ 4 share a SIMD -- the cx layout's levels 1 and
    // 0, the two-group layout's mirrored pairs -- and without the per-epoch barrier run free, so they
    // balance their issue priority by remaining work as the level-split waves do)
    const bool lc_pair = !dec && (wv ^ 4) < (int)(blockDim.x >> 6);
    if ((dec || lc_pair) && lane == 0) {
        s_rem[wv] = rem;
        s_done[wv] = 0;
    }
    // the SIMD partner (wv ^ 4) heads a split level: type A waves 6, 7 (splitA), type B 4, 6 (tB = 6)
    const bool oth_head = bid < nA ? (splitA && (wv == 2 || wv == 3)) : (tB == 6 && (wv == 0 || wv == 2));

    // ---- integrate outward from t = 0 through this direction's epochs -------------------------
    __syncthreads();  // schedule staged
    if (dec && !live && !comb) return;  // (no block barrier follows in the level-split layout)
    PROF_T(t_pro);
#ifdef RVM_PROFILE
    unsigned long long t_seg = 0, t_epo = 0;
#endif
    int redo = 0;      // speculative segments redone gated (counted in the timing build only)
    int spec_off = 0;  // wave-uniform: segments left to run gated after a redo
    int spec_bo = 4;   // wave-uniform: the next back-off, doubled by each redo (a walker whose orbit
                       // keeps needing the general solver), back to 4 after a clean segment
    double chi2 = 0.0;
    double est = 0.0;  // adaptive resolution: sum_e |(rv - o)^2 - (rv3 - o)^2| / s2 (combiner lanes)
    double c5x = 0.0, ddx = 0.0;  // the concurrent extension's chi2 and acceptance sum (cx)
    // level-split hand-off: level 1's column of P.lv_rv (one epoch row per epoch); the other levels'
    // slot in the block's LDS ring ([unit ul][local level ks][RING][WPB] doubles after the schedule)
    const int ul = wv & 1;
    const int ks = lsx ? (lvl == 3 ? 0 : (lvl == 1 ? 1 : (lvl == 0 ? 2 : 3))) : (lvl == 3 ? 0 : (lvl == 2 ? 1 : 2));
    const int RING = emax2 < RVM_LS_RING ? emax2 : RVM_LS_RING;
    double* ring = s_sched + (size_t)8 * emax2;
    gu64* lv1p = dec ? (gu64*)(P.lv_rv + ((size_t)d * P.lv_emax + e_lo) * P.lv_stride + wl) : nullptr;
    int rslot = RING > 0 ? e_lo % RING : 0;
    const int E_int = comb ? 0 : e_hi;  // the combiners integrate nothing
    bool wfault = false;  // wave-uniform: a hand-off wait of this wave gave up (RVM_ENC_FAULT)
    SpinClock clk;
    if (dec && part == 2) {
        // a tail: wait for the head's state at epoch e_lo (same block, LDS); the head (type A: wave
        // + 2, type B: wave - 1) publishes its progress at every epoch
        const int head = bid < nA ? wv + 2 : wv - 1;
        int seen = -1;
        clk.restart();
        while (__builtin_amdgcn_readfirstlane(__hip_atomic_load(&s_hof[hs], __ATOMIC_ACQUIRE,
                                                                 __HIP_MEMORY_SCOPE_WORKGROUP)) == 0) {
            const int pd = __builtin_amdgcn_readfirstlane(
                __hip_atomic_load(s_done + head, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP));
            if (pd != seen) {
                seen = pd;
                clk.restart();
            } else if (clk.expired(P.spin_ticks)) {
                wfault = true;
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
        s.rx = s_hos[hs][0][lane];
        s.ry = s_hos[hs][1][lane];
        s.vx = s_hos[hs][2][lane];
        s.vy = s_hos[hs][3][lane];
        s.rz = s_hos[hs][4][lane];
        s.vz = s_hos[hs][5][lane];
        s.r = s_hos[hs][6][lane];
        s.ir = s_hos[hs][7][lane];
        // (readfirstlane is 32-bit signed: each half through `unsigned`, or a set bit 31 -- an
        // encounter on lane 30/31 -- would sign-extend into all 32 upper lanes)
        s.encm = (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(s_hoe[hs] & 0xFFFFFFFFull)) |
                 ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(s_hoe[hs] >> 32)) << 32);
        spec_off = __builtin_amdgcn_readfirstlane(s_hosp[hs]) & 0xFFFF;
        spec_bo = __builtin_amdgcn_readfirstlane(s_hosp[hs]) >> 16;
        // the interaction at the hand-off epoch, from the same positions: the head's bits (its
        // encounter test repeats on positions the head already tested)
        kp = kick_prep<NP, L, D3>(s, 1.875);
    }
    // (LDS-coupled) this group's ring of the levels' star vx, after the lanes' t = 0 state
    const int NLC = nl + (cx ? 1 : 0);  // levels that publish (the extension wave too)
    const int RC = P.lc_ring;  // (rvm_plan_create: min(RVM_LC_RING, epochs), within RVM_LC_RING_BYTES)
    double* lring = dec ? nullptr
                        : l_init + (P.rmax > 0 ? (size_t)G * RVM_INIT_DOUBLES : 0) +
                              (size_t)grp * RC * (nl + 1) * WPB;
    // (LDS-coupled) the combiner's side: the epochs every other level has published (wave-uniform),
    // a bounded wait for epoch ec, and the combine of epoch ec -- Richardson RV, chi2, estimate, the
    // extension's sums, the RV for a refinement -- in epoch order (the bits of the barrier-coupled
    // loop), then its progress for the writers
    int next_c = 0;  // (combiner) the next epoch to combine
    auto lc_min = [&]() {
        int mn = 1 << 30;
        for (int k = 1; k < NLC; k++)
            mn = min(mn, __hip_atomic_load(&s_lcp[grp][k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
        return __builtin_amdgcn_readfirstlane(mn);
    };
    auto lc_wait = [&](const int ec) {
        int seen = -1;
        clk.restart();
        for (;;) {
            const int mn = lc_min();
            if (mn > ec) return;
            if (mn != seen) {
                seen = mn;
                clk.restart();
            } else if (clk.expired(P.spin_ticks)) {
                wfault = true;
                return;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    };
    auto lc_combine = [&](const int ec) {
        const double* rv_e = lring + (size_t)(ec % RC) * (nl + 1) * WPB;
        if (lane < WPB) {  // lane `lane` of level 0's wave owns walker slot `lane`
            double rvx = 0.0, rv3 = 0.0;
            for (int k = 0; k < nl; k++) rvx += P.lw[k] * rv_e[(size_t)k * WPB + lane];
            for (int k = 1; k < nl; k++) rv3 += P.lw3[k] * rv_e[(size_t)k * WPB + lane];
            const double r = rvx - l_rv[ec];
            chi2 += (r * r) / l_s2[ec];
            est += fabs((rvx - rv3) * (r + (rv3 - l_rv[ec]))) / l_s2[ec];
            const int wo = w0 + lane;
            if (rv_out != nullptr && wo < W) rv_out[(size_t)l_idx[ec] * W + wo] = rvx;
            if (P.ext_mult > 0 && wo < W) {  // the RV and the extension's partial sum, for a refinement
                double s5 = 0.0;
                for (int k = 0; k < nl; k++) s5 += P.lw5[k] * rv_e[(size_t)k * WPB + lane];
                const size_t xi = (size_t)(d * P.lvx_emax + ec) * P.lvx_stride + wo;
                if (cx) {  // (extend_pass's sums, from the extension wave's value of this epoch)
                    const double r5 = s5 + P.lw5[nl] * rv_e[(size_t)nl * WPB + lane];
                    const double q = r5 - l_rv[ec];
                    c5x += (q * q) / l_s2[ec];
                    ddx += fabs((r5 - rvx) * (q + (rvx - l_rv[ec]))) / l_s2[ec];
                } else {
                    P.lvx[xi] = s5;
                }
                P.rvp[xi] = rvx;
            }
        }
        // (the combiner has read epoch ec: its ring slot may be rewritten)
        if (lane == 0) __hip_atomic_store(&s_lcc[grp], ec + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    int n1 = e_lo < E ? l_n[e_lo] : 0;
    double len = e_lo < E ? l_len[e_lo] : 0.0;
    for (int e = e_lo; e < E_int; e++) {
        // prefetch the next segment while this one integrates
        const int n1_next = e + 1 < E ? l_n[e + 1] : 0;
        const double len_next = e + 1 < E ? l_len[e + 1] : 0.0;
        const int ns = n1 * mult;
        // the partner's remaining work, read now and used after the segment (latency hidden)
        int rem_oth = 0, done_oth = 0;
        if (dec || lc_pair) {
            rem_oth = __hip_atomic_load(s_rem + (wv ^ 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            done_oth = __hip_atomic_load(s_done + (wv ^ 4), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        PROF_T(ta);
        if (ns > 0) {
            const double h = len * inv_mult;  // len holds the segment's base step
            if (spec) {  // (implies nt == 6)
                // speculate unless a recent segment of this wave needed a redo: walkers whose
                // orbits keep needing the general solver (short periods, high eccentricity in a
                // wide ensemble) then run gated for a while instead of paying for redos
                if (spec_off == 0) {
                    if (segment<6, true, D3, NP, L, RVM_MAIN_G5 != 0>(s, kp, h, ns, redo)) {
                        spec_off = spec_bo;
                        spec_bo = spec_bo < 64 ? 2 * spec_bo : 64;
                    } else {
                        spec_bo = 4;
                    }
                } else {
                    segment<6, false, D3, NP, L, RVM_MAIN_G5 != 0>(s, kp, h, ns, redo);
                    spec_off--;
                }
            } else if (nt <= 6)
                segment<6, false, D3, NP, L, RVM_MAIN_G5 != 0>(s, kp, h, ns, redo);
            else if (nt == 7)
                segment<7, false, D3, NP, L, RVM_MAIN_G5 != 0>(s, kp, h, ns, redo);
            else
                segment<8, false, D3, NP, L, RVM_MAIN_G5 != 0>(s, kp, h, ns, redo);
        }
        PROF_T(tb);
        const double v0 = star_vx<NP, L>(s);
        if (dec) {
            rem -= ns * wcost;
            done += ns * wcost;
            if (lane == 0) {
                __hip_atomic_store(s_rem + wv, rem, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_store(s_done + wv, done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            // (operands through readfirstlane: a provably wave-uniform branch around each
            // s_setprio, which ignores EXEC -- cdna_hip_programming.md §5.5 T5)
            const int ro = __builtin_amdgcn_readfirstlane(rem_oth), rm = __builtin_amdgcn_readfirstlane(rem);
            const int dn = __builtin_amdgcn_readfirstlane(done), dno = __builtin_amdgcn_readfirstlane(done_oth);
            const bool high = part == 1 ? dn <= dno : (oth_head ? dn < dno : ro < rm);
            if (__builtin_amdgcn_readfirstlane((int)high))
                __builtin_amdgcn_s_setprio(2);
            else
                __builtin_amdgcn_s_setprio(1);
            if (lvl == hl) {
                if (pl_idx == 0 && valid) {
                    unsigned long long bits = (unsigned long long)__double_as_longlong(v0);
                    if (bits == RVM_LV_EMPTY) bits = 0x7FF8000000000000ULL;  // (still a NaN)
                    __hip_atomic_store(lv1p, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                lv1p += P.lv_stride;
            } else {
                // wait while the combiner is a whole ring behind (only when E > RING)
                if (E > RING && !wfault) {
                    int seen = -1;
                    for (;;) {
                        const int cp = __builtin_amdgcn_readfirstlane(
                            __hip_atomic_load(s_cprog + ul, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                        if (e - cp < RING) break;
                        if (cp != seen) {
                            seen = cp;
                            clk.restart();
                        } else if (clk.expired(P.spin_ticks)) {
                            wfault = true;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(4);
                    }
                }
                if (pl_idx == 0) ring[((ul * NK + ks) * RING + rslot) * WPB + slot] = v0;
                if (lane == 0) __hip_atomic_store(&s_lvp[ul][ks], e + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                rslot = rslot + 1 == RING ? 0 : rslot + 1;
            }
        } else {
            if (lc_pair) {
                rem -= ns * wcost;
                if (lane == 0) __hip_atomic_store(s_rem + wv, rem, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                const int ro = __builtin_amdgcn_readfirstlane(rem_oth), rm = __builtin_amdgcn_readfirstlane(rem);
                if (__builtin_amdgcn_readfirstlane((int)(ro < rm)))
                    __builtin_amdgcn_s_setprio(2);
                else
                    __builtin_amdgcn_s_setprio(1);
            }
            // publish this epoch in the group's ring.  A whole ring ahead of the combiner: a level
            // waits (only when E > RC; a wait without progress for spin_ticks gives up:
            // RVM_ENC_FAULT), the combiner itself combines the oldest epochs first
            if (lvl == 0) {
                while (!wfault && e - next_c >= RC) {
                    lc_wait(next_c);
                    if (!wfault) lc_combine(next_c++);
                }
            } else if (E > RC && !wfault && e >= RC) {
                int seen = -1;
                for (;;) {
                    const int cp = __builtin_amdgcn_readfirstlane(
                        __hip_atomic_load(&s_lcc[grp], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP));
                    if (e - cp < RC) break;
                    if (cp != seen) {
                        seen = cp;
                        clk.restart();
                    } else if (clk.expired(P.spin_ticks)) {
                        wfault = true;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(4);
                }
            }
            if (pl_idx == 0) lring[((size_t)(e % RC) * (nl + 1) + lvl) * WPB + slot] = v0;
            if (lane == 0) __hip_atomic_store(&s_lcp[grp][lvl], e + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (lvl == 0 && !wfault) {
                // the combiner integrates on and combines, without waiting, the epochs every level
                // has published (the rest after its last segment)
                const int mn = min(lc_min(), e + 1);
                while (next_c < mn) lc_combine(next_c++);
            }
        }
        n1 = n1_next;
        len = len_next;
#ifdef RVM_PROFILE
        PROF_T(tc);
        t_seg += tb - ta;
        t_epo += tc - tb;
#endif
    }
    if (!dec && lvl == 0) {  // (LDS-coupled) the combiner: the epochs the others published later
        while (!wfault && next_c < E_int) {
            lc_wait(next_c);
            if (!wfault) lc_combine(next_c++);
        }
    }
    const int encflag = (int)(((s.encm >> lane) & kick_enc_bits<NP>()) != 0) |
                        (status == RVM_STATUS_PRIOR ? 2 : 0) | (wfault ? RVM_ENC_FAULT : 0);
    // ---- the two directions of a walker meet: the second to arrive finishes it ----------------
    // (one agent-scope exchange carries the other direction's result: no fence, no barrier; the
    // slot encoding is rvm_walker.h's).  A direction arrives settled (chi2), open (the adaptive
    // resolution's lower bound lbw on its chi2: it needs halving passes) or with a status.  The
    // second arriver finishes the walker when neither direction is open; otherwise it applies the
    // walker's certain-reject test on both lower bounds (a settled direction's is its chi2; fused
    // sampler launches) and, unless that rejects, hands the walker to the refinement kernel
    // (rvm_refine.hip) through the plan's work lists.  row(r), z, u3, lnp0: the walker's proposal
    // and accept inputs (fused sampler step).
    auto finish = [&](const int wo, const double chi2w, const int enc, const bool open, const double lbw, auto&& row,
                      const double z, const double u3, const double lnp0) __attribute__((always_inline)) {
        const int st = dir_status(enc, open, chi2w);
        const unsigned long long mine =
            st != RVM_STATUS_OK ? slot_status(st)
                                : (unsigned long long)__double_as_longlong(open ? -lbw : chi2w);
        const unsigned long long old =
            __hip_atomic_exchange(slots + wo, mine, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (old == RVM_SLOT_EMPTY) return;
        __hip_atomic_store(slots + wo, RVM_SLOT_EMPTY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int st_o = RVM_STATUS_OK;
        bool open_o = false;
        double v_o = 0.0;
        if (slot_is_status(old)) {
            st_o = (int)(old & 0xFF);
        } else {
            v_o = __longlong_as_double((long long)old);
            open_o = signbit(v_o);
            v_o = fabs(v_o);
        }
        const double v_m = open ? lbw : chi2w;
        const int sf = d == 0 ? st : st_o, sb = d == 0 ? st_o : st;
        const bool of = d == 0 ? open : open_o, ob = d == 0 ? open_o : open;
        const double cf = d == 0 ? v_m : v_o, cb = d == 0 ? v_o : v_m;
        int stw = sf != RVM_STATUS_OK ? sf : sb;  // both directions see the same PRIOR verdict
        // (an encounter in one direction ends the walker whatever the other's resolution: a direction
        // left UNRESOLVED by a flag-only plan does not hide it -- oracle/rvoracle.c any_enc)
        if (stw == RVM_STATUS_UNRESOLVED && (sf == RVM_STATUS_ENCOUNTER || sb == RVM_STATUS_ENCOUNTER))
            stw = RVM_STATUS_ENCOUNTER;
        const double lp0 = -((cb + cf) / P.npoints);  // state.py:98, 109 (open: the upper bound lp_hi)
        if (stw == RVM_STATUS_OK && (of || ob)) {
            int dmode = 0;
            double dz, du, dl;
            if (P.ext_mult > 0 && P.cut) accept_inputs(sa, wo, dmode, dz, du, dl);
            if (dmode != 0 && isfinite(lp0) && !accepts_at(sa, dmode, dz, du, dl, lp0)) {
                // a certain reject: rejected whatever the refinement would give; reports lp_hi
                __hip_atomic_fetch_add(P.counters + 4, (unsigned long long)((of ? 1 : 0) + (ob ? 1 : 0)),
                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                // to the refinement kernel: list 0 both directions open, 1 forward only, 2 backward only
                const int li = of && ob ? 0 : (of ? 1 : 2);
                const int ix = __hip_atomic_fetch_add(P.rq_n + li, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (ix < P.rq_cap) {
                    P.rq_w[(size_t)li * P.rq_cap + ix] = wo;
                    P.rq_mark[wo] = (int32_t)__hip_atomic_load(P.gen_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    P.rq_c[wo] = of ? 0.0 : cf;
                    P.rq_c[(size_t)P.rq_cap + wo] = ob ? 0.0 : cb;
                    return;
                }
                // (never past the lists: counts left over from a launch whose refinement kernel did
                // not run make the walker a counted NONFINITE, not an out-of-bounds store)
                stw = RVM_STATUS_NONFINITE;
            }
        }
        if (stw == RVM_STATUS_OK && !isfinite(lp0)) stw = RVM_STATUS_NONFINITE;
        walker_out<R>(P, sa, wo, stw, stw == RVM_STATUS_OK ? lp0 : -INFINITY, logl_out, status_out, row, z, u3, lnp0);
    };
    // finishing a walker without the LDS-staged proposal (level-split layout): the slot's draws again
    // (recomputed from an opaque index rather than kept live through the integration)
    auto finish_recompute = [&](const int w_in, const double chi2w, const int enc, const bool open, const double lbw) __attribute__((always_inline)) {
        if (stretch) {
            int wo = w_in, k2, wk2, j2, jp2;
            double z2, zp2;
            asm volatile("" : "+v"(wo));
            stretch_slot(sa, wo, k2, wk2, z2, j2, zp2, jp2);
            auto row = [&](int r) { return walker_param(true, params, W, wk2, sa, r, z2, j2, k2, zp2, jp2); };
            // (lnp0 exists for the accepting kind-0 slots only: sa.lnp is n_spec long)
            finish(wo, chi2w, enc, open, lbw, row, z2,
                   stretch_u3(sa.seed, (uint64_t)(sa.s0_begin + wo), sa.iteration, sa.half), k2 == 0 ? sa.lnp[wo] : 0.0);
        } else if (mh) {
            auto row = [&](int r) { return walker_param(true, params, W, w_in, sa, r, 0.0, 0, 0, 0.0, 0); };
            finish(w_in, chi2w, enc, open, lbw, row, 0.0, mh_u(sa.seed, (uint64_t)(sa.s0_begin + w_in), sa.iteration),
                   sa.lnp[w_in]);
        } else {
            auto row = [&](int) { return 0.0; };
            finish(w_in, chi2w, enc, open, lbw, row, 0.0, 0.0, 0.0);
        }
    };

    int dummy_redo = 0;
    // ---- adaptive resolution, stage 1: the extension level ----------------------------------
    // One wave per group / unit -- its combiner wave -- integrates one more level (P.ext_mult steps
    // per base step) of direction dr from t = 0 and joins it, epoch by epoch, to the main pass's
    // levels: r5 = all nl + 1 levels (lw5), formed from the main pass's partial sum over its own
    // levels (P.lvx, sum_k lw5[k] rv_k, kept by every launch) and its RV r (P.rvp) -- two numbers per
    // epoch and walker, the same bits as summing the levels here.  A marked walker (combiner lane
    // `lane`, its bit in need_m) is settled -- chi2 from r5 -- when the extension changed chi2 by at most
    // sum |(r5-o)^2 - (r-o)^2| / s2 <= RVM_EXT_ACCEPT rtol_dir npoints (r = the main pass's RV); an
    // encounter of the extension ends it ENCOUNTER, a non-finite one NONFINITE; otherwise the
    // halving passes follow.  One wave, no barrier: each epoch's value
    // moves from the walker's first lane to its combiner lane by a shuffle, and the stored levels
    // of the next epoch load while this one integrates.
    auto extend_pass = [&](const int gr, const int dr, const uint64_t need_m, bool& need, double& chi2w, int& enc,
                           double& c5o, double& ddo) __attribute__((always_inline)) {
        const DirSched& SR = dr ? P.bwd : P.fwd;
        const int Er = SR.n_epochs;
        const double* r_dir = dec ? s_sched + (size_t)dr * 4 * emax2 : l_dir;
        const double* r_len = r_dir;
        const double* r_rv = r_dir + Er;
        const double* r_s2 = r_dir + 2 * Er;
        const int* r_n = reinterpret_cast<const int*>(r_dir + 3 * Er);
        const int* r_idx = r_n + Er;
        {
            const double* in = l_init + (size_t)gr * RVM_INIT_DOUBLES + lane;
            s.rx = in[0];
            s.ry = in[64];
            s.vx = in[128];
            s.vy = in[192];
            s.rz = in[256];
            s.vz = in[320];
            s.r = in[384];
            s.ir = in[448];
            s.encm = 0;
        }
        KickPrep<NP> kq{};
        if (Er > 0) kq = kick_prep<NP, L, D3>(s, 1.875);
        const int mx = P.ext_mult;
        const int ntx = P.ext_nt;
        const double ix = P.inv_ext;
        const int cs = lane & (WPB - 1);  // combiner lane -> walker slot
        const bool cl = lane < WPB && ((need_m >> lane) & 1);
        const int wo = w0 + cs;
        const size_t xb = (size_t)dr * P.lvx_emax * P.lvx_stride + (cl ? wo : 0);
        const double* xs = P.lvx + xb;
        const double* xr = P.rvp + xb;
        double a5 = cl && Er > 0 ? xs[0] : 0.0, a4 = cl && Er > 0 ? xr[0] : 0.0;
        double c5 = 0.0, dd = 0.0;
        int x_off = 0, x_bo = 4;  // speculation back-off (as the main pass's spec_off / spec_bo)
        for (int e = 0; e < Er; e++) {
            const bool nx = cl && e + 1 < Er;
            const double b5 = nx ? xs[(size_t)(e + 1) * P.lvx_stride] : 0.0;
            const double b4 = nx ? xr[(size_t)(e + 1) * P.lvx_stride] : 0.0;
            const int ns = r_n[e] * mx;
            if (ns > 0) {
                const double h = r_len[e] * ix;
                if (P.ext_spec && ntx <= 6) {  // (the main pass's speculation policy: same bits)
                    if (x_off == 0) {
                        if (segment<6, true, D3, NP, L, RVM_MAIN_G5 != 0>(s, kq, h, ns, dummy_redo)) {
                            x_off = x_bo;
                            x_bo = x_bo < 64 ? 2 * x_bo : 64;
                        } else {
                            x_bo = 4;
                        }
                    } else {
                        segment<6, false, D3, NP, L, RVM_MAIN_G5 != 0>(s, kq, h, ns, dummy_redo);
                        x_off--;
                    }
                } else if (ntx <= 6)
                    segment<6, false, D3, NP, L, RVM_MAIN_G5 != 0>(s, kq, h, ns, dummy_redo);
                else if (ntx == 7)
                    segment<7, false, D3, NP, L, RVM_MAIN_G5 != 0>(s, kq, h, ns, dummy_redo);
                else
                    segment<8, false, D3, NP, L, RVM_MAIN_G5 != 0>(s, kq, h, ns, dummy_redo);
            }
            const double v = star_vx<NP, L>(s);
            const double vx = __shfl(v, cs * L);
            if (cl) {
                const double r = a4;
                const double r5 = a5 + P.lw5[nl] * vx;
                const double q = r5 - r_rv[e];
                c5 += (q * q) / r_s2[e];
                dd += fabs((r5 - r) * (q + (r - r_rv[e]))) / r_s2[e];
                if (rv_out != nullptr && wo < W) rv_out[(size_t)r_idx[e] * W + wo] = r5;
            }
            a5 = b5;
            a4 = b4;
        }
        const bool xenc = ((s.encm >> (cs * L)) & kick_enc_bits<NP>()) != 0;
        if (cl) {
            c5o = c5;
            ddo = dd;
        }
        if (cl && need) {
            if (xenc) {
                enc |= 1;
                chi2w = c5;
                need = false;
            } else if (dd <= RVM_EXT_ACCEPT * P.rtol_dir * P.npoints) {  // (false for a non-finite one)
                chi2w = c5;
                need = false;
            }
        }
    };
    // The extension stage over the walker slots marked in s_need[g] of the active groups (gmask;
    // set by the caller, one barrier since) when the launch has no concurrent extension wave: the
    // combiner waves (lr == 0) run extend_pass, every wave meets at the barrier.  The combiner lanes
    // (cmb: level 0's wave, lane < WPB) update need / chi2w / enc and take the extension's chi2
    // and change (xc5, xdd) for the walker's lower bound.  Halving passes are the refinement
    // kernel's (rvm_refine.hip).
    auto extend_stage = [&](const int lr, const int gr, const int dr, bool& need, double& chi2w, int& enc,
                            double& xc5, double& xdd) __attribute__((always_inline)) {
        if (P.ext_mult > 0) {
            const uint64_t gneed = s_need[gr];
            if (lr == 0 && gneed) {
                if (lane == 0)
                    __hip_atomic_fetch_add(P.counters + 3, (unsigned long long)__builtin_popcountll(gneed),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                extend_pass(gr, dr, gneed, need, chi2w, enc, xc5, xdd);
            }
            __syncthreads();
        }
    };
    // a combiner lane's direction after the main pass and the extension: open (need) with the lower
    // bound on its chi2 (oracle/rvoracle.c dir_extend: the extension's when it is finite, else the
    // main pass's with its estimate alone), or settled; without halving passes (rmax = 0) an open
    // direction is UNRESOLVED
    auto direction_lb = [&](const bool need, const double chi2_main, const double est_raw, const bool xran,
                            const double xc5, const double xdd) __attribute__((always_inline)) {
        if (!need) return 0.0;
        if (xran && isfinite(xc5) && isfinite(xdd)) return open_lb(xc5, xdd, est_raw);
        return open_lb(chi2_main, INFINITY, est_raw);
    };

    if (!dec) {
        if (pl_idx == 0) s_enc[lvl][slot] = encflag;
        __syncthreads();
        const bool cmb = lvl == 0 && lane < WPB;  // lane `lane` of wave 0 owns walker slot `lane`
        const int wo = w0 + lane;
        int enc = 0;
        // (adaptive plans: an encounter only the coarser levels see refines the direction instead
        // of ending the walker, DevPlan::fin_level; `cenc`)
        bool cenc = false;
        if (cmb) {
            int encc = 0;
            for (int k = 0; k < nl; k++) {
                const int f = s_enc[k][lane];
                if (k == P.fin_level || !(P.rtol_dir < INFINITY)) {
                    enc |= f;
                } else {
                    enc |= f & ~1;
                    encc |= f & 1;
                }
            }
            cenc = encc != 0 && (enc & 1) == 0;
        }
        double chi2w = chi2;
        bool need = false;
        double lbw = 0.0;
        if (P.rtol_dir < INFINITY) {  // (kernel argument: uniform)
            // (a non-finite chi2 -- the fixed step blowing up on an extreme orbit -- refines too, and
            // so does a walker past the eccentricity guard: its e^2 from the walker's first lane,
            // and one whose coarser levels alone came within the exit distance -- its main pass,
            // like a non-finite one, neither settles nor bounds it: the stored RV of a refinement's
            // first step-doubling change is invalidated, oracle/rvoracle.c dir_main `bad`)
            const double e2c = __shfl(e2w, (lane & (WPB - 1)) * L);
            need = cmb && wo < W && enc == 0 &&
                   (est / P.npoints > P.rtol_dir || !isfinite(chi2w) || !isfinite(est) ||
                    (P.ext_mult > 0 && e2c > P.e2_guard) || cenc);
            if (cenc && need && P.ext_mult > 0)
                for (int e = 0; e < E; e++) P.rvp[(size_t)(d * P.lvx_emax + e) * P.lvx_stride + wo] = __builtin_nan("");
            if (P.rmax == 0) {
                if (need) enc |= RVM_ENC_UNRESOLVED;
                need = false;
            } else {
                const bool need0 = need;
                if (cx) {  // (block-uniform)
                    if (lvl == 0) {
                        // the concurrent extension's verdict (extend_pass's rule on the same sums)
                        const uint64_t nx = ballot(need);
                        if (lane == 0 && nx)
                            __hip_atomic_fetch_add(P.counters + 3, (unsigned long long)__builtin_popcountll(nx),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (need) {
                            if (s_enc[nl][lane] & 1) {
                                enc |= 1;
                                chi2w = c5x;
                                need = false;
                            } else if (!cenc && ddx <= RVM_EXT_ACCEPT * P.rtol_dir * P.npoints) {
                                chi2w = c5x;
                                need = false;
                            }
                        }
                    }
                } else if (P.ext_mult > 0) {
                    if (lvl == 0) {
                        const uint64_t nb = ballot(need);
                        if (lane == 0) s_need[grp] = nb;
                    }
                    __syncthreads();
                    if ((s_need[0] | (G > 1 ? s_need[1] : 0ull)) != 0)
                        extend_stage(lvl, grp, d, need, chi2w, enc, c5x, ddx);
                }
                // (the extension's bound only below the cut guard, DevPlan::e2_cut)
                lbw = cenc ? 0.0 : direction_lb(need, chi2, est, need0 && P.ext_mult > 0 && (e2c <= P.e2_cut || P.cut_guard_k > 0.0), c5x,
                                                   e2c <= P.e2_cut ? ddx : P.cut_guard_k * ddx);
            }
        }
        if (cmb && wo < W) {
            const int gl = grp * WPB + lane;
            auto row = [&](int r) { return l_q[r * GW + gl]; };
            if (fused)
                finish(wo, chi2w, enc, need, lbw, row, l_q[R * GW + gl], l_q[(R + 1) * GW + gl],
                       l_q[(R + 2) * GW + gl]);
            else
                finish(wo, chi2w, enc, need, lbw, row, 0.0, 0.0, 0.0);
        }
    } else {
        // level-split: level waves publish their flags; the combiner finishes the unit, or hands it
        // to the block's refinement team (all eight waves of a type-A block)
#ifdef RVM_PROFILE
        const unsigned long long rt_integ = __builtin_amdgcn_s_memrealtime();
        auto prof_dec = [&](unsigned long long rt_arr, int arr) {
            const int gw = (int)blockIdx.x * (blockDim.x >> 6) + wv;
            if (lane == 0 && gw < RVM_PROF_MAX_WAVES) {
                unsigned long long* o = rvm_prof + (size_t)gw * RVM_PROF_SLOTS;
                o[0] = t_start;
                o[1] = t_pro;
                o[2] = t_seg;
                o[3] = t_epo;
                o[4] = __builtin_readcyclecounter();
                o[5] = rt_start;
                o[6] = __builtin_amdgcn_s_memrealtime();
                // (level field 7: a combiner)
                o[7] = (unsigned long long)(comb || (part == 1 && bid < nA) ? 7 : lvl) | ((unsigned long long)d << 8) |
                       ((unsigned long long)mult << 16) |
                       ((unsigned long long)part << 24);
                o[8] = (unsigned long long)redo;
                o[9] = (unsigned long long)E;
                o[10] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);
                o[11] = rt_integ;
                o[12] = rt_arr;
                o[13] = (unsigned long long)arr | ((unsigned long long)unit_of() << 8);
                o[14] = t_p1;
                o[15] = t_p2;
                o[16] = t_p3;
                o[17] = t_p4;
            }
        };
#endif
        if (part == 1) {
            // a head: hand the state over to the tail and leave
            s_hos[hs][0][lane] = s.rx;
            s_hos[hs][1][lane] = s.ry;
            s_hos[hs][2][lane] = s.vx;
            s_hos[hs][3][lane] = s.vy;
            s_hos[hs][4][lane] = s.rz;
            s_hos[hs][5][lane] = s.vz;
            s_hos[hs][6][lane] = s.r;
            s_hos[hs][7][lane] = s.ir;
            if (lane == 0) {
                s_hoe[hs] = s.encm;
                s_hosp[hs] = spec_off | (spec_bo << 16);
                __hip_atomic_store(&s_hof[hs], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            if (bid >= nA) {  // (type-B heads have no combiner role)
#ifdef RVM_PROFILE
                prof_dec(__builtin_amdgcn_s_memrealtime(), lvl);
#endif
                return;
            }
            // type A: this wave now combines its unit
            if (lane == 0) {  // (its partner no longer keeps pace with it)
                __hip_atomic_store(s_rem + wv, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                __hip_atomic_store(s_done + wv, 1 << 30, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        if (!comb && part != 1) {
            // a level wave: publish this level's encounter / prior flags (type B: and leave)
            if (lvl == hl) {
                if (pl_idx == 0 && valid)
                    __hip_atomic_store((gi32*)(P.lv_enc + (size_t)d * P.lv_stride + w), encflag, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            } else {
                if (pl_idx == 0) s_encl[ul][ks][slot] = encflag;
                if (lane == 0) __hip_atomic_store(&s_lvp[ul][ks], E + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
#ifdef RVM_PROFILE
            prof_dec(__builtin_amdgcn_s_memrealtime(), lvl);
#endif
            if (bid >= nA) return;
        }
        // (lsx: level 0's wave, its integration done, combines its unit -- the ring holds every epoch)
        if (comb || part == 1 || (lsx && lvl == 0)) {
            // the unit's combiner: consume epoch e once the local levels have published it (LDS
            // counters) and the HBM-handed level's values have landed (every lane's slot off the
            // sentinel); lowest issue priority (it shares a SIMD with a level wave).  A plan whose
            // hand-off workspace is dirty from an earlier give-up (counters[0] != 0, until
            // rvm_plan_faults resets it) reports every walker NONFINITE without waiting.
            __builtin_amdgcn_s_setprio(0);
            bool hung = __hip_atomic_load(P.counters, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0ull;
            hung = __builtin_amdgcn_readfirstlane((int)hung) != 0;
            const bool dirty = hung;
            auto local_published = [&]() {
                int p = __hip_atomic_load(&s_lvp[ul][0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                for (int k = 1; k < NK; k++) {
                    const int pk = __hip_atomic_load(&s_lvp[ul][k], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    p = pk < p ? pk : p;
                }
                return __builtin_amdgcn_readfirstlane(p);
            };
            gu64* l1 = (gu64*)(P.lv_rv + (size_t)d * P.lv_emax * P.lv_stride + wl);
            double chi2w = 0.0;
            double c5x = 0.0, ddx = 0.0;  // lsx: the extension's chi2 and acceptance sum (as extend_pass)
            int rr = 0;
            // one epoch: the levels in order 0..3 (same arithmetic as the LDS-coupled path), b1 the
            // HBM-handed level's bits
            auto consume = [&](const int e, const unsigned long long b1) {
                double* rg = ring + (size_t)rr * WPB + slot;
                const size_t rs = (size_t)RING * WPB;
                const double vh = __longlong_as_double((long long)b1);
                double v[4];
                if (lsx) {
                    v[0] = rg[(ul * 4 + 2) * rs];
                    v[1] = rg[(ul * 4 + 1) * rs];
                    v[2] = vh;
                    v[3] = rg[(ul * 4 + 0) * rs];
                } else {
                    v[0] = rg[(ul * 3 + 2) * rs];
                    v[1] = vh;
                    v[2] = rg[(ul * 3 + 1) * rs];
                    v[3] = rg[(ul * 3 + 0) * rs];
                }
                double rvx = 0.0, rv3 = 0.0;
#pragma unroll
                for (int k = 0; k < 4; k++) rvx += P.lw[k] * v[k];
#pragma unroll
                for (int k = 1; k < 4; k++) rv3 += P.lw3[k] * v[k];
                const double r = rvx - l_rv[e];
                chi2w += (r * r) / l_s2[e];
                est += fabs((rvx - rv3) * (r + (rv3 - l_rv[e]))) / l_s2[e];
                if (rv_out != nullptr && valid && pl_idx == 0) rv_out[(size_t)l_idx[e] * W + w] = rvx;
                if (P.ext_mult > 0 && valid && pl_idx == 0) {  // the RV and the extension's partial sum
                    double s5 = 0.0;
#pragma unroll
                    for (int k = 0; k < 4; k++) s5 += P.lw5[k] * v[k];
                    const size_t xi = (size_t)(d * P.lvx_emax + e) * P.lvx_stride + w;
                    if (lsx) {  // (extend_pass's sums, from the extension wave's value of this epoch)
                        const double r5 = s5 + P.lw5[nl] * rg[(ul * 4 + 3) * rs];
                        const double q = r5 - l_rv[e];
                        c5x += (q * q) / l_s2[e];
                        ddx += fabs((r5 - rvx) * (q + (rvx - l_rv[e]))) / l_s2[e];
                        // the RV for a refinement's first step-doubling change, kept in level 0's ring
                        // slot (read; the ring holds the whole direction) and written to HBM only for
                        // the walkers the refinement kernel gets (below)
                        rg[(ul * 4 + 2) * rs] = rvx;
                    } else {
                        P.lvx[xi] = s5;
                        P.rvp[xi] = rvx;
                    }
                }
                // (the levels wait on it only when the ring wraps; a release store also waits for
                // every load in flight, the prefetched HBM values included)
                if (E > RING && lane == 0)
                    __hip_atomic_store(s_cprog + ul, e + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                rr = rr + 1 == RING ? 0 : rr + 1;
            };
            // The HBM-handed level's values are loaded PF epochs ahead, each into the register its
            // epoch's value just left (the loop is unrolled by PF: no register moves, which would
            // wait for the loads in flight): an lsx combiner starts when its own level is done and
            // finds most values landed -- one HBM latency per PF epochs.  A value still at the
            // sentinel is polled again when its epoch comes.  The hang clock restarts when a wait
            // begins (a wait's limit is time without progress).
            // The loads are unconditional (a lane past W reads walker W - 1's slot, an epoch past the
            // last re-reads the last; the values are masked afterwards): a load the compiler can
            // branch around leaves it unsure how many are in flight, and it then waits for all.
            constexpr int PF = 8;
            const int el = E > 0 ? E - 1 : 0;
            unsigned long long bq[PF];
#pragma unroll
            for (int j = 0; j < PF; j++)
                bq[j] = __hip_atomic_load(l1 + (size_t)(j < el ? j : el) * P.lv_stride, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
            gi32* e1p = (gi32*)(P.lv_enc + (size_t)d * P.lv_stride + wl);
            int f1 = __hip_atomic_load(e1p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // (early too)
            int pub = 0;  // the local levels' published epochs, as last read
            for (int e0 = 0; e0 < E; e0 += PF) {
#pragma unroll
                for (int j = 0; j < PF; j++) {
                    const int e = e0 + j;
                    if (e < E) {
                        if (pub <= e) {
                            pub = local_published();
                            if (pub <= e) clk.restart();
                            while (!hung && pub <= e) {
                                __builtin_amdgcn_s_sleep(2);
                                hung = clk.expired(P.spin_ticks);
                                pub = local_published();
                            }
                        }
                        gu64* le = l1 + (size_t)e * P.lv_stride;
                        unsigned long long b1 = valid ? bq[j] : 0ULL;
                        // (the test of the prefetched value in straight-line code, the poll as a
                        // bottom-tested loop: a loop header that reads b1 makes the compiler wait
                        // for every load in flight, vmcnt(0), at each epoch)
                        if (ballot(b1 == RVM_LV_EMPTY) != 0 && !hung) {
                            clk.restart();
                            do {
                                __builtin_amdgcn_s_sleep(2);
                                hung = clk.expired(P.spin_ticks);
                                b1 = valid ? __hip_atomic_load(le, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ULL;
                            } while (ballot(b1 == RVM_LV_EMPTY) != 0 && !hung);
                        }
                        bq[j] = __hip_atomic_load(l1 + (size_t)(e + PF < el ? e + PF : el) * P.lv_stride,
                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        if (valid && pl_idx == 0) __hip_atomic_store(le, RVM_LV_EMPTY, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        consume(e, b1);
                    }
                }
            }
            clk.restart();
            // the levels' flags: local ones after their last counter step (E + 1), level 1's from HBM
            while (!hung && local_published() <= E) {
                __builtin_amdgcn_s_sleep(2);
                hung = clk.expired(P.spin_ticks);
            }
            // (slot 0 is level 3, the finest; lsx: [3] the extension; the HBM-handed level's in f1)
            int enc = s_encl[ul][0][slot] | s_encl[ul][1][slot] | s_encl[ul][2][slot];
            int encc = 0;  // (adaptive: the coarser levels' encounter bits, DevPlan::fin_level)
            if (P.rtol_dir < INFINITY) {
                encc = (s_encl[ul][1][slot] | s_encl[ul][2][slot]) & 1;
                enc = s_encl[ul][0][slot] | ((s_encl[ul][1][slot] | s_encl[ul][2][slot]) & ~1);
            }
            {
                f1 = valid ? f1 : 0;
                if (ballot(f1 < 0) != 0 && !hung) {
                    do {
                        __builtin_amdgcn_s_sleep(2);
                        hung = clk.expired(P.spin_ticks);
                        f1 = valid ? __hip_atomic_load(e1p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
                    } while (ballot(f1 < 0) != 0 && !hung);
                }
                if (valid && pl_idx == 0) __hip_atomic_store(e1p, -1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const int f1p = f1 > 0 ? f1 : 0;
                if (P.rtol_dir < INFINITY) {
                    enc |= f1p & ~1;
                    encc |= f1p & 1;
                } else {
                    enc |= f1p;
                }
            }
            const bool cenc = encc != 0 && (enc & 1) == 0;
            if (hung) {  // never completed (or a dirty workspace): NONFINITE, and the give-up counted
                chi2w = __builtin_nan("");
                enc |= RVM_ENC_FAULT;
                if (!dirty && lane == 0)
                    __hip_atomic_fetch_add(P.counters, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
#ifdef RVM_PROFILE
            const unsigned long long rt_arr = __builtin_amdgcn_s_memrealtime();
#endif
            // adaptive resolution: settled, or open (with its lower bound) for the refinement kernel
            bool need = P.rtol_dir < INFINITY && valid && pl_idx == 0 && enc == 0 &&
                        (est / P.npoints > P.rtol_dir || !isfinite(chi2w) || !isfinite(est) ||
                         (P.ext_mult > 0 && e2w > P.e2_guard) || cenc);
            // (a coarse-only encounter's main pass neither settles nor bounds the direction: its
            // stored RV for a refinement's first step-doubling change is invalidated)
            if (cenc && need && !lsx && P.ext_mult > 0)
                for (int e = 0; e < E; e++) P.rvp[(size_t)(d * P.lvx_emax + e) * P.lvx_stride + w] = __builtin_nan("");
            if (need && P.rmax == 0) {
                enc |= RVM_ENC_UNRESOLVED;
                need = false;
            }
            const bool need0 = need;
            const double chi2m = chi2w;
            if (lsx) {  // the concurrent extension's verdict (extend_pass's rule on the same sums)
                const uint64_t nx = ballot(need);
                if (lane == 0 && nx)
                    __hip_atomic_fetch_add(P.counters + 3, (unsigned long long)__builtin_popcountll(nx),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (need) {
                    if (s_encl[ul][3][slot] & 1) {
                        enc |= 1;
                        chi2w = c5x;
                        need = false;
                    } else if (!cenc && ddx <= RVM_EXT_ACCEPT * P.rtol_dir * P.npoints) {
                        chi2w = c5x;
                        need = false;
                    }
                }
            }
            if (!lsx && P.ext_mult > 0 && ballot(need) != 0) {
                // the extension after the main pass, on this wave: its lanes take the walker slots
                // (lane = slot, extend_pass's convention) through LDS
                if (valid && pl_idx == 0) {
                    s_fchi[ul][slot] = chi2w;
                    s_fenc[ul][slot] = enc | (need ? 16 : 0) | (cenc ? 32 : 0) | (e2w > P.e2_cut ? 64 : 0);
                    s_fx[0][ul][slot] = est;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                const bool cl = lane < WPB && w0 + lane < W;
                double c2 = cl ? s_fchi[ul][lane] : 0.0;
                const int f = cl ? s_fenc[ul][lane] : 0;
                const double es = cl ? s_fx[0][ul][lane] : 0.0;
                const double cm = c2;
                int en = f & 15;
                bool nd = (f & 16) != 0;
                const bool cn = (f & 32) != 0;  // (a coarse-only encounter: the extension cannot settle it)
                const uint64_t nm = ballot(nd);
                if (lane == 0)
                    __hip_atomic_fetch_add(P.counters + 3, (unsigned long long)__builtin_popcountll(nm),
                                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                double xc5 = 0.0, xdd = 0.0;
                extend_pass(ul, d, nm, nd, c2, en, xc5, xdd);
                const double lb = cn ? 0.0 : direction_lb(nd, cm, es, (f & 16) != 0 && ((f & 64) == 0 || P.cut_guard_k > 0.0), xc5,
                                                                 (f & 64) != 0 ? P.cut_guard_k * xdd : xdd);
                if (cl) finish_recompute(w0 + lane, c2, en, nd, lb);
            } else if (valid && pl_idx == 0) {
                if (lsx && need) {  // the main pass's RV of an open direction (the ring, consume above)
                    const double* rg = ring + (size_t)(ul * 4 + 2) * RING * WPB + slot;
                    for (int e = 0; e < E; e++)
                        P.rvp[(size_t)(d * P.lvx_emax + e) * P.lvx_stride + w] = cenc ? __builtin_nan("") : rg[(size_t)e * WPB];
                }
                finish_recompute(w, chi2w, enc, need,
                                 cenc ? 0.0 : direction_lb(need, chi2m, est, lsx && need0 && (e2w <= P.e2_cut || P.cut_guard_k > 0.0), c5x,
                                                          e2w <= P.e2_cut ? ddx : P.cut_guard_k * ddx));
            }
#ifdef RVM_PROFILE
            prof_dec(rt_arr, nl - 1);
#endif
        }
        return;
    }
#ifdef RVM_PROFILE
    PROF_T(t_end);
    const int gw = (blockIdx.y * gridDim.x + blockIdx.x) * (blockDim.x >> 6) + wv;
    if (lane == 0 && gw < RVM_PROF_MAX_WAVES) {
        unsigned long long* o = rvm_prof + (size_t)gw * RVM_PROF_SLOTS;
        o[0] = t_start;
        o[1] = t_pro;
        o[2] = t_seg;
        o[3] = t_epo;
        o[4] = t_end;
        o[5] = rt_start;
        o[6] = __builtin_amdgcn_s_memrealtime();
        o[7] = (unsigned long long)lvl | ((unsigned long long)blockIdx.y << 8) | ((unsigned long long)mult << 16);
        o[8] = (unsigned long long)redo;
        o[9] = (unsigned long long)E;
        o[10] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID
        o[14] = t_p1;
        o[15] = t_p2;
        o[16] = t_p3;
        o[17] = t_p4;
    }
#endif
}

// Dynamic-LDS budget of one logl_kernel instantiation on the current device: the CU's 160 KB minus
// the kernel's own static LDS (hipFuncGetAttributes; ~28 KB), with the attribute that admits a
// dynamic request beyond 64 KB set once per device and instantiation.
template <int NPV, bool D3V, bool DECV>
static size_t lds_budget() {
    static size_t budget[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        (void)hipGetLastError();
        return 32 * 1024;
    }
    if (budget[dev] == 0) {
        const void* f = reinterpret_cast<const void*>(&logl_kernel<NPV, D3V, DECV>);
        hipFuncAttributes fa{};
        size_t b = 32 * 1024;  // (conservative if the runtime cannot tell)
        if (hipFuncGetAttributes(&fa, f) == hipSuccess && fa.sharedSizeBytes < (size_t)RVM_LDS_PER_CU) {
            const size_t lim = (size_t)RVM_LDS_PER_CU - fa.sharedSizeBytes;
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lim) == hipSuccess)
                b = lim;
            else if (fa.sharedSizeBytes < 64 * 1024)
                b = 64 * 1024 - fa.sharedSizeBytes;
        }
        (void)hipGetLastError();
        budget[dev] = b;
    }
    return budget[dev];
}

template <int NPV, bool D3V>
static hipError_t launch_logl_t(const DevPlan& P, int W, const double* params, double hill_factor,
                                unsigned long long* slots, double* logl, int32_t* status, double* rv_out,
                                const StretchArgs& sa, hipStream_t stream) {
    const int lpw = LanesPerWalker<NPV>::value;
    const int wpb = 64 / lpw;
    const int groups = (W + wpb - 1) / wpb;
    // one walker group per block while the blocks fit one per CU (every wave alone on its SIMD:
    // latency-bound); beyond that two groups with mirrored level order per block, which pairs
    // the heaviest level with the lightest on each SIMD (logl_kernel)
    // Paired one-group blocks (3 planets, round 6): where two groups would share a block, a launch of
    // at most one group per CU instead runs one group per block with the extension as its fifth wave
    // (cx below), two such blocks per CU (the 3-planet instantiation is held to 168 VGPRs for it) --
    // the extension beside the main pass instead of after it, for config 5's 4096-walker half-steps.
    // (A/B knob RVM_CX_PAIRS=0: the two-group blocks)
    static const bool pairs_env = [] {
        const char* e = getenv("RVM_CX_PAIRS");
        return !(e && e[0] == '0');
    }();
    const bool pairs = NPV == 3 && !D3V && pairs_env && P.ext_mult > 0 && rv_out == nullptr && P.n_cu > 0 &&
                       2 * groups > P.n_cu && groups <= P.n_cu && W >= RVM_CX_MIN_WALKERS;
    const int G = (!pairs && P.n_cu > 0 && 2 * groups > P.n_cu && 2 * P.n_levels * 64 <= 512) ? 2 : 1;
    dim3 grid((groups + G - 1) / G, 2);
    // one group per block (the blocks fit one per CU): the extension level as an extra wave
    // (logl_kernel, cx) when the plan has one and no model RVs are asked for.  The fifth wave shares
    // SIMD 0 with level 0 (4 + 8 steps per base step against level 3's 7 alone), which costs every
    // launch ~60 % (config 1's one-walker launch 0.335 -> 0.538 ms with nothing flagged,
    // scripts/probe/config1_probe.py): worth it only where a launch almost surely holds a flagged
    // walker.  Launches of a few walkers (the reference API's single-state calls) run the extension
    // after the main pass, only when flagged -- the same bits either way.
    const bool cx = G == 1 && P.ext_mult > 0 && rv_out == nullptr && W >= RVM_CX_MIN_WALKERS;
    dim3 block(64 * (P.n_levels + (cx ? 1 : 0)) * G);
    const int emax = P.fwd.n_epochs > P.bwd.n_epochs ? P.fwd.n_epochs : P.bwd.n_epochs;
    const size_t rows = (size_t)(D3V ? 7 : 5) * NPV;
    const bool fused = sa.c != nullptr || sa.mh_scale != nullptr;
    const size_t init = P.rmax > 0 ? (size_t)RVM_INIT_DOUBLES * sizeof(double) : 0;  // per group / unit
    // (+ the LDS-coupled layout's ring of the levels' star vx per group, logl_kernel lring)
    const size_t lc_ring = (size_t)P.lc_ring * (P.n_levels + 1) * wpb * sizeof(double);
    size_t smem = (size_t)emax * 4 * sizeof(double) + (fused ? (rows + 3) * G * wpb * sizeof(double) : 0) + G * init +
                  G * lc_ring;
    // level-split layout (logl_kernel) when it lowers the heaviest SIMD's load: in steps per base
    // step, max(m3, m2 + m0, 2 m1) for one round of <= n_cu blocks, against m3 per round of
    // single-group blocks or max_i(m_i + m_{n-1-i}) per round of two-group blocks
    int nA = 0, tB = 8, splitA = 0, lsx = 0;
    // with the adaptive resolution's extension level: where two groups would share a block (no
    // room for the concurrent extension wave), the level-split layout carries the extension as a
    // fifth level of the main pass (logl_kernel, lsx) -- the ring then holds whole directions
    if (P.lv_rv != nullptr && W <= P.lv_stride && P.n_levels == 4 && P.n_cu > 0 && P.ext_mult > 0 &&
        rv_out == nullptr && G == 2 && emax <= RVM_LS_RING) {
        const int units = 2 * groups;
        const int na = groups, nb = (units + 7) / 8;
        const size_t smem_x = (size_t)emax * 8 * sizeof(double) + (size_t)8 * emax * wpb * sizeof(double) + 2 * init;
        if (na + nb <= P.n_cu && smem_x <= lds_budget<NPV, D3V, true>()) {
            nA = na;
            tB = 8;
            lsx = 1;
            grid = dim3(na + nb, 1);
            block = dim3(8 * 64);
            smem = smem_x;
        }
    }
    if (nA == 0 && P.lv_rv != nullptr && W <= P.lv_stride && P.n_levels == 4 && P.n_cu > 0) {
        const int* m = P.mult;
        const int units = 2 * groups;
        // type-B blocks carry 6 units' level 1 (two of them split head / tail) when the CUs allow,
        // else 8
        const int na = groups;
        tB = na + (units + 5) / 6 <= P.n_cu ? 6 : 8;
        const int nb = (units + tB - 1) / tB;
        const int c_dec = std::max(m[3], std::max(m[2] + m[0], 2 * m[1]));
        const int c_cpl = G == 1 ? m[3] * ((2 * groups + P.n_cu - 1) / P.n_cu)
                                 : std::max(m[0] + m[3], m[1] + m[2]) * ((groups + P.n_cu - 1) / P.n_cu);
        const int ring = emax < RVM_LS_RING ? emax : RVM_LS_RING;
        const size_t smem_ls =
            (size_t)emax * 8 * sizeof(double) + (size_t)6 * ring * wpb * sizeof(double) + 2 * init;
        if (na + nb <= P.n_cu && c_dec < c_cpl && smem_ls <= lds_budget<NPV, D3V, true>()) {
            nA = na;
            grid = dim3(na + nb, 1);
            block = dim3(8 * 64);
            // level 0 split head / tail in the type-A blocks: the combiner starts with the head's
            // hand-off, so the ring must hold every epoch of a direction
            splitA = emax <= RVM_LS_RING ? 1 : 0;
            smem = smem_ls;
        }
    }
    if (nA > 0) {
        logl_kernel<NPV, D3V, true><<<grid, block, smem, stream>>>(P, W, params, hill_factor, slots, rv_out, logl,
                                                                   status, sa, nA, tB | (splitA << 8) | (lsx << 9));
    } else {
        if (smem > lds_budget<NPV, D3V, false>()) return hipErrorInvalidConfiguration;
        logl_kernel<NPV, D3V, false><<<grid, block, smem, stream>>>(P, W, params, hill_factor, slots, rv_out, logl,
                                                                    status, sa, nA, 8);
    }
    return hipGetLastError();
}

// rvm_plan_create: set the likelihood kernel's LDS attribute for the plan's instantiations once, so
// that launches never change function attributes (they stay capturable into a hipGraph)
// The LDS-coupled layouts' largest request for this plan (two groups per block, a fused sampler step's
// staging, the adaptive resolution's t = 0 state): the fallback every launch may take, so a plan whose
// schedule it cannot stage is refused at creation rather than failing its launches
static size_t logl_smem_worst(const DevPlan& P, int npv, bool d3) {
    const int wpb = 64 / (npv == 1 ? 1 : (npv == 2 ? 2 : 4));
    const int emax = P.fwd.n_epochs > P.bwd.n_epochs ? P.fwd.n_epochs : P.bwd.n_epochs;
    const size_t rows = (size_t)(d3 ? 7 : 5) * npv;
    const size_t init = P.rmax > 0 ? (size_t)RVM_INIT_DOUBLES * sizeof(double) : 0;
    const size_t ring = (size_t)P.lc_ring * (P.n_levels + 1) * wpb * sizeof(double);
    return (size_t)emax * 4 * sizeof(double) + (rows + 3) * 2 * wpb * sizeof(double) + 2 * init + 2 * ring;
}

hipError_t prepare_logl(const DevPlan& P) {
    const bool inc = P.inclined != 0;
    size_t budget = 0;
#define RVM_PREP(NPV)                                                                          \
    (inc ? ((void)lds_budget<NPV, true, true>(), budget = lds_budget<NPV, true, false>())      \
         : ((void)lds_budget<NPV, false, true>(), budget = lds_budget<NPV, false, false>()))
    switch (P.n_planets) {
        case 1:
            (void)RVM_PREP(1);
            break;
        case 2:
            (void)RVM_PREP(2);
            break;
        case 3:
            (void)RVM_PREP(3);
            break;
        case 4:
            (void)RVM_PREP(4);
            break;
        default:
            return hipErrorInvalidValue;
    }
#undef RVM_PREP
    return logl_smem_worst(P, P.n_planets, inc) <= budget ? hipSuccess : hipErrorInvalidConfiguration;
}

// the likelihood kernel (main pass + extension); an adaptive plan's walkers it hands on are
// finished by the refinement kernel (rvm_refine.hip launch_refine), which the caller enqueues next
// on the same stream (rvm_abi.hip run_logl): every output is final when both have run
hipError_t launch_logl(const DevPlan& P, int W, const double* params, double hill_factor, unsigned long long* slots,
                       double* logl, int32_t* status, double* rv_out, const StretchArgs& sa, hipStream_t stream) {
    const bool inc = P.inclined != 0;
    hipError_t e = hipErrorInvalidValue;
#define RVM_LAUNCH(NPV) \
    (inc ? launch_logl_t<NPV, true>(P, W, params, hill_factor, slots, logl, status, rv_out, sa, stream) \
         : launch_logl_t<NPV, false>(P, W, params, hill_factor, slots, logl, status, rv_out, sa, stream))
    switch (P.n_planets) {
        case 1:
            e = RVM_LAUNCH(1);
            break;
        case 2:
            e = RVM_LAUNCH(2);
            break;
        case 3:
            e = RVM_LAUNCH(3);
            break;
        case 4:
            e = RVM_LAUNCH(4);
            break;
        default:
            break;
    }
#undef RVM_LAUNCH
    return e;
}

}  // namespace rvm

#ifdef RVM_PROFILE
extern "C" int rvm_prof_copy(void* host, size_t bytes) {
    const size_t n = bytes < sizeof(rvm::rvm_prof) ? bytes : sizeof(rvm::rvm_prof);
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(rvm::rvm_prof), n, 0, hipMemcpyDeviceToHost);
}
extern "C" int rvm_prof_fail_copy(void* host) {
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(rvm::rvm_fail), sizeof(rvm::rvm_fail), 0, hipMemcpyDeviceToHost);
}
extern "C" int rvm_prof_clear(void) {
    static unsigned long long zf[12];
    (void)hipMemcpyToSymbol(HIP_SYMBOL(rvm::rvm_fail), zf, sizeof(zf), 0, hipMemcpyHostToDevice);
    static unsigned long long zero[RVM_PROF_MAX_WAVES * RVM_PROF_SLOTS];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(rvm::rvm_prof), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
#endif

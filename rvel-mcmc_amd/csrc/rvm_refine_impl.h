// rvm_refine_impl.h -- the adaptive resolution's halving passes, for the walkers the
// likelihood kernel (rvm_logl.hip) left with a direction above the error bound after its main pass
// and extension.
//
// Replaces, for those walkers, the reference's per-proposal step adaptivity: REBOUND's IAS15 picks
// its steps per orbit (state.py:61-73), a plan's step is fixed, and a walker far from the plan's
// reference orbit is integrated again with every step halved until its extrapolation-error
// estimate is within the bound.
//
// The rule is the WALKER's (oracle/rvoracle.c rvo_logl_whx_adapt): its two directions go through
// the passes together (rf = 1, 2, ... rmax, every open direction each time) and after every pass
//   * an encounter in either direction ends the walker (ENCOUNTER);
//   * a direction whose estimate is within the bound settles (chi2 of that pass);
//   * a direction whose estimate stopped falling (a pass from rf = 2 on at least half the previous
//     pass's: the roundoff floor of the finer steps, not the asymptotic h^8 fall) settles at its
//     best pass so far (the smallest estimate) when that is within RVM_FLOOR_BOUND x the bound --
//     counted (counters[5]); else it refines on;
//   * the certain-reject test (fused sampler launches): with each direction's lower bound on its
//     chi2 (a settled one's chi2; an open one's chi2 less min(the step-doubling change of the pass,
//     RVM_CUT_EST_FACTOR x its estimate)) the walker stops when its accept test fails even at
//     lp_hi = -(lb_f + lb_b) / npoints, and reports lp_hi;
//   * still open after rmax: UNRESOLVED (counted; the samplers raise on it).
//
// Layout.  Work lists (DevPlan rq_*): walkers with both directions open, forward only, backward
// only, in the order they met.  A workgroup of 8 waves takes WPB = 64 / L walkers of one list (a
// group; persistent blocks stride over the groups, both-direction groups first) and integrates
// their open directions LDS-coupled, one wave per (direction, level), one barrier per epoch:
// both directions open -> waves 0..3 direction 0's levels 0..3, waves 4..7 direction 1's in
// mirrored order (wave i runs on SIMD i % 4: each SIMD carries levels i and nl-1-i, 11 steps per
// base step at 4..7); one direction -> waves 0..nl-1, each alone on its SIMD (the lone-wave rate).
// More than four levels with both open: one direction after the other.  Level 0's wave of a
// direction combines (lane = walker slot): Richardson RV, chi2, estimate and the step-doubling
// change against the previous pass's RV (P.rvp, written back), then wave 0's lanes decide per walker.
// Each wave re-derives its lanes' state at t = 0 from the walker's parameters (rvm_walker.h, the
// same bits as the likelihood kernel's prologue) and finishes the walker as it would have
// (rvm_walker.h walker_out: logl, status, counters, the fused accept).
//
// Teams (round 4: two; round 6: a ladder of up to RVM_TEAMS_MAX).  At the bench's steady state about
// one walker slot in a launch needs a second halving pass, and that launch then waited pass 1 (14
// steps per base step on the longest level) and pass 2 (28) one after the other; at HD155358's and
// the 3-planet system's steady states a launch climbs to pass 3 or 4.  When every task fits the grid,
// each group has team A, which runs pass 1, team B on other CUs, which runs pass 2 at the same time,
// before pass 1's outcome is known, team C pass 3, and so on (DevPlan::n_teams, fewer when the tasks
// would not all fit).  A decides after pass 1 and publishes its walkers' state (write-through
// granules and a flag tagged with the launch generation).  If every walker of the group is done,
// A finishes them and B, which polls the flag at every epoch, stops (and passes the stop on to C).
// Otherwise B, at the end of its pass, takes A's state and applies pass 2's results to the walkers
// still open: their step-doubling change is against pass 1's RV, which A stored write-through; B
// then publishes for C in turn.  The last team goes on alone, rf = nteam + 1, ..., and finishes the
// group.  Decisions and values are the sequential passes' bit for bit; a launch whose deepest walker
// needs pass r <= nteam waits max(pass r) instead of the sum of passes 2 .. r.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

// FMA contraction only within one source expression, as in rvm_logl.hip (the same step code must
// round identically here)
#pragma clang fp contract(on)

#include "rvm_walker.h"

// the halving passes' Kepler guess (rvm_device.h drift KG): 0 the fourth-order guess, 1 the fifth-order
// one (G5).  G5 on every step
// cuts a lone wave's step on eccentric orbits at coarse resolution (933 -> 693 cycles at 32 steps per
// inner orbit, e = 0.22) but costs ~55 cycles where the fourth-order guess already takes one Halley
// step (scripts/probe/seg_bench.hip, profiles/r05g_seg_bench_g5.txt); at the passes' finer steps the
// latter dominates: steady state 1.388 ms per iteration and config 4 318k chain-steps/s with the
// fourth-order guess against 1.422 / 295k with G5 (profiles/r05h_steady_ab_refine_g5.jsonl,
// r05h_config4_ab_refine_g5.jsonl; "default" there is G5 on).  The refinement and eager kernels share
// the setting: their bits must agree.
#ifndef RVM_REFINE_GUESS
#define RVM_REFINE_GUESS 0
#endif
// the blocks' count of list-size readers (the last one resets the lists): relaxed after the reads
// have returned (1), or acquire-release (0: an agent-scope L2 writeback before, invalidate after)
#ifndef RVM_REFINE_RELAXED_COUNT
#define RVM_REFINE_RELAXED_COUNT 0
#endif

namespace rvm {

#ifdef RVM_PROFILE
// Timing build (make profile -> scripts/probe/librvmcmc_prof.so; scripts/probe/refine_prof.py): per
// wave of a block's first task, [0..3] the 100 MHz real time at kernel entry, pass-loop start,
// pass-loop end and task end; [4] shader cycles inside segments, [5] in epoch handling (star vx,
// barrier, combiner), [6] steps integrated, [7] prologue cycles, [8] pass-loop cycles,
// [9] task | team << 16 | (own + 1) << 20 | (last level + 1) << 24 | eager << 28, [10] passes
// integrated, [11] HW_REG_HW_ID, [12] cycles in the eager / team / split waits and replays,
// [13..15] cycles from entry to: the list sizes read, the schedule staged, the walker state set up;
// [16], [17] to the slot's walker index and stretch draws, and its parameter rows, loaded (this build
// waits for each there).
#define RVM_RPROF_SLOTS 20
#define RVM_RPROF_MAX_WAVES 4096
static __device__ unsigned long long rvm_rprof[RVM_RPROF_MAX_WAVES * RVM_RPROF_SLOTS];  // (per translation unit: rvm_refine_np2.hip reads it)
#define RPROF_T(v) const unsigned long long v = __builtin_readcyclecounter()
#define RPROF_RT(v) const unsigned long long v = __builtin_amdgcn_s_memrealtime()
#else
#define RPROF_T(v)
#define RPROF_RT(v)
#endif

// Claim word of one eager (pass, direction) item (DevPlan::eflag): set it to gen << 8 | code unless
// this launch generation already holds it.  Returns whether the caller now owns the item.  The eager
// block claims at its start (code 1), the refinement kernel when it needs the pass (code 3): whoever
// comes second leaves the item to the first -- so the refinement kernel only ever waits on an eager
// block that is already running, never on one that may not have been dispatched.
__device__ __forceinline__ bool claim_item(gu64* w, unsigned long long gen, unsigned long long code) {
    unsigned long long v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (;;) {
        if ((v >> 8) == gen) return false;
        unsigned long long expect = v;
        if (__hip_atomic_compare_exchange_strong(w, &expect, (gen << 8) | code, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT))
            return true;
        v = expect;
    }
}

// Bounded wait of a refinement pass's hand-off (split exchange, team B for team A): the partner
// integrates a pass of 2^rf x the base steps without publishing progress, so the allowance scales
// with the pass (a deep pass is no timeout; the timeout stays a last-resort fault)
// (capped at 60 s: a partner that is really lost -- a fault, a workgroup never co-resident -- still
// ends in a counted fault within a minute, not hours at a deep pass)
__device__ __forceinline__ unsigned long long pass_ticks(const DevPlan& P, int rf) {
    const unsigned long long t = P.spin_ticks << (rf < RVM_RESOLVE_MAX_LIMIT ? rf : RVM_RESOLVE_MAX_LIMIT);
    constexpr unsigned long long cap = 6000000000ull;  // 60 s of the 100 MHz real-time counter
    return t < cap ? t : (P.spin_ticks > cap ? P.spin_ticks : cap);
}

// NW: waves per workgroup.  8 (512 threads) runs a both-direction group's two directions side by side
// (mirrored levels) and plans of up to 8 levels; 4 (256 threads, plans of at most four levels) runs
// them one after the other when a group holds both -- the split and team layouts, the steady state's,
// give every workgroup one direction anyway, where waves 4..7 of an 8-wave group only waited at the
// barriers -- and a wave may then hold up to 512 registers (AGPRs too) instead of 256: no scratch
// spill (round 5: 400 B per lane, 13.6 MB per steady-state launch; tests/test_kernel_resources.py).
template <int NP, bool D3, int NW>
__global__ __launch_bounds__(NW * 64) void refine_kernel(const DevPlan P, const int W, const double* __restrict__ params,
                                                     const double hill_factor, double* __restrict__ rv_out,
                                                     double* __restrict__ logl_out, int32_t* __restrict__ status_out,
                                                     const StretchArgs sa, const int eager) {
    constexpr int L = LanesPerWalker<NP>::value;
    constexpr int WPB = 64 / L;
    constexpr int PR = D3 ? 7 : 5;
    constexpr int R = PR * NP;
    const int wv = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int slot = lane / L;
    const int pl_idx = lane % L;
    const int nl = P.n_levels;
    RPROF_T(pt_entry);
    RPROF_RT(prt_entry);
#ifdef RVM_PROFILE
    unsigned long long p_seg = 0, p_epo = 0, p_steps = 0, p_wait = 0, p_pass = 0;
    int p_lvl = -1;
#endif

    // the list sizes are final (the likelihood kernel has ended); the last block to read them
    // resets them for the plan's next launch and (no eager blocks in this launch: they read the
    // generation too) advances the launch generation -- every block has read it by then
    __shared__ int s_n[3];
    __shared__ unsigned long long s_gen;
    __shared__ int s_depth;
    if (threadIdx.x == 0) {
        for (int i = 0; i < 3; i++) s_n[i] = __hip_atomic_load(P.rq_n + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long g0 = __hip_atomic_load(P.gen_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_gen = g0;
        // the deepest pass the plan's previous RVM_DEPTH_WINDOW launches needed (P.depth_w, by generation
        // mod RVM_DEPTH_WINDOW + 1, tagged with it; this launch writes its own word only, so every block
        // reads the same)
        int d = P.depth_w != nullptr ? 0 : RVM_TEAMS_MAX;  // (no words: no limit)
        if (P.depth_w != nullptr) {
            unsigned long long v[RVM_DEPTH_WINDOW];
#pragma unroll
            for (int i = 0; i < RVM_DEPTH_WINDOW; i++)
                v[i] = __hip_atomic_load(P.depth_w + (g0 + 1 + i) % (RVM_DEPTH_WINDOW + 1), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
            for (int i = 0; i < RVM_DEPTH_WINDOW; i++)
                if ((v[i] >> 8) < g0 && (v[i] >> 8) + RVM_DEPTH_WINDOW >= g0 && (int)(v[i] & 0xFF) > d)
                    d = (int)(v[i] & 0xFF);
        }
        s_depth = d;
#if RVM_REFINE_RELAXED_COUNT
        // (the three loads have returned before the count is bumped: the last block's reset
        // cannot overtake them; no release / acquire -- an L2 writeback and invalidate -- needed)
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        const int done = __hip_atomic_fetch_add(P.rq_n + 3, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
        const int done = __hip_atomic_fetch_add(P.rq_n + 3, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
#endif
        if (done == (int)gridDim.x - 1) {
            for (int i = 0; i < 4; i++) __hip_atomic_store(P.rq_n + i, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!eager) __hip_atomic_store(P.gen_dev, g0 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    __syncthreads();
    RPROF_T(pt_lists);
    const unsigned long long gen = s_gen;
    const int nq[3] = {s_n[0], s_n[1], s_n[2]};
    const int depth_hint = s_depth;
    const int gq0 = (nq[0] + WPB - 1) / WPB, gq1 = (nq[1] + WPB - 1) / WPB, gq2 = (nq[2] + WPB - 1) / WPB;
    const int ng = gq0 + gq1 + gq2;
    // split: each both-direction group's two directions on two workgroups (2j, 2j + 1) -- every
    // direction's levels then alone on their SIMDs (7 x 2^rf steps per base step on the busiest
    // instead of 11 x 2^rf with both in one block) -- exchanging the walkers' per-direction state
    // after every pass; only when every task has a workgroup of its own in the grid (all co-resident
    // once dispatched; in-order dispatch leaves at most one workgroup waiting for its partner)
    const int ntask_split = 2 * gq0 + gq1 + gq2;
    // (eager: pass 1 is a replay of eager_kernel's results, both directions in one block)
    const bool split = !eager && P.rq_x != nullptr && gq0 <= P.rq_xgroups && ((int)gridDim.x & 1) == 0 &&
                       ntask_split <= (int)gridDim.x;
    // teams: team t runs pass t + 1 of the group from the start (A pass 1, B pass 2, C pass 3 ...), the
    // last one then the rest -- when the split layout holds, no RV curve is wanted (every team would
    // write it), and as many teams as the plan allows whose tasks all fit the grid (at least two), and
    // no more than the deepest pass of the plan's recent launches asks for: a team beyond it runs a
    // pass that is cancelled almost always, and its cancel latency and clock share lengthen the launch
    // (bench chain: 1.334 / 1.339 / 1.342 ms per iteration at 2 / 3 / 4 teams; HD155358 and the
    // 3-planet system, whose launches reach passes 3 and 4: 5.61 / 4.42 / 3.78 and 11.4 / 9.52 / 8.61)
    int nteam = 0;
    if (split && P.rq_t != nullptr && P.rvp != nullptr && P.rvp2 != nullptr && rv_out == nullptr &&
        ng <= P.rq_xgroups) {
        nteam = P.n_teams < P.rmax ? P.n_teams : P.rmax;
        if (nteam > (depth_hint > 2 ? depth_hint : 2)) nteam = depth_hint > 2 ? depth_hint : 2;
        while (nteam >= 2 && nteam * ntask_split > (int)gridDim.x) nteam--;
    }
    const bool team = nteam >= 2;
    const int ntask_team = nteam * ntask_split;
    // (eager: one task per group of the launch's walkers, as eager_kernel grouped them -- two, one per
    // direction, when they fit the grid: the eager split, round 6; a 4-wave block otherwise runs the
    // directions of the passes after the eager ones one after the other.  RVM_EAGER_SPLIT=0: one)
    const int ngw = (W + WPB - 1) / WPB;
    const bool esplit = eager && P.eager_split && P.rq_x != nullptr && ngw <= P.rq_xgroups &&
                        ((int)gridDim.x & 1) == 0 && 2 * ngw <= (int)gridDim.x;
    const int ntask = eager ? (esplit ? 2 * ngw : ngw) : (team ? ntask_team : (split ? ntask_split : ng));
    if ((int)blockIdx.x >= ntask) return;

    // LDS: both directions' schedules ([d][seg_h1 | obs_rv | obs_s2 | (seg_n, obs_idx)], E_d each),
    // the levels' star vx per epoch (double-buffered), encounter flags, the lanes' state at t = 0,
    // and per walker slot its directions' state
    extern __shared__ double s_sched[];
    __shared__ double s_rv[2][2][RVM_MAX_LEVELS][64];
    __shared__ int s_enc[2][RVM_MAX_LEVELS][64];
    __shared__ double s_init[8][64];
    __shared__ double s_chi[2][64], s_lb[2][64];
    __shared__ double s_pest[2][64], s_best[2][64], s_bchi[2][64];  // previous / best estimate, best chi2
    __shared__ int s_open[2][64];  // 1 open, 0 settled, 2 encounter, 3 non-finite pass
    __shared__ int s_live[64];     // the walker is still refining
    __shared__ int s_stw[64];      // its final status and logl (finished after the passes)
    __shared__ double s_lpw[64];
    __shared__ double s_acc[3][64];  // its accept inputs z, u, lnp0 (s_dmode: 0 none, 1 stretch, 2 MH)
    __shared__ int s_dmode[64];
    __shared__ unsigned long long s_mask[2];
    __shared__ int s_xfault;  // a split task's exchange gave up (its walkers end NONFINITE)
    // team B's first pass: its results per direction and walker slot (chi2, estimate, encounter),
    // applied once team A's state after pass 1 is in; the cancel poll, by epoch parity
    __shared__ double s_tc2[2][64], s_te2[2][64];
    __shared__ int s_ter[2][64];
    __shared__ int s_cancel[2];
    // eager tasks: the group's walker indices and each slot's list (-1: not listed, the likelihood
    // kernel finished it), and whether any slot is listed
    __shared__ int s_eitems[64], s_eli[64], s_eany;
    __shared__ int s_emask;  // (eager) directions of the current pass an eager block runs
    __shared__ int s_skip[64];  // the slot is a speculative variant its partner's decision rules out
    const int emax = P.fwd.n_epochs > P.bwd.n_epochs ? P.fwd.n_epochs : P.bwd.n_epochs;
    for (int dd = 0; dd < 2; dd++) {
        const DirSched& SD = dd ? P.bwd : P.fwd;
        double* b = s_sched + (size_t)dd * 4 * emax;
        const int ED = SD.n_epochs;
        int* bn = reinterpret_cast<int*>(b + 3 * ED);
        for (int i = threadIdx.x; i < ED; i += blockDim.x) {
            b[i] = SD.seg_h1[i];
            b[ED + i] = SD.obs_rv[i];
            b[2 * ED + i] = SD.obs_s2[i];
            bn[i] = SD.seg_n[i];
            bn[ED + i] = SD.obs_idx[i];
        }
    }
    RPROF_T(pt_sched);
    const bool stretch = sa.c != nullptr;
    const bool mh = sa.mh_scale != nullptr;
    const bool mapped = stretch || mh || sa.fd_x != nullptr;

    for (int t = blockIdx.x; t < ntask; t += gridDim.x) {
        // the task's group, and (split both-direction group) the direction this workgroup integrates
        int g = t, own = -1, tm = 0;  // tm: the task's team (0 = A, 1 = B, ...; always A without teams)
        if (team) {
            if (t < 2 * nteam * gq0) {
                g = t / (2 * nteam);
                const int r = t - g * 2 * nteam;
                own = r & 1;
                tm = r >> 1;
            } else {
                const int u = t - 2 * nteam * gq0;
                g = gq0 + u / nteam;
                tm = u - (u / nteam) * nteam;
            }
        } else if (esplit) {
            g = t >> 1;
            own = t & 1;
        } else if (split) {
            if (t < 2 * gq0) {
                g = t >> 1;
                own = t & 1;
            } else {
                g = t - gq0;
            }
        }
        int li = g < gq0 ? 0 : (g < gq0 + gq1 ? 1 : 2);
        const int base = (li == 0 ? g : (li == 1 ? g - gq0 : g - gq0 - gq1)) * WPB;
        int cnt = nq[li] - base < WPB ? nq[li] - base : WPB;
        const int* items = P.rq_w + (size_t)li * P.rq_cap + base;
        gu64* ef = eager ? (gu64*)(P.eflag + (size_t)g * RVM_EFLAG_WORDS) : nullptr;  // (the eager group's flags)
        if (eager) {
            // the launch's walkers g * WPB ..: which of them the lists hold, and in which
            const int w0 = g * WPB;
            __syncthreads();  // (the previous task's LDS state is no longer read)
            if (threadIdx.x < 64) {
                s_eitems[threadIdx.x] = w0 + (int)threadIdx.x < W ? w0 + (int)threadIdx.x : w0;
                s_eli[threadIdx.x] = -1;
            }
            if (threadIdx.x == 0) s_eany = 0;
            __syncthreads();
            for (int l2 = 0; l2 < 3; l2++)
                for (int i = threadIdx.x; i < nq[l2]; i += blockDim.x) {
                    const int wl = P.rq_w[(size_t)l2 * P.rq_cap + i];
                    if (wl >= w0 && wl < w0 + WPB) {
                        s_eli[wl - w0] = l2;
                        s_eany = 1;
                    }
                }
            __syncthreads();
            if (!s_eany) {  // nothing to refine here: eager_kernel's blocks of the group stop
                if (threadIdx.x == 0)
                    __hip_atomic_store(ef, (gen << 8) | 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                continue;
            }
            items = s_eitems;
            cnt = WPB;
        }
        // this lane's walker (lanes past the group's last repeat its first walker: benign values)
        const int wo = items[slot < cnt ? slot : 0];
        int kind = 0, wk = wo, jst = 0, jp = 0;
        double zst = 0.0, zp = 0.0;
        if (stretch) stretch_slot(sa, wo, kind, wk, zst, jst, zp, jp);
#ifdef RVM_PROFILE
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // (timing build: the slot's index in)
#endif
        RPROF_T(pt_slot);
        double rowv[R];
#pragma unroll
        for (int r = 0; r < R; r++) rowv[r] = walker_param(mapped, params, W, wk, sa, r, zst, jst, kind, zp, jp);
#ifdef RVM_PROFILE
        asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");  // (timing build: the rows in)
#endif
        RPROF_T(pt_rows);
        Lane<NP> s;
        int status = RVM_STATUS_OK;
        double e2w;
        walker_setup<NP, D3, L>(rowv, pl_idx, hill_factor, s, status, e2w);
        RPROF_T(pt_setup);
        __syncthreads();  // (the previous group's LDS state is no longer read)
        if (wv == 0) {
            s_init[0][lane] = s.rx;
            s_init[1][lane] = s.ry;
            s_init[2][lane] = s.vx;
            s_init[3][lane] = s.vy;
            s_init[4][lane] = s.rz;
            s_init[5][lane] = s.vz;
            s_init[6][lane] = s.r;
            s_init[7][lane] = s.ir;
            if (lane < WPB) {
                const int lli = eager ? s_eli[lane] : li;  // (eager: this slot's list, -1 none)
                // a speculative iteration's half-1 slot against the outcome of its partner j (kind 1:
                // j rejects, 2: j accepts): when j was not handed on (its mark is not this launch's)
                // the likelihood kernel has stored j's final decision, and the variant it rules out is
                // never read (rvm_stretch_iteration_end) -- skipped instead of refined
                int skip = 0;
                if (P.skip_variants && stretch && sa.n_spec > 0 && sa.dec != nullptr && lane < cnt && lli >= 0) {
                    int k2 = 0, wk2 = 0, j2 = 0, jp2 = 0;
                    double z2 = 0.0, zp2 = 0.0;
                    stretch_slot(sa, items[lane], k2, wk2, z2, j2, zp2, jp2);
                    const long long jl = (long long)j2 - sa.s0_begin;
                    if (k2 != 0 && jl >= 0 && jl < sa.n_spec && P.rq_mark[jl] != (int32_t)gen)
                        skip = (k2 == 2) != (sa.dec[jl] == 1);
                }
                s_skip[lane] = skip;
                const bool v = lane < cnt && lli >= 0 && !skip;
                const int wl = items[lane < cnt ? lane : 0];
                const bool of = v && lli != 2, ob = v && lli != 1;
                s_open[0][lane] = of ? 1 : 0;
                s_open[1][lane] = ob ? 1 : 0;
                s_chi[0][lane] = of ? 0.0 : P.rq_c[wl];
                s_chi[1][lane] = ob ? 0.0 : P.rq_c[(size_t)P.rq_cap + wl];
                s_lb[0][lane] = s_chi[0][lane];
                s_lb[1][lane] = s_chi[1][lane];
                for (int d2i = 0; d2i < 2; d2i++) {
                    s_pest[d2i][lane] = INFINITY;
                    s_best[d2i][lane] = INFINITY;
                    s_bchi[d2i][lane] = 0.0;
                }
                s_live[lane] = v ? 1 : 0;
                s_stw[lane] = RVM_STATUS_NONFINITE;  // (every pass loop ends with a decision)
                s_lpw[lane] = -INFINITY;
            }
            const int lli = lane < WPB ? (eager ? s_eli[lane] : li) : -1;
            const bool live0 = lane < WPB && lane < cnt && lli >= 0 && !s_skip[lane < WPB ? lane : 0];
            const uint64_t m0 = ballot(live0 && lli != 2);
            const uint64_t m1 = ballot(live0 && lli != 1);
            if (lane == 0) {
                s_mask[0] = m0;
                s_mask[1] = m1;
                s_xfault = 0;
                s_cancel[0] = s_cancel[1] = 0;
            }
        }
        // the decision lanes' accept inputs (wave 0, lane = walker slot), kept in LDS through the passes
        const int wme = items[lane < WPB && lane < cnt ? lane : 0];
        if (wv == 0 && lane < WPB) {
            int dmode = 0;
            double dz = 0.0, du = 0.0, dl = 0.0;
            if (lane < cnt && (!eager || s_eli[lane] >= 0) && P.ext_mult > 0 && P.cut)
                accept_inputs(sa, wme, dmode, dz, du, dl);
            s_dmode[lane] = dmode;
            s_acc[0][lane] = dz;
            s_acc[1][lane] = du;
            s_acc[2][lane] = dl;
        }
        __syncthreads();

        // team t < nteam - 1 publishes after its pass at rq_t[g][t] (16 rows of 64 values: live, status,
        // logl, then per direction open, chi2, lb, previous / best estimate, best chi2), its flag at
        // rq_tf[g][t] = (launch generation << 8) | 1 (walkers left for team t + 1) or 2 (all done);
        // team t > 0 reads team t - 1's.  rq_tf[g][n_teams - 1], the group's done word, is set with
        // the flag 2 by whichever team finishes the group: every later team polls it, so all of them
        // stop within one poll of the finish (not one poll per team down the ladder)
        const size_t ks = (size_t)(P.n_teams - 1);
        gu64* tpub = team && tm < nteam - 1 ? (gu64*)(P.rq_t + ((size_t)g * ks + tm) * 16 * 64) : nullptr;
        gu64* tflag = team && tm < nteam - 1 ? (gu64*)(P.rq_tf + (size_t)g * P.n_teams + tm) : nullptr;
        gu64* tprev = team && tm > 0 ? (gu64*)(P.rq_t + ((size_t)g * ks + tm - 1) * 16 * 64) : nullptr;
        gu64* tpflag = team && tm > 0 ? (gu64*)(P.rq_tf + (size_t)g * P.n_teams + tm - 1) : nullptr;
        gu64* tdone = team ? (gu64*)(P.rq_tf + (size_t)g * P.n_teams + ks) : nullptr;
        const size_t plane2 = (size_t)2 * P.lvx_emax * P.lvx_stride;  // (one team's RV buffer)
        bool cancelled = false;  // (team t > 0: an earlier team finished the group)
        // a pass's outcome for direction dd of walker slot `lane` (its combiner lane): encounter,
        // non-finite (the walker ends NONFINITE: a halving pass that blows up is not refined further,
        // oracle/rvoracle.c dir_halve -- the last pass would run 2^rmax x the base steps),
        // settled (estimate within the bound), settled at the roundoff floor, or still open with the
        // pass's lower bound on its chi2
        auto pass_result = [&](const int dd, const int rfp, const double c2, const double e2, const double d2,
                               const int er) __attribute__((always_inline)) {
            const bool fin = isfinite(c2) && isfinite(e2);
            if (!er && !fin) {
                s_open[dd][lane] = 3;
                return;
            }
            const double en = e2 / P.npoints;
            // (the roundoff floor: this pass's estimate no longer falls; the best pass's estimate is
            // e2 / npoints units too)
            const bool stall = fin && rfp >= 2 && !(en < 0.5 * s_pest[dd][lane]);
            if (fin && en < s_best[dd][lane]) {
                s_best[dd][lane] = en;
                s_bchi[dd][lane] = c2;
            }
            s_pest[dd][lane] = fin ? en : INFINITY;
            if (er) {
                s_open[dd][lane] = 2;
            } else if (fin && !(en > P.rtol_dir)) {
                s_open[dd][lane] = 0;
                s_chi[dd][lane] = c2;
                s_lb[dd][lane] = c2;
            } else if (stall && s_best[dd][lane] <= RVM_FLOOR_BOUND * P.rtol_dir) {
                s_open[dd][lane] = 0;
                s_chi[dd][lane] = s_bchi[dd][lane];
                s_lb[dd][lane] = s_bchi[dd][lane];
                __hip_atomic_fetch_add(P.counters + 5, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                s_chi[dd][lane] = fin ? c2 : __builtin_nan("");
                s_lb[dd][lane] = fin ? open_lb(c2, d2, e2) : 0.0;
            }
        };
        bool finisher = !team && own <= 0;  // the workgroup that finishes the walkers
        int rf_last = 0;                    // the last pass the group's decisions took
        RPROF_T(pt_loop0);
        RPROF_RT(prt_loop0);
        for (int rf = 1 + tm; rf <= P.rmax; rf++) {
            const bool bfirst = tm > 0 && rf == 1 + tm;  // a later team's pass concurrent with A's
            const uint64_t mk0 = s_mask[0], mk1 = s_mask[1];
            const int amw = (mk0 ? 1 : 0) | (mk1 ? 2 : 0);  // directions a live walker still needs
            if (amw == 0) break;
            int emask = 0;  // (eager) the directions whose pass rf an eager block runs: replayed below
            if (eager) {
                // eager_kernel's blocks of directions no open walker needs stop (every pass), and each
                // pass it runs is claimed per needed direction: a direction whose eager block has
                // started is left to it (its stored results are replayed after this workgroup's own
                // sub-passes), any other one this workgroup integrates itself -- it never waits on a
                // block that may not have been dispatched
                if (threadIdx.x == 0) {
                    int em = 0;
                    for (int d3 = 0; d3 < 2; d3++) {
                        if (own >= 0 && d3 != own) continue;  // (eager split: the partner's direction is its own)
                        if (!((amw >> d3) & 1))
                            __hip_atomic_store(ef + 6 + d3, (gen << 8) | 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        else if (rf <= P.eager_passes && !claim_item(ef + 2 + 2 * (rf - 1) + d3, gen, 3ull))
                            em |= 1 << d3;
                    }
                    s_emask = em;
                }
                __syncthreads();
                emask = s_emask;
            }
            // the ones this workgroup integrates
            const int am = (own < 0 ? amw : (amw & (1 << own))) & ~emask;
            // sub-passes: both directions at once (up to four levels), else one after the other;
            // none when a split task's own direction is done (the partner's pass only)
            const bool both = am == 3 && nl <= 4 && NW >= 8;
            const int nsub = am == 0 ? 0 : ((am == 3 && !both) ? 2 : 1);
            for (int sp = 0; sp < nsub; sp++) {
                // this wave's (direction, level) task, or none
                const int sd = am == 3 ? sp : (am == 1 ? 0 : 1);  // the sub-pass's direction (one-direction mode)
                int dd = -1, k = -1;
                if (both) {
                    const int j = wv & 3;
                    dd = wv >> 2;
                    k = j < nl ? (dd == 0 ? j : nl - 1 - j) : -1;
                } else {
                    dd = sd;
                    k = wv < nl ? wv : -1;
                }
                if (k < 0) dd = -1;
                // (wave-uniform in the compiler's eyes, SGPRs: a role derived from threadIdx would make
                // the step loops divergent loops, with their state in extra registers)
                dd = __builtin_amdgcn_readfirstlane(dd);
                k = __builtin_amdgcn_readfirstlane(k);
                const int dd_u = dd < 0 ? 0 : dd;
                const int k_u = k < 0 ? 0 : k;
                const bool work = dd >= 0;
                const DirSched& SR = dd_u ? P.bwd : P.fwd;
                const int Er = SR.n_epochs;
                // the barrier count (the same on every wave): the longer direction, or the sub-pass's
                const int eb = both ? emax : (sd ? P.bwd : P.fwd).n_epochs;
                const double* r_dir = s_sched + (size_t)dd_u * 4 * emax;
                const double* r_len = r_dir;
                const double* r_rv = r_dir + Er;
                const double* r_s2 = r_dir + 2 * Er;
                const int* r_n = reinterpret_cast<const int*>(r_dir + 3 * Er);
                const int* r_idx = r_n + Er;
                const uint64_t need = dd_u ? mk1 : mk0;
                KickPrep<NP> kq{};
                if (work) {
                    s.rx = s_init[0][lane];
                    s.ry = s_init[1][lane];
                    s.vx = s_init[2][lane];
                    s.vy = s_init[3][lane];
                    s.rz = s_init[4][lane];
                    s.vz = s_init[5][lane];
                    s.r = s_init[6][lane];
                    s.ir = s_init[7][lane];
                    s.encm = 0;
                    if (Er > 0) kq = kick_prep<NP, L, D3>(s, 1.875);
                }
                const int m_r = P.mult[k_u] << rf;
                const int nt_r = P.nt[k_u];
                const bool late = P.late_mult > 0 && m_r >= P.late_mult;  // (the late vote: the same bits)
                const double sc = ldexp(P.inv_mult[k_u], -rf);  // (exact: a power-of-two scaling)
                const bool cmb = work && k == 0 && lane < WPB && ((need >> lane) & 1);
                const bool hasp = P.rvp != nullptr;
                double c2 = 0.0, e2 = 0.0, d2 = hasp ? 0.0 : INFINITY;  // (the combiner lanes)
                // the previous pass's RV, replaced by this pass's: P.rvp (team t > 0: its own plane of
                // P.rvp2; its first pass only writes it -- the previous pass's RV is still being written
                // by team t - 1)
                double* pbuf = tm ? P.rvp2 + (size_t)(tm - 1) * plane2 : P.rvp;
                double* pp = hasp ? pbuf + (size_t)dd_u * P.lvx_emax * P.lvx_stride + (cmb ? wme : 0) : nullptr;
                for (int e = 0; e < eb; e++) {
                    const bool here = e < Er;
                    const double pv = cmb && here && hasp && !bfirst ? pp[(size_t)e * P.lvx_stride] : 0.0;  // (issued early)
                    const int ns = __builtin_amdgcn_readfirstlane(work && here ? r_n[e] * m_r : 0);
                    RPROF_T(pt_s0);
                    if (ns > 0) {
                        // (a later team's first pass stops part-way once an earlier team has finished the
                        // group: the barrier below then breaks every wave out at this epoch)
                        if (bfirst)
                            (void)segment_gated_c<D3, NP, L, RVM_REFINE_GUESS>(s, kq, r_len[e] * sc, ns, nt_r, tdone,
                                                                                 nullptr, (gen << 8) | 2ull, late);
                        else
                            segment_gated<D3, NP, L, RVM_REFINE_GUESS>(s, kq, r_len[e] * sc, ns, nt_r, late);
                    }
                    RPROF_T(pt_s1);
#ifdef RVM_PROFILE
                    p_seg += pt_s1 - pt_s0;
                    p_steps += (unsigned long long)ns;
#endif
                    if (work && here) {  // (star_vx gathers over the walker's lanes by DPP: outside the lane branch)
                        const double v0 = star_vx<NP, L>(s);
                        if (pl_idx == 0) s_rv[dd_u][e & 1][k_u][slot] = v0;
                    }
                    // a later team polls the group's done word (one load per epoch; the result by epoch
                    // parity, read by every wave after the barrier and rewritten only two barriers later)
                    if (bfirst && wv == 0 && lane == 0)
                        s_cancel[e & 1] = __hip_atomic_load(tdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                                          ((gen << 8) | 2ull);
                    __syncthreads();
                    if (bfirst && s_cancel[e & 1]) {
                        cancelled = true;
                        break;
                    }
                    if (cmb && here) {
                        double rvx = 0.0, rv3 = 0.0;
                        for (int q = 0; q < nl; q++) rvx += P.lw[q] * s_rv[dd_u][e & 1][q][lane];
                        for (int q = 1; q < nl; q++) rv3 += P.lw3[q] * s_rv[dd_u][e & 1][q][lane];
                        const double r = rvx - r_rv[e];
                        c2 += (r * r) / r_s2[e];
                        e2 += fabs((rvx - rv3) * (r + (rv3 - r_rv[e]))) / r_s2[e];
                        if (hasp) {
                            d2 += fabs((rvx - pv) * (r + (pv - r_rv[e]))) / r_s2[e];
                            if (team && tm < nteam - 1)  // (write-through: the next team reads it)
                                __hip_atomic_store((gu64*)(pp + (size_t)e * P.lvx_stride),
                                                   (unsigned long long)__double_as_longlong(rvx), __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
                            else
                                pp[(size_t)e * P.lvx_stride] = rvx;
                        }
                        if (rv_out != nullptr) rv_out[(size_t)r_idx[e] * W + wme] = rvx;
                    }
#ifdef RVM_PROFILE
                    p_epo += __builtin_readcyclecounter() - pt_s1;
#endif
                }
#ifdef RVM_PROFILE
                if (work) {
                    p_pass++;
                    p_lvl = k;
                }
#endif
                if (cancelled) break;
                if (work && pl_idx == 0) s_enc[dd_u][k_u][slot] = (int)(((s.encm >> lane) & kick_enc_bits<NP>()) != 0);
                __syncthreads();
                if (bfirst) {
                    // a later team: this pass's results aside until the previous team's state is in
                    if (work && k == 0 && lane < WPB) {
                        int er = 0;
                        for (int q = 0; q < nl; q++) er |= s_enc[dd_u][q][lane];
                        s_tc2[dd_u][lane] = c2;
                        s_te2[dd_u][lane] = e2;
                        s_ter[dd_u][lane] = er;
                    }
                    continue;
                }
                // the direction's combiner lanes: settle, open (with the pass's lower bound) or encounter
                if (work && k == 0 && lane < WPB) {
                    if ((need >> lane) & 1) {
                        int er = 0;
                        for (int q = 0; q < nl; q++) er |= s_enc[dd_u][q][lane];
                        pass_result(dd_u, rf, c2, e2, d2, er);
                    }
                    if (lane == 0 && need)
                        __hip_atomic_fetch_add(P.counters + 3, (unsigned long long)__builtin_popcountll(need),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (cancelled) break;  // (a later team: an earlier one finished the group; every wave saw the same flag)
            rf_last = rf;
            RPROF_T(pt_w0);
            __syncthreads();
            if (emask != 0 && wv == 0) {
                // the eager-run directions: once their blocks have stored pass rf (write-through values,
                // then the claim word = gen << 8 | 2), each combiner lane takes that pass's chi2,
                // estimate and encounter flag, and its step-doubling change against the previous pass's
                // RV (P.rvp: the main pass's, then pass 1's), which this pass's RV then replaces there
                const bool mine0 = (emask & 1) && lane < WPB && ((mk0 >> lane) & 1);
                const bool mine1 = (emask & 2) && lane < WPB && ((mk1 >> lane) & 1);
                gu64* f0 = ef + 2 + 2 * (rf - 1);
                const unsigned long long done = (gen << 8) | 2ull;
                SpinClock clk;
                clk.restart();
                bool ok = true;
                for (;;) {
                    const bool rdy = (!mine0 || __hip_atomic_load(f0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == done) &&
                                     (!mine1 || __hip_atomic_load(f0 + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == done);
                    if (ballot(!rdy) == 0) break;
                    // (a claimed block is running: the wait ends; the allowance is a last-resort fault)
                    if (clk.expired(pass_ticks(P, rf))) {
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                if (!ok) {
                    if (lane == 0) {
                        s_xfault = 1;
                        __hip_atomic_fetch_add(P.counters, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                } else {
                    for (int d3 = 0; d3 < 2; d3++) {
                        if (!(d3 ? mine1 : mine0)) continue;
                        const DirSched& SB = d3 ? P.bwd : P.fwd;
                        const int Eb = SB.n_epochs;
                        const double* b_dir = s_sched + (size_t)d3 * 4 * emax;
                        const double* b_rv = b_dir + Eb;
                        const double* b_s2 = b_dir + 2 * Eb;
                        const size_t plane = (size_t)P.lvx_emax * P.lvx_stride;
                        gu64* cur = (gu64*)(P.rve + ((size_t)(rf - 1) * 2 + d3) * plane + wme);
                        double* prv = P.rvp + (size_t)d3 * plane + wme;
                        double d2 = 0.0;
                        // (RCH epochs' loads in flight at once: one epoch at a time, each store
                        // waiting for its load, cost ~0.4 us per epoch on the step's critical path)
                        constexpr int RCH = 16;
                        for (int e0 = 0; e0 < Eb; e0 += RCH) {
                            double rvc[RCH], pvc[RCH];
#pragma unroll
                            for (int j = 0; j < RCH; j++) {
                                const int e = e0 + j < Eb ? e0 + j : Eb - 1;
                                rvc[j] = __longlong_as_double((long long)__hip_atomic_load(
                                    cur + (size_t)e * P.lvx_stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
                                pvc[j] = prv[(size_t)e * P.lvx_stride];
                            }
#pragma unroll
                            for (int j = 0; j < RCH; j++) {
                                const int e = e0 + j;
                                if (e < Eb) {
                                    const double rvx = rvc[j], pv = pvc[j];
                                    const double r = rvx - b_rv[e];
                                    d2 += fabs((rvx - pv) * (r + (pv - b_rv[e]))) / b_s2[e];
                                    prv[(size_t)e * P.lvx_stride] = rvx;
                                }
                            }
                        }
                        gu64* es = (gu64*)(P.esum + ((size_t)(rf - 1) * 2 + d3) * 3 * P.lvx_stride + wme);
                        auto ld = [&](size_t o) {
                            return __longlong_as_double((long long)__hip_atomic_load(es + o, __ATOMIC_RELAXED,
                                                                                     __HIP_MEMORY_SCOPE_AGENT));
                        };
                        pass_result(d3, rf, ld(0), ld(P.lvx_stride), d2, (int)ld(2 * (size_t)P.lvx_stride));
                    }
                }
                if (lane == 0) {
                    const unsigned long long nd = ((emask & 1) ? __builtin_popcountll(mk0) : 0) +
                                                  ((emask & 2) ? __builtin_popcountll(mk1) : 0);
                    __hip_atomic_fetch_add(P.counters + 3, nd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
            }
            if (bfirst) {
                // a later team: the previous team's state after its pass (wave 0; the flag is in by now
                // unless that team is late), then this pass's results for the walkers still open
                if (wv == 0) {
                    SpinClock clk;
                    clk.restart();
                    unsigned long long f = 0;
                    bool ok = true;
                    while (((f = __hip_atomic_load(tpflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 8) != gen) {
                        if (__hip_atomic_load(tdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ((gen << 8) | 2ull)) {
                            f = (gen << 8) | 2ull;  // (an earlier team finished the group)
                            break;
                        }
                        if (clk.expired(pass_ticks(P, tm))) {
                            ok = false;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(2);
                    }
                    ok = __builtin_amdgcn_readfirstlane((int)ok) != 0;
                    f = __builtin_amdgcn_readfirstlane(f);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    if (!ok) {
                        if (lane == 0) {
                            s_xfault = 1;
                            __hip_atomic_fetch_add(P.counters, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        }
                    } else if ((f & 0xFF) == 2) {
                        if (lane == 0) s_cancel[0] = 1;  // (an earlier team finished the group after all)
                    } else if (lane < WPB) {
                        // (every row's load in flight before the first LDS store)
                        unsigned long long row_v[15];
#pragma unroll
                        for (int rw = 0; rw < 15; rw++)
                            row_v[rw] = __hip_atomic_load(tprev + rw * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        auto ld = [&](int row) { return row_v[row]; };
                        s_live[lane] = (int)ld(0);
                        s_stw[lane] = (int)ld(1);
                        s_lpw[lane] = __longlong_as_double((long long)ld(2));
                        for (int d3 = 0; d3 < 2; d3++) {
                            s_open[d3][lane] = (int)ld(3 + 6 * d3);
                            s_chi[d3][lane] = __longlong_as_double((long long)ld(4 + 6 * d3));
                            s_lb[d3][lane] = __longlong_as_double((long long)ld(5 + 6 * d3));
                            s_pest[d3][lane] = __longlong_as_double((long long)ld(6 + 6 * d3));
                            s_best[d3][lane] = __longlong_as_double((long long)ld(7 + 6 * d3));
                            s_bchi[d3][lane] = __longlong_as_double((long long)ld(8 + 6 * d3));
                        }
                    }
                }
                __syncthreads();
                if (s_cancel[0]) {
                    cancelled = true;
                    break;
                }
                // the directions this workgroup integrated: the walkers still live and open there
                // take this pass's chi2 and estimate, and the step-doubling change against the previous
                // pass's RV (team t - 1's, write-through) and this pass's (team t's plane of P.rvp2)
                const double* rprev = tm == 1 ? P.rvp : P.rvp2 + (size_t)(tm - 2) * plane2;
                const double* rown = P.rvp2 + (size_t)(tm - 1) * plane2;
                for (int d3 = 0; d3 < 2; d3++) {
                    const bool mine = own < 0 ? (((d3 == 0 ? mk0 : mk1) != 0)) : d3 == own;
                    if (!mine || wv != 0 || lane >= WPB) continue;
                    const bool open_here = s_xfault == 0 && s_live[lane] != 0 && s_open[d3][lane] == 1;
                    const uint64_t needb = ballot(open_here);
                    if (open_here) {
                        const DirSched& SB = d3 ? P.bwd : P.fwd;
                        const int Eb = SB.n_epochs;
                        const double* b_dir = s_sched + (size_t)d3 * 4 * emax;
                        const double* b_rv = b_dir + Eb;
                        const double* b_s2 = b_dir + 2 * Eb;
                        const size_t off = (size_t)d3 * P.lvx_emax * P.lvx_stride + wme;
                        double d2b = 0.0;
                        constexpr int RCH = 16;  // (epochs' loads in flight at once, as the eager replay)
                        for (int e0 = 0; e0 < Eb; e0 += RCH) {
                            double pvc[RCH], rvc[RCH];
#pragma unroll
                            for (int j = 0; j < RCH; j++) {
                                const int e = e0 + j < Eb ? e0 + j : Eb - 1;
                                pvc[j] = __longlong_as_double((long long)__hip_atomic_load(
                                    (gu64*)(rprev + off + (size_t)e * P.lvx_stride), __ATOMIC_RELAXED,
                                    __HIP_MEMORY_SCOPE_AGENT));
                                rvc[j] = rown[off + (size_t)e * P.lvx_stride];
                            }
#pragma unroll
                            for (int j = 0; j < RCH; j++) {
                                const int e = e0 + j;
                                if (e < Eb) {
                                    const double pv = pvc[j], rvx = rvc[j];
                                    const double r = rvx - b_rv[e];
                                    d2b += fabs((rvx - pv) * (r + (pv - b_rv[e]))) / b_s2[e];
                                }
                            }
                        }
                        pass_result(d3, 1 + tm, s_tc2[d3][lane], s_te2[d3][lane], d2b, s_ter[d3][lane]);
                    }
                    if (lane == 0 && needb)
                        __hip_atomic_fetch_add(P.counters + 3, (unsigned long long)__builtin_popcountll(needb),
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                __syncthreads();
            }
            if (own >= 0 && wv == 0) {
                // split: publish this direction's state of every walker (the meeting slot's encoding,
                // rvm_walker.h: chi2, -lb, or the ENCOUNTER status) as write-through granules, drain,
                // one lane stores the flag (launch generation, pass); then the partner's, after its
                // flag and one agent-scope acquire (cdna_hip_programming.md §6 Guideline 16, R1).
                // Double-buffered by the pass's parity: a partner reads pass rf's values before it
                // publishes rf + 1, which this workgroup awaits before it writes rf + 2.
                // (each team of a group its own slots and flags)
                const size_t xb = ((size_t)(g * P.n_teams + tm) * 2) * 2 * 64;
                gu64* mine = (gu64*)(P.rq_x + xb + ((size_t)own * 2 + (rf & 1)) * 64);
                gu64* theirs = (gu64*)(P.rq_x + xb + ((size_t)(own ^ 1) * 2 + (rf & 1)) * 64);
                if (lane < WPB) {
                    const int o = s_open[own][lane];
                    const unsigned long long b =
                        o >= 2 ? slot_status(o == 2 ? RVM_STATUS_ENCOUNTER : RVM_STATUS_NONFINITE)
                               : (unsigned long long)__double_as_longlong(o == 1 ? -s_lb[own][lane] : s_chi[own][lane]);
                    __hip_atomic_store(mine + lane, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                const unsigned long long tag = (gen << 8) | (unsigned long long)rf;
                if (lane == 0)
                    __hip_atomic_store((gu64*)(P.rq_xf + ((size_t)g * P.n_teams + tm) * 2 + own), tag, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                gu64* tf = (gu64*)(P.rq_xf + ((size_t)g * P.n_teams + tm) * 2 + (own ^ 1));
                SpinClock clk;
                clk.restart();
                bool ok = true;
                while (__hip_atomic_load(tf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != tag) {
                    if (clk.expired(pass_ticks(P, rf))) {
                        ok = false;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
                ok = __builtin_amdgcn_readfirstlane((int)ok) != 0;
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                if (!ok) {
                    if (lane == 0) {
                        s_xfault = 1;
                        __hip_atomic_fetch_add(P.counters, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                } else if (lane < WPB) {
                    const unsigned long long b = __hip_atomic_load(theirs + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    const int od = own ^ 1;
                    if (slot_is_status(b)) {
                        s_open[od][lane] = (b & 0xFF) == RVM_STATUS_NONFINITE ? 3 : 2;
                    } else {
                        const double v = __longlong_as_double((long long)b);
                        s_open[od][lane] = signbit(v) ? 1 : 0;
                        s_chi[od][lane] = fabs(v);  // (an open direction's chi2 is not needed: only its lb)
                        s_lb[od][lane] = fabs(v);
                    }
                }
            }
#ifdef RVM_PROFILE
            p_wait += __builtin_readcyclecounter() - pt_w0;
#endif
            // the walker's decision (wave 0, lane = walker slot; a split task's two workgroups take the
            // same decisions from the same states)
            if (wv == 0) {
                bool live = lane < WPB && s_live[lane] != 0;
                if (live) {
                    const int of = s_open[0][lane], ob = s_open[1][lane];
                    int stw = RVM_STATUS_OK;
                    double lp = 0.0;
                    bool done = true;
                    if (s_xfault) {
                        stw = RVM_STATUS_NONFINITE;
                    } else if (of >= 2 || ob >= 2) {
                        // (the forward direction's end first, as the oracle integrates it first)
                        stw = (of >= 2 ? of : ob) == 2 ? RVM_STATUS_ENCOUNTER : RVM_STATUS_NONFINITE;
                    } else if (of == 0 && ob == 0) {
                        lp = -((s_chi[1][lane] + s_chi[0][lane]) / P.npoints);  // state.py:98, 109
                        if (!isfinite(lp)) stw = RVM_STATUS_NONFINITE;
                    } else {
                        const double lp_hi = -((s_lb[1][lane] + s_lb[0][lane]) / P.npoints);
                        const int dmode = s_dmode[lane];
                        if (dmode != 0 && isfinite(lp_hi) &&
                            !accepts_at(sa, dmode, s_acc[0][lane], s_acc[1][lane], s_acc[2][lane], lp_hi)) {
                            lp = lp_hi;  // a certain reject
                            if (own <= 0)
                                __hip_atomic_fetch_add(P.counters + 4,
                                                       (unsigned long long)((of ? 1 : 0) + (ob ? 1 : 0)),
                                                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        } else if (rf == P.rmax) {
                            stw = RVM_STATUS_UNRESOLVED;
                        } else {
                            done = false;
                        }
                    }
                    if (done) {
                        live = false;
                        s_live[lane] = 0;
                        s_stw[lane] = stw;
                        s_lpw[lane] = stw == RVM_STATUS_OK ? lp : -INFINITY;
                    }
                }
                const uint64_t m0 = ballot(live && s_open[0][lane] == 1);
                const uint64_t m1 = ballot(live && s_open[1][lane] == 1);
                if (lane == 0) {
                    s_mask[0] = m0;
                    s_mask[1] = m1;
                }
                if (team && tm < nteam - 1 && own <= 0) {
                    // a team before the last after its pass: publish the walkers' state for the next
                    // team (write-through granules, drain, then the flag: 2 when the group is done and
                    // the later teams may stop)
                    if (lane < WPB) {
                        auto st = [&](int row, unsigned long long v) {
                            __hip_atomic_store(tpub + row * 64 + lane, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        };
                        auto bits = [](double v) { return (unsigned long long)__double_as_longlong(v); };
                        st(0, (unsigned long long)s_live[lane]);
                        st(1, (unsigned long long)(unsigned)s_stw[lane]);
                        st(2, bits(s_lpw[lane]));
                        for (int d3 = 0; d3 < 2; d3++) {
                            st(3 + 6 * d3, (unsigned long long)(unsigned)s_open[d3][lane]);
                            st(4 + 6 * d3, bits(s_chi[d3][lane]));
                            st(5 + 6 * d3, bits(s_lb[d3][lane]));
                            st(6 + 6 * d3, bits(s_pest[d3][lane]));
                            st(7 + 6 * d3, bits(s_best[d3][lane]));
                            st(8 + 6 * d3, bits(s_bchi[d3][lane]));
                        }
                    }
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    if (lane == 0) {
                        __hip_atomic_store(tflag, (gen << 8) | ((m0 | m1) == 0 ? 2ull : 1ull), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
                        if ((m0 | m1) == 0)
                            __hip_atomic_store(tdone, (gen << 8) | 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    }
                }
            }
            __syncthreads();
            if (team && tm < nteam - 1) {
                // a team before the last ends after its pass; it finishes the group only when no walker
                // is left for the next team
                finisher = own <= 0 && (s_mask[0] | s_mask[1]) == 0;
                break;
            }
        }
        RPROF_T(pt_loop1);
        RPROF_RT(prt_loop1);
        if (team && tm == nteam - 1) finisher = own <= 0 && !cancelled;
        // a cancelled team before the last passes the cancel on (the next team polls only its flag)
        if (team && cancelled && tm < nteam - 1 && own <= 0 && threadIdx.x == 0)
            __hip_atomic_store(tflag, (gen << 8) | 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        // the group's walkers, as the likelihood kernel would have finished them (rvm_walker.h;
        // a split group's by its forward-direction workgroup, of team A or B)
        // the group's depth for the next launches' team count (generation-tagged: a larger generation
        // always wins the max)
        if (finisher && threadIdx.x == 0 && P.depth_w != nullptr && rf_last > 0)
            __hip_atomic_fetch_max(P.depth_w + gen % (RVM_DEPTH_WINDOW + 1), (gen << 8) | (unsigned long long)rf_last,
                                   __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (finisher && wv == 0 && lane < WPB && lane < cnt && s_skip[lane]) {
            logl_out[wme] = -INFINITY;
            status_out[wme] = RVM_STATUS_SKIPPED;
            __hip_atomic_fetch_add(P.counters + 6, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (finisher && wv == 0 && lane < WPB && lane < cnt && (!eager || s_eli[lane] >= 0)) {
            int k2 = 0, wk2 = wme, j2 = 0, jp2 = 0;
            double z2 = 0.0, zp2 = 0.0;
            if (stretch) stretch_slot(sa, wme, k2, wk2, z2, j2, zp2, jp2);
            auto row = [&](int r) { return walker_param(mapped, params, W, wk2, sa, r, z2, j2, k2, zp2, jp2); };
            const double u3 = stretch ? stretch_u3(sa.seed, (uint64_t)(sa.s0_begin + wme), sa.iteration, sa.half)
                                      : (mh ? mh_u(sa.seed, (uint64_t)(sa.s0_begin + wme), sa.iteration) : 0.0);
            const double lnp0 = (stretch && k2 == 0) || mh ? sa.lnp[wme] : 0.0;
            walker_out<R>(P, sa, wme, s_stw[lane], s_lpw[lane], logl_out, status_out, row, z2, u3, lnp0);
        }
        // (eager) the group is done: any of its eager blocks still running stops at its next epoch
        // (the caller's stream joins eager_kernel's after this kernel, rvm_abi.hip run_logl)
        if (eager && threadIdx.x == 0)
            __hip_atomic_store(ef, (gen << 8) | 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#ifdef RVM_PROFILE
        if (t == (int)blockIdx.x && lane == 0 && (size_t)blockIdx.x * 8 + wv < RVM_RPROF_MAX_WAVES) {
            unsigned long long* o = rvm_rprof + ((size_t)blockIdx.x * 8 + wv) * RVM_RPROF_SLOTS;
            o[0] = prt_entry;
            o[1] = prt_loop0;
            o[2] = prt_loop1;
            o[3] = __builtin_amdgcn_s_memrealtime();
            o[4] = p_seg;
            o[5] = p_epo;
            o[6] = p_steps;
            o[7] = pt_loop0 - pt_entry;
            o[8] = pt_loop1 - pt_loop0;
            o[9] = (unsigned long long)t | ((unsigned long long)tm << 16) | ((unsigned long long)(own + 1) << 20) |
                   ((unsigned long long)(p_lvl + 1) << 24) | ((unsigned long long)(eager ? 1 : 0) << 28);
            o[10] = p_pass;
            o[11] = (unsigned long long)(unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_REG_HW_ID
            o[12] = p_wait;
            o[13] = pt_lists - pt_entry;
            o[14] = pt_sched - pt_entry;
            o[15] = pt_setup - pt_entry;
            o[16] = pt_slot - pt_entry;
            o[17] = pt_rows - pt_entry;
        }
#endif
    }
}

// Eager halving passes (round 4): for a plain launch of 32..512 walkers (SMALA's centres, batched
// State evaluations), halving pass 1 (and 2 with RVM_EAGER_PASSES=2) of EVERY walker runs on the
// plan's side stream at the same time as the likelihood kernel, on CUs the launch leaves idle.
// Grid: (groups of WPB walkers) x 2 directions x eager_passes, four waves per block (one per level).
// A block first claims its (pass, direction) item of its group (DevPlan::eflag; claim_item) -- if the
// refinement kernel has claimed it, that kernel integrates the pass itself and the block exits --
// then stores its walker-directions' chi2, estimate, encounter flag and RV per epoch write-through,
// and finally the claim word gen << 8 | 2.  The refinement kernel, one task per group, replays the
// items it finds claimed by an eager block instead of integrating them (the same decisions and
// bits), and stops every block it does not need: a group none of whose walkers it holds at once
// (eflag[0]), the directions no open walker needs (eflag[6 + d]), and, when it has finished the
// group, whatever of it still runs (eflag[0]) -- blocks check these before reading their walkers and
// once per epoch.  run_logl joins the side stream back into the caller's after the refinement
// kernel (rvm_abi.hip): the launch is complete, eager blocks included, when the caller's stream is.
template <int NP, bool D3>
__global__ __launch_bounds__(256) void eager_kernel(const DevPlan P, const int W, const double* __restrict__ params,
                                                    const double hill_factor) {
    constexpr int L = LanesPerWalker<NP>::value;
    constexpr int WPB = 64 / L;
    constexpr int PR = D3 ? 7 : 5;
    constexpr int R = PR * NP;
    const int wv = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    const int slot = lane / L;
    const int pl_idx = lane % L;
    const int nl = P.n_levels;
    const int np2 = P.eager_passes == 2;  // (blocks per group: 2 directions x eager_passes)
    const int g = blockIdx.x >> (1 + np2), dd = (blockIdx.x >> np2) & 1, rf = 1 + (np2 & blockIdx.x);
    const DirSched& SR = dd ? P.bwd : P.fwd;
    const int Er = SR.n_epochs;
    __shared__ double s_rv[2][RVM_MAX_LEVELS][64];
    __shared__ int s_enc[RVM_MAX_LEVELS][64];
    __shared__ int s_cancel[2];
    __shared__ unsigned long long s_gen;
    gu64* ef = (gu64*)(P.eflag + (size_t)g * RVM_EFLAG_WORDS);
    if (threadIdx.x == 0) s_gen = __hip_atomic_load(P.gen_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const unsigned long long gen = s_gen;
    const unsigned long long ctag = (gen << 8) | 1ull;
    auto cancelled_now = [&]() {
        return __hip_atomic_load(ef, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ctag ||
               __hip_atomic_load(ef + 6 + dd, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == ctag;
    };
    gu64* item = ef + 2 + 2 * (rf - 1) + dd;
    if (threadIdx.x == 0) s_cancel[0] = cancelled_now() || !claim_item(item, gen, 1ull);
    __syncthreads();
    if (s_cancel[0]) return;  // (before the walkers are read)
    const int w0 = g * WPB;
    const int wo = w0 + slot < W ? w0 + slot : w0;  // (lanes past the last walker repeat the group's first)
    double rowv[R];
#pragma unroll
    for (int r = 0; r < R; r++) rowv[r] = params[(size_t)r * W + wo];
    Lane<NP> s;
    int status = RVM_STATUS_OK;
    double e2w;
    walker_setup<NP, D3, L>(rowv, pl_idx, hill_factor, s, status, e2w);
    int k = wv < nl ? wv : -1;
    k = __builtin_amdgcn_readfirstlane(k);
    const int k_u = k < 0 ? 0 : k;
    const bool work = k >= 0;
    KickPrep<NP> kq{};
    if (work && Er > 0) kq = kick_prep<NP, L, D3>(s, 1.875);
    const int m_r = P.mult[k_u] << rf;
    const int nt_r = P.nt[k_u];
    const bool late = P.late_mult > 0 && m_r >= P.late_mult;  // (the late vote: the same bits)
    const double sc = ldexp(P.inv_mult[k_u], -rf);
    const bool cmb = work && k == 0 && lane < WPB && w0 + lane < W;
    const size_t plane = (size_t)P.lvx_emax * P.lvx_stride;
    gu64* rvo = (gu64*)(P.rve + ((size_t)(rf - 1) * 2 + dd) * plane + (cmb ? w0 + lane : 0));
    double c2 = 0.0, e2 = 0.0;
    bool cancelled = false;
    for (int e = 0; e < Er; e++) {
        const int ns = __builtin_amdgcn_readfirstlane(work ? SR.seg_n[e] * m_r : 0);
        // (cancels are seen at the epochs: the segment-level cancel of team B's passes,
        // segment_gated_c, measured slower here -- config 4 0.645 -> 0.66 ms median step,
        // profiles/r05r_config4_ab_cancel.jsonl)
        if (ns > 0) segment_gated<D3, NP, L, RVM_REFINE_GUESS>(s, kq, SR.seg_h1[e] * sc, ns, nt_r, late);
        if (work) {
            const double v0 = star_vx<NP, L>(s);
            if (pl_idx == 0) s_rv[e & 1][k_u][slot] = v0;
        }
        if (wv == 0 && lane == 0) s_cancel[e & 1] = cancelled_now();
        __syncthreads();
        if (s_cancel[e & 1]) {
            cancelled = true;
            break;
        }
        if (cmb) {  // (the refinement kernel's combiner, expression for expression)
            double rvx = 0.0, rv3 = 0.0;
            for (int q = 0; q < nl; q++) rvx += P.lw[q] * s_rv[e & 1][q][lane];
            for (int q = 1; q < nl; q++) rv3 += P.lw3[q] * s_rv[e & 1][q][lane];
            const double ob = SR.obs_rv[e], s2 = SR.obs_s2[e];
            const double r = rvx - ob;
            c2 += (r * r) / s2;
            e2 += fabs((rvx - rv3) * (r + (rv3 - ob))) / s2;
            __hip_atomic_store(rvo + (size_t)e * P.lvx_stride, (unsigned long long)__double_as_longlong(rvx),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (cancelled) return;
    if (work && pl_idx == 0) s_enc[k_u][slot] = (int)(((s.encm >> lane) & kick_enc_bits<NP>()) != 0);
    __syncthreads();
    if (wv == 0) {
        if (cmb) {
            int er = 0;
            for (int q = 0; q < nl; q++) er |= s_enc[q][lane];
            gu64* es = (gu64*)(P.esum + ((size_t)(rf - 1) * 2 + dd) * 3 * P.lvx_stride + w0 + lane);
            auto bits = [](double v) { return (unsigned long long)__double_as_longlong(v); };
            __hip_atomic_store(es, bits(c2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(es + P.lvx_stride, bits(e2), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(es + 2 * (size_t)P.lvx_stride, bits((double)er), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(item, (gen << 8) | 2ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int NPV, bool D3V>
static hipError_t launch_eager_t(const DevPlan& P, int W, const double* params, double hill_factor, hipStream_t st) {
    constexpr int wpb = 64 / LanesPerWalker<NPV>::value;
    const int groups = (W + wpb - 1) / wpb;
    eager_kernel<NPV, D3V><<<dim3(2 * P.eager_passes * groups), dim3(256), 0, st>>>(P, W, params, hill_factor);
    return hipGetLastError();
}

// Dynamic-LDS budget of the refinement kernel on the current device (the CU's 160 KB less its static
// LDS), with the attribute admitting it set once per device and instantiation.  rvm_plan_create
// calls it (prepare_refine) so a launch never changes function attributes -- launches stay
// capturable -- and a plan whose schedule would not fit is refused there, not at launch.
template <int NPV, bool D3V, int NW>
static size_t refine_budget() {
    static size_t budget[64] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) {
        (void)hipGetLastError();
        return 32 * 1024;
    }
    if (budget[dev] == 0) {
        const void* f = reinterpret_cast<const void*>(&refine_kernel<NPV, D3V, NW>);
        hipFuncAttributes fa{};
        size_t b = 32 * 1024;
        if (hipFuncGetAttributes(&fa, f) == hipSuccess && fa.sharedSizeBytes < (size_t)RVM_LDS_PER_CU) {
            const size_t lim = (size_t)RVM_LDS_PER_CU - fa.sharedSizeBytes;
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lim) == hipSuccess) b = lim;
        }
        (void)hipGetLastError();
        budget[dev] = b;
    }
    return budget[dev];
}

template <int NPV, bool D3V>
static hipError_t launch_refine_t(const DevPlan& P, int W, const double* params, double hill_factor, double* logl,
                                  int32_t* status, double* rv_out, const StretchArgs& sa, int eager,
                                  hipStream_t stream) {
    constexpr int wpb = 64 / LanesPerWalker<NPV>::value;
    const int emax = P.fwd.n_epochs > P.bwd.n_epochs ? P.fwd.n_epochs : P.bwd.n_epochs;
    const size_t smem = (size_t)emax * 8 * sizeof(double);
    // (checked by rvm_plan_create: a launch that cannot run would leave the work lists' counts set)
    // (refine_kernel NW: four waves per workgroup for up to four levels; RVM_REFINE_W4=0 forces eight, A/B)
    static const bool w4_env = [] {
        const char* e = getenv("RVM_REFINE_W4");
        return !(e && e[0] == '0');
    }();
    const bool w4 = P.n_levels <= 4 && w4_env;
    if (smem > (w4 ? refine_budget<NPV, D3V, 4>() : refine_budget<NPV, D3V, 8>())) return hipErrorInvalidConfiguration;
    // every block reads the list sizes (the last one resets them): a grid of at most one block
    // per CU, and no more than the lists could fill
    // (an even count: a split group's two workgroups are 2j, 2j + 1)
    const int groups = (W + wpb - 1) / wpb + 2;
    int nb = std::max(2, std::min(P.n_cu > 0 ? P.n_cu : 256, 2 * groups));
    nb &= ~1;
    if (w4)
        refine_kernel<NPV, D3V, 4><<<dim3(nb), dim3(256), smem, stream>>>(P, W, params, hill_factor, rv_out, logl, status,
                                                                          sa, eager);
    else
        refine_kernel<NPV, D3V, 8><<<dim3(nb), dim3(512), smem, stream>>>(P, W, params, hill_factor, rv_out, logl, status,
                                                                          sa, eager);
    return hipGetLastError();
}

// prepare_refine's check for one instantiation (rvm_plan_create)
template <int NPV, bool D3V>
static hipError_t prepare_refine_t(const DevPlan& P) {
    const int emax = P.fwd.n_epochs > P.bwd.n_epochs ? P.fwd.n_epochs : P.bwd.n_epochs;
    const size_t smem = (size_t)emax * 8 * sizeof(double);
    const size_t b = std::min(refine_budget<NPV, D3V, 4>(), refine_budget<NPV, D3V, 8>());
    return smem <= b ? hipSuccess : hipErrorInvalidConfiguration;
}

// the per-planet-count translation units (rvm_refine_np<N>.hip: one instantiation set each, so make -j
// compiles them in parallel) export these
#define RVM_REFINE_NP_API(N)                                                                                     \
    hipError_t launch_refine_np##N(const DevPlan& P, int W, const double* params, double hill_factor, double* logl, \
                                   int32_t* status, double* rv_out, const StretchArgs& sa, int eager,            \
                                   hipStream_t stream);                                                          \
    hipError_t launch_eager_np##N(const DevPlan& P, int W, const double* params, double hill_factor,            \
                                  hipStream_t stream);                                                           \
    hipError_t prepare_refine_np##N(const DevPlan& P);
RVM_REFINE_NP_API(1)
RVM_REFINE_NP_API(2)
RVM_REFINE_NP_API(3)
RVM_REFINE_NP_API(4)
#undef RVM_REFINE_NP_API

}  // namespace rvm

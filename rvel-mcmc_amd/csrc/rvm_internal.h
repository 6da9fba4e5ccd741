// rvm_internal.h -- host/device shared launch descriptors of librvmcmc.so (not part of the ABI).
#pragma once
#include <stdint.h>

#include "../../include/rvmcmc.h"

namespace rvm {

// level-split layout: the LDS ring of a type-A block holds at most this many epochs per level
// (levels wait for the combiner beyond it); the dynamic LDS request plus the kernel's static LDS
// (read with hipFuncGetAttributes at launch) must stay within the CU's 160 KB
constexpr int RVM_LS_RING = 64;
// LDS-coupled layouts (one or two groups per block): epochs of the levels' star vx a group's ring
// holds (rvm_logl.hip; the levels wait for the combiner beyond it)
constexpr int RVM_LC_RING = 16;
// ... within this many bytes per group (the one-planet layouts, 64 walkers per group, took
// 40 KB per group at 16 epochs -- 80 KB for a two-group block -- which cut a one-planet fused launch to
// ~1150 epochs per direction and one block per CU); DevPlan::lc_ring holds the plan's ring length
constexpr int RVM_LC_RING_BYTES = 24 * 1024;
constexpr int RVM_LDS_PER_CU = 160 * 1024;
// adaptive resolution: lane state at t = 0 kept in LDS for the refinement passes, per walker group
// (rx, ry, vx, vy, rz, vz, r, ir of each of the 64 lanes)
constexpr int RVM_INIT_DOUBLES = 8 * 64;
// the extension's acceptance bound, in units of the direction's tolerance (rvm_logl.hip extend_pass;
// oracle/rvoracle.c EXT_ACCEPT).  Round 4: 1 (was 2) -- at 2 a steady-state proposal settled by the
// extension in both directions missed T2 (1.39e-6 vs IAS15, GPU and oracle alike): r5's error
// reaches 1.3 x the change d where d is in (1, 2] tol_dir, 0.43 x where d <= tol_dir
constexpr double RVM_EXT_ACCEPT = 1.0;
// the certain-reject cut's error bound after a halving pass: min(d2, this x the pass's estimate)
// (rvm_logl.hip refine_loop; oracle/rvoracle.c CUT_EST_FACTOR; measured error / estimate <= 57 on
// the main pass at the plan's step, smaller after a halving)
constexpr double RVM_CUT_EST_FACTOR = 100.0;
// the roundoff floor of a halving pass (rvm_refine.hip; oracle/rvoracle.c FLOOR_BOUND): a direction
// whose estimate stopped falling settles at its best pass when that pass's estimate is within this
// x tol_dir (round 4: a crossing-orbit walker of the wide ball reached its floor at ~1e-7..2e-6 in
// logL from the 5th halving on -- the finer steps' accumulated rounding -- and ended UNRESOLVED on
// the GPU where the oracle's rounding happened to settle it)
constexpr double RVM_FLOOR_BOUND = 4.0;
// the certain-reject cut after the extension (round 6): for a walker whose pericentre passage is
// quicker still than the eccentricity guard's -- (1 - e) below this factor x (1 - e_guard), 1.82x
// quicker -- the extension's change does not bound its error (HD155358's steady state, planets of
// e = 0.79-0.84: the extension's chi2 50-500x the true one, its change a third of the error; three
// proposals in 24576 cut that IAS15 accepts, scripts/probe/decision_mismatch_probe.py), so its bound
// stays the main pass's (chi2 - 100 est); oracle/rvoracle.c CUT_ECC_FACTOR
constexpr double RVM_CUT_ECC_FACTOR = 0.6712;
// past the cut guard the bound after the extension is chi2 - min(K d, 100 est), K = RVM_CUT_GUARD_K
// (the three wrong cuts had the extension's change d a third of the error); oracle CUT_GUARD_K
constexpr double RVM_CUT_GUARD_K = 10.0;
// launches of fewer walkers than this run the extension after the main pass (only when a walker is
// flagged) instead of as a concurrent fifth wave of the one-group-per-block layout (launch_logl_t)
constexpr int RVM_CX_MIN_WALKERS = 32;
// plain launches of at most this many walkers run the first two halving passes of every walker
// beside the likelihood kernel (rvm_refine.hip eager_kernel): 4 x 512 / 32 = 64 blocks of 4 waves
constexpr int RVM_EAGER_MAX = 512;
// ... and at least this many (a launch of a few walkers rarely refines, and the fork costs the
// scalar State API ~7 %: config 1, profiles/r04x_configs_eager_ab.jsonl)
constexpr int RVM_EAGER_MIN = 32;
// eflag words per eager group (rvm_refine.hip)
constexpr int RVM_EFLAG_WORDS = 8;
// refinement kernel teams per walker group (rvm_refine_impl.h): team t runs halving pass t + 1 from
// the launch's start, all at once; at most this many (the plan's count: DevPlan::n_teams)
constexpr int RVM_TEAMS_MAX = 4;
constexpr int RVM_TEAMS_DEFAULT = 4;
// ... and no more than the deepest pass of the plan's last this-many launches needed (at least two)
constexpr int RVM_DEPTH_WINDOW = 8;

// Epoch schedule of one integration direction (t >= 0 ascending from 0, or t < 0 descending).
struct DirSched {
    int32_t n_epochs;
    int32_t n_steps;          // sum of seg_n: base steps of the whole direction
    // level-split layout: levels 0 (type-A blocks) and 1 (type-B, tB = 6) may run as a head over
    // epochs [0, split) and a tail over [split, n_epochs) in two waves; pre = base steps before split
    int32_t split0, pre0, split1, pre1;
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
    // halving passes (rvm_refine.hip refinement and eager kernels): a level whose steps per base step
    // (mult << rf) reach late_mult runs the gated drift with the late vote (rvm_device.h drift ACC 3:
    // the same bits; ~3-6 % faster per step where few first Halley steps fail, slower where many do:
    // scripts/probe/kepler_accept_probe.hip, profiles/r06a_kepler_accept_probe.jsonl); 0: never
    int32_t late_mult;
    // LDS-coupled layouts: epochs in each group's ring of the levels' star vx (rvm_logl.hip lring; 2 ..
    // RVM_LC_RING, within RVM_LC_RING_BYTES per group; set by rvm_plan_create)
    int32_t lc_ring;
    double inv_mult[RVM_MAX_LEVELS];  // 1 / mult: level step = seg_h1 * inv_mult
    double lw[RVM_MAX_LEVELS];     // Richardson (Lagrange-at-zero in h^2) weights
    // adaptive resolution (rvm_logl.hip): lw3 = the Lagrange weights of levels
    // 1 .. n_levels-1 alone (lw3[0] = 0); a direction whose estimate
    //   est = sum_e |(rv - o)^2 - (rv3 - o)^2| / s2 / npoints   (rv3 = sum_k lw3[k] rv_k)
    // exceeds rtol_dir is integrated again with every step halved, at most rmax times
    double lw3[RVM_MAX_LEVELS];
    double rtol_dir;   // +inf: no estimate check
    int32_t rmax;
    // the finest level (largest multiplier) of the main pass: with the adaptive resolution on, an
    // encounter the main pass sees only on coarser levels does not end the walker -- those levels'
    // positions near a close approach are the least accurate (round 5: 21 of HD155358's 23
    // device-only encounters at its steady state never came within the exit distance on a densely
    // sampled trajectory) -- the direction is refined instead (oracle/rvoracle.c dir_main)
    int32_t fin_level;
    // 1: the certain-reject test runs on fused sampler launches (rvm_plan_set_certain_reject; an
    // empirical lower bound on chi2), 0: every open walker refines to the bound
    int32_t cut;
    // the extension (stage 1, rvm_logl.hip extend_pass): one more level of ext_mult steps per base
    // step (0: none) joined to the main pass's levels; lw5 = the weights of all n_levels + 1 levels.
    // Every launch keeps, per direction, epoch and walker ([2][lvx_emax][lvx_stride]), lvx = the
    // main pass's partial sum sum_k lw5[k] rv_k and rvp = its extrapolated RV (then each halving
    // pass's, the previous pass of the next)
    int32_t ext_mult, ext_nt, ext_spec;
    double inv_ext;
    double lw5[RVM_MAX_LEVELS + 1];
    double* lvx;
    double* rvp;
    // eccentricity guard (rvm_plan_set_verify_eccentricity; +inf: off): a walker with a planet of
    // e^2 above it counts as above the bound after the main pass (it gets the extension)
    double e2_guard;
    // ... and above this e^2 (from the guard: RVM_CUT_ECC_FACTOR) the extension's change gives no
    // lower bound for the certain-reject cut (+inf: always)
    double e2_cut;
    double cut_guard_k;  // past the cut guard: chi2 - min(k d, 100 est) (RVM_CUT_GUARD_K; 0: chi2 - 100 est)
    int32_t lvx_emax, lvx_stride;
    // walkers handed from the likelihood kernel to the refinement kernel (rvm_refine.hip): a walker
    // with a direction still open after the main pass and the extension (and no certain reject) is
    // appended to list 0 (both directions open), 1 (forward only) or 2 (backward only):
    // rq_n[0..2] the list sizes (the refinement kernel resets them; rq_n[3] counts its blocks),
    // rq_w [3][rq_cap] walker slots, rq_c [2][rq_cap] the settled direction's chi2 (fwd, bwd)
    int32_t* rq_n;
    int32_t* rq_w;
    double* rq_c;
    int32_t rq_cap;
    // rq_mark [rq_cap]: the low 32 bits of the launch generation at each walker slot the likelihood
    // kernel listed -- a speculative iteration's half-1 variant whose partner was NOT listed has its
    // partner's decision final in StretchArgs::dec, so the variant the decision rules out is skipped
    // (rvm_refine.hip; RVM_STATUS_SKIPPED)
    int32_t* rq_mark;
    int32_t skip_variants;  // 1: skip the ruled-out variants (RVM_SKIP_VARIANTS=0 at plan creation: refine them, A/B)
    // a both-direction group split over two workgroups exchanges its walkers' per-direction state
    // after every halving pass (rvm_refine.hip): rq_x [groups][2 directions][2 pass parities][64]
    // values in the meeting slot's encoding, rq_xf [groups][2] the flag (launch generation << 8 | pass)
    unsigned long long* rq_x;
    unsigned long long* rq_xf;
    int32_t rq_xgroups;
    // (both [groups][n_teams] since round 4: team t runs pass t + 1 from the launch's start, then hands
    // its walkers on, rvm_refine_impl.h) team t's walker state after its pass for team t + 1,
    // rq_t [groups][n_teams - 1][16][64], and its flag rq_tf [groups][n_teams] (launch generation
    // << 8 | 1, or 2 when the group is done; [n_teams - 1] the group's done word)
    unsigned long long* rq_t;
    unsigned long long* rq_tf;
    // teams 1 .. n_teams - 1: their own RV per pass (as rvp), [n_teams - 1][2][lvx_emax][lvx_stride]
    double* rvp2;
    // the plan's team count (2 .. RVM_TEAMS_MAX; a launch uses fewer when its groups' tasks would not
    // all fit the grid, or when the deepest pass of the plan's last two launches was shallower; rq_t
    // null: no teams)
    int32_t n_teams;
    // [RVM_DEPTH_WINDOW + 1] by launch generation mod RVM_DEPTH_WINDOW + 1: the deepest pass a group
    // of that launch finished at, tagged (generation << 8 | pass; atomic max)
    unsigned long long* depth_w;
    // eager halving passes (rvm_refine.hip eager_kernel; plain launches of at most eager_max
    // walkers, 0: none): passes 1 and 2 of every walker beside the likelihood kernel -- rve [2
    // passes][2 directions][lvx_emax][lvx_stride] their RV per epoch, esum [2][2][3][lvx_stride]
    // their chi2, estimate and encounter flag
    double* rve;
    double* esum;
    // [groups][8] (rvm_refine.hip): [0] cancel the group, [2 + 2 (rf - 1) + d] the claim word of
    // pass rf in direction d (generation << 8 | 1 eager block running, 2 its results stored, 3 the
    // refinement kernel integrates it itself), [6 + d] cancel direction d
    unsigned long long* eflag;
    int32_t eager_max;
    int32_t eager_passes;  // (1 or 2: how many halving passes eager_kernel runs)
    int32_t eager_split;   // 1: an eager launch's refinement runs each direction of a group on its own block
    // the launch generation (device word, >= 1): the tag of the refinement kernel's exchange flags and
    // the eager blocks' claim words.  Read on the device by both kernels and advanced on the device
    // after every launch (the refinement kernel's last block, or gen_bump_kernel after an eager
    // launch), so a launch sequence captured into a hipGraph tags every replay afresh.
    unsigned long long* gen_dev;
    // plan-owned device counters (rvm_plan_faults): [0] level-split hand-offs given up (the
    // workspace is dirty until reset), [1] NONFINITE results, [2] UNRESOLVED results,
    // [3] walker-direction refinement passes (extension + halvings), [4] refinements cut short as
    // certain rejects, [5] directions settled at their roundoff floor (RVM_FLOOR_BOUND)
    unsigned long long* counters;
    unsigned long long spin_ticks;  // hand-off waits give up after this long without progress (100 MHz)
    double npoints;
    int32_t n_obs;
    int32_t inclined;  // 1: 7 parameter rows per planet (ix, iy), 3-D integration
    int32_t n_cu;      // compute units of the plan's device (launch shape, launch_logl)
    // level-split layout (launch_logl, rvm_logl.hip): level 1 of a walker group runs in another
    // workgroup than its levels 3, 2, 0 and the unit's combiner, and hands its star velocities over
    // through HBM.  Null when the plan cannot use it.  All-ones / -1 between launches.
    double* lv_rv;     // [2][lv_emax][lv_stride] the HBM-handed level's (1; 2 with lsx) star vx per direction, epoch, walker
    int32_t* lv_enc;   // [2][lv_stride] level 1's encounter / prior flags
    int32_t lv_emax, lv_stride;
    DirSched fwd, bwd;
};

// Fused sampler step by value as a kernel argument: a stretch half-step (rvm_stretch_half_step,
// c != nullptr) or an MH step (rvm_mh_step, mh_scale != nullptr); both null for a plain
// likelihood launch.
//
// Speculative whole iteration (rvm_stretch_iteration_begin, n_spec > 0): the launch has 3 n_spec
// walker slots.  Slots [0, n) are half 0's walkers (proposal against c = half 1, accept at the
// end as a plain half-step, decision to dec[]); slots [n, 2n) and [2n, 3n) are half 1's walkers
// proposed against their partner j in half 0 as it will be after this iteration's first
// half-step, both ways: c = c0[j] (the partner rejects) and c = q0(j) (it accepts; q0 recomputed
// from c0, c and the partner's own draws).  Their logl go to logl_out[n + v n + k]; the second
// half-step's accepts run afterwards (rvm_stretch_iteration_end) once dec[] is known.
struct StretchArgs {
    const double* c;    // complement half, walker-major [n1][dim] (one contiguous row per c_j)
    double* x;          // this half's free parameters [dim][xstride] (accepted proposals written back)
    double* x_aos;      // walker-major mirror of x [W][dim] kept in step on accept (nullable)
    double* lnp;        // their log-probabilities [W]
    int32_t* accepted;  // accept counters [W] (nullable)
    int64_t s0_begin;   // global index of walker 0 of x (Philox key)
    uint64_t seed, iteration;
    double a;
    int32_t n1, dim;
    uint32_t half;
    int32_t xstride;    // row stride of x (W for a half-step, n_spec for a speculative iteration)
    // speculative iteration only (n_spec = 0 otherwise)
    int32_t n_spec;     // walkers per half on this rank
    const double* c0;   // half 0 walker-major [n1][dim] as at the start of the iteration
    const double* x1;   // half 1's free parameters [dim][n_spec]
    int64_t s1_begin;   // global index of half 1's walker 0 (Philox key)
    int32_t* dec;       // [n_spec] half 0's accept decisions (1 accepted)
    const double* lnp1;  // [n_spec] half 1's log-probabilities (nullable): its accept inputs, for the
                         // adaptive resolution's certain-reject test
    // fused MH step (rvm_mh_step; c == nullptr, mh_scale != nullptr): walker w is chain w with
    // free parameters x [dim][xstride], proposal q = x + mh_step * mh_scale[p] * N(0,1) formed in the
    // prologue (Philox keyed by s0_begin + w), MH accept at the end against lnp
    const double* mh_scale;  // [dim]
    double mh_step;
    // fused SMALA stencil (rvm_smala_stencil_logl; fd_x != nullptr, no accept in the launch):
    // walker w = s * fd_n + c is point s of chain c's central-difference stencil around
    // fd_x [dim][fd_n], formed as rvm_fd_params does (fd_point)
    const double* fd_x;
    const double* fd_floor;  // [dim]
    double fd_rel;
    int32_t fd_n;
    int32_t src[RVM_MAX_PARAM_ROWS];  // rvm_param_map
    double base[RVM_MAX_PARAM_ROWS];
};

// Second half of a speculative stretch iteration (rvm_stretch_iteration_end) by value.
struct IterEndArgs {
    int32_t dim, n, n_half;     // free parameters, walkers per half on this rank, walkers per half
    int64_t s0_begin, s1_begin;  // global index of this rank's first walker of half 0 / half 1
    const double* x0;           // half 0 [dim][n] after the first half-step
    double* x0_aos;             // its walker-major mirror [n][dim], refreshed here (nullable)
    const int32_t* dec_local;   // [n] half 0's decisions on this rank
    const int32_t* dec_all;     // [n_half] half 0's decisions, global order
    double* x1;                 // half 1 [dim][n], updated in place
    double* x1_aos;             // its walker-major mirror [n][dim] (nullable)
    double* lnp1;               // [n]
    const double* c0;           // half 0 walker-major [n_half][dim] at the start of the iteration
    const double* c1;           // half 1 walker-major [n_half][dim] at the start of the iteration
    const double* lnp_spec;     // [3 n] logl of the begin launch (half 1's two variants at n and 2n)
    const int32_t* st_spec;     // [3 n] their statuses
    double a;
    uint64_t seed, iteration;
    int32_t* accepted1;         // [n] (nullable)
    double* lnp_new_out;        // [n] logl of half 1's chosen proposals (nullable)
    int32_t* status_new_out;    // [n] (nullable)
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

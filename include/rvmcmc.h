/*
 * rvmcmc.h -- C ABI of librvmcmc.so, the MI355X (gfx950) radial-velocity MCMC hot path.
 *
 * The reference (MrSwordFish/rvel-mcmc, Python 2 + REBOUND) has no native interface of its own;
 * its hot path is reached through three Python call sites, which this ABI replaces in batch:
 *
 *   reference call site                                   replaced by
 *   ----------------------------------------------------  ----------------------------------------
 *   state.py:103-110  State.get_logp(obs) -> float         rvm_logl_batch (W walkers per call)
 *     (state.py:36-47 setup_sim, :61-73 get_rv,
 *      :89-98 get_chi2, :299-315 priorHard, and
 *      REBOUND sim.add/move_to_com/integrate/Encounter)
 *   mcmc.py:28-35     lnprob(x, e) (emcee callback)         rvm_logl_batch
 *   observations.py:6-69 Observation.{tf,tb,rvf,rvb,       rvm_plan_create (epoch schedule, obs data)
 *     errorf,errorb,Npoints}
 *   mcmc.py:57-65 Ensemble.step -> emcee 2.2.1 stretch     rvm_stretch_propose / rvm_stretch_accept,
 *     move (EnsembleSampler._propose_stretch)                or fused: rvm_stretch_half_step
 *   mcmc.py:89-121 Mh.generate_proposal / Mh.step          rvm_mh_propose / rvm_mh_accept, or fused:
 *                                                            rvm_mh_step
 *   state.py:218-294 get_chi2_d_dd / get_logp_d_dd         rvm_logl_derivs (exact gradient + Hessian,
 *     (REBOUND 1st/2nd-order variational equations)         hyper-dual forward mode)
 *   mcmc.py:144-187 Smala.generate_proposal/step           rvm_fd_params (finite-difference stencil)
 *     mcmc.py:135-139 Smala.softabs,                         + rvm_smala_derive, or rvm_logl_derivs +
 *     mcmc.py:158-162 Smala.transitionProbability              rvm_smala_metric; rvm_smala_propose /
 *                                                              rvm_smala_accept
 *
 * Conventions
 *   - All array pointers passed to launch functions are DEVICE pointers (hipMalloc / torch CUDA
 *     tensors), caller-owned.  Launch functions never allocate, never synchronise, and are
 *     stream-ordered on `stream` (a hipStream_t; NULL = the null stream): everything a launch
 *     enqueues is complete once `stream` is -- including the eager halving pass a plain launch of
 *     32..512 walkers runs on the plan's own side stream, which is forked from `stream` and joined
 *     back into it within the launch -- so inputs may be reused right after `stream` is synchronised.
 *     They are capturable into a hipGraph: no host-side state changes per launch (the launch
 *     generation that tags the kernels' hand-off flags advances on the device) and kernel
 *     attributes are set by rvm_plan_create.  rvm_plan_create is the only call that allocates
 *     (device buffers owned by the plan) and it synchronises once.
 *   - A plan is single-stream: it owns per-launch workspace (the direction-exchange slots and the
 *     level-split hand-off slots, left empty by every completed launch), so launches that use one plan must be
 *     serialised on one stream at a time.  Concurrent launches on two streams need two plans (the
 *     Python layer keys its plan cache by stream, rvmcmc/engine.py).
 *   - Walker parameters are SoA, [n_params][n_walkers] float64, n_params = 5*n_planets with the
 *     canonical per-planet key order  m, a, h, k, l  (the Python layer maps a
 *     State's dict order onto it), or 7*n_planets (m, a, h, k, l, ix, iy) for inclined plans.
 *   - Return code: 0 = success, < 0 = argument / launch error (rvm_last_error() explains).
 *     Per-walker physics outcomes are never errors: they are status codes plus logl = -INFINITY
 *     (the reference raises rebound.Encounter / returns -inf from priorHard; mcmc.py:28-35 maps
 *     every exception to -inf).
 */
#ifndef RVMCMC_H
#define RVMCMC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RVM_ABI_VERSION 12

/* per-walker status codes (status_out) */
#define RVM_STATUS_OK 0
#define RVM_STATUS_PRIOR 1     /* State.priorHard() true (state.py:299-315) -> logl = -inf        */
#define RVM_STATUS_ENCOUNTER 2 /* pair distance < exit_min_distance (REBOUND Encounter) -> -inf   */
#define RVM_STATUS_NONFINITE 3 /* non-finite chi2 (a main pass that blows up is refined; a halving pass
                                  that blows up ends the walker), or a hand-off that gave up -> -inf */
#define RVM_STATUS_UNRESOLVED 4 /* adaptive resolution: the extrapolation-error estimate still above
                                   rvm_config.resolve_tol after resolve_max refinements -> -inf      */
#define RVM_STATUS_SKIPPED 5    /* rvm_stretch_iteration_begin's status_spec only: a half-1 variant
                                   slot whose partner's first-half decision (already final) rules it
                                   out, not refined by the adaptive resolution; rvm_stretch_iteration_end
                                   never reads it.  logl -inf                                          */

#define RVM_MAX_PLANETS 4
#define RVM_MAX_LEVELS 6
#define RVM_MAX_EPOCHS_PER_DIRECTION 1700 /* epochs with t >= 0, and with t < 0, per plan */
#define RVM_SMALA_MAX_PARAMS 20           /* free parameters per SMALA chain                 */
#define RVM_RESOLVE_MAX_LIMIT 12          /* rvm_config.resolve_max                          */

/* Integrator configuration of a plan. */
typedef struct {
    int32_t n_planets;     /* 1..RVM_MAX_PLANETS                                                  */
    double dt;             /* base step in code units (yr/2pi); the segment between two epochs is
                              cut into n = ceil(len/dt) base steps                                 */
    int32_t n_levels;      /* Richardson levels, 1..RVM_MAX_LEVELS                                  */
    double npoints_norm;   /* obs.Npoints: chi2 is divided by this (state.py:98), NOT the epoch count */
    int32_t level_mult[RVM_MAX_LEVELS]; /* level k integrates each segment with n * level_mult[k]
                              steps (distinct, >= 1, at most 64); all zero = harmonic 1, 2, ..., n_levels */
    double period_hint;    /* shortest orbital period the walkers are expected to have (code units):
                              sizes the per-level Stumpff series (performance only, results are
                              exact for any orbit); 0 = longest series on every level              */
    int32_t inclined;      /* 0: coplanar, params [5*n_planets][W] (m, a, h, k, l); 1: inclined,
                              params [7*n_planets][W] (m, a, h, k, l, ix, iy; REBOUND's Pal ix, iy),
                              3-D integration, prior adds ix^2 + iy^2 >= 4 (state.py:311-313)      */
    double resolve_tol;    /* adaptive resolution: bound on a walker's |logL| error as
                              estimated from the extrapolation itself -- the change of chi2/npoints
                              when the coarsest level is dropped -- split evenly over its two
                              directions.  A direction above its half first gets one extra level
                              (the extension, rvm_plan_extension) joined to its stored levels; if
                              that does not settle it, the walker's open directions are integrated
                              again together with every step halved, up to resolve_max times (the
                              reference's IAS15 adapts its step to the orbit; a fixed plan step
                              does not).  The halving passes run in a second kernel on the launch's
                              stream; every launch function of an adaptive plan
                              enqueues both.  <= 0: off                                            */
    int32_t resolve_max;   /* 0..RVM_RESOLVE_MAX_LIMIT halvings; 0 with resolve_tol > 0: flag
                              (UNRESOLVED) only                                                    */
} rvm_config;

typedef struct rvm_plan rvm_plan;

/* Build the epoch schedule for one observation set (host arrays, n_obs epochs in any order and
 * sign; t = 0 is the initial condition).  Allocates device memory and workspace for up to
 * max_walkers walkers per launch -- with four increasing levels and max_walkers large enough for
 * the level-split launch layout (more walker groups than half the CUs) also its hand-off
 * workspace, 16 * max(epochs per direction) * max_walkers + 8 * max_walkers bytes.
 * observations.py:6-69 (tf/tb/rvf/rvb/errorf/errorb). */
int rvm_plan_create(const rvm_config* cfg, const double* t, const double* rv, const double* sigma, int32_t n_obs,
                    int32_t max_walkers, rvm_plan** out);
void rvm_plan_destroy(rvm_plan* plan);
/* schedule introspection: total level-1 steps per direction (fwd, bwd), epochs per direction */
int rvm_plan_info(const rvm_plan* plan, int32_t* steps_fwd, int32_t* steps_bwd, int32_t* epochs_fwd,
                  int32_t* epochs_bwd);
/* The adaptive resolution's extension level of a plan: *ext_mult = its steps per base step
 * (max(level_mult) + 1), or 0 when the plan has none -- resolution off or flag-only, n_levels < 2 or
 * = RVM_MAX_LEVELS, or its stored main-pass values (2 doubles per direction, epoch and walker:
 * 32 * max(epochs per direction) * max_walkers bytes of device memory, written by every launch)
 * above RVM_EXT_MAX_BYTES. */
#define RVM_EXT_MAX_BYTES (4ull << 30)
int rvm_plan_extension(const rvm_plan* plan, int32_t* ext_mult);
/* Eccentricity guard of the adaptive resolution (plans with an extension level): a walker with a
 * planet of eccentricity above e counts as above the bound after the main pass whatever its
 * estimate, so the extension verifies it -- the estimate under-reads on orbits whose pericentre
 * passage is much quicker than the plan's reference orbit.  e <= 0: off (default). */
int rvm_plan_set_verify_eccentricity(rvm_plan* plan, double e);

/* The certain-reject test of the adaptive resolution (on: default).  On fused sampler launches a
 * walker whose accept test fails even at the upper bound on its logL that both directions' lower
 * bounds on chi2 give stops refining and reports that bound (a certain reject).  The bound of an
 * open direction is empirical (chi2 less the change its last stage brought, capped at 100 x its
 * estimate; the measured error / estimate stays <= 57), so on = 0 lets every
 * open walker refine to the plan's tolerance instead.  Replaces nothing in the reference (IAS15
 * integrates every proposal in full, state.py:61-73). */
int rvm_plan_set_certain_reject(rvm_plan* plan, int32_t on);

/* Counters of a plan since its creation or the last reset, read in order on `stream` (the call
 * synchronises that stream; any output pointer may be NULL):
 *   handoff_timeouts  level-split hand-off waits that gave up (rvm_plan_set_handoff_timeout): their
 *                     walkers report RVM_STATUS_NONFINITE, the plan's hand-off workspace is dirty
 *                     and every later level-split launch on the plan reports NONFINITE until reset
 *   nonfinite         walkers finished with RVM_STATUS_NONFINITE (any launch on the plan)
 *   unresolved        walkers finished with RVM_STATUS_UNRESOLVED
 *   refined           walker-direction passes of the adaptive resolution (extension + halvings)
 *   truncated         walker-directions whose refinement stopped because the proposal's accept
 *                     test fails even at the upper bound on its logL both directions give
 *                     (fused sampler launches): such a proposal is rejected and
 *                     reports that upper bound
 * reset != 0: zero the counters and restore the hand-off workspace, after the stream's earlier work.
 * The samplers (rvmcmc) check this and raise on timeouts / non-finite results (mcmc.py:28-35: emcee
 * refuses NaN log-probabilities) rather than treating them as ordinary rejections. */
int rvm_plan_faults(rvm_plan* plan, int32_t reset, int64_t* handoff_timeouts, int64_t* nonfinite,
                    int64_t* unresolved, int64_t* refined, int64_t* truncated, void* stream);
/* All of a plan's counters as an array (the same reset): out[0..4] as rvm_plan_faults, out[5]
 * walker-directions the adaptive resolution settled at their roundoff floor (a halving pass whose
 * estimate no longer fell: the direction keeps its best pass, whose estimate was within
 * RVM_FLOOR_BOUND = 4 x the bound), out[6] speculative variant slots skipped
 * (RVM_STATUS_SKIPPED); entries past RVM_N_COUNTERS read 0. */
#define RVM_N_COUNTERS 7
int rvm_plan_counters(rvm_plan* plan, int32_t reset, int64_t* out, int32_t n, void* stream);
/* Kernel timing (benchmarks): the plan's next max_launches likelihood evaluations (any entry point)
 * record HIP events on their stream around the likelihood kernel and around the refinement kernel
 * that follows it (0..4096; 0 stops).  rvm_plan_kernel_times waits for those events and returns
 * each evaluation's two kernel durations in ms (logl_ms[i], refine_ms[i]; either may be NULL; up
 * to max of them, *n_out = how many), then stops timing. */
int rvm_plan_time_kernels(rvm_plan* plan, int32_t max_launches);
int rvm_plan_kernel_times(rvm_plan* plan, float* logl_ms, float* refine_ms, int32_t max, int32_t* n_out);
/* Level-split hand-off waits give up after `seconds` without progress (default 2 s; > 0). */
int rvm_plan_set_handoff_timeout(rvm_plan* plan, double seconds);

/* logl_out[w] = -chi2/npoints_norm or -INF; status_out[w]; rv_out (nullable) = model RV
 * [n_obs][n_walkers] in the plan's input epoch order.  hill_factor = State.hillRadiusFactor
 * as the caller sees it (1.0 inside the reference samplers after deepcopy, state.py:212-213). */
int rvm_logl_batch(const rvm_plan* plan, int32_t n_walkers, const double* params, double hill_factor,
                   double* logl_out, int32_t* status_out, double* rv_out, void* stream);

/* ---- samplers (device-side proposal / accept; counter-based Philox4x32-10 RNG) ------------------
 * Draws are keyed by (seed, iteration, stream_id, global walker index), so results do not depend
 * on how walkers are sharded across ranks.  Every launch takes optional `draws` (device, nullable):
 * when non-NULL the documented uniforms/normals are read from it instead of Philox (tests inject
 * the same draws into the oracle). */

/* emcee 2.2.1 stretch move, half-step (S0 = walkers [s0_begin, s0_begin+n_s0) of the GLOBAL
 * ensemble, complement S1 given as a device array [n_params][n_s1] of positions).
 * propose: z = ((a-1)u1+1)^2/a, j = floor(u2*n_s1), q = c_j - z (c_j - x)
 *   writes q_out [n_params][n_s0] and z_out [n_s0].  draws layout: [2][n_s0] (u1, u2).
 * accept: lnpdiff = (n_params-1) ln z + lnp_new - lnp_old > ln(u3) -> x <- q, lnp <- lnp_new.
 *   x, lnp: [n_params][n_s0], [n_s0] (in place).  accepted: int32 counters [n_s0] (+= 1).
 *   draws layout: [n_s0] (u3). */
int rvm_stretch_propose(int32_t n_params, int32_t n_s0, int64_t s0_begin, const double* x, int32_t n_s1,
                        const double* c, double a, uint64_t seed, uint64_t iteration, uint32_t half,
                        const double* draws, double* q_out, double* z_out, void* stream);
int rvm_stretch_accept(int32_t n_params, int32_t n_s0, int64_t s0_begin, double* x, double* lnp, const double* q,
                       const double* lnp_new, const double* z, uint64_t seed, uint64_t iteration, uint32_t half,
                       const double* draws, int32_t* accepted, void* stream);

/* Mapping of a State's free-parameter vector onto the kernel's parameter rows (rvmcmc.engine.
 * ParamMap): row r (5 or 7 per planet, see Conventions) takes free parameter src[r], or the fixed
 * value base[r] when src[r] < 0 (state.py:26-31 ignore_vars / ignore_params). */
#define RVM_MAX_PARAM_ROWS (7 * RVM_MAX_PLANETS)
typedef struct rvm_param_map {
    int32_t n_rows;
    int32_t src[RVM_MAX_PARAM_ROWS];
    double base[RVM_MAX_PARAM_ROWS];
} rvm_param_map;

/* One whole stretch-move half-step in ONE likelihood launch: the proposal (as
 * rvm_stretch_propose, Philox draws), the walker log-likelihood of the proposals (as
 * rvm_logl_batch on map(q)), and the accept (as rvm_stretch_accept), bit-identical to the
 * three-call sequence.  x: [n_params][n_s0] free parameters (in place), lnp [n_s0] (in place),
 * c_aos: the complement WALKER-MAJOR, [n_s1][n_params] (each c_j one contiguous row: one cache line
 * per gathered walker instead of n_params), n_s0 <= the plan's max_walkers.  x_aos (nullable): a
 * walker-major mirror [n_s0][n_params] of x that accepted proposals are written to as well (the
 * next half-step's c_aos).  lnp_new_out / status_out (nullable): the proposals' logl and status;
 * accepted (nullable): int32 counters += 1. */
int rvm_stretch_half_step(const rvm_plan* plan, const rvm_param_map* map, int32_t n_params, int32_t n_s0,
                          int64_t s0_begin, double* x, double* x_aos, double* lnp, int32_t n_s1, const double* c_aos,
                          double a, uint64_t seed, uint64_t iteration, uint32_t half, double hill_factor,
                          double* lnp_new_out, int32_t* status_out, int32_t* accepted, void* stream);

/* One whole stretch-move ITERATION (both half-steps, mcmc.py:57-65 / emcee 2.2.1 sample()) in one
 * likelihood launch plus one small accept launch, bit-identical to two rvm_stretch_half_step calls.
 * The second half's proposal against partner j depends on j's first-half decision, so begin
 * evaluates it both ways (partner rejected: c0[j]; accepted: its proposal q0(j)) next to the first
 * half's own proposals -- 3 n_loc walker slots in one launch, which keeps a chip that one half-step
 * fills only partly busy (n_loc walkers of each half per rank; the plan needs max_walkers >= 3 n_loc).
 *
 * begin: half 0's proposals against c1, its logl and accepts (x0, lnp0 in place; accepted0 +=);
 *   half 1's proposals x1 against both variants of its partner in c0; logl of all 3 n_loc slots to
 *   lnp_spec / status_spec [3 n_loc] (slot n_loc + v n_loc + k: half 1's walker k, variant v);
 *   half 0's decisions to dec [n_loc] (1 accepted).  c0, c1: both halves walker-major
 *   [n_half][n_params] as at the start of the iteration, global order (on one rank: the walker-major
 *   mirrors); they must not be written before end has run.  s0_begin / s1_begin: global index of
 *   this rank's first walker of half 0 (its index within the half) and of half 1 (n_half + its
 *   index within half 1): the Philox keys.  lnp1 (nullable): half 1's log-probabilities [n_loc] as at the start of
 *   the iteration -- its accept inputs, which lets the adaptive resolution cut a refinement short
 *   on a certain reject (rvm_plan_faults `truncated`); NULL refines half 1's slots fully.
 * end: half 1's accepts with the variant dec_all[j] selects (dec_all: half 0's decisions in
 *   global order, [n_half]; on one rank dec itself); x1, lnp1 in place, x1_aos / x0_aos (nullable)
 *   mirrors updated; lnp_new_out / status_new_out (nullable): the chosen proposals' logl, status. */
int rvm_stretch_iteration_begin(const rvm_plan* plan, const rvm_param_map* map, int32_t n_params, int32_t n_loc,
                                int64_t s0_begin, int64_t s1_begin, double* x0, double* lnp0, const double* x1,
                                const double* lnp1, int32_t n_half, const double* c0, const double* c1, double a,
                                uint64_t seed, uint64_t iteration, double hill_factor, double* lnp_spec,
                                int32_t* status_spec, int32_t* dec, int32_t* accepted0, void* stream);
int rvm_stretch_iteration_end(int32_t n_params, int32_t n_loc, int64_t s0_begin, int64_t s1_begin, const double* x0,
                              double* x0_aos, const int32_t* dec, const int32_t* dec_all, double* x1, double* x1_aos,
                              double* lnp1, int32_t n_half, const double* c0, const double* c1,
                              const double* lnp_spec, const int32_t* status_spec, double a, uint64_t seed,
                              uint64_t iteration, int32_t* accepted1, double* lnp_new_out, int32_t* status_new_out,
                              void* stream);

/* Gaussian random-walk Metropolis-Hastings (mcmc.py:89-121), n_chains independent chains:
 * propose: q = x + step_size * scales[p] * N(0,1)        draws layout: [n_params][n_chains]
 * accept : exp(lnp_new - lnp_old) > u -> x <- q, lnp <- lnp_new   draws layout: [n_chains] */
int rvm_mh_propose(int32_t n_params, int32_t n_chains, int64_t chain_begin, const double* x, const double* scales,
                   double step_size, uint64_t seed, uint64_t iteration, const double* draws, double* q_out,
                   void* stream);
int rvm_mh_accept(int32_t n_params, int32_t n_chains, int64_t chain_begin, double* x, double* lnp, const double* q,
                  const double* lnp_new, uint64_t seed, uint64_t iteration, const double* draws, int32_t* accepted,
                  void* stream);
/* One whole MH step of n_chains chains (mcmc.py:107-121 for every chain) in ONE likelihood launch:
 * the proposal (as rvm_mh_propose, Philox draws), the walker log-likelihood of map(q) (as
 * rvm_logl_batch) and the accept (as rvm_mh_accept), bit-identical to the three-call sequence.
 * x [n_params][n_chains] and lnp [n_chains] in place; scales [n_params]; n_chains <= the plan's
 * max_walkers.  lnp_new_out / status_out (nullable): the proposals' logl and status; accepted
 * (nullable): int32 counters += 1.  Prior / encounter proposals are rejected through -inf. */
int rvm_mh_step(const rvm_plan* plan, const rvm_param_map* map, int32_t n_params, int32_t n_chains,
                int64_t chain_begin, double* x, double* lnp, const double* scales, double step_size, uint64_t seed,
                uint64_t iteration, double hill_factor, double* lnp_new_out, int32_t* status_out, int32_t* accepted,
                void* stream);

/* Central finite-difference stencil for SMALA's gradient/metric (x: [n_params][n_chains]).
 * out: SoA [n_params][(2P+1) * n_chains]; stencil point s of chain c is walker s*n_chains + c with
 * s = 0: x, s = 1+2p: x + eps_p e_p, s = 2+2p: x - eps_p e_p, eps_p = rel_step*max(|x_p|, floor[p]).
 * One rvm_logl_batch over (2P+1)*n_chains walkers then gives logp, its gradient and (rv_out) the
 * per-epoch RV Jacobian. */
int rvm_fd_params(int32_t n_params, int32_t n_chains, const double* x, double rel_step, const double* floor_,
                  double* out, void* stream);

/* ---- SMALA (mcmc.py:126-187) on device, one thread per chain ---------------------------------
 * Per-chain quantities a SMALA step needs at a point x; all device arrays, C = n_chains,
 * P = n_params (<= RVM_SMALA_MAX_PARAMS), matrices row-major per chain: element (i, j) of chain c
 * at [(i * P + j) * C + c]. */
typedef struct {
    double* lp;      /* [C]       logp(x)                                                          */
    double* grad;    /* [P][C]    central-difference gradient of logp                              */
    double* mu;      /* [P][C]    drift x + eps^2/2 G^-1 grad                  (mcmc.py:150)        */
    double* L;       /* [P*P][C]  Cholesky factor of G^-1, lower                (mcmc.py:149)        */
    double* G;       /* [P*P][C]  SoftAbs metric Q diag(lambda coth(alpha lambda)) Q^T of eig(-H)  */
    double* logdet;  /* [C]       log det G^-1                                                     */
    int32_t* ok;     /* [C]       1: clean stencil and positive-definite metric                    */
} rvm_smala_cache;

/* From one rvm_logl_batch launch over rvm_fd_params' stencil of x (same x, rel_step, floor_;
 * walkers s * C + c, with rv_out): the gradient from the stencil's logp, the Gauss-Newton Hessian
 * H = -(2/npoints) J^T diag(inv_sigma2) J from its per-epoch model RVs (rv_stencil
 * [n_obs][(2P+1) C], rows in the plan's input epoch order; inv_sigma2 [n_obs] in the same order),
 * the SoftAbs metric of -H (cyclic Jacobi eigen-solver), G^-1, its Cholesky factor and the drift.
 * Replaces state.py:253-294 (variational derivatives) + mcmc.py:135-150. */
int rvm_smala_derive(int32_t n_params, int32_t n_chains, int32_t n_obs, const double* x, double rel_step,
                     const double* floor_, const double* lp_stencil, const int32_t* status_stencil,
                     const double* rv_stencil, const double* inv_sigma2, double npoints_norm, double alpha,
                     double eps, const rvm_smala_cache* out, void* stream);
/* The same cache from exact derivatives (rvm_logl_derivs outputs: lp [C], status [C], grad [P][C],
 * hess [P*P][C]): the reference's Hessian (state.py:253-294) instead of the Gauss-Newton one.
 * Chains with status != 0 or non-finite derivatives get ok = 0.  mcmc.py:135-150. */
int rvm_smala_metric(int32_t n_params, int32_t n_chains, const double* x, const double* lp, const int32_t* status,
                     const double* grad, const double* hess, double alpha, double eps, const rvm_smala_cache* out,
                     void* stream);
/* x_prop = mu + eps chol(G^-1) z (x where the cache is not ok); z ~ N(0,1) from Philox keyed by
 * (seed, chain_begin + c, iteration, 5 | p << 8) or from draws [P][C].  mcmc.py:144-153. */
int rvm_smala_propose(int32_t n_params, int32_t n_chains, int64_t chain_begin, const double* x,
                      const rvm_smala_cache* cur, double eps, uint64_t seed, uint64_t iteration,
                      const double* draws, double* x_prop, void* stream);
/* exp(lp* - lp + log q(x | x*) - log q(x* | x)) > u  (u from Philox stream 6 or draws [C]), both
 * caches ok and lp* finite -> x <- x_prop, cur <- prop (per chain), accepted[c] += 1.
 * failures[c] += 1 (nullable) when the proposal's metric failed with a finite logp.
 * mcmc.py:158-187. */
int rvm_smala_accept(int32_t n_params, int32_t n_chains, int64_t chain_begin, double* x, const rvm_smala_cache* cur,
                     const double* x_prop, const rvm_smala_cache* prop, double eps, uint64_t seed,
                     uint64_t iteration, const double* draws, int32_t* accepted, int32_t* failures, void* stream);

/* Fused SMALA step, three launches instead of five (mcmc.py:167-187 for every chain):
 *   rvm_smala_propose                       x* (unchanged)
 *   rvm_smala_stencil_logl                  rvm_fd_params' stencil of x* formed inside ONE likelihood
 *                                           launch (walker s * n_chains + c, as rvm_fd_params; map:
 *                                           free parameters -> kernel rows, as rvm_stretch_half_step)
 *                                           -> logl / status [(2P+1) C], rv_out [n_obs][(2P+1) C]
 *   rvm_smala_derive_accept                 rvm_smala_derive of x* into prop, then rvm_smala_accept,
 *                                           in one kernel (one wave per chain)
 * bit-identical to rvm_fd_params + rvm_logl_batch + rvm_smala_derive + rvm_smala_accept.
 * rvm_smala_metric_accept is the exact-Hessian counterpart (rvm_smala_metric + rvm_smala_accept). */
int rvm_smala_stencil_logl(const rvm_plan* plan, const rvm_param_map* map, int32_t n_params, int32_t n_chains,
                           const double* x, double rel_step, const double* floor_, double hill_factor,
                           double* logl_out, int32_t* status_out, double* rv_out, void* stream);
int rvm_smala_derive_accept(int32_t n_params, int32_t n_chains, int64_t chain_begin, int32_t n_obs, double* x,
                            const double* x_prop, double rel_step, const double* floor_, const double* lp_stencil,
                            const int32_t* status_stencil, const double* rv_stencil, const double* inv_sigma2,
                            double npoints_norm, double alpha, double eps, const rvm_smala_cache* cur,
                            const rvm_smala_cache* prop, uint64_t seed, uint64_t iteration, const double* draws,
                            int32_t* accepted, int32_t* failures, void* stream);
/* The fused step with the centres' logp on a second (adaptive) plan, launched on another stream
 * (mcmc.py:167-187; the reference's logp is IAS15's):
 *   rvm_smala_derive_sides    rvm_smala_derive of x* without the stencil's centre row (its status and
 *                             logp are not read): gradient, Hessian, metric, drift, Cholesky into prop,
 *                             on the stencil's stream while the centres' launch still runs
 *   rvm_smala_center_accept   prop's logp from lp_center, prop ok only if status_center is 0, then
 *                             rvm_smala_accept, once the centres' launch is done
 * bit-identical to copying the centres' logp / status into the stencil's row 0 and calling
 * rvm_smala_derive_accept (the other cache entries do not depend on that row). */
int rvm_smala_derive_sides(int32_t n_params, int32_t n_chains, int32_t n_obs, const double* x, double rel_step,
                           const double* floor_, const double* lp_stencil, const int32_t* status_stencil,
                           const double* rv_stencil, const double* inv_sigma2, double npoints_norm, double alpha,
                           double eps, const rvm_smala_cache* out, void* stream);
int rvm_smala_center_accept(int32_t n_params, int32_t n_chains, int64_t chain_begin, double* x, const double* x_prop,
                            const double* lp_center, const int32_t* status_center, const rvm_smala_cache* cur,
                            const rvm_smala_cache* prop, double eps, uint64_t seed, uint64_t iteration,
                            const double* draws, int32_t* accepted, int32_t* failures, void* stream);
int rvm_smala_metric_accept(int32_t n_params, int32_t n_chains, int64_t chain_begin, double* x, const double* x_prop,
                            const double* lp, const int32_t* status, const double* grad, const double* hess,
                            double alpha, double eps, const rvm_smala_cache* cur, const rvm_smala_cache* prop,
                            uint64_t seed, uint64_t iteration, const double* draws, int32_t* accepted,
                            int32_t* failures, void* stream);

/* ---- exact derivatives (state.py:218-294) ----------------------------------------------------
 * logp, its gradient and its Hessian for n_chains parameter vectors (params: kernel rows
 * [5|7 * n_planets][n_chains], as rvm_logl_batch), differentiated along n_dirs kernel rows
 * dir_rows[0..n_dirs) (host array; the free parameters of the State, in its order):
 *   logl_out [n_chains]            -chi2/npoints_norm (or -INF with status != 0)
 *   grad_out [n_dirs][n_chains]    d logp / d p_i
 *   hess_out [n_dirs*n_dirs][n_chains]  d2 logp / d p_i d p_j, row-major per chain (symmetric)
 *   status_out [n_chains]          as rvm_logl_batch; gradient and Hessian are NaN unless 0
 * The reference integrates REBOUND's order-1 and order-2 variational equations (one variation per
 * parameter, one per pair); here every parameter pair (i >= j) is one hyper-dual integration of the
 * plan's own discrete integrator (same steps, levels and Richardson weights as rvm_logl_batch),
 * so the results are the exact derivatives of that likelihood.  workspace: device buffer of
 * rvm_logl_derivs_workspace_bytes(n_chains, n_dirs) bytes (no allocation inside).  No limit from
 * the plan's max_walkers. */
size_t rvm_logl_derivs_workspace_bytes(int32_t n_chains, int32_t n_dirs);
int rvm_logl_derivs(const rvm_plan* plan, int32_t n_chains, const double* params, int32_t n_dirs,
                    const int32_t* dir_rows, double hill_factor, double* logl_out, double* grad_out, double* hess_out,
                    int32_t* status_out, void* workspace, void* stream);

const char* rvm_last_error(void);
int rvm_abi_version(void);

#ifdef __cplusplus
}
#endif

#endif /* RVMCMC_H */

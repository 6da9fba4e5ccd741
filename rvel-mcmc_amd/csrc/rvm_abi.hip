// rvm_abi.hip -- the extern "C" surface of librvmcmc.so (declared in include/rvmcmc.h).
//
// Host-side work here is limited to building the epoch schedule once per observation set
// (rvm_plan_create) and to argument checking; every per-step entry point only enqueues kernels on
// the caller's stream.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rvm_internal.h"

// the eager first halving pass for small plain launches (rvm_refine.hip), unless RVM_EAGER says otherwise
#ifndef RVM_EAGER_DEFAULT
#define RVM_EAGER_DEFAULT true
#endif
// eager halving passes run beside the likelihood kernel: pass 1 only (pass 2 as well, RVM_EAGER_PASSES=2,
// measured slower: config 4 at 0.90 -> 1.07 ms per step -- the side stream's next launch queues behind
// the longer eager kernel)
#ifndef RVM_EAGER_PASSES_DEFAULT
#define RVM_EAGER_PASSES_DEFAULT 1
#endif

namespace rvm {
hipError_t launch_logl(const DevPlan& P, int W, const double* params, double hill_factor, unsigned long long* slots,
                       double* logl, int32_t* status, double* rv_out, const StretchArgs& sa, hipStream_t stream);
hipError_t launch_refine(const DevPlan& P, int W, const double* params, double hill_factor, double* logl,
                         int32_t* status, double* rv_out, const StretchArgs& sa, int eager, hipStream_t stream);
hipError_t launch_eager(const DevPlan& P, int W, const double* params, double hill_factor, hipStream_t stream);
hipError_t launch_gen_bump(const DevPlan& P, hipStream_t stream);
hipError_t prepare_logl(const DevPlan& P);
hipError_t prepare_refine(const DevPlan& P);
hipError_t launch_stretch_propose(int P, int n0, int64_t s0b, const double* x, int n1, const double* c, double a,
                                  uint64_t seed, uint64_t it, uint32_t half, const double* draws, double* q,
                                  double* z, hipStream_t st);
hipError_t launch_stretch_accept(int P, int n0, int64_t s0b, double* x, double* lnp, const double* q,
                                 const double* lnp_new, const double* z, uint64_t seed, uint64_t it, uint32_t half,
                                 const double* draws, int32_t* acc, hipStream_t st);
hipError_t launch_mh_propose(int P, int n, int64_t b, const double* x, const double* scales, double step,
                             uint64_t seed, uint64_t it, const double* draws, double* q, hipStream_t st);
hipError_t launch_mh_accept(int P, int n, int64_t b, double* x, double* lnp, const double* q, const double* lnp_new,
                            uint64_t seed, uint64_t it, const double* draws, int32_t* acc, hipStream_t st);
hipError_t launch_stretch_iteration_end(const IterEndArgs& g, hipStream_t st);
hipError_t launch_fd_params(int P, int n, const double* x, double rel, const double* fl, double* out, hipStream_t st);
hipError_t launch_smala_derive(int P, int C, int E, const double* x, double rel, const double* fl,
                               const double* lp_st, const int32_t* st_st, const double* rv, const double* w,
                               double npoints, double alpha, double eps, const SmalaCache& out, int sides,
                               hipStream_t st);
hipError_t launch_smala_center_accept(int P, int C, int64_t begin, double* x, const SmalaCache& cur, const double* xs,
                                      const SmalaCache& prop, const double* lpc, const int32_t* stc, double eps,
                                      uint64_t seed, uint64_t it, const double* draws, int32_t* accepted,
                                      int32_t* failures, hipStream_t st);
hipError_t launch_smala_metric(int P, int C, const double* x, const double* lp, const int32_t* status,
                               const double* grad, const double* hess, double alpha, double eps, const SmalaCache& out,
                               hipStream_t st);
hipError_t launch_smala_propose(int P, int C, int64_t begin, const double* x, const SmalaCache& cur, double eps,
                                uint64_t seed, uint64_t it, const double* draws, double* xs, hipStream_t st);
hipError_t launch_smala_accept(int P, int C, int64_t begin, double* x, const SmalaCache& cur, const double* xs,
                               const SmalaCache& prop, double eps, uint64_t seed, uint64_t it, const double* draws,
                               int32_t* accepted, int32_t* failures, hipStream_t st);
hipError_t launch_smala_derive_accept(int P, int C, int E, const double* xs, double rel, const double* fl,
                                      const double* lp_st, const int32_t* st_st, const double* rv, const double* w,
                                      double npoints, double alpha, double eps, const SmalaCache& prop,
                                      int64_t begin, double* x, const SmalaCache& cur, uint64_t seed, uint64_t it,
                                      const double* draws, int32_t* accepted, int32_t* failures, hipStream_t st);
hipError_t launch_smala_metric_accept(int P, int C, const double* xs, const double* lp, const int32_t* status,
                                      const double* grad, const double* hess, double alpha, double eps,
                                      const SmalaCache& prop, int64_t begin, double* x, const SmalaCache& cur,
                                      uint64_t seed, uint64_t it, const double* draws, int32_t* accepted,
                                      int32_t* failures, hipStream_t st);
hipError_t launch_derivs(const DevPlan& P, int C, const double* params, int n_dirs, const int32_t* dir_rows,
                         double hill_factor, double* ws, int32_t* wst, double* logl, double* grad, double* hess,
                         int32_t* status, hipStream_t stream);
}  // namespace rvm

struct rvm_plan {
    rvm::DevPlan dev;
    void* dmem = nullptr;        // one device allocation: schedule + workspace
    void* lvmem = nullptr;       // level-split layout workspace (DevPlan::lv_*), when usable
    size_t lv_bytes = 0;
    void* xmem = nullptr;        // the extension's stored levels (DevPlan::lvx), when the plan has one
    void* rqmem = nullptr;       // the refinement kernel's work lists (DevPlan::rq_*), adaptive plans
    unsigned long long* slots = nullptr;  // [max_walkers] direction meeting slots (rvm_logl.hip)
    int32_t max_walkers = 0;
    int32_t steps[2] = {0, 0};
    // rvm_plan_time_kernels: event triples around the likelihood and refinement kernels of the next
    // `cap` launches (the kernels' own durations on their stream, for the bench's roofline)
    mutable std::vector<hipEvent_t> tev;
    mutable int32_t tcap = 0, tn = 0;
    void* emem = nullptr;                // eager passes' results (DevPlan::rve, esum), small plans
    hipStream_t side = nullptr;          // their stream, forked from and joined to the caller's
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
};

// One likelihood evaluation as every entry point runs it: the likelihood kernel, then (adaptive
// plans) the refinement kernel for the walkers it handed on, stream-ordered.  Everything it enqueues
// is complete when the caller's stream is (the header's conventions): an eager launch forks the
// plan's side stream from the caller's and joins it back after the refinement kernel, which by then
// has stopped every eager block it did not wait for (rvm_refine.hip).  No host-side state changes
// per launch -- the launch generation lives on the device -- so a captured hipGraph replays it.
static hipError_t run_logl(const rvm_plan* plan, int W, const double* params, double hill_factor, double* logl,
                           int32_t* status, double* rv_out, const rvm::StretchArgs& sa, hipStream_t st) {
    const bool tm = plan->tn < plan->tcap;
    // eager halving passes (rvm_refine.hip): plain launches of 32..512 walkers, no RV curve wanted
    const bool mapped = sa.c != nullptr || sa.mh_scale != nullptr || sa.fd_x != nullptr;
    const int eager = plan->side != nullptr && !mapped && rv_out == nullptr && params != nullptr &&
                      W >= rvm::RVM_EAGER_MIN && W <= plan->dev.eager_max;
    hipError_t e = hipSuccess;
    if (eager) {
        e = hipEventRecord(plan->ev_fork, st);
        if (e == hipSuccess) e = hipStreamWaitEvent(plan->side, plan->ev_fork, 0);
        if (e == hipSuccess) e = rvm::launch_eager(plan->dev, W, params, hill_factor, plan->side);
        if (e != hipSuccess) {
            // (join whatever was enqueued on the side stream before reporting)
            if (hipEventRecord(plan->ev_join, plan->side) == hipSuccess) (void)hipStreamWaitEvent(st, plan->ev_join, 0);
            return e;
        }
    }
    if (tm) (void)hipEventRecord(plan->tev[3 * plan->tn], st);
    e = rvm::launch_logl(plan->dev, W, params, hill_factor, plan->slots, logl, status, rv_out, sa, st);
    if (tm) (void)hipEventRecord(plan->tev[3 * plan->tn + 1], st);
    // (the refinement kernel runs even after a failed likelihood launch: it resets the work lists)
    const hipError_t er = rvm::launch_refine(plan->dev, W, params, hill_factor, logl, status, rv_out, sa, eager, st);
    if (e == hipSuccess) e = er;
    if (tm) (void)hipEventRecord(plan->tev[3 * plan->tn + 2], st);
    if (tm) plan->tn++;
    if (eager) {
        hipError_t ej = hipEventRecord(plan->ev_join, plan->side);
        if (ej == hipSuccess) ej = hipStreamWaitEvent(st, plan->ev_join, 0);
        if (ej == hipSuccess) ej = rvm::launch_gen_bump(plan->dev, st);
        if (e == hipSuccess) e = ej;
    }
    return e;
}

static thread_local std::string g_err;

static int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

static int hip_fail(hipError_t e, const char* where) {
    return fail(-3, std::string(where) + ": " + hipGetErrorString(e));
}

extern "C" {

const char* rvm_last_error(void) { return g_err.c_str(); }
int rvm_abi_version(void) { return RVM_ABI_VERSION; }

int rvm_plan_create(const rvm_config* cfg, const double* t, const double* rv, const double* sigma, int32_t n_obs,
                    int32_t max_walkers, rvm_plan** out) {
    if (!cfg || !t || !rv || !sigma || !out) return fail(-1, "rvm_plan_create: null argument");
    if (cfg->n_planets < 1 || cfg->n_planets > RVM_MAX_PLANETS) return fail(-1, "rvm_plan_create: n_planets out of range");
    if (cfg->n_levels < 1 || cfg->n_levels > RVM_MAX_LEVELS) return fail(-1, "rvm_plan_create: n_levels out of range");
    if (!(cfg->dt > 0.0) || !std::isfinite(cfg->dt)) return fail(-1, "rvm_plan_create: dt must be > 0");
    if (n_obs < 0 || max_walkers < 1) return fail(-1, "rvm_plan_create: bad sizes");
    if (!(cfg->npoints_norm != 0.0)) return fail(-1, "rvm_plan_create: npoints_norm must be nonzero");
    int mult[RVM_MAX_LEVELS];
    bool harmonic = true;
    for (int k = 0; k < cfg->n_levels; k++) harmonic = harmonic && cfg->level_mult[k] == 0;
    int max_mult = 1;
    for (int k = 0; k < cfg->n_levels; k++) {
        mult[k] = harmonic ? k + 1 : cfg->level_mult[k];
        if (mult[k] < 1 || mult[k] > 64) return fail(-1, "rvm_plan_create: level_mult out of range (1..64)");
        for (int j = 0; j < k; j++)
            if (mult[j] == mult[k]) return fail(-1, "rvm_plan_create: level_mult entries must be distinct");
        max_mult = mult[k] > max_mult ? mult[k] : max_mult;
    }
    if (!(cfg->period_hint >= 0.0) || !std::isfinite(cfg->period_hint))
        return fail(-1, "rvm_plan_create: period_hint must be >= 0");
    if (std::isnan(cfg->resolve_tol) || cfg->resolve_max < 0 || cfg->resolve_max > RVM_RESOLVE_MAX_LIMIT)
        return fail(-1, "rvm_plan_create: resolve_tol must be a number and resolve_max in 0..12");
    const int rmax = cfg->resolve_tol > 0.0 ? cfg->resolve_max : 0;
    for (int i = 0; i < n_obs; i++) {
        if (!std::isfinite(t[i]) || !std::isfinite(rv[i]) || !std::isfinite(sigma[i]))
            return fail(-1, "rvm_plan_create: non-finite observation");
    }

    // split epochs by direction, sort by |t| (stable), cut segments into ceil(len/dt) steps
    struct Dir {
        std::vector<int32_t> idx, seg_n;
        std::vector<double> seg_len, orv, os2;
    } dir[2];
    long long total_steps[2] = {0, 0};
    for (int dd = 0; dd < 2; dd++) {
        Dir& D = dir[dd];
        for (int i = 0; i < n_obs; i++)
            if ((dd == 0) == (t[i] >= 0.0)) D.idx.push_back(i);
        std::stable_sort(D.idx.begin(), D.idx.end(), [&](int a, int b) { return std::fabs(t[a]) < std::fabs(t[b]); });
        const double sign = dd == 0 ? 1.0 : -1.0;
        double tprev = 0.0;
        for (int i : D.idx) {
            const double at = std::fabs(t[i]);
            const double len = at - tprev;
            tprev = at;
            int n = len > 0.0 ? (int)std::ceil(len / cfg->dt - 1e-9) : 0;
            if (len > 0.0 && n < 1) n = 1;
            D.seg_n.push_back(n);
            D.seg_len.push_back(n > 0 ? sign * len / n : 0.0);  // base step; level step = this / mult
            D.orv.push_back(rv[i]);
            D.os2.push_back(sigma[i] * sigma[i]);
            total_steps[dd] += n;
        }
        if ((total_steps[dd] * (long long)max_mult) << rmax > (1LL << 30))
            return fail(-1, "rvm_plan_create: dt too small for the epoch span");
        if (D.idx.size() > (size_t)RVM_MAX_EPOCHS_PER_DIRECTION)
            return fail(-1, "rvm_plan_create: too many epochs in one direction (the schedule is staged in LDS)");
    }

    // device layout: per direction [seg_n | obs_idx] int32 and [seg_len | obs_rv | obs_s2] f64, + workspace
    const size_t nf = dir[0].idx.size(), nb = dir[1].idx.size();
    const size_t n_dbl = 3 * (nf + nb) + (size_t)max_walkers + RVM_N_COUNTERS;  // schedule f64 | slots | counters (u64)
    const size_t n_int = 2 * (nf + nb);
    const size_t bytes = n_dbl * sizeof(double) + n_int * sizeof(int32_t) + 64;
    rvm_plan* plan = new rvm_plan();
    hipError_t e = hipMalloc(&plan->dmem, bytes);
    if (e != hipSuccess) {
        delete plan;
        return hip_fail(e, "rvm_plan_create: hipMalloc");
    }
    std::vector<unsigned char> host(bytes, 0);
    double* hd = reinterpret_cast<double*>(host.data());
    int32_t* hi = reinterpret_cast<int32_t*>(host.data() + n_dbl * sizeof(double));
    double* dd_base = reinterpret_cast<double*>(plan->dmem);
    int32_t* di_base = reinterpret_cast<int32_t*>(reinterpret_cast<unsigned char*>(plan->dmem) + n_dbl * sizeof(double));
    size_t od = 0, oi = 0;
    rvm::DirSched* S[2] = {&plan->dev.fwd, &plan->dev.bwd};
    for (int dd = 0; dd < 2; dd++) {
        const Dir& D = dir[dd];
        const size_t n = D.idx.size();
        S[dd]->n_epochs = (int32_t)n;
        S[dd]->n_steps = (int32_t)total_steps[dd];
        // head / tail split points (rvm_logl.hip level-split roles): level 0 at the share f0 of the
        // steps that balances SIMD loads m2 + f0 m0 = m3 + (1 - f0) m0, level 1 at one half
        {
            const int nlv = cfg->n_levels;
            double f0 = 0.5;
            // (+0.11: the tail's SIMD runs level 3 alone until the head ends, at the lone-wave rate;
            // measured at 6144 slots, scripts/probe/prof_clock.py with RVM_LS_F0: 0.625 -> SIMD 0/1
            // end 6 % after SIMD 2/3, 0.74 -> within 1 %)
            if (nlv == 4) f0 = (double)(mult[3] + mult[0] - mult[2]) / (2.0 * mult[0]) + 0.11;
#ifdef RVM_PROFILE
            if (const char* ef = getenv("RVM_LS_F0")) f0 = atof(ef);  // (timing build only: scripts/probe)
#endif
            f0 = std::min(1.0, std::max(0.0, f0));
            const double fr[2] = {f0, 0.5};
            int32_t sp[2] = {0, 0}, pr[2] = {0, 0};
            for (int q = 0; q < 2; q++) {
                const double target = fr[q] * (double)total_steps[dd];
                long long cum = 0, best_cum = 0;
                int best = 0;
                double best_d = target;  // split at 0
                for (size_t i = 0; i < n; i++) {
                    cum += D.seg_n[i];
                    const double dist = std::fabs((double)cum - target);
                    if (dist < best_d) {
                        best_d = dist;
                        best = (int)i + 1;
                        best_cum = cum;
                    }
                }
                sp[q] = best;
                pr[q] = (int32_t)best_cum;
            }
            S[dd]->split0 = sp[0];
            S[dd]->pre0 = pr[0];
            S[dd]->split1 = sp[1];
            S[dd]->pre1 = pr[1];
        }
        std::memcpy(hd + od, D.seg_len.data(), n * sizeof(double));
        S[dd]->seg_h1 = dd_base + od;
        od += n;
        std::memcpy(hd + od, D.orv.data(), n * sizeof(double));
        S[dd]->obs_rv = dd_base + od;
        od += n;
        std::memcpy(hd + od, D.os2.data(), n * sizeof(double));
        S[dd]->obs_s2 = dd_base + od;
        od += n;
        std::memcpy(hi + oi, D.seg_n.data(), n * sizeof(int32_t));
        S[dd]->seg_n = di_base + oi;
        oi += n;
        std::memcpy(hi + oi, D.idx.data(), n * sizeof(int32_t));
        S[dd]->obs_idx = di_base + oi;
        oi += n;
        plan->steps[dd] = (int32_t)total_steps[dd];
    }
    plan->slots = reinterpret_cast<unsigned long long*>(dd_base + od);
    for (int32_t i = 0; i < max_walkers; i++)  // empty between launches (the kernel restores this)
        reinterpret_cast<unsigned long long*>(hd + od)[i] = 0x7FF4DEADBEEF0001ULL;
    plan->dev.counters = reinterpret_cast<unsigned long long*>(dd_base + od + max_walkers);  // (zeroed)
    plan->max_walkers = max_walkers;
    e = hipMemcpy(plan->dmem, host.data(), bytes, hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(plan->dmem);
        delete plan;
        return hip_fail(e, "rvm_plan_create: hipMemcpy");
    }

    rvm::DevPlan& P = plan->dev;
    P.n_planets = cfg->n_planets;
    P.n_levels = cfg->n_levels;
    P.npoints = cfg->npoints_norm;
    P.n_obs = n_obs;
    P.inclined = cfg->inclined ? 1 : 0;
    {
        int dev = 0, ncu = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
            ncu = 0;
        P.n_cu = ncu;
    }
    // Richardson weights for the h^2 expansion: level k steps dt/mult[k]; Lagrange at 0 in x = 1/mult^2
    for (int k = 0; k < RVM_MAX_LEVELS; k++) {
        P.mult[k] = k < cfg->n_levels ? mult[k] : 1;
        P.inv_mult[k] = 1.0 / P.mult[k];
        P.lw[k] = 0.0;
        P.nt[k] = 8;
        P.spec[k] = 0;
    }
    // adaptive resolution: the weights of levels 1 .. n-1 alone (the estimate drops the coarsest)
    for (int k = 0; k < RVM_MAX_LEVELS; k++) P.lw3[k] = 0.0;
    for (int k = 1; k < cfg->n_levels; k++) {
        const double xk = 1.0 / ((double)mult[k] * mult[k]);
        double wk = 1.0;
        for (int j = 1; j < cfg->n_levels; j++) {
            if (j == k) continue;
            const double xj = 1.0 / ((double)mult[j] * mult[j]);
            wk *= xj / (xj - xk);
        }
        P.lw3[k] = wk;
    }
    P.rtol_dir = cfg->resolve_tol > 0.0 && cfg->n_levels >= 2 ? 0.5 * cfg->resolve_tol : INFINITY;
    P.fin_level = 0;
    for (int k = 1; k < cfg->n_levels; k++)
        if (mult[k] > mult[P.fin_level]) P.fin_level = k;
    P.rmax = P.rtol_dir < INFINITY ? rmax : 0;
    P.cut = 1;
    P.spin_ticks = 200000000ull;  // 2 s of the 100 MHz real-time counter without progress
    for (int k = 0; k < cfg->n_levels; k++) {
        const double xk = 1.0 / ((double)mult[k] * mult[k]);
        double wk = 1.0;
        for (int j = 0; j < cfg->n_levels; j++) {
            if (j == k) continue;
            const double xj = 1.0 / ((double)mult[j] * mult[j]);
            wk *= xj / (xj - xk);
        }
        P.lw[k] = wk;
        // Stumpff series length (rvm_device.h stumpff_bound): nominal z = (2 pi h / P)^2 on a
        // circular orbit, x2 for the pericentre of e ~ 0.25 orbits; lanes beyond the bound take
        // the general evaluation, so this choice only affects speed.  Levels whose nominal z is
        // small enough that the first Halley step is accepted almost always (fine levels) run
        // their segments speculatively (rvm_logl.hip segment<>)
        if (cfg->period_hint > 0.0) {
            const double nh = 2.0 * M_PI * cfg->dt / (mult[k] * cfg->period_hint);
            const double zn = 2.0 * nh * nh;
            P.nt[k] = zn <= 0.1 ? 6 : (zn <= 0.3 ? 7 : 8);
            P.spec[k] = zn <= 0.04 ? 1 : 0;
        }
    }
    // the LDS-coupled layouts' ring (DevPlan::lc_ring): up to RVM_LC_RING epochs, within
    // RVM_LC_RING_BYTES per group, at least 2 (a level runs at most a ring ahead of its combiner)
    {
        const int wpb = cfg->n_planets == 1 ? 64 : (cfg->n_planets == 2 ? 32 : 16);
        const int emax = (int)std::max<size_t>(std::max(nf, nb), 1);
        const int fit = (int)(rvm::RVM_LC_RING_BYTES / ((size_t)(cfg->n_levels + 1) * wpb * sizeof(double)));
        P.lc_ring = std::max(2, std::min(std::min(rvm::RVM_LC_RING, emax), fit));
    }
    {
        const char* sv = getenv("RVM_SKIP_VARIANTS");
        P.skip_variants = sv && sv[0] == '0' ? 0 : 1;
    }
    // the halving passes' late vote (DevPlan::late_mult): levels of at least RVM_LATE_SPO (default 96)
    // steps per period_hint; RVM_LATE_SPO=0 turns it off (A/B)
    P.late_mult = 0;
    {
        const char* ls = getenv("RVM_LATE_SPO");
        const double spo = ls ? atof(ls) : 96.0;
        if (spo > 0.0 && cfg->period_hint > 0.0) P.late_mult = (int32_t)std::ceil(spo * cfg->dt / cfg->period_hint - 1e-9);
        if (P.late_mult < 1 && spo > 0.0 && cfg->period_hint > 0.0) P.late_mult = 1;
    }
    // level-split layout (rvm_logl.hip launch_logl): four strictly increasing levels and batches
    // big enough that the plan's largest launch would need two-group blocks
    P.lv_rv = nullptr;
    P.lv_enc = nullptr;
    P.lv_emax = 0;
    P.lv_stride = 0;
    {
        const int wpb = cfg->n_planets == 1 ? 64 : (cfg->n_planets == 2 ? 32 : 16);
        const int64_t groups = ((int64_t)max_walkers + wpb - 1) / wpb;
        bool inc = cfg->n_levels == 4;
        for (int k = 1; inc && k < 4; k++) inc = mult[k] > mult[k - 1];
#ifdef RVM_PROFILE
        // RVM_NO_LEVEL_SPLIT=1 forces the LDS-coupled layout (timing build only: scripts/probe)
        const char* nols = getenv("RVM_NO_LEVEL_SPLIT");
        if (nols && nols[0] == '1') inc = false;
#endif
        if (inc && P.n_cu > 0 && 2 * groups > P.n_cu) {
            const int64_t emax = (int64_t)(nf > nb ? nf : nb) > 0 ? (int64_t)(nf > nb ? nf : nb) : 1;
            const size_t b_rv = (size_t)(2 * emax * max_walkers) * sizeof(double);
            const size_t b_enc = (size_t)(2 * (int64_t)max_walkers) * sizeof(int32_t);
            if (hipMalloc(&plan->lvmem, b_rv + b_enc) != hipSuccess) {
                plan->lvmem = nullptr;
                (void)hipGetLastError();  // the fallback is not an error: clear the runtime's sticky status
            } else {
                unsigned char* base = reinterpret_cast<unsigned char*>(plan->lvmem);
                P.lv_rv = reinterpret_cast<double*>(base);
                P.lv_enc = reinterpret_cast<int32_t*>(base + b_rv);
                P.lv_emax = (int32_t)emax;
                P.lv_stride = max_walkers;
                plan->lv_bytes = b_rv + b_enc;
                // every slot empty (all-ones: the NaN sentinel / -1); the combiners restore this
                if (hipMemset(plan->lvmem, 0xFF, b_rv + b_enc) != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
                    (void)hipFree(plan->lvmem);
                    plan->lvmem = nullptr;
                    P.lv_rv = nullptr;
                    P.lv_enc = nullptr;
                    (void)hipGetLastError();
                }
            }
            // (no workspace: launches keep the LDS-coupled layout)
        }
    }
    // the extension level (rvm_logl.hip extend_pass): max(mult) + 1 steps per base step, its
    // Stumpff series as the finest level's, and room for every launch's main-pass levels
    P.ext_mult = 0;
    P.ext_nt = 8;
    P.inv_ext = 1.0;
    P.lvx = nullptr;
    P.rvp = nullptr;
    P.rvp2 = nullptr;
    // refinement teams (A/B knob RVM_REFINE_TEAMS: 0 or 1 runs the passes one after the other, 2 ..
    // RVM_TEAMS_MAX that many passes at once)
    int n_teams = rvm::RVM_TEAMS_DEFAULT;
    if (const char* tp = getenv("RVM_REFINE_TEAMS")) n_teams = std::max(1, std::min(atoi(tp), rvm::RVM_TEAMS_MAX));
    P.n_teams = n_teams;
    P.rve = nullptr;
    P.esum = nullptr;
    P.eflag = nullptr;
    P.eager_max = 0;
    P.eager_passes = 0;
    {
        const char* es = getenv("RVM_EAGER_SPLIT");  // (A/B knob: 0 keeps both directions in one block)
        P.eager_split = es && es[0] == '0' ? 0 : 1;
    }
    P.e2_guard = INFINITY;
    P.e2_cut = INFINITY;
    P.cut_guard_k = 0.0;
    P.lvx_emax = 0;
    P.lvx_stride = 0;
    P.ext_spec = 0;
    for (int k = 0; k <= RVM_MAX_LEVELS; k++) P.lw5[k] = 0.0;
    // (A/B knob RVM_NO_EXTENSION=1: no extension stage, flagged directions go straight to halving passes)
    const char* noext = getenv("RVM_NO_EXTENSION");
    if (P.rmax > 0 && cfg->n_levels >= 2 && cfg->n_levels < RVM_MAX_LEVELS && !(noext && noext[0] == '1')) {
        const int nl = cfg->n_levels;
        const size_t emax = std::max<size_t>(std::max(nf, nb), 1);
        const size_t bl = 2 * emax * (size_t)max_walkers * sizeof(double);  // partial sums
        const size_t bx = (1 + (size_t)n_teams) * bl;                       // + last RV (per team)
        // (a failed allocation is not an error: the plan refines by halving passes alone, ext_mult 0)
        if (bx <= RVM_EXT_MAX_BYTES && hipMalloc(&plan->xmem, bx) != hipSuccess) {
            plan->xmem = nullptr;
            (void)hipGetLastError();  // (clear the runtime's sticky status)
        }
        if (plan->xmem != nullptr) {
            int m5[RVM_MAX_LEVELS + 1];
            int fin = 0;
            for (int k = 0; k < nl; k++) {
                m5[k] = mult[k];
                if (mult[k] > mult[fin]) fin = k;
            }
            m5[nl] = mult[fin] + 1;
            auto lagrange = [&](int k0, int n, double* w) {  // Lagrange-at-zero weights of levels k0 .. n-1 of m5
                for (int k = k0; k < n; k++) {
                    const double xk = 1.0 / ((double)m5[k] * m5[k]);
                    double wk = 1.0;
                    for (int j = k0; j < n; j++) {
                        if (j == k) continue;
                        const double xj = 1.0 / ((double)m5[j] * m5[j]);
                        wk *= xj / (xj - xk);
                    }
                    w[k] = wk;
                }
            };
            lagrange(0, nl + 1, P.lw5);
            P.ext_mult = m5[nl];
            P.ext_nt = P.nt[fin];
            P.ext_spec = P.spec[fin];  // (a finer step than the finest level's: speculate where it does)
            P.inv_ext = 1.0 / m5[nl];
            // and as plan level slot nl (lw[nl] = 0): the concurrent extension wave of the
            // LDS-coupled layout integrates it like any level (rvm_logl.hip, cx)
            P.mult[nl] = P.ext_mult;
            P.nt[nl] = P.ext_nt;
            P.spec[nl] = P.ext_spec;
            P.inv_mult[nl] = P.inv_ext;
            P.lvx = reinterpret_cast<double*>(plan->xmem);
            P.rvp = reinterpret_cast<double*>(reinterpret_cast<unsigned char*>(plan->xmem) + bl);
            P.rvp2 = n_teams >= 2 ? reinterpret_cast<double*>(reinterpret_cast<unsigned char*>(plan->xmem) + 2 * bl)
                                  : nullptr;
            P.lvx_emax = (int32_t)emax;
            P.lvx_stride = max_walkers;
        }
    }
    // the refinement kernel's work lists (rvm_refine.hip): sizes [4] (zero), walkers [3][max_walkers],
    // settled directions' chi2 [2][max_walkers]
    P.rq_n = nullptr;
    P.rq_w = nullptr;
    P.rq_c = nullptr;
    P.rq_cap = 0;
    P.rq_x = nullptr;
    P.rq_xf = nullptr;
    P.rq_xgroups = 0;
    P.rq_t = nullptr;
    P.rq_tf = nullptr;
    P.gen_dev = nullptr;
    P.depth_w = nullptr;
    P.rq_mark = nullptr;
    if (P.rmax > 0) {
        // (+ the split exchange: flags and double-buffered values per both-direction group of up to 64
        // walkers and team; groups of 16 walkers at 3-4 planets; + team A's published state and flag)
        const int64_t xg = ((int64_t)max_walkers + 15) / 16 + 1;
        const size_t nt = (size_t)std::max(n_teams, 2);
        const size_t b_x = (size_t)xg * nt * 2 * 2 * 64 * sizeof(unsigned long long);
        const size_t b_xf = (size_t)xg * nt * 2 * sizeof(unsigned long long);
        const size_t b_t = (size_t)xg * (nt - 1) * 16 * 64 * sizeof(unsigned long long);
        const size_t b_tf = (size_t)xg * nt * sizeof(unsigned long long);  // (+ the group's done word)
        const size_t b_c = 2 * (size_t)max_walkers * sizeof(double);
        const size_t b_w = 3 * (size_t)max_walkers * sizeof(int32_t);
        const size_t b_m = ((size_t)max_walkers * sizeof(int32_t) + 63) & ~(size_t)63;  // rq_mark
        const size_t b_d = (rvm::RVM_DEPTH_WINDOW + 1) * sizeof(unsigned long long);    // depth_w
        const size_t b_all = b_x + b_xf + b_t + b_tf + b_c + b_w + 64 + b_m + b_d;  // (+ rq_n [4], the launch generation)
        if (hipMalloc(&plan->rqmem, b_all) != hipSuccess || hipMemset(plan->rqmem, 0, b_all) != hipSuccess ||
            hipDeviceSynchronize() != hipSuccess) {
            (void)hipGetLastError();
            rvm_plan_destroy(plan);
            return fail(-3, "rvm_plan_create: hipMalloc of the refinement work lists failed");
        }
        unsigned char* base = reinterpret_cast<unsigned char*>(plan->rqmem);
        P.rq_x = reinterpret_cast<unsigned long long*>(base);
        P.rq_xf = reinterpret_cast<unsigned long long*>(base + b_x);
        P.rq_t = reinterpret_cast<unsigned long long*>(base + b_x + b_xf);
        P.rq_tf = reinterpret_cast<unsigned long long*>(base + b_x + b_xf + b_t);
        P.rq_c = reinterpret_cast<double*>(base + b_x + b_xf + b_t + b_tf);
        P.rq_w = reinterpret_cast<int32_t*>(base + b_x + b_xf + b_t + b_tf + b_c);
        P.rq_n = reinterpret_cast<int32_t*>(base + b_x + b_xf + b_t + b_tf + b_c + b_w);
        P.gen_dev = reinterpret_cast<unsigned long long*>(base + b_x + b_xf + b_t + b_tf + b_c + b_w + 32);
        // (zeroed: generation 0, older than any launch)
        P.depth_w = reinterpret_cast<unsigned long long*>(base + b_x + b_xf + b_t + b_tf + b_c + b_w + 64 + b_m);
        P.rq_mark = reinterpret_cast<int32_t*>(base + b_x + b_xf + b_t + b_tf + b_c + b_w + 64);  // (zeroed)
        const unsigned long long gen1 = 1;  // (every flag word starts at generation 0)
        if (hipMemcpy(P.gen_dev, &gen1, sizeof(gen1), hipMemcpyHostToDevice) != hipSuccess) {
            (void)hipGetLastError();
            rvm_plan_destroy(plan);
            return fail(-3, "rvm_plan_create: initialising the launch generation failed");
        }
        P.rq_cap = max_walkers;
        P.rq_xgroups = (int32_t)xg;
        if (const char* sp = getenv("RVM_REFINE_SPLIT"))  // (A/B knob: 0 keeps both directions in one block)
            if (sp[0] == '0') P.rq_x = nullptr;
        if (n_teams < 2) P.rq_t = nullptr;
        if (const char* th = getenv("RVM_TEAMS_HINT"))  // (A/B knob: 0 always runs the plan's team count)
            if (th[0] == '0') P.depth_w = nullptr;
        P.n_teams = (int32_t)nt;
    }
    // eager halving passes for the plan's plain launches of RVM_EAGER_MIN..RVM_EAGER_MAX walkers
    // (SMALA's centres, batched State evaluations): results of passes 1 and 2, a side stream and two
    // events -- only for plans that can make such a launch (a one-walker scalar plan never does, and
    // its stream would only add to the hardware queues).  Any failure: no eager passes,
    // the refinement kernel integrates as usual.
    {
        const char* eg = getenv("RVM_EAGER");  // (A/B knob: 0 turns the eager pass off, 1 on)
        const bool eager_on = eg ? eg[0] == '1' : RVM_EAGER_DEFAULT;
        const int emw = std::min<int>(max_walkers, rvm::RVM_EAGER_MAX);
        if (P.rmax >= 2 && P.rvp != nullptr && P.gen_dev != nullptr && cfg->n_levels <= 4 && eager_on &&
            max_walkers >= rvm::RVM_EAGER_MIN) {
            // passes 1 and 2: RV [2][2][emax][stride], sums [2][2][3][stride]; flags [groups][8] (zeroed)
            const size_t plane = (size_t)P.lvx_emax * P.lvx_stride;
            const size_t nflag = rvm::RVM_EFLAG_WORDS * (size_t)((rvm::RVM_EAGER_MAX + 15) / 16) + 8;
            const size_t b = (4 * plane + 12 * (size_t)P.lvx_stride + nflag) * sizeof(double);
            if (hipMalloc(&plan->emem, b) == hipSuccess && hipMemset(plan->emem, 0, b) == hipSuccess &&
                hipDeviceSynchronize() == hipSuccess &&
                hipStreamCreateWithFlags(&plan->side, hipStreamNonBlocking) == hipSuccess &&
                hipEventCreateWithFlags(&plan->ev_fork, hipEventDisableTiming) == hipSuccess &&
                hipEventCreateWithFlags(&plan->ev_join, hipEventDisableTiming) == hipSuccess) {
                P.rve = reinterpret_cast<double*>(plan->emem);
                P.esum = P.rve + 4 * plane;
                P.eflag = reinterpret_cast<unsigned long long*>(P.esum + 12 * (size_t)P.lvx_stride);
                P.eager_max = emw;
                const char* ep = getenv("RVM_EAGER_PASSES");  // (A/B knob: 1 or 2)
                P.eager_passes = ep && ep[0] == '1' ? 1 : (ep && ep[0] == '2' ? 2 : RVM_EAGER_PASSES_DEFAULT);
            } else {
                (void)hipGetLastError();
                if (plan->ev_fork) (void)hipEventDestroy(plan->ev_fork);
                if (plan->side) (void)hipStreamDestroy(plan->side);
                if (plan->emem) (void)hipFree(plan->emem);
                plan->emem = nullptr;
                plan->side = nullptr;
                plan->ev_fork = plan->ev_join = nullptr;
            }
        }
    }
    // kernel attributes (dynamic LDS) set once here, so launches stay capturable; a schedule the
    // refinement kernel cannot stage is refused now rather than failing every launch
    {
        const hipError_t pe = rvm::prepare_logl(P);
        if (pe != hipSuccess) {
            rvm_plan_destroy(plan);
            return fail(-1, pe == hipErrorInvalidConfiguration
                                ? "rvm_plan_create: the epoch schedule does not fit the likelihood kernel's LDS "
                                  "(too many epochs in one direction)"
                                : "rvm_plan_create: n_planets has no kernel instantiation");
        }
    }
    if (rvm::prepare_refine(P) != hipSuccess) {
        rvm_plan_destroy(plan);
        return fail(-1, "rvm_plan_create: the epoch schedule does not fit the refinement kernel's LDS "
                        "(too many epochs in one direction for the adaptive resolution)");
    }
    *out = plan;
    return 0;
}

void rvm_plan_destroy(rvm_plan* plan) {
    if (!plan) return;
    if (plan->side) (void)hipStreamSynchronize(plan->side);
    if (plan->ev_fork) (void)hipEventDestroy(plan->ev_fork);
    if (plan->ev_join) (void)hipEventDestroy(plan->ev_join);
    if (plan->side) (void)hipStreamDestroy(plan->side);
    if (plan->emem) (void)hipFree(plan->emem);
    for (hipEvent_t ev : plan->tev) (void)hipEventDestroy(ev);
    if (plan->rqmem) (void)hipFree(plan->rqmem);
    if (plan->lvmem) (void)hipFree(plan->lvmem);
    if (plan->xmem) (void)hipFree(plan->xmem);
    if (plan->dmem) (void)hipFree(plan->dmem);
    delete plan;
}

int rvm_plan_set_certain_reject(rvm_plan* plan, int32_t on) {
    if (!plan) return fail(-1, "rvm_plan_set_certain_reject: null plan");
    plan->dev.cut = on ? 1 : 0;
    return 0;
}

int rvm_plan_set_verify_eccentricity(rvm_plan* plan, double e) {
    if (!plan) return fail(-1, "rvm_plan_set_verify_eccentricity: null plan");
    if (std::isnan(e) || e >= 1.0) return fail(-1, "rvm_plan_set_verify_eccentricity: e must be < 1 (<= 0: off)");
    plan->dev.e2_guard = e > 0.0 ? e * e : INFINITY;
    {
        const char* cf = getenv("RVM_CUT_FACTOR");  // (A/B knob: the guard's factor)
        const double ec = 1.0 - (1.0 - e) * (cf ? atof(cf) : rvm::RVM_CUT_ECC_FACTOR);
        const char* cg = getenv("RVM_CUT_GUARD");  // (A/B knob: 0 turns the cut guard off)
        plan->dev.e2_cut = e > 0.0 && !(cg && atoi(cg) == 0) ? ec * ec : INFINITY;
        const char* ck = getenv("RVM_CUT_GUARD_K");  // (A/B knob: past the guard, chi2 - min(k d, 100 est))
        plan->dev.cut_guard_k = ck ? atof(ck) : rvm::RVM_CUT_GUARD_K;
    }
    return 0;
}

int rvm_plan_extension(const rvm_plan* plan, int32_t* ext_mult) {
    if (!plan) return fail(-1, "rvm_plan_extension: null plan");
    if (ext_mult) *ext_mult = plan->dev.ext_mult;
    return 0;
}

int rvm_plan_counters(rvm_plan* plan, int32_t reset, int64_t* out, int32_t n, void* stream) {
    if (!plan) return fail(-1, "rvm_plan_counters: null plan");
    if (n < 0 || (n > 0 && !out)) return fail(-1, "rvm_plan_counters: bad output array");
    hipStream_t st = (hipStream_t)stream;
    unsigned long long h[RVM_N_COUNTERS] = {};
    hipError_t e = hipMemcpyAsync(h, plan->dev.counters, sizeof(h), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) return hip_fail(e, "rvm_plan_counters");
    for (int i = 0; i < n; i++) out[i] = i < RVM_N_COUNTERS ? (int64_t)h[i] : 0;
    if (reset) {
        // the hand-off slots back to their sentinels (late level-1 stores of a launch that gave up
        // have landed: the stream's earlier work is complete), then the counters
        if (plan->lvmem) e = hipMemsetAsync(plan->lvmem, 0xFF, plan->lv_bytes, st);
        if (e == hipSuccess) e = hipMemsetAsync(plan->dev.counters, 0, sizeof(h), st);
        if (e == hipSuccess) e = hipStreamSynchronize(st);
        if (e != hipSuccess) return hip_fail(e, "rvm_plan_counters: reset");
    }
    return 0;
}

int rvm_plan_faults(rvm_plan* plan, int32_t reset, int64_t* handoff_timeouts, int64_t* nonfinite,
                    int64_t* unresolved, int64_t* refined, int64_t* truncated, void* stream) {
    if (!plan) return fail(-1, "rvm_plan_faults: null plan");
    int64_t c[RVM_N_COUNTERS] = {};
    const int rc = rvm_plan_counters(plan, reset, c, RVM_N_COUNTERS, stream);
    if (rc != 0) return rc;
    if (handoff_timeouts) *handoff_timeouts = c[0];
    if (nonfinite) *nonfinite = c[1];
    if (unresolved) *unresolved = c[2];
    if (refined) *refined = c[3];
    if (truncated) *truncated = c[4];
    return 0;
}

int rvm_plan_time_kernels(rvm_plan* plan, int32_t max_launches) {
    if (!plan) return fail(-1, "rvm_plan_time_kernels: null plan");
    if (max_launches < 0 || max_launches > 4096) return fail(-1, "rvm_plan_time_kernels: max_launches out of range");
    while ((int32_t)plan->tev.size() < 3 * max_launches) {
        hipEvent_t ev;
        const hipError_t e = hipEventCreate(&ev);
        if (e != hipSuccess) return hip_fail(e, "rvm_plan_time_kernels: hipEventCreate");
        plan->tev.push_back(ev);
    }
    plan->tcap = max_launches;
    plan->tn = 0;
    return 0;
}

int rvm_plan_kernel_times(rvm_plan* plan, float* logl_ms, float* refine_ms, int32_t max, int32_t* n_out) {
    if (!plan || max < 0) return fail(-1, "rvm_plan_kernel_times: bad arguments");
    const int n = std::min(plan->tn, max);
    for (int i = 0; i < n; i++) {
        hipError_t e = hipEventSynchronize(plan->tev[3 * i + 2]);
        float a = 0.0f, b = 0.0f;
        if (e == hipSuccess) e = hipEventElapsedTime(&a, plan->tev[3 * i], plan->tev[3 * i + 1]);
        if (e == hipSuccess) e = hipEventElapsedTime(&b, plan->tev[3 * i + 1], plan->tev[3 * i + 2]);
        if (e != hipSuccess) return hip_fail(e, "rvm_plan_kernel_times");
        if (logl_ms) logl_ms[i] = a;
        if (refine_ms) refine_ms[i] = b;
    }
    if (n_out) *n_out = n;
    plan->tn = 0;
    plan->tcap = 0;
    return 0;
}

int rvm_plan_set_handoff_timeout(rvm_plan* plan, double seconds) {
    if (!plan) return fail(-1, "rvm_plan_set_handoff_timeout: null plan");
    if (!(seconds > 0.0) || !(seconds < 1e9)) return fail(-1, "rvm_plan_set_handoff_timeout: seconds out of range");
    const double ticks = seconds * 1e8;  // 100 MHz real-time counter
    plan->dev.spin_ticks = ticks < 1.0 ? 1ull : (unsigned long long)ticks;
    return 0;
}

int rvm_plan_info(const rvm_plan* plan, int32_t* sf, int32_t* sb, int32_t* ef, int32_t* eb) {
    if (!plan) return fail(-1, "rvm_plan_info: null plan");
    if (sf) *sf = plan->steps[0];
    if (sb) *sb = plan->steps[1];
    if (ef) *ef = plan->dev.fwd.n_epochs;
    if (eb) *eb = plan->dev.bwd.n_epochs;
    return 0;
}

int rvm_logl_batch(const rvm_plan* plan, int32_t n_walkers, const double* params, double hill_factor,
                   double* logl_out, int32_t* status_out, double* rv_out, void* stream) {
    if (!plan) return fail(-1, "rvm_logl_batch: null plan");
    if (n_walkers == 0) return 0;
    if (n_walkers < 0 || n_walkers > plan->max_walkers)
        return fail(-1, "rvm_logl_batch: n_walkers exceeds the plan's max_walkers");
    if (!params || !logl_out || !status_out) return fail(-1, "rvm_logl_batch: null buffer");
    if (!(hill_factor >= 0.0)) return fail(-1, "rvm_logl_batch: hill_factor must be >= 0");
    rvm::StretchArgs none{};
    hipError_t e = run_logl(plan, n_walkers, params, hill_factor, logl_out, status_out, rv_out, none, (hipStream_t)stream);
    if (e != hipSuccess) return hip_fail(e, "rvm_logl_batch");
    return 0;
}

int rvm_stretch_half_step(const rvm_plan* plan, const rvm_param_map* map, int32_t n_params, int32_t n_s0,
                          int64_t s0_begin, double* x, double* x_aos, double* lnp, int32_t n_s1, const double* c,
                          double a, uint64_t seed, uint64_t iteration, uint32_t half, double hill_factor,
                          double* lnp_new_out, int32_t* status_out, int32_t* accepted, void* stream) {
    if (!plan || !map) return fail(-1, "rvm_stretch_half_step: null plan or map");
    if (n_s0 == 0) return 0;
    if (n_s0 < 0 || n_s0 > plan->max_walkers)
        return fail(-1, "rvm_stretch_half_step: n_s0 exceeds the plan's max_walkers");
    if (n_params < 1 || n_s1 < 1 || !x || !lnp || !c) return fail(-1, "rvm_stretch_half_step: bad arguments");
    if (!(a > 1.0)) return fail(-1, "rvm_stretch_half_step: stretch scale a must be > 1");
    if (!(hill_factor >= 0.0)) return fail(-1, "rvm_stretch_half_step: hill_factor must be >= 0");
    const int rows = (plan->dev.inclined ? 7 : 5) * plan->dev.n_planets;
    if (map->n_rows != rows) return fail(-1, "rvm_stretch_half_step: map rows do not match the plan");
    rvm::StretchArgs sa{};
    sa.c = c;
    sa.x = x;
    sa.x_aos = x_aos;
    sa.lnp = lnp;
    sa.accepted = accepted;
    sa.s0_begin = s0_begin;
    sa.seed = seed;
    sa.iteration = iteration;
    sa.a = a;
    sa.n1 = n_s1;
    sa.dim = n_params;
    sa.half = half;
    sa.xstride = n_s0;
    for (int r = 0; r < RVM_MAX_PARAM_ROWS; r++) {
        const int k = r < rows ? map->src[r] : -1;
        if (k >= n_params) return fail(-1, "rvm_stretch_half_step: map source index out of range");
        sa.src[r] = k < 0 ? -1 : k;
        sa.base[r] = r < rows ? map->base[r] : 0.0;
    }
    hipError_t e = run_logl(plan, n_s0, nullptr, hill_factor, lnp_new_out, status_out, nullptr, sa, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_stretch_half_step");
}

int rvm_stretch_iteration_begin(const rvm_plan* plan, const rvm_param_map* map, int32_t n_params, int32_t n_loc,
                                int64_t s0_begin, int64_t s1_begin, double* x0, double* lnp0, const double* x1,
                                const double* lnp1, int32_t n_half, const double* c0, const double* c1, double a,
                                uint64_t seed, uint64_t iteration, double hill_factor, double* lnp_spec,
                                int32_t* status_spec, int32_t* dec, int32_t* accepted0, void* stream) {
    if (!plan || !map) return fail(-1, "rvm_stretch_iteration_begin: null plan or map");
    if (n_loc == 0) return 0;
    if (n_loc < 0 || (int64_t)3 * n_loc > plan->max_walkers)
        return fail(-1, "rvm_stretch_iteration_begin: 3 n_loc exceeds the plan's max_walkers");
    if (n_params < 1 || n_half < n_loc || !x0 || !lnp0 || !x1 || !c0 || !c1 || !lnp_spec || !status_spec || !dec)
        return fail(-1, "rvm_stretch_iteration_begin: bad arguments");
    if (s0_begin < 0 || s0_begin + n_loc > n_half || s1_begin < n_half || s1_begin + n_loc > 2 * (int64_t)n_half)
        return fail(-1, "rvm_stretch_iteration_begin: walker ranges outside the halves");
    if (!(a > 1.0)) return fail(-1, "rvm_stretch_iteration_begin: stretch scale a must be > 1");
    if (!(hill_factor >= 0.0)) return fail(-1, "rvm_stretch_iteration_begin: hill_factor must be >= 0");
    const int rows = (plan->dev.inclined ? 7 : 5) * plan->dev.n_planets;
    if (map->n_rows != rows) return fail(-1, "rvm_stretch_iteration_begin: map rows do not match the plan");
    rvm::StretchArgs sa{};
    sa.c = c1;
    sa.x = x0;
    sa.x_aos = nullptr;  // c0 must stay as it was until rvm_stretch_iteration_end
    sa.lnp = lnp0;
    sa.accepted = accepted0;
    sa.s0_begin = s0_begin;
    sa.seed = seed;
    sa.iteration = iteration;
    sa.a = a;
    sa.n1 = n_half;
    sa.dim = n_params;
    sa.half = 0;
    sa.xstride = n_loc;
    sa.n_spec = n_loc;
    sa.c0 = c0;
    sa.x1 = x1;
    sa.s1_begin = s1_begin;
    sa.dec = dec;
    sa.lnp1 = lnp1;
    for (int r = 0; r < RVM_MAX_PARAM_ROWS; r++) {
        const int k = r < rows ? map->src[r] : -1;
        if (k >= n_params) return fail(-1, "rvm_stretch_iteration_begin: map source index out of range");
        sa.src[r] = k < 0 ? -1 : k;
        sa.base[r] = r < rows ? map->base[r] : 0.0;
    }
    hipError_t e = run_logl(plan, 3 * n_loc, nullptr, hill_factor, lnp_spec, status_spec, nullptr, sa, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_stretch_iteration_begin");
}

int rvm_stretch_iteration_end(int32_t n_params, int32_t n_loc, int64_t s0_begin, int64_t s1_begin, const double* x0,
                              double* x0_aos, const int32_t* dec, const int32_t* dec_all, double* x1, double* x1_aos,
                              double* lnp1, int32_t n_half, const double* c0, const double* c1,
                              const double* lnp_spec, const int32_t* status_spec, double a, uint64_t seed,
                              uint64_t iteration, int32_t* accepted1, double* lnp_new_out, int32_t* status_new_out,
                              void* stream) {
    if (n_loc == 0) return 0;
    if (n_params < 1 || n_loc < 0 || n_half < n_loc || !x0 || !dec || !dec_all || !x1 || !lnp1 || !c0 || !c1 ||
        !lnp_spec || !status_spec)
        return fail(-1, "rvm_stretch_iteration_end: bad arguments");
    if (s0_begin < 0 || s0_begin + n_loc > n_half || s1_begin < n_half || s1_begin + n_loc > 2 * (int64_t)n_half)
        return fail(-1, "rvm_stretch_iteration_end: walker ranges outside the halves");
    if (!(a > 1.0)) return fail(-1, "rvm_stretch_iteration_end: stretch scale a must be > 1");
    rvm::IterEndArgs g{};
    g.dim = n_params;
    g.n = n_loc;
    g.n_half = n_half;
    g.s0_begin = s0_begin;
    g.s1_begin = s1_begin;
    g.x0 = x0;
    g.x0_aos = x0_aos;
    g.dec_local = dec;
    g.dec_all = dec_all;
    g.x1 = x1;
    g.x1_aos = x1_aos;
    g.lnp1 = lnp1;
    g.c0 = c0;
    g.c1 = c1;
    g.lnp_spec = lnp_spec;
    g.st_spec = status_spec;
    g.a = a;
    g.seed = seed;
    g.iteration = iteration;
    g.accepted1 = accepted1;
    g.lnp_new_out = lnp_new_out;
    g.status_new_out = status_new_out;
    hipError_t e = rvm::launch_stretch_iteration_end(g, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_stretch_iteration_end");
}

int rvm_stretch_propose(int32_t n_params, int32_t n_s0, int64_t s0_begin, const double* x, int32_t n_s1,
                        const double* c, double a, uint64_t seed, uint64_t iteration, uint32_t half,
                        const double* draws, double* q_out, double* z_out, void* stream) {
    if (n_s0 == 0) return 0;
    if (n_params < 1 || n_s0 < 0 || n_s1 < 1 || !x || !c || !q_out || !z_out)
        return fail(-1, "rvm_stretch_propose: bad arguments");
    if (!(a > 1.0)) return fail(-1, "rvm_stretch_propose: stretch scale a must be > 1");
    hipError_t e = rvm::launch_stretch_propose(n_params, n_s0, s0_begin, x, n_s1, c, a, seed, iteration, half, draws,
                                               q_out, z_out, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_stretch_propose");
}

int rvm_stretch_accept(int32_t n_params, int32_t n_s0, int64_t s0_begin, double* x, double* lnp, const double* q,
                       const double* lnp_new, const double* z, uint64_t seed, uint64_t iteration, uint32_t half,
                       const double* draws, int32_t* accepted, void* stream) {
    if (n_s0 == 0) return 0;
    if (n_params < 1 || n_s0 < 0 || !x || !lnp || !q || !lnp_new || !z)
        return fail(-1, "rvm_stretch_accept: bad arguments");
    hipError_t e = rvm::launch_stretch_accept(n_params, n_s0, s0_begin, x, lnp, q, lnp_new, z, seed, iteration, half,
                                              draws, accepted, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_stretch_accept");
}

int rvm_mh_propose(int32_t n_params, int32_t n_chains, int64_t chain_begin, const double* x, const double* scales,
                   double step_size, uint64_t seed, uint64_t iteration, const double* draws, double* q_out,
                   void* stream) {
    if (n_chains == 0) return 0;
    if (n_params < 1 || n_chains < 0 || !x || !scales || !q_out) return fail(-1, "rvm_mh_propose: bad arguments");
    hipError_t e = rvm::launch_mh_propose(n_params, n_chains, chain_begin, x, scales, step_size, seed, iteration, draws,
                                          q_out, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_mh_propose");
}

int rvm_mh_accept(int32_t n_params, int32_t n_chains, int64_t chain_begin, double* x, double* lnp, const double* q,
                  const double* lnp_new, uint64_t seed, uint64_t iteration, const double* draws, int32_t* accepted,
                  void* stream) {
    if (n_chains == 0) return 0;
    if (n_params < 1 || n_chains < 0 || !x || !lnp || !q || !lnp_new) return fail(-1, "rvm_mh_accept: bad arguments");
    hipError_t e = rvm::launch_mh_accept(n_params, n_chains, chain_begin, x, lnp, q, lnp_new, seed, iteration, draws,
                                         accepted, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_mh_accept");
}

int rvm_mh_step(const rvm_plan* plan, const rvm_param_map* map, int32_t n_params, int32_t n_chains,
                int64_t chain_begin, double* x, double* lnp, const double* scales, double step_size, uint64_t seed,
                uint64_t iteration, double hill_factor, double* lnp_new_out, int32_t* status_out, int32_t* accepted,
                void* stream) {
    if (!plan || !map) return fail(-1, "rvm_mh_step: null plan or map");
    if (n_chains == 0) return 0;
    if (n_chains < 0 || n_chains > plan->max_walkers)
        return fail(-1, "rvm_mh_step: n_chains exceeds the plan's max_walkers");
    if (n_params < 1 || !x || !lnp || !scales) return fail(-1, "rvm_mh_step: bad arguments");
    if (!(hill_factor >= 0.0)) return fail(-1, "rvm_mh_step: hill_factor must be >= 0");
    const int rows = (plan->dev.inclined ? 7 : 5) * plan->dev.n_planets;
    if (map->n_rows != rows) return fail(-1, "rvm_mh_step: map rows do not match the plan");
    rvm::StretchArgs sa{};
    sa.x = x;
    sa.lnp = lnp;
    sa.accepted = accepted;
    sa.s0_begin = chain_begin;
    sa.seed = seed;
    sa.iteration = iteration;
    sa.dim = n_params;
    sa.xstride = n_chains;
    sa.mh_scale = scales;
    sa.mh_step = step_size;
    for (int r = 0; r < RVM_MAX_PARAM_ROWS; r++) {
        const int k = r < rows ? map->src[r] : -1;
        if (k >= n_params) return fail(-1, "rvm_mh_step: map source index out of range");
        sa.src[r] = k < 0 ? -1 : k;
        sa.base[r] = r < rows ? map->base[r] : 0.0;
    }
    hipError_t e = run_logl(plan, n_chains, nullptr, hill_factor, lnp_new_out, status_out, nullptr, sa, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_mh_step");
}

int rvm_smala_stencil_logl(const rvm_plan* plan, const rvm_param_map* map, int32_t n_params, int32_t n_chains,
                           const double* x, double rel_step, const double* floor_, double hill_factor,
                           double* logl_out, int32_t* status_out, double* rv_out, void* stream) {
    if (!plan || !map) return fail(-1, "rvm_smala_stencil_logl: null plan or map");
    if (n_chains == 0) return 0;
    const int64_t W = (int64_t)(2 * n_params + 1) * n_chains;
    if (n_params < 1 || n_chains < 0 || !x || !floor_ || !logl_out || !status_out || !(rel_step > 0.0))
        return fail(-1, "rvm_smala_stencil_logl: bad arguments");
    if (W > plan->max_walkers) return fail(-1, "rvm_smala_stencil_logl: (2 n_params + 1) n_chains exceeds max_walkers");
    if (!(hill_factor >= 0.0)) return fail(-1, "rvm_smala_stencil_logl: hill_factor must be >= 0");
    const int rows = (plan->dev.inclined ? 7 : 5) * plan->dev.n_planets;
    if (map->n_rows != rows) return fail(-1, "rvm_smala_stencil_logl: map rows do not match the plan");
    rvm::StretchArgs sa{};
    sa.dim = n_params;
    sa.fd_x = x;
    sa.fd_floor = floor_;
    sa.fd_rel = rel_step;
    sa.fd_n = n_chains;
    for (int r = 0; r < RVM_MAX_PARAM_ROWS; r++) {
        const int k = r < rows ? map->src[r] : -1;
        if (k >= n_params) return fail(-1, "rvm_smala_stencil_logl: map source index out of range");
        sa.src[r] = k < 0 ? -1 : k;
        sa.base[r] = r < rows ? map->base[r] : 0.0;
    }
    hipError_t e = run_logl(plan, (int)W, nullptr, hill_factor, logl_out, status_out, rv_out, sa, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_smala_stencil_logl");
}

int rvm_fd_params(int32_t n_params, int32_t n_chains, const double* x, double rel_step, const double* floor_,
                  double* out, void* stream) {
    if (n_chains == 0) return 0;
    if (n_params < 1 || n_chains < 0 || !x || !floor_ || !out || !(rel_step > 0.0))
        return fail(-1, "rvm_fd_params: bad arguments");
    hipError_t e = rvm::launch_fd_params(n_params, n_chains, x, rel_step, floor_, out, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_fd_params");
}

size_t rvm_logl_derivs_workspace_bytes(int32_t n_chains, int32_t n_dirs) {
    if (n_chains < 0 || n_dirs < 0) return 0;
    const size_t items = (size_t)n_chains * (size_t)(n_dirs * (n_dirs + 1) / 2);
    return items * 2 * (4 * sizeof(double) + sizeof(int32_t));
}

int rvm_logl_derivs(const rvm_plan* plan, int32_t n_chains, const double* params, int32_t n_dirs,
                    const int32_t* dir_rows, double hill_factor, double* logl_out, double* grad_out, double* hess_out,
                    int32_t* status_out, void* workspace, void* stream) {
    if (!plan) return fail(-1, "rvm_logl_derivs: null plan");
    if (n_chains == 0) return 0;
    const int rows = (plan->dev.inclined ? 7 : 5) * plan->dev.n_planets;
    if (n_chains < 0 || n_dirs < 1 || n_dirs > rows || !dir_rows || !params || !grad_out || !hess_out || !workspace)
        return fail(-1, "rvm_logl_derivs: bad arguments");
    if ((size_t)n_chains * (size_t)(n_dirs * (n_dirs + 1) / 2) > (size_t)(1 << 30))
        return fail(-1, "rvm_logl_derivs: too many chains x parameter pairs");
    if (!(hill_factor >= 0.0)) return fail(-1, "rvm_logl_derivs: hill_factor must be >= 0");
    for (int k = 0; k < n_dirs; k++) {
        if (dir_rows[k] < 0 || dir_rows[k] >= rows) return fail(-1, "rvm_logl_derivs: dir_rows entry out of range");
        for (int q = 0; q < k; q++)
            if (dir_rows[q] == dir_rows[k]) return fail(-1, "rvm_logl_derivs: dir_rows entries must be distinct");
    }
    const size_t items = (size_t)n_chains * (size_t)(n_dirs * (n_dirs + 1) / 2);
    double* ws = reinterpret_cast<double*>(workspace);
    int32_t* wst = reinterpret_cast<int32_t*>(ws + 2 * 4 * items);
    hipError_t e = rvm::launch_derivs(plan->dev, n_chains, params, n_dirs, dir_rows, hill_factor, ws, wst, logl_out,
                                      grad_out, hess_out, status_out, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_logl_derivs");
}

static bool smala_cache_ok(const rvm_smala_cache* c) {
    return c && c->lp && c->grad && c->mu && c->L && c->G && c->logdet && c->ok;
}

static rvm::SmalaCache smala_cache(const rvm_smala_cache* c) {
    return rvm::SmalaCache{c->lp, c->grad, c->mu, c->L, c->G, c->logdet, c->ok};
}

int rvm_smala_derive(int32_t n_params, int32_t n_chains, int32_t n_obs, const double* x, double rel_step,
                     const double* floor_, const double* lp_stencil, const int32_t* status_stencil,
                     const double* rv_stencil, const double* inv_sigma2, double npoints_norm, double alpha,
                     double eps, const rvm_smala_cache* out, void* stream) {
    if (n_chains == 0) return 0;
    if (n_params < 1 || n_params > RVM_SMALA_MAX_PARAMS || n_chains < 0 || n_obs < 0 || !x || !floor_ ||
        !lp_stencil || !status_stencil || (n_obs > 0 && (!rv_stencil || !inv_sigma2)) || !smala_cache_ok(out) ||
        !(rel_step > 0.0) || !(npoints_norm != 0.0) || !(alpha > 0.0))
        return fail(-1, "rvm_smala_derive: bad arguments");
    hipError_t e = rvm::launch_smala_derive(n_params, n_chains, n_obs, x, rel_step, floor_, lp_stencil,
                                            status_stencil, rv_stencil, inv_sigma2, npoints_norm, alpha, eps,
                                            smala_cache(out), 0, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_smala_derive");
}

int rvm_smala_derive_sides(int32_t n_params, int32_t n_chains, int32_t n_obs, const double* x, double rel_step,
                           const double* floor_, const double* lp_stencil, const int32_t* status_stencil,
                           const double* rv_stencil, const double* inv_sigma2, double npoints_norm, double alpha,
                           double eps, const rvm_smala_cache* out, void* stream) {
    if (n_chains == 0) return 0;
    if (n_params < 1 || n_params > RVM_SMALA_MAX_PARAMS || n_chains < 0 || n_obs < 0 || !x || !floor_ ||
        !lp_stencil || !status_stencil || (n_obs > 0 && (!rv_stencil || !inv_sigma2)) || !smala_cache_ok(out) ||
        !(rel_step > 0.0) || !(npoints_norm != 0.0) || !(alpha > 0.0))
        return fail(-1, "rvm_smala_derive_sides: bad arguments");
    hipError_t e = rvm::launch_smala_derive(n_params, n_chains, n_obs, x, rel_step, floor_, lp_stencil,
                                            status_stencil, rv_stencil, inv_sigma2, npoints_norm, alpha, eps,
                                            smala_cache(out), 1, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_smala_derive_sides");
}

int rvm_smala_center_accept(int32_t n_params, int32_t n_chains, int64_t chain_begin, double* x, const double* x_prop,
                            const double* lp_center, const int32_t* status_center, const rvm_smala_cache* cur,
                            const rvm_smala_cache* prop, double eps, uint64_t seed, uint64_t iteration,
                            const double* draws, int32_t* accepted, int32_t* failures, void* stream) {
    if (n_chains == 0) return 0;
    if (n_params < 1 || n_params > RVM_SMALA_MAX_PARAMS || n_chains < 0 || !x || !x_prop || !lp_center ||
        !status_center || !smala_cache_ok(cur) || !smala_cache_ok(prop))
        return fail(-1, "rvm_smala_center_accept: bad arguments");
    hipError_t e = rvm::launch_smala_center_accept(n_params, n_chains, chain_begin, x, smala_cache(cur), x_prop,
                                                   smala_cache(prop), lp_center, status_center, eps, seed, iteration,
                                                   draws, accepted, failures, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_smala_center_accept");
}

int rvm_smala_metric(int32_t n_params, int32_t n_chains, const double* x, const double* lp, const int32_t* status,
                     const double* grad, const double* hess, double alpha, double eps, const rvm_smala_cache* out,
                     void* stream) {
    if (n_chains == 0) return 0;
    if (n_params < 1 || n_params > RVM_SMALA_MAX_PARAMS || n_chains < 0 || !x || !lp || !status || !grad || !hess ||
        !smala_cache_ok(out) || !(alpha > 0.0))
        return fail(-1, "rvm_smala_metric: bad arguments");
    hipError_t e = rvm::launch_smala_metric(n_params, n_chains, x, lp, status, grad, hess, alpha, eps, smala_cache(out),
                                            (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_smala_metric");
}

int rvm_smala_derive_accept(int32_t n_params, int32_t n_chains, int64_t chain_begin, int32_t n_obs, double* x,
                            const double* x_prop, double rel_step, const double* floor_, const double* lp_stencil,
                            const int32_t* status_stencil, const double* rv_stencil, const double* inv_sigma2,
                            double npoints_norm, double alpha, double eps, const rvm_smala_cache* cur,
                            const rvm_smala_cache* prop, uint64_t seed, uint64_t iteration, const double* draws,
                            int32_t* accepted, int32_t* failures, void* stream) {
    if (n_chains == 0) return 0;
    if (n_params < 1 || n_params > RVM_SMALA_MAX_PARAMS || n_chains < 0 || n_obs < 0 || !x || !x_prop || !floor_ ||
        !lp_stencil || !status_stencil || (n_obs > 0 && (!rv_stencil || !inv_sigma2)) || !smala_cache_ok(cur) ||
        !smala_cache_ok(prop) || !(rel_step > 0.0) || !(npoints_norm != 0.0) || !(alpha > 0.0))
        return fail(-1, "rvm_smala_derive_accept: bad arguments");
    hipError_t e = rvm::launch_smala_derive_accept(n_params, n_chains, n_obs, x_prop, rel_step, floor_, lp_stencil,
                                                   status_stencil, rv_stencil, inv_sigma2, npoints_norm, alpha, eps,
                                                   smala_cache(prop), chain_begin, x, smala_cache(cur), seed,
                                                   iteration, draws, accepted, failures, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_smala_derive_accept");
}

int rvm_smala_metric_accept(int32_t n_params, int32_t n_chains, int64_t chain_begin, double* x, const double* x_prop,
                            const double* lp, const int32_t* status, const double* grad, const double* hess,
                            double alpha, double eps, const rvm_smala_cache* cur, const rvm_smala_cache* prop,
                            uint64_t seed, uint64_t iteration, const double* draws, int32_t* accepted,
                            int32_t* failures, void* stream) {
    if (n_chains == 0) return 0;
    if (n_params < 1 || n_params > RVM_SMALA_MAX_PARAMS || n_chains < 0 || !x || !x_prop || !lp || !status || !grad ||
        !hess || !smala_cache_ok(cur) || !smala_cache_ok(prop) || !(alpha > 0.0))
        return fail(-1, "rvm_smala_metric_accept: bad arguments");
    hipError_t e = rvm::launch_smala_metric_accept(n_params, n_chains, x_prop, lp, status, grad, hess, alpha, eps,
                                                   smala_cache(prop), chain_begin, x, smala_cache(cur), seed,
                                                   iteration, draws, accepted, failures, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_smala_metric_accept");
}

int rvm_smala_propose(int32_t n_params, int32_t n_chains, int64_t chain_begin, const double* x,
                      const rvm_smala_cache* cur, double eps, uint64_t seed, uint64_t iteration,
                      const double* draws, double* x_prop, void* stream) {
    if (n_chains == 0) return 0;
    if (n_params < 1 || n_params > RVM_SMALA_MAX_PARAMS || n_chains < 0 || !x || !x_prop || !smala_cache_ok(cur))
        return fail(-1, "rvm_smala_propose: bad arguments");
    hipError_t e = rvm::launch_smala_propose(n_params, n_chains, chain_begin, x, smala_cache(cur), eps, seed, iteration,
                                             draws, x_prop, (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_smala_propose");
}

int rvm_smala_accept(int32_t n_params, int32_t n_chains, int64_t chain_begin, double* x, const rvm_smala_cache* cur,
                     const double* x_prop, const rvm_smala_cache* prop, double eps, uint64_t seed,
                     uint64_t iteration, const double* draws, int32_t* accepted, int32_t* failures, void* stream) {
    if (n_chains == 0) return 0;
    if (n_params < 1 || n_params > RVM_SMALA_MAX_PARAMS || n_chains < 0 || !x || !x_prop || !smala_cache_ok(cur) ||
        !smala_cache_ok(prop))
        return fail(-1, "rvm_smala_accept: bad arguments");
    hipError_t e = rvm::launch_smala_accept(n_params, n_chains, chain_begin, x, smala_cache(cur), x_prop,
                                            smala_cache(prop), eps, seed, iteration, draws, accepted, failures,
                                            (hipStream_t)stream);
    return e == hipSuccess ? 0 : hip_fail(e, "rvm_smala_accept");
}

}  // extern "C"

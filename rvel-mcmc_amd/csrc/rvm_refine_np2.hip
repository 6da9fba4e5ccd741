// rvm_refine_np2.hip -- the refinement and eager kernels for 2-planet plans (rvm_refine_impl.h);
// one translation unit per planet count so that the build compiles them in parallel
#include "rvm_refine_impl.h"

namespace rvm {

hipError_t launch_refine_np2(const DevPlan& P, int W, const double* params, double hill_factor, double* logl,
                              int32_t* status, double* rv_out, const StretchArgs& sa, int eager, hipStream_t stream) {
    return P.inclined ? launch_refine_t<2, true>(P, W, params, hill_factor, logl, status, rv_out, sa, eager, stream)
                      : launch_refine_t<2, false>(P, W, params, hill_factor, logl, status, rv_out, sa, eager, stream);
}

hipError_t launch_eager_np2(const DevPlan& P, int W, const double* params, double hill_factor, hipStream_t stream) {
    return P.inclined ? launch_eager_t<2, true>(P, W, params, hill_factor, stream)
                      : launch_eager_t<2, false>(P, W, params, hill_factor, stream);
}

hipError_t prepare_refine_np2(const DevPlan& P) {
    return P.inclined ? prepare_refine_t<2, true>(P) : prepare_refine_t<2, false>(P);
}

}  // namespace rvm

// (timing build: the 2-planet refinement kernel's per-wave records, scripts/probe/refine_prof.py)
#ifdef RVM_PROFILE
extern "C" int rvm_rprof_copy(void* host, size_t bytes) {
    const size_t n = bytes < sizeof(rvm::rvm_rprof) ? bytes : sizeof(rvm::rvm_rprof);
    return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(rvm::rvm_rprof), n, 0, hipMemcpyDeviceToHost);
}
extern "C" int rvm_rprof_clear(void) {
    static unsigned long long zero[RVM_RPROF_MAX_WAVES * RVM_RPROF_SLOTS];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(rvm::rvm_rprof), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
#endif

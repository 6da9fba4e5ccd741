// rvm_refine_np3.hip -- the refinement and eager kernels for 3-planet plans (rvm_refine_impl.h);
// one translation unit per planet count so that the build compiles them in parallel
#include "rvm_refine_impl.h"

namespace rvm {

hipError_t launch_refine_np3(const DevPlan& P, int W, const double* params, double hill_factor, double* logl,
                              int32_t* status, double* rv_out, const StretchArgs& sa, int eager, hipStream_t stream) {
    return P.inclined ? launch_refine_t<3, true>(P, W, params, hill_factor, logl, status, rv_out, sa, eager, stream)
                      : launch_refine_t<3, false>(P, W, params, hill_factor, logl, status, rv_out, sa, eager, stream);
}

hipError_t launch_eager_np3(const DevPlan& P, int W, const double* params, double hill_factor, hipStream_t stream) {
    return P.inclined ? launch_eager_t<3, true>(P, W, params, hill_factor, stream)
                      : launch_eager_t<3, false>(P, W, params, hill_factor, stream);
}

hipError_t prepare_refine_np3(const DevPlan& P) {
    return P.inclined ? prepare_refine_t<3, true>(P) : prepare_refine_t<3, false>(P);
}

}  // namespace rvm

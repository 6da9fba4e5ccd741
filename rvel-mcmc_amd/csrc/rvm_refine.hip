// rvm_refine.hip -- dispatch of the refinement and eager kernels (rvm_refine_impl.h; instantiated per
// planet count in rvm_refine_np<N>.hip) and the launch-generation bump.
#include "rvm_refine_impl.h"

namespace rvm {

// After an eager launch (run_logl, once the side stream has joined): the next launch generation
// (the refinement kernel advances it itself when no eager blocks share its generation)
__global__ void gen_bump_kernel(unsigned long long* gen_dev) {
    if (threadIdx.x == 0) __hip_atomic_fetch_add(gen_dev, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

hipError_t launch_gen_bump(const DevPlan& P, hipStream_t stream) {
    gen_bump_kernel<<<dim3(1), dim3(64), 0, stream>>>(P.gen_dev);
    return hipGetLastError();
}

hipError_t launch_eager(const DevPlan& P, int W, const double* params, double hill_factor, hipStream_t stream) {
    switch (P.n_planets) {
        case 1:
            return launch_eager_np1(P, W, params, hill_factor, stream);
        case 2:
            return launch_eager_np2(P, W, params, hill_factor, stream);
        case 3:
            return launch_eager_np3(P, W, params, hill_factor, stream);
        case 4:
            return launch_eager_np4(P, W, params, hill_factor, stream);
        default:
            return hipErrorInvalidValue;
    }
}

hipError_t launch_refine(const DevPlan& P, int W, const double* params, double hill_factor, double* logl,
                         int32_t* status, double* rv_out, const StretchArgs& sa, int eager, hipStream_t stream) {
    if (P.rmax <= 0 || P.rq_n == nullptr) return hipSuccess;
    switch (P.n_planets) {
        case 1:
            return launch_refine_np1(P, W, params, hill_factor, logl, status, rv_out, sa, eager, stream);
        case 2:
            return launch_refine_np2(P, W, params, hill_factor, logl, status, rv_out, sa, eager, stream);
        case 3:
            return launch_refine_np3(P, W, params, hill_factor, logl, status, rv_out, sa, eager, stream);
        case 4:
            return launch_refine_np4(P, W, params, hill_factor, logl, status, rv_out, sa, eager, stream);
        default:
            return hipErrorInvalidValue;
    }
}

// rvm_plan_create: set the refinement kernel's LDS attribute for the plan's instantiation and check
// that the plan's schedule fits it (hipErrorInvalidConfiguration otherwise)
hipError_t prepare_refine(const DevPlan& P) {
    if (P.rmax <= 0 || P.rq_n == nullptr) return hipSuccess;
    switch (P.n_planets) {
        case 1:
            return prepare_refine_np1(P);
        case 2:
            return prepare_refine_np2(P);
        case 3:
            return prepare_refine_np3(P);
        case 4:
            return prepare_refine_np4(P);
        default:
            return hipErrorInvalidValue;
    }
}

}  // namespace rvm

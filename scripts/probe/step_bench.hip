// Cycles per Wisdom-Holman step of the 2-planet lane state on one wave (gfx950), by component:
// kick2 + drift<NT>, drift only, kick only.  State: the S2 benchmark system (tests/conftest.py)
// at the finest Richardson level's step (P_min/96) unless argv[1] gives steps per orbit.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 step_bench.hip -o step_bench && ./step_bench [spo]
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>

#include "../../rvel-mcmc_amd/csrc/rvm_device.h"
using namespace rvm;

#define NSTEP 2000

template <int NT, int MODE>
__global__ void step_bench(double h, long long* cyc, double* sink) {
    const int lane = threadIdx.x & 63;
    const int p = lane & 1;
    // S2: planet 1 {m 1.2e-3, a 0.88, h 0.218, k 0.015, l 0.3}, planet 2 {2.1e-3, 1.55, 0.16, 0.02, 2.2}
    const double m[2] = {1.2e-3, 2.1e-3}, a[2] = {0.88, 1.55}, hh[2] = {0.218, 0.16}, kk[2] = {0.015, 0.02},
                 ll[2] = {0.3 + 1e-3 * lane, 2.2};
    Lane<2> s;
    s.m[0] = m[0];
    s.m[1] = m[1];
    s.iMi[0] = 1.0;
    s.iMi[1] = 1.0 / (1.0 + m[0]);
    s.iMi[2] = 1.0 / (1.0 + m[0] + m[1]);
    s.mu[0] = m[0] * s.iMi[1];
    s.mu[1] = m[1] * s.iMi[2];
    s.p = p;
    s.GM = p ? 1.0 + m[0] + m[1] : 1.0 + m[0];
    s.dmin2 = 1e-6;
    double X, Y, VX, VY;
    pal_to_cart(1.0 + m[p], a[p], ll[p], kk[p], hh[p], X, Y, VX, VY);
    const double x1 = grp_get<2, 0>(X), y1 = grp_get<2, 0>(Y), vx1 = grp_get<2, 0>(VX), vy1 = grp_get<2, 0>(VY);
    s.rx = p ? X - m[0] * x1 * s.iMi[1] : X;
    s.ry = p ? Y - m[0] * y1 * s.iMi[1] : Y;
    s.vx = p ? VX - m[0] * vx1 * s.iMi[1] : VX;
    s.vy = p ? VY - m[0] * vy1 * s.iMi[1] : VY;
    s.r = sqrt(s.rx * s.rx + s.ry * s.ry);
    s.ir = 1.0 / s.r;
    s.encm = 0;
    lane_finish(s);
    __syncthreads();
    const long long t0 = clock64();
#pragma unroll 2
    for (int j = 0; j < NSTEP; j++) {
        if (MODE != 2) kick<2, 2>(s, h);
        if (MODE != 1) drift<NT>(s, h);
    }
    const long long t1 = clock64();
    sink[blockIdx.x * 64 + lane] = s.rx + s.vy + (s.encm ? 1.0 : 0.0);
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int NT, int MODE>
static void run(const char* name, double h, int blocks, long long* cyc, double* sink) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    step_bench<NT, MODE><<<blocks, 64>>>(h, cyc, sink);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    step_bench<NT, MODE><<<blocks, 64>>>(h, cyc, sink);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c[1024];
    hipMemcpy(c, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < blocks; i++) mx = c[i] > mx ? c[i] : mx;
    printf("%-22s blocks=%4d  %7.1f clk/step  %6.1f ns/step (wall)\n", name, blocks, mx / NSTEP, ms * 1e6 / NSTEP);
}

int main(int argc, char** argv) {
    long long* cyc;
    double* sink;
    hipMalloc(&cyc, 1024 * sizeof(long long));
    hipMalloc(&sink, 1024 * 64 * sizeof(double));
    for (int a = 1; a < (argc > 1 ? argc : 2); a++) {
        const double spo = argc > 1 ? atof(argv[a]) : 96.0;
        const double h = 2.0 * M_PI * sqrt(0.88 * 0.88 * 0.88 / (1.0 + 1.2e-3)) / spo;
        printf("steps per orbit %.0f, h = %.5f\n", spo, h);
        const int blocks = 256;
        run<6, 0>("kick+drift<6>", h, blocks, cyc, sink);
        run<7, 0>("kick+drift<7>", h, blocks, cyc, sink);
        run<8, 0>("kick+drift<8>", h, blocks, cyc, sink);
        run<6, 2>("drift<6>", h, blocks, cyc, sink);
        run<7, 2>("drift<7>", h, blocks, cyc, sink);
    }
    return 0;
}

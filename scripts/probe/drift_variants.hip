// Cycle cost of drift variants on one wave (gfx950): the product drift<NT> and experimental
// restructurings built from the same rvm_device.h pieces.  S2 inner/outer planets, step P/spo.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 drift_variants.hip -o drift_variants && ./drift_variants 56
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <math.h>

#include "../../rvel-mcmc_amd/csrc/rvm_device.h"
using namespace rvm;

#define NSTEP 2000

// V1: guess order 3 or 4 (GO), one Halley step, single early gate (no second-step stage)
template <int NT, int GO, int NP>
__device__ __forceinline__ void drift_v1(Lane<NP>& s, double dt) {
    const double GM = s.GM, r0 = s.r, ir0 = s.ir;
    const double v2 = fma(s.vx, s.vx, s.vy * s.vy);
    const double eta = fma(s.rx, s.vx, s.ry * s.vy);
    const double beta = fma(s.GM2, ir0, -v2);
    const double zeta = fma(-beta, r0, GM);
    const double u = dt * ir0, sg = eta * ir0, g = GM * ir0;
    const double hs = 0.5 * sg;
    const double T3 = fma(hs, sg, (beta - g) * (1.0 / 6.0));
    double x;
    if constexpr (GO >= 4) {
        const double T4 = sg * fma(-0.625 * sg, sg, fma(5.0 / 12.0, g, -0.375 * beta));
        x = u * fma(u, fma(u, fma(u, T4, T3), -hs), 1.0);
    } else {
        x = u * fma(u, fma(u, T3, -hs), 1.0);
    }
    double G0, G1, G2, G3, fp, fpp, Q, z, x3, f0;
    halley<NT>(x, beta, r0, eta, zeta, GM, dt, G0, G1, G2, G3, fp, fpp, Q, z, x3, vconsts_for<NT>().k2, vconsts_for<NT>().k3, f0);
    constexpr double B = stumpff_bound<NT>();
    const double X = x - Q;
    const bool hard = fabs(beta) * (u * u) > 0.5;
    const uint64_t bad = ballot(!(fabs(z) <= B)) | ballot(!halley_done(Q, z, x3)) | ballot(hard);
    if (__builtin_expect(bad != 0, 0)) {
        const bool ok = fabs(z) <= B && halley_done(Q, z, x3) && !hard;
        if (!ok) kepler_rare(r0, eta, zeta, beta, GM, dt, fabs(z) <= B ? X : x, hard, G0, G1, G2, G3, fp, fpp, Q);
    }
    const DriftOut o = drift_apply<false>(s, dt, beta, eta, zeta, G0, G1, G2, G3, fp, fpp, Q);
    s.rx = o.rx;
    s.ry = o.ry;
    s.vx = o.vx;
    s.vy = o.vy;
    s.r = o.r;
    s.ir = o.ir;
}

// V2: no gate at all (INCORRECT for rare lanes -- measures the gate's cost only)
template <int NT, int NP>
__device__ __forceinline__ void drift_v2(Lane<NP>& s, double dt) {
    const double GM = s.GM, r0 = s.r, ir0 = s.ir;
    const double v2 = fma(s.vx, s.vx, s.vy * s.vy);
    const double eta = fma(s.rx, s.vx, s.ry * s.vy);
    const double beta = fma(s.GM2, ir0, -v2);
    const double zeta = fma(-beta, r0, GM);
    const double u = dt * ir0, sg = eta * ir0, g = GM * ir0;
    const double hs = 0.5 * sg;
    const double T3 = fma(hs, sg, (beta - g) * (1.0 / 6.0));
    const double T4 = sg * fma(-0.625 * sg, sg, fma(5.0 / 12.0, g, -0.375 * beta));
    const double x = u * fma(u, fma(u, fma(u, T4, T3), -hs), 1.0);
    double G0, G1, G2, G3, fp, fpp, Q, z, x3, f0;
    halley<NT>(x, beta, r0, eta, zeta, GM, dt, G0, G1, G2, G3, fp, fpp, Q, z, x3, vconsts_for<NT>().k2, vconsts_for<NT>().k3, f0);
    const DriftOut o = drift_apply<false>(s, dt, beta, eta, zeta, G0, G1, G2, G3, fp, fpp, Q);
    s.rx = o.rx;
    s.ry = o.ry;
    s.vx = o.vx;
    s.vy = o.vy;
    s.r = o.r;
    s.ir = o.ir;
}

template <int V, int NT>
__device__ __forceinline__ void do_drift(Lane<2>& s, double h) {
    if constexpr (V == 0) drift<NT>(s, h);
    if constexpr (V == 1) drift_v1<NT, 3>(s, h);
    if constexpr (V == 2) drift_v1<NT, 4>(s, h);
    if constexpr (V == 3) drift_v2<NT>(s, h);
}

template <int V, int NT, int MODE>
__global__ void bench(double h, long long* cyc, double* sink) {
    const int lane = threadIdx.x & 63;
    const int p = lane & 1;
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
        if (MODE == 0) kick<2, 2>(s, h);
        do_drift<V, NT>(s, h);
    }
    const long long t1 = clock64();
    sink[blockIdx.x * 64 + lane] = s.rx + s.vy + (s.encm ? 1.0 : 0.0);
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int V, int NT, int MODE>
static void run(const char* name, double h, long long* cyc, double* sink) {
    const int blocks = 256;
    bench<V, NT, MODE><<<blocks, 64>>>(h, cyc, sink);
    hipDeviceSynchronize();
    bench<V, NT, MODE><<<blocks, 64>>>(h, cyc, sink);
    hipDeviceSynchronize();
    long long c[256];
    hipMemcpy(c, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < blocks; i++) mx = c[i] > mx ? c[i] : mx;
    double r[64];
    hipMemcpy(r, sink, 64 * sizeof(double), hipMemcpyDeviceToHost);
    printf("%-34s %7.1f clk/step   (state %.15e)\n", name, mx / NSTEP, r[0]);
}

int main(int argc, char** argv) {
    long long* cyc;
    double* sink;
    hipMalloc(&cyc, 1024 * sizeof(long long));
    hipMalloc(&sink, 1024 * 64 * sizeof(double));
    for (int a = 1; a < (argc > 1 ? argc : 2); a++) {
        const double spo = argc > 1 ? atof(argv[a]) : 56.0;
        const double h = 2.0 * M_PI * sqrt(0.88 * 0.88 * 0.88 / (1.0 + 1.2e-3)) / spo;
        printf("steps per orbit %.0f\n", spo);
        run<0, 6, 0>("product drift<6> +kick", h, cyc, sink);
        run<1, 6, 0>("v1 guess3 single gate +kick", h, cyc, sink);
        run<2, 6, 0>("v1 guess4 single gate +kick", h, cyc, sink);
        run<3, 6, 0>("v2 no gate (incorrect) +kick", h, cyc, sink);
        run<0, 6, 1>("product drift<6>", h, cyc, sink);
        run<1, 6, 1>("v1 guess3 single gate", h, cyc, sink);
        run<2, 6, 1>("v1 guess4 single gate", h, cyc, sink);
        run<3, 6, 1>("v2 no gate (incorrect)", h, cyc, sink);
    }
    return 0;
}

// Why the gated drift's first Halley step fails on steady-state walkers (round 6 study): for 2-planet
// walkers read from a file (kernel rows m, a, h, k, l per planet; scripts/probe/kepler_accept_probe.py
// writes them from the steady-state slots), integrate NSTEP kick-drift-kick steps of size P1 / SPO
// (P1: the S2 inner period) with the gated drift the refinement passes run, and classify every drift's
// first Halley step before it is taken:
//   [0] drifts   [1] fail the cheap test (|z| > B or |q| > tol |x|)   [2] of those, fail the z-aware
//   test |q|^3 |z| <= 7.3e-17 |x|^3 (with |z| <= B)   [3] of those, |q| <= 1e-4 |x| (a Taylor second
//   step would do)   [4] wave-steps with any lane failing the cheap test   [5] ... failing the z-aware one
// Encountered lanes are counted as the kernel treats them (converged).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 kepler_accept_probe.hip -o kepler_accept_probe
//   ./kepler_accept_probe walkers.bin N SPO NSTEP
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#pragma clang fp contract(on)
#include "../../rvel-mcmc_amd/csrc/rvm_walker.h"
using namespace rvm;

__global__ __launch_bounds__(64) void probe(const double* rows, int n, double h, int nstep, unsigned long long* cnt,
                                            long long* cyc) {
    const int lane = threadIdx.x & 63;
    const int slot = lane >> 1, p = lane & 1;
    int w = blockIdx.x * 32 + slot;
    if (w >= n) w = n - 1;
    double rowv[10];
    for (int r = 0; r < 10; r++) rowv[r] = rows[(size_t)w * 10 + r];
    Lane<2> s;
    int status = RVM_STATUS_OK;
    double e2w;
    walker_setup<2, false, 2>(rowv, p, 1.0, s, status, e2w);
    KickPrep<2> kp = kick_prep<2, 2, false>(s, 1.875);
    lane_set_step(s, h);
    const VConsts vk = vconsts_for<6>();
    unsigned long long c[6] = {0, 0, 0, 0, 0, 0};
    kick_apply<2, true, false>(s, kp);
    const long long t0 = clock64();
    for (int j = 0; j < nstep; j++) {
        {  // the drift's first Halley step, as rvm_device.h drift computes it
            const double GM = s.GM, r0 = s.r, ir0 = s.ir;
            const double v2 = fma(s.vx, s.vx, s.vy * s.vy);
            const double eta = fma(s.rx, s.vx, s.ry * s.vy);
            const double beta = fma(s.GM2, ir0, -v2);
            const double zeta = fma(-beta, r0, GM);
            const double u = h * ir0, sg = eta * ir0, g = GM * ir0;
            const double hs = 0.5 * sg;
            const double T3 = fma(hs, sg, (beta - g) * (1.0 / 6.0));
            const double T4 = sg * fma(-0.625 * sg, sg, fma(5.0 / 12.0, g, -0.375 * beta));
            const double x = u * fma(u, fma(u, fma(u, T4, T3), -hs), 1.0);
            double G0, G1, G2, G3, fp, fpp, Q, z, x3, f0;
            halley<6>(x, beta, r0, eta, zeta, GM, h, G0, G1, G2, G3, fp, fpp, Q, z, x3, vk.k2, vk.k3, f0);
            const bool enc = lane_encountered(s);
            const bool zok = fabs(z) <= stumpff_bound<6>();
            const bool cheap = (zok && halley_ok<6>(Q, x)) || enc;
            const bool zaw = cheap || (zok && fabs((Q * Q) * (Q * z)) <= 7.3e-17 * fabs(x3));
            const bool tay = zaw || (zok && fabs(Q) <= 1e-4 * fabs(x));
            c[0] += 1;
            c[1] += cheap ? 0 : 1;
            c[2] += zaw ? 0 : 1;
            c[3] += (!zaw && tay) ? 1 : 0;
            c[4] += ballot(!cheap) ? 1 : 0;
            c[5] += ballot(!zaw) ? 1 : 0;
        }
        bool bad = false;
        drift<6, true, false, 2>(s, h, bad, vk);
        kp = kick_prep<2, 2, false>(s, vk.c1875);
        kick_apply<2, false, false>(s, kp);
    }
    const long long t1 = clock64();
    for (int k = 0; k < 4; k++) atomicAdd(cnt + k, c[k]);
    if (lane == 0) {
        atomicAdd(cnt + 4, c[4]);
        atomicAdd(cnt + 5, c[5]);
        cyc[blockIdx.x] = t1 - t0;
    }
    if (!isfinite(s.rx)) atomicAdd(cnt + 6, 1ull);
}

// timing: the plain segment loop (segments of NS steps, the refinement passes' rf = 1 finest level at
// ~2.3 base steps per segment) with the gated drift's second chance ACC, or ungated (ACC = -1)
template <int ACC, int KG = 0>
__global__ __launch_bounds__(64) void timing(const double* rows, int n, double h, int nseg, int ns, long long* cyc,
                                             double* sink) {
    const int lane = threadIdx.x & 63;
    const int slot = lane >> 1, p = lane & 1;
    int w = blockIdx.x * 32 + slot;
    if (w >= n) w = n - 1;
    double rowv[10];
    for (int r = 0; r < 10; r++) rowv[r] = rows[(size_t)w * 10 + r];
    Lane<2> s;
    int status = RVM_STATUS_OK;
    double e2w;
    walker_setup<2, false, 2>(rowv, p, 1.0, s, status, e2w);
    KickPrep<2> kp = kick_prep<2, 2, false>(s, 1.875);
    bool bad = false;
    __syncthreads();
    const long long t0 = clock64();
    for (int g = 0; g < nseg; g++) {
        if constexpr (ACC < 0)
            segment_steps<6, false, false, 2, 2, KG, 0>(s, kp, h, ns, bad);
        else
            segment_steps<6, true, false, 2, 2, KG, ACC>(s, kp, h, ns, bad);
    }
    const long long t1 = clock64();
    sink[blockIdx.x * 64 + lane] = s.rx + s.vy + s.ry + s.vx;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int ACC, int KG = 0>
static double run_timing(const double* rows, int n, double h, int nseg, int ns, long long* cyc, double* sink,
                         double* out_sink) {
    const int blocks = (n + 31) / 32;
    timing<ACC, KG><<<blocks, 64>>>(rows, n, h, nseg, ns, cyc, sink);
    hipDeviceSynchronize();
    long long* hc = (long long*)malloc(blocks * sizeof(long long));
    hipMemcpy(hc, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    hipMemcpy(out_sink, sink, (size_t)blocks * 64 * sizeof(double), hipMemcpyDeviceToHost);
    double mean = 0;
    for (int b = 0; b < blocks; b++) mean += hc[b];
    free(hc);
    return mean / blocks / ((double)nseg * ns);
}

int main(int argc, char** argv) {
    if (argc < 5) {
        fprintf(stderr, "usage: %s walkers.bin N SPO NSTEP\n", argv[0]);
        return 2;
    }
    const int n = atoi(argv[2]);
    const double spo = atof(argv[3]);
    const int nstep = atoi(argv[4]);
    double* hw = (double*)malloc((size_t)n * 10 * sizeof(double));
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(hw, sizeof(double), (size_t)n * 10, f) != (size_t)n * 10) {
        fprintf(stderr, "cannot read %s\n", argv[1]);
        return 2;
    }
    fclose(f);
    double *rows;
    unsigned long long* cnt;
    long long* cyc;
    const int blocks = (n + 31) / 32;
    hipMalloc(&rows, (size_t)n * 10 * sizeof(double));
    hipMalloc(&cnt, 8 * sizeof(unsigned long long));
    hipMalloc(&cyc, blocks * sizeof(long long));
    hipMemcpy(rows, hw, (size_t)n * 10 * sizeof(double), hipMemcpyHostToDevice);
    hipMemset(cnt, 0, 8 * sizeof(unsigned long long));
    const double P1 = 2.0 * M_PI * sqrt(0.88 * 0.88 * 0.88 / (1.0 + 1.2e-3));
    probe<<<blocks, 64>>>(rows, n, P1 / spo, nstep, cnt, cyc);
    if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "kernel failed\n");
        return 1;
    }
    unsigned long long c[8];
    hipMemcpy(c, cnt, sizeof(c), hipMemcpyDeviceToHost);
    long long* hc = (long long*)malloc(blocks * sizeof(long long));
    hipMemcpy(hc, cyc, blocks * sizeof(long long), hipMemcpyDeviceToHost);
    double mean = 0;
    for (int b = 0; b < blocks; b++) mean += hc[b];
    mean /= blocks;
    const double ws = (double)blocks * nstep;
    printf("{\"spo\": %.1f, \"walkers\": %d, \"steps\": %d, \"lane_fail_cheap\": %.5f, \"lane_fail_zaware\": %.5f, "
           "\"lane_taylor_ok_of_zaware_fail\": %.5f, \"wave_fail_cheap\": %.4f, \"wave_fail_zaware\": %.4f, "
           "\"cyc_per_step_probe\": %.1f, \"nonfinite_lanes\": %llu}\n",
           spo, n, nstep, (double)c[1] / c[0], (double)c[2] / c[0], c[2] ? (double)c[3] / c[2] : 0.0, c[4] / ws,
           c[5] / ws, mean / nstep, c[6]);
    // timing of the step variants on the same walkers (256 blocks at a time: one wave per CU)
    const int nt_walk = n < 256 * 32 ? n : 256 * 32;
    double* sink;
    hipMalloc(&sink, (size_t)blocks * 64 * sizeof(double));
    double* s0 = (double*)malloc((size_t)blocks * 64 * sizeof(double));
    double* s1 = (double*)malloc((size_t)blocks * 64 * sizeof(double));
    const int ns = 32, nseg = nstep / ns;
    const double h = P1 / spo;
    const double tu = run_timing<-1>(rows, nt_walk, h, nseg, ns, cyc, sink, s0);
    const double t0c = run_timing<0>(rows, nt_walk, h, nseg, ns, cyc, sink, s0);
    const double t1c = run_timing<1>(rows, nt_walk, h, nseg, ns, cyc, sink, s1);
    double d1 = 0;
    for (int i = 0; i < ((nt_walk + 31) / 32) * 64; i++) d1 = fmax(d1, fabs(s1[i] - s0[i]) / fmax(1e-300, fabs(s0[i])));
    const double t3c = run_timing<3>(rows, nt_walk, h, nseg, ns, cyc, sink, s1);
    int n3 = 0;
    for (int i = 0; i < ((nt_walk + 31) / 32) * 64; i++) n3 += !(s1[i] == s0[i]) && (s1[i] == s1[i] || s0[i] == s0[i]);
    const double t4c = run_timing<4>(rows, nt_walk, h, nseg, ns, cyc, sink, s1);
    const double g5u = run_timing<-1, 1>(rows, nt_walk, h, nseg, ns, cyc, sink, s1);
    const double g5g = run_timing<0, 1>(rows, nt_walk, h, nseg, ns, cyc, sink, s1);
    const double g5l = run_timing<3, 1>(rows, nt_walk, h, nseg, ns, cyc, sink, s1);
    printf("{\"spo\": %.1f, \"g5_cyc_per_step\": {\"ungated\": %.1f, \"acc0\": %.1f, \"late3\": %.1f}}\n", spo, g5u, g5g, g5l);
    printf("{\"spo\": %.1f, \"cyc_per_step\": {\"ungated\": %.1f, \"acc0\": %.1f, \"acc1\": %.1f, \"late3\": %.1f, "
           "\"late4\": %.1f}, \"lanes_acc3_differing_from_acc0\": %d}\n", spo, tu, t0c, t1c, t3c, t4c, n3);
    return 0;
}

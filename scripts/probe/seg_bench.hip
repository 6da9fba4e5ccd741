// Lone-wave cost of the segment loop the refinement passes run (rvm_walker.h segment_steps: the
// KDK step with the gated drift, as segment_gated) against the ungated (speculative) loop, on
// 2-planet walkers whose inner orbit has eccentricity E (S2's planets otherwise), one wave per block
// (32 walkers x 2 planet lanes, each walker's mean longitude offset), one block per CU: cycles per
// step (clock64 over NSEG segments of NS steps) at a step of P_inner / SPO.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 seg_bench.hip -o seg_bench && ./seg_bench E SPO ...
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#pragma clang fp contract(on)
#include "../../rvel-mcmc_amd/csrc/rvm_walker.h"
using namespace rvm;

#define NSEG 16
#define NS 140

template <int NT, bool GATED, int G5 = 0, int CAN = 0>
__global__ __launch_bounds__(64) void seg_bench(double ecc, double h, long long* cyc, double* sink, int* nbad,
                                                const unsigned long long* flag) {
    const int lane = threadIdx.x & 63;
    const int slot = lane >> 1, p = lane & 1;
    // S2 (mcmc_benchmark_mh.py:32) with planet 1's eccentricity set to ecc (h = ecc sin w, k = ecc cos w)
    const double w1 = 0.07 * slot;
    double rowv[10] = {1.2e-3, 0.88, ecc * sin(w1), ecc * cos(w1), 0.3 + 0.19 * slot,
                       2.1e-3, 1.55, 0.16, 0.02, 2.2 + 0.05 * slot};
    Lane<2> s;
    int status = RVM_STATUS_OK;
    double e2w;
    walker_setup<2, false, 2>(rowv, p, 1.0, s, status, e2w);
    s.dmin2 = 0.0;  // (no encounter exits: every lane integrates)
    s.idmin2 = INFINITY;
    KickPrep<2> kp = kick_prep<2, 2, false>(s, 1.875);
    bool bad = false;
    __syncthreads();
    const long long t0 = clock64();
    if constexpr (CAN) {  // (the cancellable gated segment: a flag that never reaches the tag)
        for (int g = 0; g < NSEG; g++)
            (void)segment_steps_c<NT, false, 2, 2, G5, CAN == 1 ? 16 : (CAN == 2 ? 32 : 64)>(s, kp, h, NS,
                                                                                          (const gu64*)flag, nullptr, 1ull);
    } else {
        for (int g = 0; g < NSEG; g++) segment_steps<NT, GATED, false, 2, 2, G5>(s, kp, h, NS, bad);
    }
    const long long t1 = clock64();
    sink[blockIdx.x * 64 + lane] = s.rx + s.vy;
    const uint64_t b = ballot(bad);
    if (lane == 0) {
        cyc[blockIdx.x] = t1 - t0;
        nbad[blockIdx.x] = __builtin_popcountll(b);
    }
}

template <int NT, bool GATED, int G5 = 0, int CAN = 0>
static void run(const char* name, double ecc, double h, long long* cyc, double* sink, int* nbad) {
    const int blocks = 256;
    static unsigned long long* flag = nullptr;
    if (!flag) {
        hipMalloc(&flag, sizeof(unsigned long long));
        hipMemset(flag, 0, sizeof(unsigned long long));
    }
    seg_bench<NT, GATED, G5, CAN><<<blocks, 64>>>(ecc, h, cyc, sink, nbad, flag);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    seg_bench<NT, GATED, G5, CAN><<<blocks, 64>>>(ecc, h, cyc, sink, nbad, flag);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    long long c[256];
    int nb[256];
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    hipMemcpy(nb, nbad, sizeof(nb), hipMemcpyDeviceToHost);
    double mx = 0, mean = 0;
    for (int i = 0; i < blocks; i++) {
        mx = c[i] > mx ? c[i] : mx;
        mean += c[i];
    }
    mean /= blocks;
    const double steps = (double)NSEG * NS;
    printf("%-20s e=%.2f  %7.1f clk/step (max %7.1f)  %6.1f ns/step wall  lanes ever bad %d\n", name, ecc, mean / steps,
           mx / steps, ms * 1e6 / steps, nb[0]);
}

int main(int argc, char** argv) {
    long long* cyc;
    double* sink;
    int* nbad;
    hipMalloc(&cyc, 256 * sizeof(long long));
    hipMalloc(&sink, 256 * 64 * sizeof(double));
    hipMalloc(&nbad, 256 * sizeof(int));
    const double P1 = 2.0 * M_PI * sqrt(0.88 * 0.88 * 0.88 / (1.0 + 1.2e-3));
    for (int a = 1; a + 1 < argc; a += 2) {
        const double ecc = atof(argv[a]), spo = atof(argv[a + 1]);
        const double h = P1 / spo;
        printf("-- e %.2f, steps per inner orbit %.0f\n", ecc, spo);
        run<6, true>("gated<6>", ecc, h, cyc, sink, nbad);
        run<6, true, 1>("gated<6> G5", ecc, h, cyc, sink, nbad);
        run<6, true, 0, 1>("gated<6> cancellable", ecc, h, cyc, sink, nbad);
        run<6, true, 0, 2>("gated<6> cancel 32", ecc, h, cyc, sink, nbad);
        run<6, true, 0, 3>("gated<6> cancel 64", ecc, h, cyc, sink, nbad);
        run<6, false>("ungated<6>", ecc, h, cyc, sink, nbad);
        run<7, true>("gated<7>", ecc, h, cyc, sink, nbad);
        run<7, true, 0, 1>("gated<7> cancellable", ecc, h, cyc, sink, nbad);
        run<8, true>("gated<8>", ecc, h, cyc, sink, nbad);
        run<8, true, 0, 1>("gated<8> cancellable", ecc, h, cyc, sink, nbad);
    }
    return 0;
}

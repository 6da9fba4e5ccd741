// Latency / issue-rate probe for the fp64 instruction mix of the WH step on gfx950.
// One workgroup of `waves` waves on one CU (waves land on different SIMDs first); each wave runs a
// timed loop of N iterations of a dependent chain (ILP 1) or k independent chains (ILP k), timed
// with clock64 (s_memtime) and with events (wall clock); one round = one op on every chain.
//   hipcc -O3 --offload-arch=gfx950 latency.hip -o latency && ./latency
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define N 4096

template <int ILP>
__global__ void fma_chain(double* out, double a, double b, long long* cyc) {
    double x[ILP];
#pragma unroll
    for (int k = 0; k < ILP; k++) x[k] = threadIdx.x * 1e-3 + k;
    long long t0 = clock64();
    for (int i = 0; i < N; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
#pragma unroll
            for (int k = 0; k < ILP; k++) x[k] = fma(x[k], a, b);
        }
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int k = 0; k < ILP; k++) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int ILP>
__global__ void rcp_chain(double* out, long long* cyc) {
    double x[ILP];
#pragma unroll
    for (int k = 0; k < ILP; k++) x[k] = 1.0 + threadIdx.x * 1e-3 + k;
    long long t0 = clock64();
    for (int i = 0; i < N; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) {
#pragma unroll
            for (int k = 0; k < ILP; k++) x[k] = __builtin_amdgcn_rcp(x[k]);
        }
    }
    long long t1 = clock64();
    double s = 0;
#pragma unroll
    for (int k = 0; k < ILP; k++) s += x[k];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

__global__ void dpp_chain(double* out, long long* cyc) {
    int x = threadIdx.x;
    long long t0 = clock64();
    for (int i = 0; i < N; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) x = __builtin_amdgcn_mov_dpp(x, 0x4E, 0xF, 0xF, false) + 1;
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

__global__ void mul_chain(double* out, double a, long long* cyc) {
    double x = threadIdx.x * 1e-3;
    long long t0 = clock64();
    for (int i = 0; i < N; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) x = x * a;
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

__global__ void f32_chain(double* out, float a, float b, long long* cyc) {
    float x = threadIdx.x * 1e-3f;
    long long t0 = clock64();
    for (int i = 0; i < N; i++) {
#pragma unroll
        for (int j = 0; j < 8; j++) x = fmaf(x, a, b);
    }
    long long t1 = clock64();
    out[blockIdx.x * blockDim.x + threadIdx.x] = x;
    if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

static void report(const char* name, long long* dcyc, int nw, float ms) {
    long long h[64];
    hipMemcpy(h, dcyc, nw * sizeof(long long), hipMemcpyDeviceToHost);
    double mx = 0;
    for (int i = 0; i < nw; i++) mx = h[i] > mx ? h[i] : mx;
    printf("%-28s waves/CU=%2d  clock64 cycles per round = %7.2f   wall %.3f ms -> %.2f ns/round\n", name, nw,
           mx / (N * 8.0), ms, ms * 1e6 / (N * 8.0));
}

int main() {
    double* out;
    long long* cyc;
    hipMalloc(&out, 1 << 20);
    hipMalloc(&cyc, 1 << 16);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    float ms;
    for (int w : {1, 4, 8}) {
        dim3 blk(64 * w);
#define RUN(NAME, ...)                                      \
    __VA_ARGS__;                                            \
    hipDeviceSynchronize();                                 \
    hipEventRecord(e0);                                     \
    __VA_ARGS__;                                            \
    hipEventRecord(e1);                                     \
    hipEventSynchronize(e1);                                \
    hipEventElapsedTime(&ms, e0, e1);                       \
    report(NAME, cyc, w, ms);
        RUN("fma f64 ILP1", fma_chain<1><<<1, blk>>>(out, 0.999, 1e-3, cyc));
        RUN("fma f64 ILP2 (per chain)", fma_chain<2><<<1, blk>>>(out, 0.999, 1e-3, cyc));
        RUN("fma f64 ILP4 (per chain)", fma_chain<4><<<1, blk>>>(out, 0.999, 1e-3, cyc));
        RUN("mul f64 ILP1", mul_chain<<<1, blk>>>(out, 0.999, cyc));
        RUN("fma f32 ILP1", f32_chain<<<1, blk>>>(out, 0.999f, 1e-3f, cyc));
        RUN("rcp f64 ILP1", rcp_chain<1><<<1, blk>>>(out, cyc));
        RUN("rcp f64 ILP4 (per chain)", rcp_chain<4><<<1, blk>>>(out, cyc));
        RUN("dpp+add i32 ILP1", dpp_chain<<<1, blk>>>(out, cyc));
    }
    return 0;
}

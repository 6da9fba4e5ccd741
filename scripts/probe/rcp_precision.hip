// probe: relative error of v_rcp_f64 / v_rsq_f64 and after one Newton step (diagnostic only)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
__global__ void k(const double* x, double* out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double a = x[i];
    double r = __builtin_amdgcn_rcp(a);
    double e = fma(-a, r, 1.0);
    double r1 = fma(r, e, r);
    double y = __builtin_amdgcn_rsq(a);
    double f = fma(-a * y, y, 1.0);
    double y1 = fma(0.5 * y, f, y);
    out[4 * i + 0] = r; out[4 * i + 1] = r1; out[4 * i + 2] = y; out[4 * i + 3] = y1;
}
int main() {
    const int n = 1 << 20;
    std::vector<double> x(n), o(4 * n);
    unsigned long long s = 88172645463325252ull;
    for (int i = 0; i < n; i++) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; x[i] = std::ldexp(1.0 + (s >> 11) * 0x1.0p-53, (int)(s % 40) - 20); }
    double *dx, *dout;
    hipMalloc(&dx, n * 8); hipMalloc(&dout, 4 * n * 8);
    hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
    k<<<(n + 255) / 256, 256>>>(dx, dout, n);
    hipMemcpy(o.data(), dout, 4 * n * 8, hipMemcpyDeviceToHost);
    double m[4] = {0, 0, 0, 0};
    for (int i = 0; i < n; i++) {
        long double rr = 1.0L / x[i], ry = 1.0L / sqrtl((long double)x[i]);
        double e0 = fabs((double)((o[4*i] - rr) / rr)), e1 = fabs((double)((o[4*i+1] - rr) / rr));
        double e2 = fabs((double)((o[4*i+2] - ry) / ry)), e3 = fabs((double)((o[4*i+3] - ry) / ry));
        m[0] = fmax(m[0], e0); m[1] = fmax(m[1], e1); m[2] = fmax(m[2], e2); m[3] = fmax(m[3], e3);
    }
    printf("max rel err: rcp %.3e  rcp+1NR %.3e  rsq %.3e  rsq+1NR %.3e  (ulp 1.1e-16)\n", m[0], m[1], m[2], m[3]);
    return 0;
}

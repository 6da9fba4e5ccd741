// ISA probe: one kick + one drift of the 2-planet lane state (count instructions per step)
#include "../../rvel-mcmc_amd/csrc/rvm_device.h"
using namespace rvm;
template <int NT>
__global__ void step_probe(double* buf, int n, double h) {
    Lane<2> s;
    const int i = threadIdx.x;
    s.rx = buf[i]; s.ry = buf[i + 64]; s.vx = buf[i + 128]; s.vy = buf[i + 192];
    s.r = buf[i + 256]; s.ir = buf[i + 320]; s.GM = buf[i + 384];
    s.m[0] = buf[448]; s.m[1] = buf[449]; s.iMi[0] = 1.0; s.iMi[1] = buf[450]; s.iMi[2] = buf[451];
    s.mu[0] = buf[452]; s.mu[1] = buf[453]; s.dmin2 = buf[454]; s.p = i & 1; s.encm = 0; lane_finish(s);
    for (int j = 0; j < n; j++) {
        asm volatile("; STEP_BEGIN" ::: "memory");
        kick<2, 2>(s, h);
        drift<NT>(s, h);
        asm volatile("; STEP_END" ::: "memory");
    }
    buf[i] = s.rx; buf[i + 64] = s.ry; buf[i + 128] = s.vx; buf[i + 192] = s.vy; buf[i + 256] = (double)(s.encm & 1);
}

template __global__ void step_probe<6>(double*, int, double);

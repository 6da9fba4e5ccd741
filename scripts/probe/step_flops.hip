// ISA probe for the frozen algorithmic flop count (roofline.py): one Wisdom-Holman
// kick-drift-kick step exactly as the segment loop runs it (rvm_walker.h segment_steps: drift,
// kick_prep, kick_apply) on the 2-planet lane layout, between two asm markers.  scripts/step_flops.py
// compiles this for gfx950 and counts the fp64 VALU instructions between the markers.
//   SPEC = 1: the ungated drift of the speculative fine levels (no wave vote); 0: the gated drift.
#include "../../rvel-mcmc_amd/csrc/rvm_device.h"
using namespace rvm;

template <int NT, bool GATED>
__global__ void step_flops(double* buf, int n, double h) {
    Lane<2> s;
    const int i = threadIdx.x;
    s.rx = buf[i];
    s.ry = buf[i + 64];
    s.vx = buf[i + 128];
    s.vy = buf[i + 192];
    s.r = buf[i + 256];
    s.ir = buf[i + 320];
    s.GM = buf[i + 384];
    s.m[0] = buf[448];
    s.m[1] = buf[449];
    s.iMi[0] = 1.0;
    s.iMi[1] = buf[450];
    s.iMi[2] = buf[451];
    s.mu[0] = buf[452];
    s.mu[1] = buf[453];
    s.dmin2 = buf[454];
    s.p = i & 1;
    s.q = i & 1;
    s.encm = 0;
    lane_finish(s);
    lane_set_step(s, h);
    const VConsts vk = vconsts_for<NT>();
    KickPrep<2> kp = kick_prep<2, 2, false>(s, vk.c1875);
    bool bad = false;
    for (int j = 0; j < n; j++) {
        asm volatile("; STEP_BEGIN" ::: "memory");
        drift<NT, GATED, false>(s, h, bad, vk);
        kp = kick_prep<2, 2, false>(s, vk.c1875);
        kick_apply<2, false, false>(s, kp);
        asm volatile("; STEP_END" ::: "memory");
    }
    buf[i] = s.rx;
    buf[i + 64] = s.ry;
    buf[i + 128] = s.vx;
    buf[i + 192] = s.vy;
    buf[i + 256] = (double)(s.encm & 1) + (bad ? 1.0 : 0.0);
}

template __global__ void step_flops<6, false>(double*, int, double);
template __global__ void step_flops<6, true>(double*, int, double);

"""Plain-Python restatement of the device RNG (rvm_device.h: philox / uniform2).

Philox4x32-10 (Salmon et al., SC'11) keyed by the 64-bit seed, counter
(item lo, item hi, iteration lo, (iteration hi & 0xFFFF) | stream << 16); two uniforms in (0, 1)
with 53-bit resolution: ((x >> 5) * 2^26 + (y >> 6) + 0.5) / 2^53.
"""
import numpy as np

M0, M1 = 0xD2511F53, 0xCD9E8D57
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK = 0xFFFFFFFF


def philox4x32_10(c, k0, k1):
    x, y, z, w = c
    for _ in range(10):
        p0 = M0 * x
        p1 = M1 * z
        hi0, lo0 = (p0 >> 32) & MASK, p0 & MASK
        hi1, lo1 = (p1 >> 32) & MASK, p1 & MASK
        x, y, z, w = (hi1 ^ y ^ k0) & MASK, lo1, (hi0 ^ w ^ k1) & MASK, lo0
        k0 = (k0 + W0) & MASK
        k1 = (k1 + W1) & MASK
    return x, y, z, w


def uniform2(seed, item, iteration, stream):
    c = (item & MASK, (item >> 32) & MASK, iteration & MASK, (((iteration >> 32) & 0xFFFF) | (stream << 16)) & MASK)
    x, y, z, w = philox4x32_10(c, seed & MASK, (seed >> 32) & MASK)
    a = ((x >> 5) << 26) | (y >> 6)
    b = ((z >> 5) << 26) | (w >> 6)
    return (a + 0.5) / 9007199254740992.0, (b + 0.5) / 9007199254740992.0


RNG_STRETCH_PROPOSE = 1
RNG_STRETCH_ACCEPT = 2
RNG_MH_PROPOSE = 3
RNG_MH_ACCEPT = 4


def stretch_uniforms(seed, begin, n, iteration, half):
    """(u1, u2, u3) arrays for walkers begin..begin+n-1 as the device draws them."""
    u1 = np.empty(n)
    u2 = np.empty(n)
    u3 = np.empty(n)
    for i in range(n):
        u1[i], u2[i] = uniform2(seed, begin + i, iteration, RNG_STRETCH_PROPOSE | (half << 8))
        u3[i], _ = uniform2(seed, begin + i, iteration, RNG_STRETCH_ACCEPT | (half << 8))
    return u1, u2, u3

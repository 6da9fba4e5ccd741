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


def uniform2_vec(seed, items, iteration, stream):
    """uniform2 for an array of items at once (numpy uint64 lanes; same bits as uniform2)."""
    u64 = np.uint64
    items = np.asarray(items, dtype=np.uint64)
    m = u64(MASK)
    x, y = items & m, (items >> u64(32)) & m
    z = np.full_like(items, iteration & MASK)
    w = np.full_like(items, (((iteration >> 32) & 0xFFFF) | (stream << 16)) & MASK)
    k0, k1 = u64(seed & MASK), u64((seed >> 32) & MASK)
    for _ in range(10):
        p0 = u64(M0) * x
        p1 = u64(M1) * z
        x, y, z, w = ((p1 >> u64(32)) ^ y ^ k0) & m, p1 & m, ((p0 >> u64(32)) ^ w ^ k1) & m, p0 & m
        k0 = (k0 + u64(W0)) & m
        k1 = (k1 + u64(W1)) & m
    a = ((x >> u64(5)) << u64(26)) | (y >> u64(6))
    b = ((z >> u64(5)) << u64(26)) | (w >> u64(6))
    return (a.astype(np.float64) + 0.5) / 9007199254740992.0, (b.astype(np.float64) + 0.5) / 9007199254740992.0


def stretch_uniforms(seed, begin, n, iteration, half):
    """(u1, u2, u3) arrays for walkers begin..begin+n-1 as the device draws them."""
    items = np.arange(begin, begin + n, dtype=np.uint64)
    u1, u2 = uniform2_vec(seed, items, iteration, RNG_STRETCH_PROPOSE | (half << 8))
    u3, _ = uniform2_vec(seed, items, iteration, RNG_STRETCH_ACCEPT | (half << 8))
    return u1, u2, u3

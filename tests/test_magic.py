"""The planner's magic-number division (ghx_internal.hpp make_magic + ghx_kernels.hip fastdiv),
restated bit-for-bit in numpy and checked against exact division on edge and random cases."""
import numpy as np


def make_magic(d):
    d = max(d, 1)
    l = 0
    while (1 << l) < d:
        l += 1
    m = ((1 << 32) * ((1 << l) - d)) // d + 1
    return m & 0xFFFFFFFF, min(l, 1), max(l - 1, 0)


def fastdiv(n, mag):
    m, s1, s2 = mag
    n = n.astype(np.uint64)
    t = (n * np.uint64(m)) >> np.uint64(32)
    return ((t + ((n - t) >> np.uint64(s1))) >> np.uint64(s2)).astype(np.uint64)


def test_fastdiv_exact():
    rng = np.random.default_rng(0)
    divisors = list(range(1, 300)) + [512, 516, 1023, 1024, 1025, 4095, 4096, 4128, 65535, 65536,
                                     262144, 266256, 2 ** 20 + 7, 2 ** 30 - 1, 2 ** 31 - 1, 2 ** 31]
    ns = np.concatenate([np.arange(0, 5000, dtype=np.uint64),
                         rng.integers(0, 2 ** 32, size=20000, dtype=np.uint64),
                         np.array([2 ** 32 - 1, 2 ** 32 - 2, 2 ** 31, 2 ** 31 - 1], dtype=np.uint64)])
    for d in divisors:
        got = fastdiv(ns, make_magic(d))
        assert np.array_equal(got, ns // np.uint64(d)), d
        # multiples and neighbours of d
        k = np.arange(0, min(2 ** 32 // d, 5000), dtype=np.uint64) * np.uint64(d)
        for delta in (0, 1):
            x = k + np.uint64(delta)
            x = x[x < 2 ** 32]
            assert np.array_equal(fastdiv(x, make_magic(d)), x // np.uint64(d)), d
        x = k[k > 0] - np.uint64(1)
        assert np.array_equal(fastdiv(x, make_magic(d)), x // np.uint64(d)), d

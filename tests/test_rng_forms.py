"""The kernel's rearranged RNG draws (crt_device.hip: rnd_pm1, rnd_01) against the reference's own
expression, rand_double(min, max) = min + (max - min) * double(seed) * SCALE (rand_util.h:110-116),
in IEEE f64 round-to-nearest (numpy on the host rounds like the GPU's v_mul_f64 / v_add_f64).
Every edge state and a large random sample must give the same bits."""
import numpy as np

SCALE = 1 / float(4294967295 - 1)


def reference(x, lo, hi):
    return lo + (hi - lo) * x * SCALE


def states():
    rng = np.random.default_rng(7)
    edges = np.array([0, 1, 2, 3, 2**31 - 2, 2**31 - 1, 2**31, 2**31 + 1, 2**32 - 3, 2**32 - 2, 2**32 - 1],
                     dtype=np.uint64)
    return np.concatenate([edges, rng.integers(0, 2**32, size=1 << 22, dtype=np.uint64)]).astype(np.float64)


def test_rnd_pm1_bit_identical():
    x = states()
    want = reference(x, -1.0, 1.0)
    got = x * (2 * SCALE) + -1.0
    assert np.array_equal(want.view(np.uint64), got.view(np.uint64))


def test_rnd_01_bit_identical():
    x = states()
    want = reference(x, 0.0, 1.0)
    got = x * SCALE
    assert np.array_equal(want.view(np.uint64), got.view(np.uint64))
    assert not np.signbit(got).any()

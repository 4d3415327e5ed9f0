"""The Newton site's acceptance test norm(perp) > 0.01f (reference/bezierTriangle.cpp:165) is evaluated on the
GPU as dot(perp, perp) > 0x38d1b718 (patch_math.hpp sqrt_above_hundredth): correctly rounded sqrt is
monotone, and 0x38d1b718 is the largest float whose rounded square root is <= 0.01f.  The equivalence was
checked over all 2^32 float32 bit patterns; this test repeats it around the threshold, on the special
values and on a random sample (numpy's float32 sqrt is the correctly rounded IEEE operation)."""
import numpy as np

X_BITS = 0x38D1B718


def _check(bits):
    f = np.asarray(bits, dtype=np.uint32).view(np.float32)
    x = np.array([X_BITS], np.uint32).view(np.float32)[0]
    with np.errstate(invalid="ignore"):
        return np.array_equal(np.sqrt(f) > np.float32(0.01), f > x)


def test_threshold_is_the_last_float_with_sqrt_at_most_a_hundredth():
    x = np.array([X_BITS, X_BITS + 1], np.uint32).view(np.float32)
    assert np.sqrt(x[0]) <= np.float32(0.01) < np.sqrt(x[1])


def test_squared_threshold_equals_sqrt_comparison():
    near = np.arange(X_BITS - (1 << 22), X_BITS + (1 << 22), dtype=np.int64).astype(np.uint32)
    special = np.array([0, 0x80000000, 1, 0x007FFFFF, 0x00800000, 0x7F7FFFFF, 0x7F800000, 0xFF800000,
                        0x7FC00000, 0xFFC00000, 0x3F800000, 0xBF800000], np.uint32)
    rng = np.random.default_rng(3)
    sample = rng.integers(0, 1 << 32, 1 << 22, dtype=np.uint64).astype(np.uint32)
    assert _check(near) and _check(special) and _check(sample)

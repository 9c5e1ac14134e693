"""Kernel 2's division reciprocal (u256.cuh mg_reciprocal_fp): the Moller-Granlund
reciprocal v = floor((2^64 - 1) / d) - 2^32 of a normalised 32-bit divisor, taken
from the fp64 quotient 2^64 / d and corrected once against the defining
inequality.  The same arithmetic in numpy (IEEE fp64, as the GPU's correctly
rounded division) must equal the exact integer reciprocal on the edges of the
range and on a dense sample of it (the whole range is checked by a C program
during development: 2^31 divisors, no mismatch)."""
import numpy as np

M64 = (1 << 64) - 1


def _fits(v, d):
    # (2^32 + v) d <= 2^64 - 1, i.e. d * 2^32 + v * d does not carry out of 2^64
    vd = v.astype(object) * d.astype(object)
    return np.array([(int(dd) << 32) + int(x) <= M64 for dd, x in zip(d, vd)])


def _fp(d):
    e = np.float64(2.0 ** 64) / d.astype(np.float64) - np.float64(2.0 ** 32)
    e = np.clip(e, 0.0, 4294967295.0)
    v = e.astype(np.uint64)
    ok = _fits(v, d)
    v = np.where(ok, v, v - 1)
    up = ok & (v != 0xFFFFFFFF) & _fits(np.minimum(v + 1, 0xFFFFFFFF), d)
    return np.where(up, v + 1, v)


def _exact(d):
    return np.array([(M64 // int(x)) - (1 << 32) for x in d], dtype=np.uint64)


def test_reciprocal_from_fp64_is_exact():
    rng = np.random.default_rng(11)
    d = np.concatenate([
        np.arange(0x80000000, 0x80000000 + 4096, dtype=np.uint64),
        np.arange(0xFFFFFFFF - 4095, 0xFFFFFFFF + 1, dtype=np.uint64),
        (rng.integers(0, 1 << 31, 60000, dtype=np.uint64) | np.uint64(0x80000000)),
        np.array([1 << 31, (1 << 31) + 1, 3 << 30, 0xFFFFFFFF], dtype=np.uint64),
    ])
    assert np.array_equal(_fp(d), _exact(d))

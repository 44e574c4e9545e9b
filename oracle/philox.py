"""Philox4x32-10 counter-based RNG (Salmon et al., SC'11 / Random123) in numpy.

ORACLE — test infrastructure only.  The HIP noise kernel uses the same stream;
this module is checked against Random123's published known-answer vectors in
``tests/test_oracle.py``.
"""
import numpy as np

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
_MASK = np.uint64(0xFFFFFFFF)
_S32 = np.uint64(32)


def philox4x32(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10.  Inputs broadcastable uint32 arrays; returns 4 uint32 arrays."""
    c0 = np.asarray(c0, dtype=np.uint32).astype(np.uint64)
    c1 = np.asarray(c1, dtype=np.uint32).astype(np.uint64)
    c2 = np.asarray(c2, dtype=np.uint32).astype(np.uint64)
    c3 = np.asarray(c3, dtype=np.uint32).astype(np.uint64)
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = np.uint64(np.uint32(k0))
    k1 = np.uint64(np.uint32(k1))
    for r in range(10):
        if r > 0:
            k0 = (k0 + np.uint64(W0)) & _MASK
            k1 = (k1 + np.uint64(W1)) & _MASK
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> _S32, p0 & _MASK
        hi1, lo1 = p1 >> _S32, p1 & _MASK
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0), lo1, (hi0 ^ c3 ^ k1), lo0
    return (c0.astype(np.uint32), c1.astype(np.uint32),
            c2.astype(np.uint32), c3.astype(np.uint32))


def u53(hi, lo):
    """53-bit uniform double in [0, 1) from two 32-bit words: ((hi<<32|lo) >> 11) * 2^-53."""
    a = (np.asarray(hi, np.uint64) << _S32) | np.asarray(lo, np.uint64)
    return (a >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def u53_open0(hi, lo):
    """53-bit uniform double in (0, 1]: (((hi<<32|lo) >> 11) + 1) * 2^-53."""
    a = (np.asarray(hi, np.uint64) << _S32) | np.asarray(lo, np.uint64)
    return ((a >> np.uint64(11)) + np.uint64(1)).astype(np.float64) * (2.0 ** -53)


def mulhi32(x, n):
    """floor(x * n / 2^32) for uint32 x and n < 2^32 (Lemire-style bounded draw)."""
    return ((np.asarray(x, np.uint64) * np.uint64(n)) >> _S32).astype(np.int64)

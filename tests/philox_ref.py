"""numpy restatement of the device Philox-4x32-10 (csrc/common.h philox(ctr_lo, ctr_hi, key)): the
checker for the device RNG consumers whose results must match bit for bit (random subset)."""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
MASK = np.uint64(0xFFFFFFFF)
S32 = np.uint64(32)


def philox(ctr_lo, ctr_hi, key):
    """ctr_lo: uint64 array (or scalar), ctr_hi / key: python ints.  Returns four uint64 arrays
    holding the 32-bit outputs (x, y, z, w)."""
    lo = np.asarray(ctr_lo, dtype=np.uint64)
    c0, c1 = lo & MASK, lo >> S32
    c2 = np.full_like(lo, np.uint64(ctr_hi) & MASK)
    c3 = np.full_like(lo, np.uint64(ctr_hi) >> S32)
    k0, k1 = np.uint64(key) & MASK, np.uint64(key) >> S32
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        c0, c1, c2, c3 = (p1 >> S32) ^ c1 ^ k0, p1 & MASK, (p0 >> S32) ^ c3 ^ k1, p0 & MASK
        k0 = (k0 + W0) & MASK
        k1 = (k1 + W1) & MASK
    return c0, c1, c2, c3


def random_subset(n, k, seed, offset, sub):
    """gpi_random_subset: the first k indices ordered by (Philox x of counter offset + i, i)."""
    x = philox(np.uint64(offset) + np.arange(n, dtype=np.uint64), sub, seed)[0]
    order = np.lexsort((np.arange(n), x))
    return order[:k].astype(np.int32)

"""Philox4x32-10 in numpy — TEST INFRASTRUCTURE (see oracle/__init__.py).

Mirrors ``deap_amd/csrc/common.hpp`` (``philox4x32_10``, ``Rng``,
``prob_threshold``, ``bounded64``, ``u01_32``, ``u01_53``) bit for bit, so the
integer-valued native decisions (tournament aspirants, crossover flags and cut
points, per-gene masks of float genomes, cxBlend ``u``) can be recomputed on
the host.  Pinned by the Random123 known-answer vectors in
``tests/test_oracle.py``.
"""
import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)

ST_SEL, ST_CX, ST_BLEND, ST_MUT, ST_MASK, ST_GAUSS, ST_FLIP, ST_VAROR, ST_INIT = range(1, 10)


def philox4x32_10(ctr, key):
    """ctr: (..., 4) uint32-valued; key: (k0, k1).  Returns (..., 4) uint32."""
    c = np.asarray(ctr, dtype=np.uint64) & MASK32
    c0, c1, c2, c3 = (c[..., i].copy() for i in range(4))
    k0, k1 = int(key[0]) & 0xFFFFFFFF, int(key[1]) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c0
        p1 = M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & MASK32
        hi1, lo1 = p1 >> np.uint64(32), p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ np.uint64(k0)), lo1, (hi0 ^ c3 ^ np.uint64(k1)), lo0
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return np.stack([c0, c1, c2, c3], axis=-1).astype(np.uint32)


class Rng:
    """dm_rng: key = seed, ctr = {item, sub, gen, (stage << 16) | island}."""

    def __init__(self, seed, island=0, gen=0):
        self.k = (seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF)
        self.gen = gen & 0xFFFFFFFF
        self.island = island & 0xFFFF

    def __call__(self, stage, item, sub):
        item = np.asarray(item, dtype=np.uint64)
        sub = np.broadcast_to(np.asarray(sub, dtype=np.uint64), item.shape)
        ctr = np.stack([item, sub, np.full(item.shape, self.gen, np.uint64),
                        np.full(item.shape, (stage << 16) | self.island, np.uint64)], axis=-1)
        return philox4x32_10(ctr, self.k)


def prob_threshold(p):
    if not p > 0.0:
        return 0
    if p >= 1.0:
        return 1 << 32
    return int(p * 4294967296.0)


def bounded64(lo, hi, n):
    v = (np.asarray(hi, np.uint64) << np.uint64(32)) | np.asarray(lo, np.uint64)
    # floor(v * n / 2^64) without 128-bit ints: split v in 32-bit halves
    n = np.uint64(n)
    a = (v >> np.uint64(32)) * n
    b = (v & MASK32) * n
    return ((a + (b >> np.uint64(32))) >> np.uint64(32)).astype(np.int64)


def u01_32(w):
    return np.asarray(w, np.float64) * 2.3283064365386963e-10


def u01_53(lo, hi):
    v = ((np.asarray(hi, np.uint64) << np.uint64(32)) | np.asarray(lo, np.uint64)) >> np.uint64(11)
    return v.astype(np.float64) * 1.1102230246251565e-16


def gene_slot(g, itemsize):
    """Philox slot (sub, word) of gene g in the per-gene streams ST_BLEND /
    ST_MASK (deap_amd/csrc/generation.hpp gene4_words): the four words of a
    call feed the four genes one lane holds in a 256-gene chunk of the hot
    kernel's layout — fp64 rows: genes {256c + 2L, +1, 256c + 128 + 2L, +1};
    fp32 rows: genes 256c + 4L .. +3 — with call sub = 64c + L."""
    g = np.asarray(g, np.int64)
    if itemsize == 4:
        return g >> 2, g & 3
    r = g & 255
    return ((g >> 8) << 6) + ((r & 127) >> 1), ((r >> 7) << 1) | (r & 1)

"""CPU check of the identities behind the bitset dominance pass
(deap_amd/csrc/bitdom.hip), restated in numpy: over a 512-v chunk C of the
objective-0 order,

* row u of D over C = prefix0(u) & P_1[k_1] & ... & P_{m-1}[k_{m-1}] without
  bit u, k_i = #{v in C : r_i(v) <= r_i(u)}, P_i[k] = the k positions of C
  with the smallest (r_i, position);
* the dominators of v inside C = popcount(suffix0(v) & ~(P_1[lb_1] | ...)) -
  [v in C], lb_i = #{u in C : r_i(u) < r_i(v)};

against Fitness.dominates (deap/base.py:209-224) by brute force on the dense
ranks, with ties in every objective and objective-0 tie groups wider than a
chunk.  The device kernels are checked against the oracle and the compare
kernel in tests/test_gpu_parity.py::test_bitset_dominance_equals_compare_kernel;
this test pins the algebra those kernels implement, on CPU."""
import numpy as np
import pytest

CW = 512


def _dense_ranks(fit):
    """Unique fitness rows, their dense ranks per objective (larger value,
    larger rank), in objective-0 (q) order."""
    uf = np.unique(fit, axis=0)
    r = np.stack([np.searchsorted(np.unique(uf[:, i]), uf[:, i]) for i in range(uf.shape[1])], 1)
    order = np.lexsort(tuple(r[:, i] for i in reversed(range(r.shape[1]))))
    return r[order]


def _tables(r, c):
    """Sorted ranks and prefix sets of chunk c for each objective i >= 1."""
    U, m = r.shape
    pos = np.arange(c * CW, min(U, c * CW + CW))
    sets, srt = [], []
    for i in range(1, m):
        rv = np.full(CW, np.iinfo(np.int64).max)
        rv[:len(pos)] = r[pos, i]
        lr = np.lexsort((np.arange(CW), rv)).argsort()  # local rank by (rank, position)
        srt.append(np.sort(rv))
        sets.append(lr[None, :] < np.arange(CW + 1)[:, None])  # P[k] = {local rank < k}
    return srt, sets


@pytest.mark.parametrize("n,m,kind", [(700, 2, "ties"), (1300, 3, "obj0"), (1100, 3, "cont"),
                                      (900, 4, "ties")])
def test_bitset_rows_and_counts_equal_brute_force(n, m, kind):
    rng = np.random.default_rng(n + m)
    if kind == "ties":
        fit = rng.integers(0, 6, size=(n, m)).astype(float)
    elif kind == "obj0":
        fit = np.concatenate([rng.integers(0, 2, size=(n, 1)).astype(float),
                              rng.integers(0, 40, size=(n, m - 1)).astype(float)], 1)
    else:
        fit = rng.uniform(size=(n, m))
    r = _dense_ranks(fit)
    U = len(r)
    dom = np.all(r[:, None, :] >= r[None, :, :], axis=2)  # dom[u, v]: u dominates v (or u == v)
    np.fill_diagonal(dom, False)
    first = {int(x): int(np.argmax(r[:, 0] == x)) for x in np.unique(r[:, 0])}
    last = {int(x): int(U - 1 - np.argmax(r[::-1, 0] == x)) for x in np.unique(r[:, 0])}
    counts = np.zeros(U, int)
    for c in range((U + CW - 1) // CW):
        srt, sets = _tables(r, c)
        v0 = c * CW
        nv = min(CW, U - v0)
        p = np.arange(CW)
        for u in range(U):  # rows
            w = p <= last[int(r[u, 0])] - v0
            for i in range(1, m):
                w &= sets[i - 1][int(np.searchsorted(srt[i - 1], r[u, i], side="right"))]
            if 0 <= u - v0 < CW:
                w[u - v0] = False
            assert np.array_equal(w[:nv], dom[u, v0:v0 + nv]), (u, c)
        for v in range(U):  # dominator counts contributed by chunk c
            o = np.zeros(CW, bool)
            for i in range(1, m):
                o |= sets[i - 1][int(np.searchsorted(srt[i - 1], r[v, i], side="left"))]
            x = ~o & (p >= first[int(r[v, 0])] - v0) & (p < nv)
            counts[v] += int(x.sum()) - (1 if 0 <= v - v0 < CW else 0)
    assert np.array_equal(counts, dom.sum(axis=0))

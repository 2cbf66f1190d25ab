"""Vectorised closed form of DEAP's sortNondominated front ORDER and of the
standard selNSGA2 choice -- TEST INFRASTRUCTURE (the checker of the device
path at the benched size, never imported by the product path).

The reference (deap/tools/emo.py:53-117) groups individuals by equal
fitness in first-appearance order (``map_fit_ind``, a dict), counts
dominators over all unique-fitness pairs in that order (``dominating_fits``)
and lists, per unique fit p, the fits it dominates (``dominated_fits[p]``,
appended in the order the pair loop meets them: ascending unique index).  The
peel then walks front r in order and, for each p, decrements the counts of
dominated_fits[p]; a fit whose count reaches 0 is appended to front r+1.  So
(SURVEY.md §8a-a21):

* front 0 = the undominated unique fits in unique (first-appearance) order;
* a fit v of rank r+1 has every dominator in fronts <= r and at least one in
  front r; it is released while its LAST dominator in front r is processed,
  and within that dominator's list in unique-index order: front r+1 is
  ordered by (max position in front r of a dominator of v, unique index of v);
* each unique fit expands to its individuals in population order;
* fronts are produced until at least min(n, k) individuals are sorted
  (emo.py:100-115), or only front 0 with ``first_front_only``.

Only CONSECUTIVE front pairs are compared, so the order costs
sum_r |F_r| x |F_r+1| x M element compares (seconds at 2^18 rows).  The
Pareto ranks themselves come from ``oracle/deap_port.py``'s Fortin log sort
(emo.py:234-441 restated; bit-exact against the reference on
tests/golden/nsga2*.npz, tests/test_support_port.py), whose ranks equal the
standard sort's.  This module is checked against
``oracle.ops.sort_nondominated`` (the literal restatement of emo.py:53-117)
and the reference-generated tests/golden/nsga2.npz in tests/test_oracle.py.
"""
import numpy as np

from . import deap_port, ops


def unique_first_appearance(wvalues):
    """(ufit[U][M], ui[n]): the distinct fitness rows in first-appearance
    order (emo.py:72-75, a dict keyed by Fitness, whose hash/eq compare
    wvalues: -0.0 == 0.0) and each row's unique index."""
    w = np.ascontiguousarray(wvalues, dtype=np.float64) + 0.0  # -0.0 -> 0.0
    if np.isnan(w).any():
        raise ValueError("closed form: NaN fitnesses are not supported")
    _, first, inv = np.unique(w, axis=0, return_index=True, return_inverse=True)
    order = np.argsort(first, kind="stable")
    uid = np.empty(len(order), np.int64)
    uid[order] = np.arange(len(order))
    return w[first[order]], uid[np.asarray(inv).ravel()]


def pareto_ranks(ufit):
    """Pareto rank of every unique fit from the port's Fortin sort
    (emo.py:246-265: ``fits.sort(reverse=True)``, sortNDHelperA)."""
    fits = [tuple(float(x) for x in row) for row in ufit]
    rank = dict.fromkeys(fits, 0)
    srt = sorted(fits, reverse=True)
    deap_port._nd_a(srt, ufit.shape[1] - 1, rank)
    return np.fromiter((rank[f] for f in fits), np.int64, len(fits))


def last_dominator_position(prev_fit, cur_fit, block=1024):
    """For every row v of cur_fit: the largest position p in prev_fit (front r
    in order) such that prev_fit[p] dominates v.  The fits are distinct, so
    ">= in every objective" is domination (base.py:209-224)."""
    P = len(prev_fit)
    key = np.empty(len(cur_fit), np.int64)
    rev = prev_fit[::-1]
    for a in range(0, len(cur_fit), block):
        c = cur_fit[a:a + block]
        dom = rev[:, None, 0] >= c[None, :, 0]
        for o in range(1, prev_fit.shape[1]):
            dom &= rev[:, None, o] >= c[None, :, o]
        hit = dom.any(axis=0)
        if not hit.all():
            raise AssertionError("a rank-(r+1) fit has no dominator in front r")
        key[a:a + block] = P - 1 - np.argmax(dom, axis=0)
    return key


def sort_nondominated(wvalues, k, first_front_only=False, ranks=None):
    """emo.py:53-117 by the closed form: a list of fronts (numpy arrays of row
    indices) in the reference's order.  ``ranks``: optional Pareto rank per
    unique fit (unique_first_appearance order), e.g. from the device, only to
    save the Fortin sort when the caller has checked them separately."""
    if k == 0:
        return []
    ufit, ui = unique_first_appearance(wvalues)
    n = len(ui)
    urank = pareto_ranks(ufit) if ranks is None else np.asarray(ranks, np.int64)
    counts = np.bincount(ui, minlength=len(ufit))
    rows = np.argsort(ui, kind="stable")  # rows grouped by unique fit, population order
    starts = np.concatenate([[0], np.cumsum(counts)[:-1]])
    by_rank = np.argsort(urank, kind="stable")  # unique index ascending inside a rank
    rstart = np.searchsorted(urank[by_rank], np.arange(urank.max() + 2))

    def members(r):
        return by_rank[rstart[r]:rstart[r + 1]]

    def expand(us):
        c = counts[us]
        off = np.repeat(starts[us] - np.concatenate([[0], np.cumsum(c)[:-1]]), c)
        return rows[off + np.arange(c.sum())]

    fronts_u = [members(0)]
    total = int(counts[fronts_u[0]].sum())
    if not first_front_only:
        target = min(n, k)
        r = 0
        while total < target:
            prev, cur = fronts_u[-1], members(r + 1)
            key = last_dominator_position(ufit[prev], ufit[cur])
            fronts_u.append(cur[np.lexsort((cur, key))])
            total += int(counts[cur].sum())
            r += 1
    return [expand(f) for f in fronts_u]


def sel_nsga2(wvalues, weights, k, fronts=None):
    """emo.py:15-50 (nd='standard') on the closed-form fronts: crowding per
    front by oracle.ops.assign_crowding_dist (emo.py:119-143), the fronts but
    the last concatenated, then ``sorted(last, key=crowding_dist,
    reverse=True)[:k - len(chosen)]`` -- a stable sort, so equal distances
    keep front order (emo.py:44-48).  Returns (chosen rows, crowding per row
    of the sorted fronts as a dict)."""
    if fronts is None:
        fronts = sort_nondominated(wvalues, k)
    w = np.asarray(wvalues, np.float64)
    wt = np.asarray(weights, np.float64)
    crowd = {}
    for f in fronts:
        vals = w[f] / wt
        for i, d in zip(f.tolist(), ops.assign_crowding_dist(vals.tolist())):
            crowd[i] = d
    chosen = [int(i) for f in fronts[:-1] for i in f]
    kk = k - len(chosen)
    if kk > 0:
        last = sorted(fronts[-1].tolist(), key=lambda i: crowd[i], reverse=True)
        chosen.extend(last[:kk])
    return chosen, crowd

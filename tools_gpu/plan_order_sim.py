import numpy as np, time
rng = np.random.default_rng(1)
n = 1 << 20
t = 3
fit = rng.standard_normal(n)
asp = rng.integers(0, n, size=(n, t))
win = asp[np.arange(n), np.argmax(fit[asp], axis=1)]
a, b = win[0::2], win[1::2]
E = len(a)
deg = np.bincount(win, minlength=n)
V = int((deg > 0).sum())
print("pairs", E, "distinct rows", V, V / n)

def reads(order, run):
    # rows read per run of `run` consecutive pairs (perfect reuse inside a run, none across)
    aa, bb = a[order], b[order]
    g = np.arange(E) // run
    rows = np.concatenate([aa, bb]); gg = np.concatenate([g, g])
    key = gg.astype(np.int64) * n + rows
    return len(np.unique(key)) / n

# current: key = parent with more slots (ties: a?), sort by key (stable by pair)
key = np.where(deg[a] >= deg[b], a, b)
order_cur = np.argsort(key, kind="stable")
other = np.where(key == a, b, a)
for run in (8, 32, 128):
    print("run", run, "pair order", round(reads(np.arange(E), run), 3), "degree key", round(reads(order_cur, run), 3))
# alternative 1: secondary sort within equal key by the other parent's key-star position
# alternative 2: order stars by their highest-degree non-key neighbour
okey = np.where(deg[other] > 1, other, -1)
# star representative: max-degree non-key neighbour of each key
rep = np.full(n, -1)
dd = deg[other]
o2 = np.lexsort((dd, key))  # last per key has max degree
last = np.r_[key[o2][1:] != key[o2][:-1], True]
rep[key[o2][last]] = other[o2][last]
starrep = rep[key]
order_alt = np.lexsort((np.arange(E), key, starrep))
for run in (8, 32, 128):
    print("run", run, "stars grouped by max-degree neighbour", round(reads(order_alt, run), 3))
# alternative 3: key = the other parent's... union-find-ish: sort by min(key, other key-star id)

def label_prop(iters, init=None):
    lab = np.arange(n) if init is None else init.copy()
    for _ in range(iters):
        m = np.minimum(lab[a], lab[b])
        new = lab.copy()
        np.minimum.at(new, a, m)
        np.minimum.at(new, b, m)
        lab = new
    return lab
for it in (1, 2, 3, 5, 8):
    lab = label_prop(it)
    el = np.minimum(lab[a], lab[b])
    order_lp = np.lexsort((np.arange(E), key, el))
    print("label prop", it, [round(reads(order_lp, r), 3) for r in (8, 32, 128)])
# random-priority labels (min of random ranks) -> balanced clusters
pri = rng.permutation(n)
for it in (1, 2, 3):
    lab = label_prop(it, pri)
    el = np.minimum(lab[a], lab[b])
    order_lp = np.lexsort((np.arange(E), key, el))
    print("random-priority label prop", it, [round(reads(order_lp, r), 3) for r in (8, 32, 128)])
print("--- run 256/512 and label-only orders")
print("degree key", [round(reads(order_cur, r), 3) for r in (256, 512)])
for it in (1, 2, 3):
    lab = label_prop(it)
    el = np.minimum(lab[a], lab[b])
    o_only = np.argsort(el, kind="stable")
    o_two = np.lexsort((np.arange(E), key, el))
    # label of the key parent only (cheaper: one lookup)
    ek = lab[key]
    o_k = np.lexsort((np.arange(E), key, ek))
    print("lp", it, "label only", [round(reads(o_only, r), 3) for r in (32, 256, 512)],
          "label+key", [round(reads(o_two, r), 3) for r in (32, 256, 512)],
          "keylabel+key", [round(reads(o_k, r), 3) for r in (32, 256, 512)])

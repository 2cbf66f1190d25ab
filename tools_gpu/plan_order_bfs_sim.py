import numpy as np, scipy.sparse as sp
from scipy.sparse.csgraph import reverse_cuthill_mckee, connected_components
exec(open(__file__.replace('plan_order_bfs_sim.py', 'plan_order_sim.py')).read().split("def label_prop")[0])
G = sp.coo_matrix((np.ones(E), (a, b)), shape=(n, n)).tocsr()
G = (G + G.T).tocsr()
ncomp, comp = connected_components(G, directed=False)
used = np.unique(np.concatenate([a, b]))
cs = np.bincount(comp[used])
print("components with edges", (cs > 1).sum(), "largest", cs.max(), "of", len(used), flush=True)
perm = reverse_cuthill_mckee(G, symmetric_mode=True)
pos = np.empty(n, np.int64); pos[perm] = np.arange(n)
for name, ek in (("max", np.maximum(pos[a], pos[b])), ("min", np.minimum(pos[a], pos[b]))):
    o = np.argsort(ek, kind="stable")
    print("RCM order", name, [round(reads(o, r), 3) for r in (32, 256, 512)], flush=True)

"""Diagnostic: the nsga2.npz golden cases one by one (sync + print after
each step), to attribute a device fault to a case and a call."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from deap_amd import tools
from deap_amd.device import DevicePopulation
d = np.load(os.path.join(os.path.dirname(__file__), "..", "tests", "golden", "nsga2.npz"))
order = [int(x) for x in sys.argv[1:]] or range(6)
for j in order:
    k = "nd%d_" % j
    wv, weights, kk = d[k + "wv"], tuple(d[k + "weights"]), int(d[k + "k"])
    n = len(wv)
    print("case", j, "n", n, "m", wv.shape[1], "k", kk, flush=True)
    pop = DevicePopulation.from_numpy(np.zeros((n, 2)), weights=weights, gtype="f64", wvalues=wv,
                                      valid=np.ones(n))
    fronts = tools.sortNondominated(pop, kk)
    torch.cuda.synchronize()
    flat = np.concatenate([f.cpu().numpy() for f in fronts]).tolist()
    print("  sort ok", flat == d[k + "order"].tolist(), flush=True)
    chosen = tools.selNSGA2(pop, kk)
    torch.cuda.synchronize()
    print("  sel ok", chosen.cpu().numpy().tolist() == d[k + "chosen"].tolist(), flush=True)
    ff = tools.sortNondominated(pop, kk, first_front_only=True)
    torch.cuda.synchronize()
    print("  ff ok", len(ff[0]) == d[k + "first"][0], flush=True)

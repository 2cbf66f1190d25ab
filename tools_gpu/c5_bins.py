"""Bin sizes of the front ordering on an evolved C5 population (diagnostic).

front_order_kernel counting-sorts the released candidates of front r+1 by the
position l of their last dominator in front r and ranks inside a bin by unique
index; a bin of more than ORDER_BIN_MAX candidates sends the whole front to the
bitonic sort.  This prints, per front, the unique count, the largest bin and
how many bins exceed 64 -- from the device's fronts, with the l keys computed
on the host.
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deap_amd import algorithms, base, benchmarks, tools  # noqa: E402
from deap_amd.ops import RandomStream  # noqa: E402


def last_dominator_position(prev_fit, cur_fit, block=1024):
    """Per row of cur_fit: the largest position in prev_fit of a dominator."""
    rev = prev_fit[::-1]
    key = np.empty(len(cur_fit), np.int64)
    for a in range(0, len(cur_fit), block):
        c = cur_fit[a:a + block]
        dom = np.all(rev[:, None, :] >= c[None, :, :], axis=2)
        key[a:a + block] = len(prev_fit) - 1 - np.argmax(dom, axis=0)
    return key


def main():
    n, m, dim = 1 << 17, 3, 12
    stream = RandomStream(1234)
    pop = tools.initPopulation(n=n, dim=dim, low=0.0, high=1.0, gtype="f64",
                               weights=(-1.0,) * m, device="cuda:0", stream=stream)
    tb = base.Toolbox()
    tb.register("evaluate", benchmarks.dtlz2, obj=m)
    tb.register("mate", tools.cxBlend, alpha=0.5)
    tb.register("mutate", tools.mutGaussian, mu=0, sigma=0.1, indpb=1.0 / dim)
    tb.register("select", tools.selNSGA2)
    benchmarks.dtlz2(pop, obj=m)
    step = algorithms.MuPlusLambdaStep(pop, tb, n, n, 0.6, 0.3)
    for _ in range(int(os.environ.get("GENS", "6"))):
        step.step(stream)
    comb = step.combined
    off = algorithms.varOr(comb, tb, n, 0.6, 0.3, evaluate=True, stream=stream)
    two = comb.like(2 * n, capacity=2 * n)
    two.wvalues[:n].copy_(comb.wvalues[:n])
    two.wvalues[n:].copy_(off.wvalues[:n])
    two.valid.fill_(1)
    fronts = tools.sortNondominated(two, n)
    wv = two.wvalues[:2 * n].double().cpu().numpy()
    prev = None
    tot_big = 0
    for r, f in enumerate(fronts):
        rows = f.cpu().numpy()
        fit = wv[rows] + 0.0
        _, first = np.unique(fit, axis=0, return_index=True)
        ufit = fit[np.sort(first)]
        if prev is not None:
            key = last_dominator_position(prev, ufit)
            cnt = np.bincount(key, minlength=len(prev))
            big = int((cnt > 64).sum())
            tot_big += big > 0
            print(f"front {r:3d} U {len(ufit):6d} prevU {len(prev):6d} maxbin {cnt.max():5d} "
                  f"bins>64 {big:4d}", flush=True)
        prev = ufit
    print(f"fronts {len(fronts)}; fronts with a bin > 64: {tot_big}", flush=True)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()

"""Run lengths of equal sort keys on an evolved C5 population (diagnostic):
objective-0 ordered keys compared whole and by their top 32 bits, and the
unique fitnesses' objective-1/2 keys by their top 32 bits -- how long the runs
a 4-pass (32-bit) radix sort would leave for a fix-up would be."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from deap_amd import algorithms, base, benchmarks, tools  # noqa: E402
from deap_amd.ops import RandomStream  # noqa: E402


def okey(x):
    b = np.ascontiguousarray(x, np.float64).view(np.uint64)
    neg = (b >> np.uint64(63)) == 1
    return np.where(neg, ~b, b | np.uint64(1 << 63))


def runs(k):
    k = np.sort(k)
    br = np.flatnonzero(np.diff(k) != 0) + 1
    lens = np.diff(np.concatenate([[0], br, [len(k)]]))
    return int(lens.max()), int((lens > 64).sum()), int((lens > 1).sum())


def main():
    n, m, dim = 1 << 17, 3, 12
    stream = RandomStream(4321)
    pop = tools.initPopulation(n=n, dim=dim, low=0.0, high=1.0, gtype="f64",
                               weights=(-1.0,) * m, device="cuda:0", stream=stream)
    tb = base.Toolbox()
    tb.register("evaluate", benchmarks.dtlz2, obj=m)
    tb.register("mate", tools.cxBlend, alpha=0.5)
    tb.register("mutate", tools.mutGaussian, mu=0, sigma=0.1, indpb=1.0 / dim)
    tb.register("select", tools.selNSGA2)
    benchmarks.dtlz2(pop, obj=m)
    step = algorithms.MuPlusLambdaStep(pop, tb, n, n, 0.6, 0.3)
    for g in range(int(os.environ.get("GENS", "30"))):
        step.step(stream)
        if g % 10 == 9 or g < 2:
            wv = step.combined.wvalues[:n].cpu().numpy()
            u = np.unique(wv, axis=0)
            k0 = okey(wv[:, 0])
            print("gen %3d: obj0 whole-key runs (max, >64, >1) %s; top-32 %s; uniques %d: "
                  "obj1 top-32 %s obj2 top-32 %s" % (
                      g + 1, runs(k0), runs(k0 >> np.uint64(32)), len(u),
                      runs(okey(u[:, 1]) >> np.uint64(32)), runs(okey(u[:, 2]) >> np.uint64(32))),
                  flush=True)


if __name__ == "__main__":
    main()

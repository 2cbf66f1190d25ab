"""Unique-fitness sizes of the fronts selNSGA2 peels in C5's generations
(bench.py --config c5 setup): ``python tools_gpu/c5_front_sizes.py [GENS]``.
Prints per generation the number of fronts, the largest and the count above
4,096 / 8,192 / 16,384 unique fitnesses."""
import sys

import numpy as np
import torch

from deap_amd import algorithms, base, benchmarks, tools
from deap_amd.ops import RandomStream

gens = int(sys.argv[1]) if len(sys.argv) > 1 else 12
n, m, dim = 1 << 17, 3, 12
stream = RandomStream(1)
pop = tools.initPopulation(n=n, dim=dim, low=0.0, high=1.0, gtype="f64", weights=(-1.0,) * m,
                           device="cuda", stream=stream)
tb = base.Toolbox()
tb.register("evaluate", benchmarks.dtlz2, obj=m)
tb.register("mate", tools.cxBlend, alpha=0.5)
tb.register("mutate", tools.mutGaussian, mu=0, sigma=0.1, indpb=1.0 / dim)
tb.register("select", tools.selNSGA2)
benchmarks.dtlz2(pop, obj=m)
step = algorithms.MuPlusLambdaStep(pop, tb, n, n, 0.6, 0.3)
import ctypes
from deap_amd import _lib
two = pop.like(2 * n, capacity=2 * n)
for g in range(1, gens + 1):
    step.step(stream)
    if g in (1, 2, 3, 4, 5, 6, 8, 12, 20, 50, 100, 200, 300):
        # the pool the next step selects from: the parents and one varOr batch
        comb = step.combined
        ctx = comb.ctx.bind()
        _lib.call("dm_gather", ctx, ctypes.byref(comb.c_pop()), None, ctypes.byref(two.c_pop(0, n)))
        off = algorithms.varOr(comb, tb, n, 0.6, 0.3, evaluate=True, stream=RandomStream(7 + g))
        _lib.call("dm_gather", ctx, ctypes.byref(off.c_pop()), None, ctypes.byref(two.c_pop(n, n)))
        fr = tools.sortNondominated(two, n)
        wv = two.wvalues[:2 * n].cpu().numpy()
        us = [int(len(np.unique(wv[f.cpu().numpy()], axis=0))) for f in fr]
        print("gen %3d fronts %3d max %6d >4096: %3d >8192: %3d >16384: %3d  sizes %s" % (
            g, len(us), max(us), sum(u > 4096 for u in us), sum(u > 8192 for u in us),
            sum(u > 16384 for u in us), us[:6] + ["..."] + us[-4:]), flush=True)
torch.cuda.synchronize()

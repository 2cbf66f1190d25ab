"""Profiling helper (not a test): eaSimple at 2^20 Rastrigin-1000D with
Statistics + HallOfFame(10), to see the bookkeeping's GPU time per generation
under rocprofv3 --kernel-trace --stats."""
import sys
import time
import numpy as np
import torch
sys.path.insert(0, ".")
from deap_amd import algorithms, base, benchmarks, tools
from deap_amd.ops import RandomStream

n, dim = 1 << 20, 1000
tb = base.Toolbox()
tb.register("evaluate", benchmarks.rastrigin)
tb.register("select", tools.selTournament, tournsize=3)
tb.register("mate", tools.cxBlend, alpha=0.5)
tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
st = RandomStream(5)
pop = tools.initPopulation(n=n, dim=dim, low=-5.12, high=5.12, gtype="f64", weights=(-1.0,), stream=st)
stats = tools.Statistics(lambda ind: ind.fitness.values)
for name, fn in (("avg", np.mean), ("std", np.std), ("min", np.min), ("max", np.max)):
    stats.register(name, fn)
hof = tools.HallOfFame(10)
algorithms.eaSimple(pop, tb, 0.5, 0.2, 2, stats=stats, halloffame=hof, verbose=False, stream=st)
torch.cuda.synchronize()
ng = int(sys.argv[1]) if len(sys.argv) > 1 else 10
t0 = time.perf_counter()
algorithms.eaSimple(pop, tb, 0.5, 0.2, ng, stats=stats, halloffame=hof, verbose=False, stream=st)
torch.cuda.synchronize()
print("ms/gen with stats+hof: %.3f" % ((time.perf_counter() - t0) / ng * 1e3))

# host-side breakdown per generation
import collections
from deap_amd import algorithms as A
acc = collections.defaultdict(float)


def timed(name, fn):
    def w(*a, **k):
        t = time.perf_counter()
        try:
            return fn(*a, **k)
        finally:
            acc[name] += time.perf_counter() - t
    return w


A._Bookkeeping.complete_hof = timed("complete_hof", A._Bookkeeping.complete_hof)
A._Bookkeeping.record = timed("record", A._Bookkeeping.record)
A.GenerationStep.step = timed("step", A.GenerationStep.step)
tools.HallOfFame._fetch_candidates = timed("fetch", tools.HallOfFame._fetch_candidates)
tools.HallOfFame._try_candidates = timed("try", tools.HallOfFame._try_candidates)
tools.Statistics.compile = timed("stats", tools.Statistics.compile)
torch.cuda.synchronize()
t0 = time.perf_counter()
algorithms.eaSimple(pop, tb, 0.5, 0.2, ng, stats=stats, halloffame=hof, verbose=False, stream=st)
torch.cuda.synchronize()
print("instrumented ms/gen: %.3f" % ((time.perf_counter() - t0) / ng * 1e3))
for k, v in sorted(acc.items()):
    print("  %-14s %.3f ms/gen" % (k, v / ng * 1e3))

"""Front sizes of the C5 bench's selNSGA2 input (2N DTLZ2 fitnesses after one
generation), for correlating per-front peel times in a kernel trace."""
import sys
sys.path.insert(0, ".")
import torch  # noqa: E402
from deap_amd import algorithms, base, benchmarks, tools, _lib  # noqa: E402
from deap_amd.ops import RandomStream  # noqa: E402
import ctypes  # noqa: E402

n, m, dim = 1 << 17, 3, 12
stream = RandomStream(0)
pop = tools.initPopulation(n=n, dim=dim, low=0.0, high=1.0, gtype="f64", weights=(-1.0,) * m,
                           stream=stream)
tb = base.Toolbox()
tb.register("evaluate", benchmarks.dtlz2, obj=m)
tb.register("mate", tools.cxBlend, alpha=0.5)
tb.register("mutate", tools.mutGaussian, mu=0, sigma=0.1, indpb=1.0 / dim)
tb.register("select", tools.selNSGA2)
benchmarks.dtlz2(pop, obj=m)
step = algorithms.MuPlusLambdaStep(pop, tb, n, n, 0.6, 0.3)
for _ in range(3):
    step.step(stream)
comb = step.combined
two = pop.like(2 * n, capacity=2 * n)
_lib.call("dm_gather", comb.ctx.bind(), ctypes.byref(comb.c_pop()), None, ctypes.byref(two.c_pop(0, n)))
off = algorithms.varOr(comb, tb, n, 0.6, 0.3, evaluate=True, stream=stream)
_lib.call("dm_gather", comb.ctx.bind(), ctypes.byref(off.c_pop()), None, ctypes.byref(two.c_pop(n, n)))
fr = tools.sortNondominated(two, n)
sizes = [len(f) for f in fr]
print("fronts", len(sizes), "sum", sum(sizes))
print(sizes)

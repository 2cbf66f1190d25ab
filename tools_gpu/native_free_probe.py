"""Probe (not a test): the product loops launch library kernels only (VERDICT
r4 item 4).  Run under ``rocprofv3 --kernel-trace``; after the set-up a
marker (``dm_philox_blocks`` -> philox_blocks_kernel) separates the set-up
from the loop, and ``tools_gpu/trace_names.py`` lists every kernel launched
after it (no ``at::native`` kernel may appear).

  python tools_gpu/native_free_probe.py PHASE
PHASE: easimple  eaSimple on 2^18 Rastrigin-1000D with Statistics (mean, std,
                 min, max, argmin per objective; mean / max over all values of
                 a 2-objective population; a non-numpy reducer) + HallOfFame(10)
       c5        MuPlusLambdaStep (varOr + evaluate + selNSGA2 + crowding carry),
                 DTLZ2 M=3, 2^15
       c5x       the examples/ga/nsga2.py loop body: selTournamentDCD ->
                 varBounded -> dtlz2 -> selNSGA2(pop + offspring) + gathers"""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
from deap_amd import _lib, algorithms, base, benchmarks, tools  # noqa: E402
from deap_amd.device import zeros  # noqa: E402
from deap_amd.ops import RandomStream  # noqa: E402


def marker(ctx):
    out = zeros((64,), torch.int32, "cuda")
    c0 = (ctypes.c_uint32 * 4)(0x4D41524B, 0, 0, 0)
    k = (ctypes.c_uint32 * 2)(1, 2)
    _lib.call("dm_philox_blocks", ctx, c0, k, 16, ctypes.c_void_p(out.data_ptr()))
    torch.cuda.synchronize()


def easimple():
    stream = RandomStream(5)
    pop = tools.initPopulation(n=1 << 18, dim=1000, low=-5.12, high=5.12, gtype="f64",
                               weights=(-1.0,), stream=stream)
    tb = base.Toolbox()
    tb.register("evaluate", benchmarks.rastrigin)
    tb.register("mate", tools.cxBlend, alpha=0.5)
    tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
    tb.register("select", tools.selTournament, tournsize=3)
    stats = tools.Statistics(key=lambda ind: ind.fitness.values)
    stats.register("avg", np.mean, axis=0)
    stats.register("std", np.std, axis=0)
    stats.register("min", np.min, axis=0)
    stats.register("max", np.max, axis=0)
    stats.register("best", np.argmin, axis=0)
    stats.register("median", lambda v: float(np.median([x[0] for x in v])))
    hof = tools.HallOfFame(10)
    algorithms.eaSimple(pop, tb, 0.5, 0.2, 1, stats=stats, halloffame=hof, verbose=False,
                        stream=stream)
    two = tools.initPopulation(n=1 << 16, dim=12, low=0.0, high=1.0, gtype="f64",
                               weights=(-1.0, -1.0), stream=stream)
    benchmarks.zdt1(two)
    s2 = tools.Statistics(key=lambda ind: ind.fitness.values)
    s2.register("avg", np.mean)
    s2.register("max", np.max)
    s2.compile(two)
    marker(pop.ctx.bind())
    algorithms.eaSimple(pop, tb, 0.5, 0.2, 6, stats=stats, halloffame=hof, verbose=False,
                        stream=stream)
    print(stats.compile(pop), s2.compile(two), hof[0].fitness.values, flush=True)
    torch.cuda.synchronize()


def c5():
    n, m = 1 << 15, 3
    stream = RandomStream(6)
    pop = tools.initPopulation(n=n, dim=12, low=0.0, high=1.0, gtype="f64",
                               weights=(-1.0,) * m, stream=stream)
    tb = base.Toolbox()
    tb.register("evaluate", benchmarks.dtlz2, obj=m)
    tb.register("mate", tools.cxBlend, alpha=0.5)
    tb.register("mutate", tools.mutGaussian, mu=0, sigma=0.1, indpb=1.0 / 12)
    tb.register("select", tools.selNSGA2)
    benchmarks.dtlz2(pop, obj=m)
    step = algorithms.MuPlusLambdaStep(pop, tb, n, n, 0.6, 0.3)
    step.step(stream)
    marker(pop.ctx.bind())
    for _ in range(4):
        step.step(stream)
    torch.cuda.synchronize()


def c5x():
    n, m, dim = 1 << 15, 3, 12
    stream = RandomStream(7)
    pop = tools.initPopulation(n=n, dim=dim, low=0.0, high=1.0, gtype="f64",
                               weights=(-1.0,) * m, stream=stream)
    tb = base.Toolbox()
    tb.register("mate", tools.cxSimulatedBinaryBounded, low=0.0, up=1.0, eta=20.0)
    tb.register("mutate", tools.mutPolynomialBounded, low=0.0, up=1.0, eta=20.0, indpb=1.0 / dim)
    benchmarks.dtlz2(pop, obj=m)
    two = pop.like(2 * n, capacity=2 * n)
    ctx = pop.ctx.bind()
    tmp = zeros((n,), torch.float64, pop.device)

    def carry(dst, src, idx):
        _lib.call("dm_gather_f64", ctx, ctypes.c_void_p(src.data_ptr()),
                  ctypes.c_void_p(idx.data_ptr()), n, ctypes.c_void_p(tmp.data_ptr()))
        if dst.crowding_dist is None:
            dst.crowding_dist = zeros((dst.capacity,), torch.float64, dst.device)
        _lib.call("dm_gather_f64", ctx, ctypes.c_void_p(tmp.data_ptr()), None, n,
                  ctypes.c_void_p(dst.crowding_dist.data_ptr()))

    idx0 = tools.selNSGA2(pop, n)
    carry(pop, pop.crowding_dist, idx0)
    _lib.call("dm_gather", ctx, ctypes.byref(pop.c_pop()), ctypes.c_void_p(idx0.data_ptr()),
              ctypes.byref(two.c_pop(0, n)))
    _lib.call("dm_gather", ctx, ctypes.byref(two.c_pop(0, n)), None, ctypes.byref(pop.c_pop()))

    def gen():
        sel = tools.selTournamentDCD(pop, n, stream=stream)
        off = algorithms.varBounded(pop, tb, 0.9, sel, stream=stream)
        benchmarks.dtlz2(off, obj=m)
        _lib.call("dm_gather", ctx, ctypes.byref(pop.c_pop()), None, ctypes.byref(two.c_pop(0, n)))
        _lib.call("dm_gather", ctx, ctypes.byref(off.c_pop()), None, ctypes.byref(two.c_pop(n, n)))
        idx = tools.selNSGA2(two, n)
        _lib.call("dm_gather", ctx, ctypes.byref(two.c_pop()), ctypes.c_void_p(idx.data_ptr()),
                  ctypes.byref(pop.c_pop()))
        carry(pop, two.crowding_dist, idx)
    gen()
    marker(ctx)
    for _ in range(4):
        gen()
    torch.cuda.synchronize()


{"easimple": easimple, "c5": c5, "c5x": c5x}[sys.argv[1]]()

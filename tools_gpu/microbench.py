#!/usr/bin/env python3
"""Ablation microbenchmarks of the fused generation on one GPU (C3 shape):
bandwidth ceilings of the access pattern (row gather random / identity) and
the generation kernel with stages switched off through its parameters."""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from deap_amd import _lib, algorithms, base, benchmarks, tools  # noqa: E402
from deap_amd.ops import RandomStream  # noqa: E402


def timeit(fn, reps=10, warm=2):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return sorted(a.elapsed_time(b) for a, b in ev)[reps // 2]


def main():
    n = int(os.environ.get("MB_POP", 1 << 20))
    dim = int(os.environ.get("MB_DIM", 1000))
    problem = os.environ.get("MB_PROBLEM", "rastrigin")
    gt = os.environ.get("MB_GTYPE", "f64")
    dev = torch.device("cuda", 0)
    stream = RandomStream(5)
    pop = tools.initPopulation(n=n, dim=dim, low=-5.12, high=5.12, gtype=gt, weights=(-1.0,),
                               device=dev, stream=stream)
    getattr(benchmarks, problem)(pop)
    off = pop.like(n, capacity=n)
    row = pop.stride
    out = {}
    ctx = pop.ctx.bind()
    perm = torch.randperm(n, device=dev).to(torch.int32)
    ident = torch.arange(n, device=dev, dtype=torch.int32)
    for name, idx in (("gather_random", perm), ("gather_identity", ident)):
        ms = timeit(lambda: _lib.call("dm_gather", ctx, ctypes.byref(pop.c_pop()),
                                      ctypes.c_void_p(idx.data_ptr()), ctypes.byref(off.c_pop())))
        out[name] = {"ms": round(ms, 4), "GB/s": round(2 * n * row / ms / 1e6, 1)}
    # torch copy ceiling
    ms = timeit(lambda: off.genes.copy_(pop.genes))
    out["torch_copy"] = {"ms": round(ms, 4), "GB/s": round(2 * n * row / ms / 1e6, 1)}

    def tb_for(cx, mut):
        tb = base.Toolbox()
        tb.register("evaluate", getattr(benchmarks, problem))
        tb.register("select", tools.selTournament, tournsize=3)
        tb.register("mate", tools.cxBlend, alpha=0.5) if cx == "blend" else \
            tb.register("mate", tools.cxTwoPoint)
        tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
        return tb

    for name, cxpb, mutpb in (("gen_select_copy", 0.0, 0.0), ("gen_cx_only", 0.5, 0.0),
                              ("gen_mut_only", 0.0, 0.2), ("gen_full", 0.5, 0.2),
                              ("gen_all_cx_all_mut", 1.0, 1.0)):
        step = algorithms.GenerationStep(pop, tb_for("blend", None), cxpb, mutpb)

        def run():
            step.step(pop, off, stream)
        ms = timeit(run)
        out[name] = {"ms": round(ms, 4), "GB/s_alg": round(n * (2 * dim * 8 + 32) / ms / 1e6, 1)}
    # evaluation alone (all rows)
    pop.valid.zero_()
    ms = timeit(lambda: getattr(benchmarks, problem)(pop, only_invalid=False))
    out["eval_all"] = {"ms": round(ms, 4), "GB/s": round(n * row / ms / 1e6, 1)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()

"""In-process A/B of a runtime switch of the C3 / C2 generation kernel (not a
test).  The same population buffers serve every variant, alternating in
rounds, so the buffer-placement effect cannot bias the
comparison as it does across processes.

  python tools_gpu/ab_inproc.py CONFIG VAR VALUE [VALUE ...]
e.g.  python tools_gpu/ab_inproc.py c3 DM_PIPE_BPC 32 64   (value "unset" removes the variable)
Prints each value's mean generation-kernel time (library HIP events)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, ".")
from deap_amd import _lib, algorithms, base, benchmarks, tools  # noqa: E402
from deap_amd.ops import RandomStream  # noqa: E402

cfg, var, values = sys.argv[1], sys.argv[2], sys.argv[3:]
rounds, G = int(os.environ.get("AB_ROUNDS", "6")), int(os.environ.get("AB_GENS", "8"))
tb = base.Toolbox()
if cfg == "c2":
    dim, gt, w, lo, hi = 4096, "bits", (1.0,), 0, 1
    tb.register("evaluate", benchmarks.onemax)
    tb.register("mate", tools.cxTwoPoint)
    tb.register("mutate", tools.mutFlipBit, indpb=0.05)
else:
    dim, gt, w, lo, hi = 1000, "f64", (-1.0,), -5.12, 5.12
    tb.register("evaluate", benchmarks.rastrigin)
    tb.register("mate", tools.cxBlend, alpha=0.5)
    tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
tb.register("select", tools.selTournament, tournsize=3)
n = 1 << 20
st = RandomStream(1234)
pop = tools.initPopulation(n=n, dim=dim, low=lo, high=hi, gtype=gt, weights=w, stream=st)
tb.evaluate(pop)
off = pop.like(n, capacity=n)
step = algorithms.GenerationStep(pop, tb, 0.5, 0.2)
nev = torch.zeros(1, dtype=torch.int64, device=pop.device)
ctx = pop.ctx.bind()
for _ in range(3):
    step.step(pop, off, st, ctypes.c_void_p(nev.data_ptr()))
    pop.swap_storage(off)
torch.cuda.synchronize()
res = {v: [] for v in values}
for r in range(rounds):
    for v in values:
        if v == "unset":
            os.environ.pop(var, None)
        else:
            os.environ[var] = v
        _lib.call("dm_ctx_reload_knobs", ctx)  # the switches are read per context
        _lib.call("dm_ctx_set_timing", ctx, G)
        for _ in range(G):
            step.step(pop, off, st, ctypes.c_void_p(nev.data_ptr()))
            pop.swap_storage(off)
        torch.cuda.synchronize()
        times = (ctypes.c_float * G)()
        cnt = ctypes.c_int32(0)
        _lib.call("dm_ctx_kernel_times", ctx, times, G, ctypes.byref(cnt))
        res[v].extend(times[:cnt.value])
_lib.call("dm_ctx_set_timing", ctx, 0)
for v in values:
    t = sorted(res[v])
    print("%s %s=%s: mean %.4f ms  median %.4f ms  (%d launches)" % (
        cfg, var, v, sum(t) / len(t), t[len(t) // 2], len(t)), flush=True)

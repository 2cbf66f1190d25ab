"""Probe (not a test): does the C3 kernel's speed on a deme's buffer pair
depend on what was allocated before / between the two buffers?  (VERDICT r4
item 6; profiles/r05_gap: one process's later-allocated demes run 2.64-2.80 ms
per launch, a one-deme process 2.93 ms.)

  python tools_gpu/alloc_order_probe.py MODE [GENS]
MODE: base        parent buffer, child buffer (bench.py's C3)
      pre:G       G GiB held in a spacer first, then parent, child
      mid:G       parent, G GiB spacer, child
      post:G      parent, child, then a G GiB spacer
      sep         parent, child, then a second parent/child pair; times both
Prints the mean gen_pipe_kernel time (library HIP events) per buffer pair."""
import ctypes
import json
import sys

import torch

sys.path.insert(0, ".")
from deap_amd import _lib, algorithms, base, benchmarks, tools  # noqa: E402
from deap_amd.ops import RandomStream  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "base"
G = int(sys.argv[2]) if len(sys.argv) > 2 else 20
n = 1 << 20
tb = base.Toolbox()
tb.register("evaluate", benchmarks.rastrigin)
tb.register("select", tools.selTournament, tournsize=3)
tb.register("mate", tools.cxBlend, alpha=0.5)
tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
keep = []


def spacer(gib):
    keep.append(torch.empty(int(gib * (1 << 30)), dtype=torch.uint8, device="cuda"))


kind, _, arg = mode.partition(":")
gib = float(arg) if arg else 0.0
if kind == "pre":
    spacer(gib)
demes = []
for d in range(2 if kind == "sep" else 1):
    s = RandomStream(1234, island=d)
    p = tools.initPopulation(n=n, dim=1000, low=-5.12, high=5.12, gtype="f64", weights=(-1.0,),
                             stream=s)
    if kind == "mid":
        spacer(gib)
    o = p.like(n, capacity=n)
    benchmarks.rastrigin(p)
    demes.append((p, o, s, algorithms.GenerationStep(p, tb, 0.5, 0.2)))
if kind == "post":
    spacer(gib)
ctx = demes[0][0].ctx.bind()
out = {"mode": mode}
for d, (p, o, s, step) in enumerate(demes):
    for _ in range(3):
        step.step(p, o, s)
        p.swap_storage(o)
    _lib.call("dm_ctx_set_timing", ctx, G)
    for _ in range(G):
        step.step(p, o, s)
        p.swap_storage(o)
    torch.cuda.synchronize()
    times = (ctypes.c_float * G)()
    cnt = ctypes.c_int32(0)
    _lib.call("dm_ctx_kernel_times", ctx, times, G, ctypes.byref(cnt))
    _lib.call("dm_ctx_set_timing", ctx, 0)
    out["pair%d_ms" % d] = round(sum(times) / G, 4)
    out["pair%d_ptrs" % d] = [hex(p.genes.data_ptr()), hex(o.genes.data_ptr())]
print(json.dumps(out), flush=True)

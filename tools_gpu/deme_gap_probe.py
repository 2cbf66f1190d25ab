"""Probe (not a test): why C4's per-deme gen_pipe_kernel runs faster than C3's
(2.638 vs 2.922 ms on one box, profiles/r04fin6).

  python tools_gpu/deme_gap_probe.py DEMES GENS

Allocates DEMES 2^20 Rastrigin-1000D demes exactly as bench.py does (every
parent population first, then every child buffer), then runs phases and
prints the mean generation-kernel time (library HIP events) per deme and
phase:
  rr      every deme in turn per generation (bench.py's C4 loop)
  alone:d deme d only, GENS generations back to back (C3's loop on d's buffers)
  rr      again (drift check)
The plan/order kernels run in every phase exactly as in the bench."""
import ctypes
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from deap_amd import _lib, algorithms, base, benchmarks, tools  # noqa: E402
from deap_amd.ops import RandomStream  # noqa: E402

ndemes = int(sys.argv[1]) if len(sys.argv) > 1 else 8
G = int(sys.argv[2]) if len(sys.argv) > 2 else 20
n = 1 << 20
tb = base.Toolbox()
tb.register("evaluate", benchmarks.rastrigin)
tb.register("select", tools.selTournament, tournsize=3)
tb.register("mate", tools.cxBlend, alpha=0.5)
tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
streams = [RandomStream(1234, island=d) for d in range(ndemes)]
pops = [tools.initPopulation(n=n, dim=1000, low=-5.12, high=5.12, gtype="f64", weights=(-1.0,),
                             stream=s) for s in streams]
for p in pops:
    benchmarks.rastrigin(p)
steps = [algorithms.GenerationStep(p, tb, 0.5, 0.2) for p in pops]
offs = [p.like(n, capacity=n) for p in pops]
ctx = pops[0].ctx.bind()


def run(seq):
    """Launch one generation per entry of seq (deme ids); per-launch ms."""
    _lib.call("dm_ctx_set_timing", ctx, len(seq))
    t0 = time.perf_counter()
    for d in seq:
        steps[d].step(pops[d], offs[d], streams[d])
        pops[d].swap_storage(offs[d])
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e3 / len(seq)
    times = (ctypes.c_float * len(seq))()
    cnt = ctypes.c_int32(0)
    _lib.call("dm_ctx_kernel_times", ctx, times, len(seq), ctypes.byref(cnt))
    _lib.call("dm_ctx_set_timing", ctx, 0)
    assert cnt.value == len(seq)
    return list(times), wall


def report(name, seq, times, wall):
    per = {}
    for d, t in zip(seq, times):
        per.setdefault(d, []).append(t)
    row = {"phase": name, "wall_ms_per_launch": round(wall, 4),
           "kernel_ms": {str(d): round(sum(v) / len(v), 4) for d, v in sorted(per.items())},
           "genes_ptr": {str(d): hex(pops[d].genes.data_ptr()) for d in sorted(per)}}
    print(json.dumps(row), flush=True)


run([d for _ in range(3) for d in range(ndemes)])  # warm-up
phases = [("rr", [d for _ in range(G) for d in range(ndemes)])]
for d in sorted({0, 1, ndemes - 1}):
    if d < ndemes:
        phases.append(("alone:%d" % d, [d] * G))
phases.append(("rr", [d for _ in range(G) for d in range(ndemes)]))
for name, seq in phases:
    t, w = run(seq)
    report(name, seq, t, w)

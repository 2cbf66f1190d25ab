"""Probe (not a test): per-channel HBM request counters of the C3 hot kernel
on demes whose buffers run fast and slow.

    rocprofv3 -E tools_gpu/tcc_channels.yaml --pmc DM_RD_CH0 ... \
        --kernel-include-regex gen_pipe -- python3 tools_gpu/placement_pmc_probe.py DEMES GENS

Allocates DEMES 2^20 Rastrigin-1000D demes as bench.py does (every parent
population, then every child buffer), warms up, then runs GENS round-robin
generations (deme 0, 1, ..., DEMES - 1 per generation).  The hot kernel's
dispatch k of the timed phase belongs to deme k % DEMES; the probe prints the
library-timed kernel ms per deme so the fast and slow demes of this process
are known beside the counters."""
import ctypes
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from deap_amd import _lib, algorithms, base, benchmarks, tools  # noqa: E402
from deap_amd.ops import RandomStream  # noqa: E402

ndemes = int(sys.argv[1]) if len(sys.argv) > 1 else 4
G = int(sys.argv[2]) if len(sys.argv) > 2 else 4
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
seq = [d for _ in range(G) for d in range(ndemes)]
warm = [d for _ in range(2) for d in range(ndemes)]
for d in warm:
    steps[d].step(pops[d], offs[d], streams[d])
    pops[d].swap_storage(offs[d])
torch.cuda.synchronize()
_lib.call("dm_ctx_set_timing", ctx, len(seq))
for d in seq:
    steps[d].step(pops[d], offs[d], streams[d])
    pops[d].swap_storage(offs[d])
torch.cuda.synchronize()
times = (ctypes.c_float * len(seq))()
cnt = ctypes.c_int32(0)
_lib.call("dm_ctx_kernel_times", ctx, times, len(seq), ctypes.byref(cnt))
per = {}
for d, t in zip(seq, times):
    per.setdefault(d, []).append(t)
print(json.dumps({"warm_dispatches": len(warm), "timed_dispatches": len(seq), "demes": ndemes,
                  "kernel_ms": {str(d): round(sum(v) / len(v), 4) for d, v in sorted(per.items())},
                  "parent_ptr": {str(d): hex(pops[d].genes.data_ptr()) for d in range(ndemes)},
                  "child_ptr": {str(d): hex(offs[d].genes.data_ptr()) for d in range(ndemes)}}),
      flush=True)

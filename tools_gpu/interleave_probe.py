"""Probe (not a test): does the C3 generation kernel of a 2^20 deme run faster
when another deme's generation runs between two of its generations?  Modes:
'alone' (one deme), 'tiny' (a 2^12 deme interleaved), 'big' (a second 2^20
deme interleaved).  Prints the big deme's mean kernel time (library HIP events)."""
import ctypes
import sys
import torch
sys.path.insert(0, ".")
from deap_amd import _lib, algorithms, base, benchmarks, tools
from deap_amd.ops import RandomStream

mode = sys.argv[1]
tb = base.Toolbox()
tb.register("evaluate", benchmarks.rastrigin)
tb.register("select", tools.selTournament, tournsize=3)
tb.register("mate", tools.cxBlend, alpha=0.5)
tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
sizes = {"alone": [1 << 20], "tiny": [1 << 20, 1 << 12], "big": [1 << 20, 1 << 20],
         "pad": [1 << 20], "many": [1 << 20] * 4, "bigrev": [1 << 20, 1 << 20],
         "isl": [1 << 20], "seed": [1 << 20], "swap": [1 << 20, 1 << 20],
         "swapoff": [1 << 20, 1 << 20], "realloc": [1 << 20], "realloc1g": [1 << 20], "dummy": [1 << 20]}[mode]
if mode == "dummy":  # an unused population (and its offspring buffer) allocated first
    _st = RandomStream(3, island=9)
    _d = tools.initPopulation(n=int(float(sys.argv[2])) if len(sys.argv) > 2 else 1 << 20, dim=1000,
                              low=-1, high=1, gtype="f64", weights=(-1.0,), stream=_st)
    _d2 = _d.like(len(_d), capacity=_d.capacity)
order = [1, 0] if mode == "bigrev" else None
if mode == "pad":  # a dummy allocation first: does the placement of the buffers matter?
    _pad = torch.empty((int(float(sys.argv[2])) if len(sys.argv) > 2 else 17 << 30,),
                       dtype=torch.uint8, device="cuda")
    if len(sys.argv) > 3 and sys.argv[3] == "free":
        del _pad
pops, offs, steps, streams = [], [], [], []
for i, n in enumerate(sizes):
    st = RandomStream(int(sys.argv[3]) if mode == "seed" else 9,
                      island=int(sys.argv[2]) if mode in ("isl", "seed") else i)
    p = tools.initPopulation(n=n, dim=1000, low=-5.12, high=5.12, gtype="f64", weights=(-1.0,), stream=st)
    benchmarks.rastrigin(p)
    pops.append(p); offs.append(p.like(n, capacity=n)); streams.append(st)
    steps.append(algorithms.GenerationStep(p, tb, 0.5, 0.2))
if mode in ("realloc", "realloc1g"):  # genome buffers allocated back to back (rounded up to 1 GiB)
    for p in (pops[0], offs[0]):
        nb = p.genes.numel()
        if mode == "realloc1g":
            nb = (nb + (1 << 30) - 1) >> 30 << 30
        t = torch.empty((nb,), dtype=torch.uint8, device=p.device)
        t[: p.genes.numel()].copy_(p.genes.view(-1))
        p.genes = t[: p.genes.numel()].view(p.genes.shape)
    torch.cuda.synchronize()
if mode == "swap":  # deme 0 runs on deme 1's buffers and vice versa
    pops[0].swap_storage(pops[1])
    offs[0].swap_storage(offs[1])
if mode == "swapoff":  # only the offspring buffers exchanged
    offs[0].swap_storage(offs[1])
nev = torch.zeros(64, dtype=torch.int64, device=pops[0].device)
ctx = pops[0].ctx.bind()
for g in range(3):
    for i in range(len(pops)):
        steps[i].step(pops[i], offs[i], streams[i], ctypes.c_void_p(nev.data_ptr()))
        pops[i].swap_storage(offs[i])
torch.cuda.synchronize()
G = 20
_lib.call("dm_ctx_set_timing", ctx, G * len(pops))
for g in range(G):
    for i in (order or range(len(pops))):
        steps[i].step(pops[i], offs[i], streams[i], ctypes.c_void_p(nev.data_ptr()))
        pops[i].swap_storage(offs[i])
torch.cuda.synchronize()
n_l = G * len(pops)
times = (ctypes.c_float * n_l)()
cnt = ctypes.c_int32(0)
_lib.call("dm_ctx_kernel_times", ctx, times, n_l, ctypes.byref(cnt))
seq = order or list(range(len(pops)))
for d in range(len(pops)):
    t = [times[j] for j in range(cnt.value) if seq[j % len(pops)] == d]
    print("%s: deme %d (n=%d) kernel %.4f ms (%d launches)" % (mode, d, sizes[d], sum(t) / len(t), len(t)))
for d, p in enumerate(pops):
    print("   deme %d genes at 0x%x, offspring at 0x%x" % (d, p.genes.data_ptr(), offs[d].genes.data_ptr()))

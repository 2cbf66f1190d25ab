"""Probe (not a test): the C3 generation kernel's speed against how its genome
buffers are allocated (the same kernel took 3.18 ms on
deme 0's buffers and 2.76-2.84 ms on demes 1-3's).

  python tools_gpu/alloc_probe.py MODE DEMES
MODE: torch   — PyTorch caching allocator (what DevicePopulation does)
      raw     — one hipMalloc per genome buffer
      contig  — hipExtMallocWithFlags(hipDeviceMallocContiguous) per buffer
      arena   — ONE hipMalloc holding every genome buffer, 2 MiB aligned
      pair    — per deme ONE hipMalloc for both genome buffers, the child
                buffer argv[4] bytes past the parent buffer's 2 MiB-rounded end
Prints each deme's mean kernel time (library HIP events) and the addresses."""
import ctypes
import sys

import torch

sys.path.insert(0, ".")
from deap_amd import _lib, algorithms, base, benchmarks, tools  # noqa: E402
from deap_amd.ops import RandomStream  # noqa: E402

mode = sys.argv[1]
ndemes = int(sys.argv[2]) if len(sys.argv) > 2 else 1
G = int(sys.argv[3]) if len(sys.argv) > 3 else 20
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                      ctypes.c_uint]


class Raw:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1",
                                         "data": (ptr, False), "version": 2}


def hip_alloc(nbytes, flags=None):
    p = ctypes.c_void_p()
    rc = hip.hipMalloc(ctypes.byref(p), nbytes) if flags is None else \
        hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, flags)
    assert rc == 0, "allocation failed rc=%d" % rc
    return p.value


tb = base.Toolbox()
tb.register("evaluate", benchmarks.rastrigin)
tb.register("select", tools.selTournament, tournsize=3)
tb.register("mate", tools.cxBlend, alpha=0.5)
tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
n = 1 << 20
pops, offs, steps, streams = [], [], [], []
keep = []
arena = None
for i in range(ndemes):
    st = RandomStream(9, island=i)
    p = tools.initPopulation(n=n, dim=1000, low=-5.12, high=5.12, gtype="f64", weights=(-1.0,),
                             stream=st)
    o = p.like(n, capacity=n)
    if mode != "torch":
        nb = p.genes.numel()
        for q in (p, o):
            if mode == "raw":
                ptr = hip_alloc(nb)
            elif mode == "contig":
                ptr = hip_alloc(nb, 0x4)
            elif mode == "pair":
                # both genome buffers of the deme in ONE allocation, the child
                # buffer DELTA bytes past the 2 MiB-rounded end of the parent
                # buffer (argv[4], default 0)
                if q is p:
                    delta = int(float(sys.argv[4])) if len(sys.argv) > 4 else 0
                    per = (nb + (2 << 20) - 1) // (2 << 20) * (2 << 20)
                    b0 = hip_alloc(2 * per + delta + (2 << 20))
                    b0 = (b0 + (2 << 20) - 1) // (2 << 20) * (2 << 20)
                    ptr = b0
                else:
                    ptr = b0 + per + delta
            elif mode == "arena":
                if arena is None:
                    per = (nb + (2 << 20) - 1) // (2 << 20) * (2 << 20)
                    arena = [hip_alloc(per * 2 * ndemes + (2 << 20)), 0, per]
                    arena[0] = (arena[0] + (2 << 20) - 1) // (2 << 20) * (2 << 20)
                ptr = arena[0] + arena[1] * arena[2]
                arena[1] += 1
            else:
                raise SystemExit("unknown mode " + mode)
            t = torch.as_tensor(Raw(ptr, nb), device=p.device)
            t.copy_(q.genes.view(-1))
            keep.append(t)
            q.genes = t.view(q.genes.shape)
        torch.cuda.synchronize()
    benchmarks.rastrigin(p)
    pops.append(p)
    offs.append(o)
    streams.append(st)
    steps.append(algorithms.GenerationStep(p, tb, 0.5, 0.2))
nev = torch.zeros(64, dtype=torch.int64, device=pops[0].device)
ctx = pops[0].ctx.bind()
for g in range(3):
    for i in range(ndemes):
        steps[i].step(pops[i], offs[i], streams[i], ctypes.c_void_p(nev.data_ptr()))
        pops[i].swap_storage(offs[i])
torch.cuda.synchronize()
_lib.call("dm_ctx_set_timing", ctx, G * ndemes)
for g in range(G):
    for i in range(ndemes):
        steps[i].step(pops[i], offs[i], streams[i], ctypes.c_void_p(nev.data_ptr()))
        pops[i].swap_storage(offs[i])
torch.cuda.synchronize()
nl = G * ndemes
times = (ctypes.c_float * nl)()
cnt = ctypes.c_int32(0)
_lib.call("dm_ctx_kernel_times", ctx, times, nl, ctypes.byref(cnt))
for d in range(ndemes):
    t = [times[j] for j in range(cnt.value) if j % ndemes == d]
    even = [t[j] for j in range(0, len(t), 2)]
    odd = [t[j] for j in range(1, len(t), 2)]
    print("%s: deme %d kernel %.4f ms (A->B %.4f, B->A %.4f)  genes 0x%x / 0x%x" % (
        mode, d, sum(t) / len(t), sum(even) / len(even), sum(odd) / len(odd),
        pops[d].genes.data_ptr(), offs[d].genes.data_ptr()), flush=True)

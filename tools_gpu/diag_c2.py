"""Diagnostic (not a test): native packed-bit hot kernel vs the dump-mode
replay kernel on one generation; prints which children differ (by child % 8,
i.e. by lane of the fused kernel) and whether parents / flags explain it."""
import ctypes
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from deap_amd import algorithms, base, benchmarks, tools
from deap_amd.ops import RandomStream

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
dim = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
stream = RandomStream(1234)
pop = tools.initPopulation(n=n, dim=dim, low=0, high=1, gtype="bits", weights=(1.0,), stream=stream)
benchmarks.onemax(pop)
tb = base.Toolbox()
tb.register("evaluate", benchmarks.onemax)
tb.register("select", tools.selTournament, tournsize=3)
tb.register("mate", tools.cxTwoPoint)
tb.register("mutate", tools.mutFlipBit, indpb=0.05)
step = algorithms.GenerationStep(pop, tb, 0.5, 0.2)
nev = torch.zeros(2, dtype=torch.int64, device=pop.device)
state = stream.getstate()
nat = pop.like(n, capacity=n)
step.step(pop, nat, stream, ctypes.c_void_p(nev.data_ptr()))
stream.setstate(state)
dmp = pop.like(n, capacity=n)
decs = []
step.step(pop, dmp, stream, ctypes.c_void_p(nev.data_ptr() + 8), mode="dump", decisions=decs)
torch.cuda.synchronize()
words = (dim + 63) // 64
gn = nat.genes[:n, :words * 8].cpu().numpy()
gd = dmp.genes[:n, :words * 8].cpu().numpy()
bad = np.nonzero((gn != gd).any(1))[0]
print("nevals native/dump", nev.cpu().tolist())
print("differing children: %d of %d" % (len(bad), n))
if len(bad):
    print("by child %% 8:", np.bincount(bad % 8, minlength=8).tolist())
    print("first:", bad[:20].tolist())
    d = decs[0]
    asp = d.aspirants.cpu().numpy().reshape(n, -1)
    cxf = d.cx_flag.cpu().numpy()
    mf = d.mut_flag.cpu().numpy()
    pg = pop.genes[:n, :words * 8].cpu().numpy()
    wv = pop.wvalues[:n, 0].cpu().numpy()
    for c in bad[:8]:
        a = asp[c]
        win = a[0]
        for x in a[1:]:
            if not (wv[x] <= wv[win]):
                win = x
        match = [int(r) for r in np.nonzero((pg == gn[c]).all(1))[0][:3]]
        print("child", c, "asp", a.tolist(), "winner", int(win), "cx", int(cxf[c // 2]),
              "mut", int(mf[c]), "native row equals parent rows", match)
wn = nat.wvalues[:n, 0].cpu().numpy()
wd = dmp.wvalues[:n, 0].cpu().numpy()
print("fitness differs:", int((wn != wd).sum()))
# crossed pairs without mutation: the cut slice the native child implies
if len(bad):
    cxr = d.cx_raw.cpu().numpy().reshape(-1, 2) if d.cx_raw is not None else None
    shown = 0
    for c in bad:
        p = c // 2
        if c % 2 or not cxf[p] or mf[2 * p] or mf[2 * p + 1]:
            continue
        a0, a1 = asp[2 * p], asp[2 * p + 1]
        w0 = a0[0]
        for x in a0[1:]:
            if not (wv[x] <= wv[w0]):
                w0 = x
        bits_par = np.unpackbits(pg[w0].view(np.uint8), bitorder="little")[:dim]
        bits_nat = np.unpackbits(gn[c].view(np.uint8), bitorder="little")[:dim]
        diff = np.nonzero(bits_par != bits_nat)[0]
        r1, r2 = cxr[p]
        if r2 >= r1:
            r2 += 1
        else:
            r1, r2 = r2, r1
        print("pair", p, "dump slice [%d,%d)" % (r1, r2), "native differs from parent0 at",
              (int(diff.min()), int(diff.max())) if len(diff) else None, "p%%8", p % 8)
        shown += 1
        if shown >= 10:
            break

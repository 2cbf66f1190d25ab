"""Per-launch phase clocks of the front chain (peel_order_kernel; diagnostic
library built with -DDM_PEEL_PROF, via DEAPMI_LIB), round 6: the chunk (peel)
workgroups AND the search workgroups of every launch, so the per-front floor
can be split into the launch gap, the state read, the member / search work,
the release and the last search workgroup's sort.  Input as
peel_phase_probe.py (``c5``: the C5 bench's own selection input).  Times in
us from wall_clock64 (100 MHz)."""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from deap_amd import tools, _lib
from deap_amd.device import DevicePopulation
m = 3
n = 1 << 18
if len(sys.argv) > 1 and sys.argv[1] == "c5":
    # the C5 bench's own selection input: 2^17 DTLZ2 individuals after a few
    # eaMuPlusLambda generations plus one varOr batch (bench.py bench_nsga2)
    from deap_amd import algorithms, base, benchmarks
    from deap_amd.ops import RandomStream
    half = n // 2
    stream = RandomStream(1234)
    p0 = tools.initPopulation(n=half, dim=12, low=0.0, high=1.0, gtype="f64",
                              weights=(-1.0,) * m, stream=stream)
    tb = base.Toolbox()
    tb.register("evaluate", benchmarks.dtlz2, obj=m)
    tb.register("mate", tools.cxBlend, alpha=0.5)
    tb.register("mutate", tools.mutGaussian, mu=0, sigma=0.1, indpb=1.0 / 12)
    tb.register("select", tools.selNSGA2)
    benchmarks.dtlz2(p0, obj=m)
    step = algorithms.MuPlusLambdaStep(p0, tb, half, half, 0.6, 0.3)
    for _ in range(int(sys.argv[2]) if len(sys.argv) > 2 else 12):
        step.step(stream)
    comb = step.combined
    off = algorithms.varOr(comb, tb, half, 0.6, 0.3, evaluate=True, stream=stream)
    wv = np.concatenate([comb.wvalues[:half].cpu().numpy(), off.wvalues[:half].cpu().numpy()])
else:
    rng = np.random.default_rng(103)
    d = np.abs(rng.normal(size=(n, m)))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    wv = -(d * (1.0 + rng.exponential(0.3, size=(n, 1))))
pop = DevicePopulation.from_numpy(np.zeros((n, 1)), weights=(-1.0,) * m, gtype="f64", wvalues=wv,
                                  valid=np.ones(n))
lib = ctypes.CDLL(_lib.LIB_PATH)
fn = lib.dm_debug_peel_prof
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_int64]
buf = np.zeros((1 << 17, 8), np.uint64)
ctx = pop.ctx.bind()
cap = 1024
stamps = []
for rep in range(3):
    if rep == 2:  # the last selection also timed per peel launch by library events
        _lib.call("dm_ctx_set_timing_target", ctx, _lib.DM_TIME_PEEL)
        _lib.call("dm_ctx_set_timing", ctx, cap)
    tools.selNSGA2(pop, n // 2)
    torch.cuda.synchronize()
    k = fn(buf.ctypes.data, 1 << 17)
    stamps.append(buf[:k].copy())
times = (ctypes.c_float * cap)()
cnt = ctypes.c_int32(0)
_lib.call("dm_ctx_kernel_times", ctx, times, cap, ctypes.byref(cnt))
_lib.call("dm_ctx_set_timing", ctx, 0)
ev_us = [t * 1e3 for t in times[:cnt.value]]
# stamps of selection 1 (no per-launch events: the bench's timed steps record
# none); selection 2 ran with an event pair around every launch
a = stamps[1].astype(np.int64)
kind = a[:, 7] & 0xFF
jj = a[:, 7] >> 8
rows = []
prev_end = None
print("  j  front  peelWG  gap   peel:pro  mem  rel  end | srch:state  search  arrive->sort  end | span  event")
for j in sorted(set(jj.tolist())):
    P = a[(jj == j) & (kind == 0)]
    S = a[(jj == j) & (kind != 0)]
    allr = np.concatenate([P, S]) if len(S) else P
    t0 = allr[:, 3].min()
    us = lambda x: (x - t0) / 100.0
    gap = (t0 - prev_end) / 100.0 if prev_end is not None else float("nan")
    end = allr[:, 6].max()
    prev_end = end
    n = int(P[0, 2]) if len(P) else (int(S[0, 2]) if len(S) else 0)
    pro = ((P[:, 4] - P[:, 3]) / 100.0).max() if len(P) else 0
    mem = ((P[:, 5] - P[:, 4]) / 100.0).max() if len(P) else 0
    rel = ((P[:, 6] - P[:, 5]) / 100.0).max() if len(P) else 0
    pend = us(P[:, 6].max()) if len(P) else 0
    if len(S):
        st = ((S[:, 4] - S[:, 3]) / 100.0).max()
        se = ((S[:, 5] - S[:, 4]) / 100.0).max()
        L = S[(S[:, 7] & 2) != 0]
        srt = ((L[:, 6] - L[:, 5]) / 100.0).max() if len(L) else float("nan")
        send = us(S[:, 6].max())
    else:
        st = se = srt = send = float("nan")
    span = us(end)
    ev = ev_us[len(rows)] if len(rows) < len(ev_us) else float("nan")
    rows.append(dict(j=j, n=n, peel_wgs=len(P), gap=gap, pro=pro, mem=mem, rel=rel, peel_end=pend,
                     state=st, search=se, sort=srt, search_end=send, span=span, event=ev))
    print("%3d %6d %6d %5.1f   %6.1f %5.1f %4.1f %5.1f | %6.1f %7.1f %8.1f %6.1f | %5.1f %6.1f" % (
        j, n, len(P), gap, pro, mem, rel, pend, st, se, srt, send, span, ev))
small = [r for r in rows if r["n"] < 500]
if small:
    keys = ("gap", "pro", "mem", "rel", "peel_end", "state", "search", "sort", "search_end", "span", "event")
    print("fronts < 500 members (%d launches), means:" % len(small))
    print("  " + "  ".join("%s %.1f" % (k_, np.nanmean([r[k_] for r in small])) for k_ in keys))
import json
json.dump(rows, open(sys.argv[3] if len(sys.argv) > 3 else "/tmp/peel_phase2.json", "w"))
b2 = stamps[2].astype(np.int64)
jb = b2[:, 7] >> 8
gaps, prev = [], None
for j in sorted(set(jb.tolist())):
    g = b2[jb == j]
    if prev is not None:
        gaps.append((g[:, 3].min() - prev) / 100.0)
    prev = g[:, 6].max()
print("with per-launch events (selection 2): mean launch gap %.1f us over %d launches" %
      (float(np.mean(gaps)), len(gaps)))

"""Phase clocks of the table peel (diagnostic library built with
-DDM_PEEL_PROF, via DEAPMI_LIB): one fixed-input selNSGA2 at 2^18 -> 2^17
(DTLZ2-shaped, as c5_dom_probe.py), then per peel launch: F, workgroups,
launch span and the slowest workgroup's prologue / member / release times
(wall_clock64 ticks at 100 MHz)."""
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
for rep in range(3):
    if rep == 2:  # the last selection also timed per peel launch by library events
        _lib.call("dm_ctx_set_timing_target", ctx, _lib.DM_TIME_PEEL)
        _lib.call("dm_ctx_set_timing", ctx, cap)
    tools.selNSGA2(pop, n // 2)
    torch.cuda.synchronize()
    k = fn(buf.ctypes.data, 1 << 17)
times = (ctypes.c_float * cap)()
cnt = ctypes.c_int32(0)
_lib.call("dm_ctx_kernel_times", ctx, times, cap, ctypes.byref(cnt))
_lib.call("dm_ctx_set_timing", ctx, 0)
ev_us = [t * 1e3 for t in times[:cnt.value]]
a = buf[:k].astype(np.int64)
# launches: a new launch starts when F changes or the start clock jumps
order = np.argsort(a[:, 3], kind="stable")
a = a[order]
cut = np.flatnonzero(np.diff(a[:, 3]) > 300) + 1  # > 3 us gap between workgroup starts
tot = 0.0
print("launch  F  wgs  span_us  max(pro) max(mem) max(rel)  mean(mem) mean(rel)  event_us  [us]")
for i, g in enumerate(np.split(a, cut)):
    span = (g[:, 6].max() - g[:, 3].min()) / 100.0
    pro = (g[:, 4] - g[:, 3]) / 100.0
    mem = (g[:, 5] - g[:, 4]) / 100.0
    rel = (g[:, 6] - g[:, 5]) / 100.0
    tot += span
    print("%3d %6d %5d %7.1f %7.1f %7.1f %7.1f %7.1f %7.1f %7.1f" % (i, g[0, 2], len(g), span, pro.max(),
          mem.max(), rel.max(), mem.mean(), rel.mean(), ev_us[i] if i < len(ev_us) else -1))
print("sum of spans %.1f us over %d launches" % (tot, len(cut) + 1))

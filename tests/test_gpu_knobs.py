"""Every tuning switch the library reads from the environment (csrc/capi.hip
read_knobs, dm_knobs in csrc/common.hpp) selects between bit-identical
kernels: each one is run here against the default on the same input and
stream state.  The C3 plan-order switches are covered by
test_gpu_fullsize.py::test_plan_orders_give_identical_children.

* generation switches at the benched size (2^20, C3 / C2): the children's
  genomes, fitness, validity and nevals are equal;
* grouping switches (DM_LEX_FULL, DM_LEX_NO32) on the near-clone NSGA-II
  populations of test_gpu_parity.py: fronts and the selNSGA2 choice equal
  the oracle (deap/tools/emo.py:15-117);
* DM_SELBEST_FULLSORT: selBest / selWorst equal the stable sort
  (deap/tools/selection.py:38-52)."""
import contextlib
import ctypes
import os

import numpy as np
import pytest

from oracle import ops

pytestmark = pytest.mark.gpu

N = 1 << 20


@contextlib.contextmanager
def knob(ctx, setting):
    """``NAME`` or ``NAME=VALUE`` set in the environment and re-read by the
    context (dm_ctx_reload_knobs), restored afterwards."""
    from deap_amd import _lib
    name, _, val = setting.partition("=")
    old = os.environ.get(name)
    os.environ[name] = val or "1"
    try:
        _lib.call("dm_ctx_reload_knobs", ctx)
        yield
    finally:
        if old is None:
            del os.environ[name]
        else:
            os.environ[name] = old
        _lib.call("dm_ctx_reload_knobs", ctx)


def _generation_pair(cfg, setting):
    """One generation from the same parents and stream state with the default
    kernels and with ``setting``: (default children, knob children, nevals)."""
    import torch
    from deap_amd import algorithms, base, benchmarks, tools
    from deap_amd.ops import RandomStream
    if cfg == "c3":
        gt, dim, obj, w, lo, hi = "f64", 1000, "rastrigin", (-1.0,), -5.12, 5.12
    else:
        gt, dim, obj, w, lo, hi = "bits", 4096, "onemax", (1.0,), 0, 1
    stream = RandomStream(4321)
    pop = tools.initPopulation(n=N, dim=dim, low=lo, high=hi, gtype=gt, weights=w, stream=stream)
    getattr(benchmarks, obj)(pop)
    tb = base.Toolbox()
    tb.register("evaluate", getattr(benchmarks, obj))
    tb.register("select", tools.selTournament, tournsize=3)
    if cfg == "c3":
        tb.register("mate", tools.cxBlend, alpha=0.5)
        tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
    else:
        tb.register("mate", tools.cxTwoPoint)
        tb.register("mutate", tools.mutFlipBit, indpb=0.05)
    step = algorithms.GenerationStep(pop, tb, 0.5, 0.2)
    nev = torch.zeros(2, dtype=torch.int64, device=pop.device)
    state = stream.getstate()
    ref = pop.like(N, capacity=N)
    step.step(pop, ref, stream, ctypes.c_void_p(nev.data_ptr()))
    other = pop.like(N, capacity=N)
    with knob(pop.ctx.bind(), setting):
        stream.setstate(state)
        step.step(pop, other, stream, ctypes.c_void_p(nev.data_ptr() + 8))
        torch.cuda.synchronize()
    return ref, other, nev.cpu().tolist()


@pytest.mark.parametrize("cfg,setting", [
    ("c3", "DM_DISABLE_PIPE"),      # general gen_float_kernel instead of the pipe
    ("c3", "DM_PIPE_BPC=64"),       # the pair-order grid on ordered plans
    ("c3", "DM_PIPE_BPC=8"),
    ("c2", "DM_DISABLE_PIPE"),      # general gen_bits_kernel instead of the fused one
    ("c2", "DM_BITS_PLAN"),         # plan kernel + burst kernel (t > 8's path)
    ("c2", "DM_BITS_NOKEYS"),       # tournaments on wvalues, no int16 keys
])
def test_generation_knobs_are_bit_identical(gpu, cfg, setting):
    """deap/algorithms.py:163-181 (one eaSimple generation): the switch picks a
    different kernel or grid for the same plans / Philox counters.  One
    exception to bit-identical fitness: C3 under DM_DISABLE_PIPE evaluates
    Rastrigin's cos(2 pi x) with the fdlibm-style cosine of the general
    kernel, the hot kernel with its LDS table (DESIGN.md §3 Numerics): the
    genomes are bit-identical, the fitness within north_star's 1e-12
    relative."""
    import torch
    ref, other, (a, b) = _generation_pair(cfg, setting)
    assert torch.equal(ref.genes[:N], other.genes[:N])
    if cfg == "c3" and setting == "DM_DISABLE_PIPE":
        x, y = ref.wvalues[:N].cpu().numpy(), other.wvalues[:N].cpu().numpy()
        assert np.all(np.abs(x - y) <= 1e-12 * np.maximum(1.0, np.abs(y)))
    else:
        assert torch.equal(ref.wvalues[:N], other.wvalues[:N])
    assert torch.equal(ref.valid[:N], other.valid[:N])
    assert a == b > 0


@pytest.mark.parametrize("setting", ["DM_LEX_FULL", "DM_LEX_NO32"])
@pytest.mark.parametrize("m", [2, 3, 4])
def test_grouping_knobs_match_the_oracle(gpu, setting, m):
    """The grouping's lexicographic order (nsga2.hip): the full sort
    (DM_LEX_FULL) and the whole-key objective-0 sort (DM_LEX_NO32) on
    near-clones a few ulps apart, fronts and choice equal to emo.py."""
    from deap_amd import tools
    from deap_amd.device import DevicePopulation
    from test_gpu_parity import _near_clone_fitness
    rng = np.random.default_rng(900 + m)
    wv = _near_clone_fitness(rng, m, 500, True, True)
    n = len(wv)
    w = (-1.0,) * m
    pop = DevicePopulation.from_numpy(np.zeros((n, 1)), weights=w, gtype="f64", wvalues=wv,
                                      valid=np.ones(n))
    with knob(pop.ctx.bind(), setting):
        fronts = [f.cpu().numpy().tolist() for f in tools.sortNondominated(pop, n)]
        chosen = tools.selNSGA2(pop, n // 2).cpu().numpy().tolist()
    assert fronts == ops.sort_nondominated(wv, n)
    assert chosen == ops.sel_nsga2(wv, w, n // 2)[0]


@pytest.mark.parametrize("k", [1, 64, 100])
def test_selbest_fullsort_knob(gpu, k):
    """DM_SELBEST_FULLSORT: selBest / selWorst by the full stable radix sort
    instead of the top-k bucket selection; both equal the stable sort with
    ties (selection.py:38-52)."""
    from deap_amd import tools
    from deap_amd.device import DevicePopulation
    rng = np.random.default_rng(k)
    n = 1 << 18
    wv = rng.integers(0, 5000, size=(n, 1)).astype(np.float64)  # many ties
    pop = DevicePopulation.from_numpy(np.zeros((n, 1)), weights=(1.0,), gtype="f64",
                                      wvalues=wv, valid=np.ones(n))
    with knob(pop.ctx.bind(), "DM_SELBEST_FULLSORT"):
        best = tools.selBest(pop, k).cpu().numpy().tolist()
        worst = tools.selWorst(pop, k).cpu().numpy().tolist()
    assert best == ops.sel_best(wv, k).tolist()
    assert worst == ops.sel_worst(wv, k).tolist()


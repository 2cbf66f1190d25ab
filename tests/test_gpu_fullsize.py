"""Parity of the BENCHED kernels at the BENCHED size (BASELINE.json configs C3
and C2: pop 2^20).  One generation of the native hot path (per-pair plan
kernel + gen_pipe_kernel / gen_bits_burst_kernel, 64 persistent workgroups
per CU, the row ring wrapping hundreds of times per wave) against one
generation of the dump-mode replay kernel from the same stream state: every
genome bit-exact, every fitness within 1e-12 relative (exact for OneMax),
the same `nevals`.  A random sample of 4,096 children is then replayed in the
CPU oracle (deap/algorithms.py:163-181 restated in oracle/ops.py) from the
dumped decisions and the parent rows."""
import numpy as np
import pytest

from oracle import ops

pytestmark = pytest.mark.gpu

N = 1 << 20


def _rel_close(a, b, tol):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= tol * np.maximum(1.0, np.abs(b)))


CASES = {
    "c3": ("f64", 1000, "blend", "gaussian", "rastrigin", (-1.0,), (-5.12, 5.12)),
    "c3r": ("f64", 1000, "blend", "gaussian", "rosenbrock", (-1.0,), (-2.048, 2.048)),
    "c2": ("bits", 4096, "twopoint", "flipbit", "onemax", (1.0,), (0, 1)),
}


@pytest.mark.parametrize("cfg", ["c3", "c2", "c3r"])
def test_benched_kernel_at_full_size(gpu, cfg):
    import ctypes
    import torch
    from deap_amd import algorithms, base, benchmarks, tools
    from deap_amd.ops import RandomStream
    gt, dim, cx, mut, obj, w, (low, high) = CASES[cfg]
    stream = RandomStream(1234)
    pop = tools.initPopulation(n=N, dim=dim, low=low, high=high, gtype=gt, weights=w,
                               stream=stream)
    getattr(benchmarks, obj)(pop)
    tb = base.Toolbox()
    tb.register("evaluate", getattr(benchmarks, obj))
    tb.register("select", tools.selTournament, tournsize=3)
    if cx == "blend":
        tb.register("mate", tools.cxBlend, alpha=0.5)
        tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
    else:
        tb.register("mate", tools.cxTwoPoint)
        tb.register("mutate", tools.mutFlipBit, indpb=0.05)
    step = algorithms.GenerationStep(pop, tb, 0.5, 0.2)
    nev = torch.zeros(2, dtype=torch.int64, device=pop.device)
    state = stream.getstate()
    native = pop.like(N, capacity=N)
    step.step(pop, native, stream, ctypes.c_void_p(nev.data_ptr()))
    stream.setstate(state)
    dumped = pop.like(N, capacity=N)
    decs = []
    step.step(pop, dumped, stream, ctypes.c_void_p(nev.data_ptr() + 8), mode="dump",
              decisions=decs)
    torch.cuda.synchronize()
    nbytes = (dim + 63) // 64 * 8 if gt == "bits" else dim * 8
    # bit-exact genomes over all 2^20 rows (compared as raw bytes on the device)
    assert torch.equal(native.genes[:N, :nbytes], dumped.genes[:N, :nbytes])
    assert bool(native.valid[:N].bool().all()) and bool(dumped.valid[:N].bool().all())
    wn, wd = native.wvalues[:N, 0], dumped.wvalues[:N, 0]
    if gt == "bits":
        assert torch.equal(wn, wd)
    else:
        assert bool((torch.abs(wn - wd) <= 1e-12 * torch.clamp(torch.abs(wd), min=1.0)).all())
    n_nat, n_dump = nev.cpu().tolist()
    assert n_nat == n_dump and 0.55 * N < n_nat < 0.65 * N  # 1-(1-cxpb)(1-mutpb) = 0.6

    # a random sample of 2,048 pairs replayed in the oracle
    d = decs[0]
    rng = np.random.default_rng(7)
    pairs = np.sort(rng.choice(N // 2, 2048, replace=False))
    ch = np.stack([2 * pairs, 2 * pairs + 1], 1).ravel()
    cht = torch.from_numpy(ch).to(pop.device)
    pt = torch.from_numpy(pairs).to(pop.device)
    asp = d.aspirants[cht].cpu().numpy()
    parent_wv = pop.wvalues[:N].cpu().numpy()
    winners = ops.sel_tournament(parent_wv, asp)
    g0, wv0, ok0 = pop.rows_numpy(winners.tolist())
    dec = {"cx_flag": d.cx_flag[pt].cpu().numpy().astype(bool),
           "mut_flag": d.mut_flag[cht].cpu().numpy().astype(bool),
           "mut_mask": ops.unpack_mask(d.mut_mask[cht].cpu().numpy().view(np.uint64), dim)}
    if cx == "blend":
        dec["blend_u"] = d.blend_u[pt].cpu().numpy()
        dec["gauss"] = d.gauss[cht].cpu().numpy()
    else:
        dec["cx_raw"] = d.cx_raw[pt].cpu().numpy()
    g, wv, ok = ops.var_and(g0, wv0, ok0, 0.5, 0.2, cx, mut, dec)
    inv = np.nonzero(~ok)[0]
    wv[inv] = ops.evaluate(g, obj, w, rows=inv)[inv]
    got_g, got_wv, _ = dumped.rows_numpy(ch.tolist())
    assert np.array_equal(got_g, g)
    assert _rel_close(got_wv, wv, 0 if gt == "bits" else 1e-12)
    assert (~ok).sum() > 1000  # the sample exercised crossover and mutation

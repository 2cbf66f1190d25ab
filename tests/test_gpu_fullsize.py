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


def _dp():
    from deap_amd.device import DevicePopulation
    return DevicePopulation


def _rel_close(a, b, tol):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= tol * np.maximum(1.0, np.abs(b)))


CASES = {
    "c3": ("f64", 1000, "blend", "gaussian", "rastrigin", (-1.0,), (-5.12, 5.12)),
    "c3r": ("f64", 1000, "blend", "gaussian", "rosenbrock", (-1.0,), (-2.048, 2.048)),
    "c2": ("bits", 4096, "twopoint", "flipbit", "onemax", (1.0,), (0, 1)),
    # round 6: the genome shapes bench.py measures beside the benched ones
    "c3d30": ("f64", 30, "blend", "gaussian", "rastrigin", (-1.0,), (-5.12, 5.12)),
    "c3f32": ("f32", 1000, "blend", "gaussian", "rastrigin", (-1.0,), (-5.12, 5.12)),
    "c3d2000": ("f64", 2000, "blend", "gaussian", "rastrigin", (-1.0,), (-5.12, 5.12)),
    "c2b8192": ("bits", 8192, "twopoint", "flipbit", "onemax", (1.0,), (0, 1)),
}


@pytest.mark.parametrize("cfg", ["c3", "c2", "c3r", "c3d30", "c3f32", "c3d2000", "c2b8192"])
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
    nbytes = (dim + 63) // 64 * 8 if gt == "bits" else dim * (4 if gt == "f32" else 8)
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


def _sphere_fitness(n, m, seed):
    """DTLZ2-shaped objective vectors: random directions on the positive unit
    sphere scaled by 1 + g, g >= 0 (the C5 population's fitness layout)."""
    rng = np.random.default_rng(seed)
    d = np.abs(rng.normal(size=(n, m)))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return d * (1.0 + rng.exponential(0.3, size=(n, 1)))


@pytest.mark.parametrize("m", [3, 2])
def test_sel_nsga2_at_full_size(gpu, m):
    """C5 at its benched size (selNSGA2 over 2N = 2^18 DTLZ2-shaped fitnesses
    -> N = 2^17, deap/tools/emo.py:15-50): the bitset dominance + table peel
    (default) against the fp64 ballot kernel (the DM_DOM_BALLOT cross-check
    path): the same fronts, chosen indices and crowding distances."""
    import torch
    from deap_amd import tools
    from deap_amd.device import dominance_path
    n = 1 << 18
    wv = -_sphere_fitness(n, m, 100 + m)  # minimisation: weights -1
    pop = _dp().from_numpy(np.zeros((n, 1)), weights=(-1.0,) * m, gtype="f64",
                           wvalues=wv, valid=np.ones(n))
    got = []
    for path in ("default", "ballot"):
        with dominance_path(path):
            fronts = [f.cpu().numpy() for f in tools.sortNondominated(pop, n // 2)]
            chosen = tools.selNSGA2(pop, n // 2).cpu().numpy()
        crowd = pop.crowding_dist[:n].cpu().numpy().copy()
        got.append((fronts, chosen, crowd))
    (f0, c0, d0), (f1, c1, d1) = got
    assert len(f0) == len(f1) > 5
    assert all(np.array_equal(a, b) for a, b in zip(f0, f1))
    assert np.array_equal(c0, c1)
    assert np.array_equal(d0[c0], d1[c1])
    torch.cuda.synchronize()


def test_sort_nondominated_objective0_ties(gpu):
    """Objective 0 takes 7 values only (most block pairs straddle a tie, the
    full-compare path), the others are continuous: fast path == LDS kernel."""
    from deap_amd import tools
    rng = np.random.default_rng(77)
    n = 40013
    wv = np.concatenate([rng.integers(0, 7, size=(n, 1)).astype(np.float64),
                         rng.uniform(0, 1, size=(n, 2))], 1)
    wv[rng.integers(0, n, 500)] = wv[rng.integers(0, n, 500)]  # duplicated fitnesses
    pop = _dp().from_numpy(np.zeros((n, 1)), weights=(1.0, -1.0, 1.0), gtype="f64",
                           wvalues=wv, valid=np.ones(n))
    from deap_amd.device import dominance_path
    fast = [f.cpu().numpy().tolist() for f in tools.sortNondominated(pop, n)]
    with dominance_path("lds"):
        ref = [f.cpu().numpy().tolist() for f in tools.sortNondominated(pop, n)]
    assert fast == ref
    assert sum(len(f) for f in fast) == n


def _shell_fitness(n, m, seed, levels=12):
    """Directions on the positive unit sphere scaled by one of a few radii:
    fronts of thousands of members (the member-slice peel path, >= 1,024
    members per 1,024-v segment)."""
    rng = np.random.default_rng(seed)
    d = np.abs(rng.normal(size=(n, m)))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    return d * (1.0 + 0.02 * rng.integers(0, levels, size=(n, 1)))


def _dup_shell_fitness(n, m, seed, levels=6):
    """Shells of ~n/levels unique members each (fronts of ~9,500 unique fits:
    the table peel splits every chunk's members into 2-4 slices, >= 2 x 2,048
    members), 5 % of the rows duplicates of other rows (equal fitnesses,
    emo.py:72-75 grouping)."""
    rng = np.random.default_rng(seed)
    wv = _shell_fitness(n, m, seed + 1, levels)
    wv[rng.integers(0, n, n // 20)] = wv[rng.integers(0, n, n // 20)]
    return wv


def _grid_fitness(n, m, seed):
    """Directions rounded to a 1/64 grid: duplicated fitnesses and equal
    crowding distances everywhere (ties at the selNSGA2 cut)."""
    return np.round(_sphere_fitness(n, m, seed) * 64.0) / 64.0


def _port_ranks(wv, fronts):
    """Pareto rank per unique fit (oracle.nsga2_closed order) from the port's
    log fronts (the ranks of the Fortin sort, emo.py:234-276); fits beyond
    the last front get one rank past it."""
    from oracle import nsga2_closed
    ufit, ui = nsga2_closed.unique_first_appearance(wv)
    urank = np.full(len(ufit), len(fronts), np.int64)
    for r, f in enumerate(fronts):
        urank[ui[np.asarray(f, np.int64)]] = r
    return urank, ui


def _check_standard_order(pop, wv, weights, k, ref_fronts):
    """The benched standard path against the closed form (SURVEY §8a-a21,
    oracle/nsga2_closed.py): every sortNondominated front equal IN ORDER, and
    the standard selNSGA2 chosen ORDER equal to emo.py:40-48 on those fronts
    (crowding by oracle.ops, the stable reverse sort of the last front, ties
    at the cut included); crowding distances bitwise."""
    from deap_amd import tools
    from oracle import nsga2_closed
    urank, ui = _port_ranks(wv, ref_fronts)
    want = nsga2_closed.sort_nondominated(wv, k, ranks=urank)
    got = [f.cpu().numpy() for f in tools.sortNondominated(pop, k)]
    assert [len(f) for f in got] == [len(f) for f in want]
    for i, (a, b) in enumerate(zip(got, want)):
        assert np.array_equal(a, b), "front %d differs from the closed form" % i
    want_c, want_crowd = nsga2_closed.sel_nsga2(wv, weights, k, fronts=want)
    chosen = tools.selNSGA2(pop, k).cpu().numpy()
    assert chosen.tolist() == want_c
    crowd = pop.crowding_dist[:len(wv)].cpu().numpy()
    assert np.array_equal(crowd[chosen], np.array([want_crowd[i] for i in want_c]))
    # the unique-fit sizes of the fronts (the table peel's slicing input)
    return [len(np.unique(ui[f])) for f in want], want, want_crowd


@pytest.mark.parametrize("n,m,kind", [(1 << 18, 3, "sphere"), (1 << 18, 2, "sphere"),
                                      (1 << 18, 4, "sphere"),
                                      (40000, 3, "shells"), (40000, 2, "shells"),
                                      (60000, 3, "dupshells"), (60000, 2, "dupshells"),
                                      (60000, 4, "dupshells"), (60000, 3, "grid")])
def test_nsga2_at_full_size_against_reference_port(gpu, n, m, kind):
    """C5 at its benched size against reference-pinned restatements (VERDICT
    r2 item 2, r3 item 1): ``oracle/deap_port.py``'s Fortin log sort and
    selNSGA2 (bit-exact with the reference on tests/golden/nsga2*.npz,
    test_support_port.py) and the closed form of the standard order
    (``oracle/nsga2_closed.py``, checked against oracle.ops and nsga2.npz in
    test_oracle.py) on the same 2N fitnesses (deap/tools/emo.py:15-117,
    234-276):

    * device ``sortLogNondominated`` fronts == the port's, member for member;
    * device ``selNSGA2(nd='log')`` chosen order == the port's;
    * every device ``sortNondominated`` front (bitset dominance + table peel,
      the benched path) == the closed form IN ORDER, with the ranks of the
      port's sort;
    * the standard ``selNSGA2`` chosen order == emo.py:40-48 on those fronts,
      ties at the cut included, crowding distances bitwise.

    M = 4 (DTLZ's free objective count, deap/benchmarks/__init__.py:495-521)
    takes the integer compare kernel + D-matrix peel: the
    same checks at 2^18 (34 fronts of up to ~22,000 members) and on the
    duplicated shells."""
    from deap_amd import tools
    from oracle import deap_port
    k = n // 2
    base = {"sphere": lambda: _sphere_fitness(n, m, 500 + m),
            "shells": lambda: _shell_fitness(n, m, 600 + m),
            "dupshells": lambda: _dup_shell_fitness(n, m, 700 + m),
            "grid": lambda: _grid_fitness(n, m, 800 + m)}[kind]
    wv = -base()
    weights = (-1.0,) * m
    pop = _dp().from_numpy(np.zeros((n, 1)), weights=weights, gtype="f64", wvalues=wv,
                           valid=np.ones(n))
    # the port on host individuals (row index kept by identity)
    inds = deap_port.nsga2_population(wv, weights)
    row = {id(ind): i for i, ind in enumerate(inds)}
    ref_chosen, ref_fronts = deap_port.sel_nsga2(inds, k, "log", return_fronts=True)
    ref_fronts = [[row[id(x)] for x in f] for f in ref_fronts]
    ref_chosen = [row[id(x)] for x in ref_chosen]
    ref_crowd = np.array([getattr(x.fitness, "crowding_dist", np.nan) for x in inds])
    # log sort: exact order
    got_log = [f.cpu().numpy().tolist() for f in tools.sortLogNondominated(pop, k)]
    assert [len(f) for f in got_log] == [len(f) for f in ref_fronts]
    assert got_log == ref_fronts
    assert tools.selNSGA2(pop, k, nd="log").cpu().numpy().tolist() == ref_chosen
    # standard sort (the benched path): exact order against the closed form
    usizes, want, want_crowd = _check_standard_order(pop, wv, weights, k, ref_fronts)
    # crowding of a front depends on its order only through duplicates: the
    # port's (log-order) distances agree on rows without an equal twin
    if kind == "shells":  # fronts of ~3,500 unique fits: one slice per chunk
        assert max(usizes) > 1024, usizes
    if kind == "dupshells" and m <= 3:  # >= 2 x 2,048: the table peel's member slices
        assert max(usizes) >= 8192, usizes
    if kind == "grid":
        last = want[-1]
        need = k - sum(len(f) for f in want[:-1])
        cut = np.sort([want_crowd[i] for i in last.tolist()])[::-1]
        assert 0 < need < len(last) and cut[need - 1] == cut[need], "no tie at the cut"


def test_nsga2_on_an_evolved_c5_population(gpu):
    """The C5 benched workload itself: 2^17 DTLZ2 (M=3, D=12) individuals after
    12 eaMuPlusLambda generations on the device (cxBlend of clones leaves
    near-clones and exact duplicates), plus one varOr batch -> 2N = 2^18
    (bench.py's stage breakdown input).  The standard sortNondominated /
    selNSGA2 on the device against the closed form with the port's ranks,
    every front in order and the chosen order (emo.py:15-117)."""
    import ctypes
    from deap_amd import _lib, algorithms, base, benchmarks, tools
    from deap_amd.ops import RandomStream
    from oracle import deap_port
    n, m, dim = 1 << 17, 3, 12
    stream = RandomStream(1234)
    pop = tools.initPopulation(n=n, dim=dim, low=0.0, high=1.0, gtype="f64",
                               weights=(-1.0,) * m, stream=stream)
    tb = base.Toolbox()
    tb.register("evaluate", benchmarks.dtlz2, obj=m)
    tb.register("mate", tools.cxBlend, alpha=0.5)
    tb.register("mutate", tools.mutGaussian, mu=0, sigma=0.1, indpb=1.0 / dim)
    tb.register("select", tools.selNSGA2)
    benchmarks.dtlz2(pop, obj=m)
    step = algorithms.MuPlusLambdaStep(pop, tb, n, n, 0.6, 0.3)
    for _ in range(12):
        step.step(stream)
    comb = step.combined
    two = pop.like(2 * n, capacity=2 * n)
    ctx = comb.ctx.bind()
    _lib.call("dm_gather", ctx, ctypes.byref(comb.c_pop()), None, ctypes.byref(two.c_pop(0, n)))
    off = algorithms.varOr(comb, tb, n, 0.6, 0.3, evaluate=True, stream=stream)
    _lib.call("dm_gather", ctx, ctypes.byref(off.c_pop()), None, ctypes.byref(two.c_pop(n, n)))
    wv = two.wvalues[:2 * n].cpu().numpy().copy()
    weights = (-1.0,) * m
    inds = deap_port.nsga2_population(wv, weights)
    row = {id(ind): i for i, ind in enumerate(inds)}
    ref_fronts = [[row[id(x)] for x in f] for f in deap_port.sort_log_nondominated(inds, n)]
    usizes, want, _ = _check_standard_order(two, wv, weights, n, ref_fronts)
    assert len(np.unique(wv, axis=0)) < 2 * n  # the population holds duplicates
    assert len(want) > 5


def _row_hashes(pop):
    """int64 hash of every genome row, computed on the device (test
    infrastructure: a wrapping multiply-add over the row's 64-bit words)."""
    import torch
    g = pop.genes[:len(pop)].view(torch.int64)
    rng = np.random.default_rng(1234)
    mult = torch.from_numpy(rng.integers(1, 2**62, size=g.shape[1], dtype=np.int64) | 1).to(g.device)
    out = torch.empty(g.shape[0], dtype=torch.int64, device=g.device)
    for a in range(0, g.shape[0], 1 << 16):
        out[a:a + (1 << 16)] = (g[a:a + (1 << 16)] * mult).sum(dim=1)
    return out.cpu().numpy()


def test_c4_migration_at_full_size(gpu):
    """C4 at its benched size: two demes of 2^20
    Rastrigin-1000D fp64 after one eaSimple generation each (clones of the
    tournament winners make equal genomes common), then migRing(k=15,
    selBest) along the ring 0 -> 1 -> 0 (deap/tools/migration.py:4-51).  The
    reference loop is replayed on the host over the full demes: for every
    immigrant, ``list.index`` = the FIRST row whose genome equals it in the
    deme as the earlier placements left it (candidate rows found through a
    hash of every row, each confirmed by an exact genome compare), then the
    emigrant replaces it.  The device result must equal that replay on every
    row (hashes of all 2^20 rows of both demes; placed rows' genomes and
    fitness bit for bit), and the emigrants must be a selBest of each deme."""
    import ctypes
    import torch
    from deap_amd import algorithms, base, benchmarks, tools
    from deap_amd.ops import RandomStream
    n, dim, k = N, 1000, 15
    tb = base.Toolbox()
    tb.register("evaluate", benchmarks.rastrigin)
    tb.register("mate", tools.cxBlend, alpha=0.5)
    tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
    tb.register("select", tools.selTournament, tournsize=3)
    demes = []
    for d in range(2):
        st = RandomStream(1234, island=d)
        p = tools.initPopulation(n=n, dim=dim, low=-5.12, high=5.12, gtype="f64", weights=(-1.0,),
                                 stream=st)
        benchmarks.rastrigin(p)
        off = p.like(n, capacity=n)
        nev = torch.zeros(1, dtype=torch.int64, device=p.device)
        algorithms.GenerationStep(p, tb, 0.5, 0.2).step(p, off, st, ctypes.c_void_p(nev.data_ptr()))
        p.swap_storage(off)
        del off
        demes.append(p)
    torch.cuda.synchronize()
    em = [tools.selBest(p, k).cpu().numpy().astype(np.int64) for p in demes]
    wv0 = [p.wvalues[:n, 0].cpu().numpy().copy() for p in demes]
    for d in range(2):  # selBest: the k largest weighted fitnesses (1e-12 tolerance)
        assert _rel_close(np.sort(wv0[d][em[d]])[::-1], np.sort(wv0[d])[::-1][:k], 1e-12)
    h0 = [_row_hashes(p) for p in demes]
    # host copies of every row a placement can touch: the emigrants and every
    # row sharing a hash with an immigrant
    need = [set(em[d].tolist()) | set(np.nonzero(np.isin(h0[d], h0[d][em[d]]))[0].tolist())
            for d in range(2)]
    rows = []
    for d in range(2):
        idx = sorted(need[d])
        g, w, _ = demes[d].rows_numpy(idx)
        rows.append({r: (g[i], w[i, 0]) for i, r in enumerate(idx)})
    # the reference loop (migarray [1, 0], immigrants = emigrants)
    cur_h = [h.copy() for h in h0]
    cur = [dict(r) for r in rows]  # row -> (genome, wvalue) as placements leave it
    placed = [[], []]
    for frm, to in enumerate([1, 0]):
        for j in range(k):
            target = rows[to][int(em[to][j])][0]
            slot = None
            for c in np.nonzero(cur_h[to] == h0[to][em[to][j]])[0]:
                if np.array_equal(cur[to][int(c)][0], target):
                    slot = int(c)
                    break
            assert slot is not None, "immigrant %d of deme %d not found" % (j, to)
            src = rows[frm][int(em[frm][j])]
            cur[to][slot] = src
            cur_h[to][slot] = h0[frm][em[frm][j]]
            placed[to].append((slot, src))
    rec = []
    tools.migRing(demes, k, tools.selBest, record=rec)
    assert all(np.array_equal(rec[0]["emigrants"][d], em[d]) for d in range(2))
    for d in range(2):
        assert np.array_equal(_row_hashes(demes[d]), cur_h[d]), "deme %d differs from the replay" % d
        slots = [s for s, _ in placed[d]]
        g, w, ok = demes[d].rows_numpy(slots)
        final = {}
        for s_, src in placed[d]:
            final[s_] = src  # a slot placed twice keeps the later emigrant
        for i, s_ in enumerate(slots):
            assert np.array_equal(g[i], final[s_][0]) and w[i, 0] == final[s_][1] and ok[i]


@pytest.mark.parametrize("knob", ["DM_PIPE_NOORDER", "DM_PIPE_LABEL_ROUNDS=0",
                                  "DM_PIPE_LABEL_ROUNDS=1", "DM_PIPE_LABEL_ROUNDS=3",
                                  "DM_PIPE_KEY_FITTER"])
def test_plan_orders_give_identical_children(gpu, knob):
    """The C3 hot kernel's plan order -- label-propagation bins (default),
    degree keys, fitter-parent keys, pair order -- only changes which pairs
    a workgroup varies together: every child is a function of its own plan
    and Philox counters, so one generation at 2^19 must be bit-identical under
    every order (genomes, fitness, nevals)."""
    import ctypes
    import os
    import torch
    from deap_amd import _lib, algorithms, base, benchmarks, tools
    from deap_amd.ops import RandomStream
    n = 1 << 19
    stream = RandomStream(99)
    pop = tools.initPopulation(n=n, dim=1000, low=-5.12, high=5.12, gtype="f64", weights=(-1.0,),
                               stream=stream)
    benchmarks.rastrigin(pop)
    tb = base.Toolbox()
    tb.register("evaluate", benchmarks.rastrigin)
    tb.register("select", tools.selTournament, tournsize=3)
    tb.register("mate", tools.cxBlend, alpha=0.5)
    tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=0.05)
    step = algorithms.GenerationStep(pop, tb, 0.5, 0.2)
    nev = torch.zeros(2, dtype=torch.int64, device=pop.device)
    state = stream.getstate()
    ref = pop.like(n, capacity=n)
    step.step(pop, ref, stream, ctypes.c_void_p(nev.data_ptr()))
    name, _, val = knob.partition("=")
    ctx = pop.ctx.bind()
    os.environ[name] = val or "1"
    try:
        _lib.call("dm_ctx_reload_knobs", ctx)
        stream.setstate(state)
        other = pop.like(n, capacity=n)
        step.step(pop, other, stream, ctypes.c_void_p(nev.data_ptr() + 8))
        torch.cuda.synchronize()
    finally:
        del os.environ[name]
        _lib.call("dm_ctx_reload_knobs", ctx)
    assert torch.equal(ref.genes[:n, :8000], other.genes[:n, :8000])  # 1,000 fp64 genes
    assert torch.equal(ref.wvalues[:n], other.wvalues[:n])
    assert torch.equal(ref.valid[:n], other.valid[:n])
    a, b = nev.cpu().tolist()
    assert a == b > 0

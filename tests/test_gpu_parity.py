"""GPU parity: every hot-path kernel against the golden vectors of the
reference and against the CPU oracle, through the C ABI (libdeapmi.so)."""
import ast
import ctypes
import functools

import numpy as np
import pytest

from conftest import golden
from oracle import ops, philox

pytestmark = pytest.mark.gpu


def _rel_close(a, b, tol):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return np.all(np.abs(a - b) <= tol * np.maximum(1.0, np.abs(b)))


def _dp():
    from deap_amd.device import DevicePopulation
    return DevicePopulation


def _toolbox(cx, mut, indpb=0.05, alpha=0.5, evaluate=None, select=None, tournsize=3, **ev_kw):
    from deap_amd import base, tools, benchmarks
    tb = base.Toolbox()
    if cx == "twopoint":
        tb.register("mate", tools.cxTwoPoint)
    else:
        tb.register("mate", tools.cxBlend, alpha=alpha)
    if mut == "flipbit":
        tb.register("mutate", tools.mutFlipBit, indpb=indpb)
    else:
        tb.register("mutate", tools.mutGaussian, mu=0, sigma=1.0, indpb=indpb)
    if evaluate:
        tb.register("evaluate", getattr(benchmarks, evaluate), **ev_kw)
    tb.register("select", tools.selTournament, tournsize=tournsize)
    return tb


# ---------------------------------------------------------------------------
def test_philox_blocks_match_oracle(gpu):
    import torch
    from deap_amd import _lib
    from deap_amd.device import Context
    ctx = Context.get()
    n = 4096
    out = torch.empty((n, 4), dtype=torch.int32, device=gpu)
    c0 = (ctypes.c_uint32 * 4)(7, 3, 11, (5 << 16) | 2)
    key = (ctypes.c_uint32 * 2)(0xDEADBEEF, 0x12345678)
    _lib.call("dm_philox_blocks", ctx.bind(), c0, key, n, ctypes.c_void_p(out.data_ptr()))
    got = out.cpu().numpy().view(np.uint32)
    ctr = np.stack([7 + np.arange(n), np.full(n, 3), np.full(n, 11), np.full(n, (5 << 16) | 2)], 1)
    want = philox.philox4x32_10(ctr.astype(np.uint64), (0xDEADBEEF, 0x12345678))
    assert np.array_equal(got, want)


def test_eval_matches_reference(gpu):
    from deap_amd import benchmarks
    d = golden("eval.npz")
    j = 0
    while "eval%d_x" % j in d:
        name, kw = d["eval%d_meta" % j]
        kw = ast.literal_eval(kw)
        f = d["eval%d_f" % j]
        pop = _dp().from_numpy(d["eval%d_x" % j], weights=(1.0,) * f.shape[1], gtype="f64")
        got = getattr(benchmarks, name)(pop, **kw).cpu().numpy()
        assert _rel_close(got, f, 1e-12), (name, np.max(np.abs(got - f)))
        assert pop.valid[: len(pop)].bool().all()
        j += 1
    pop = _dp().from_numpy(d["onemax_x"], weights=(1.0,), gtype="bits")
    assert np.array_equal(benchmarks.onemax(pop).cpu().numpy()[:, 0], d["onemax_f"])
    pop = _dp().from_numpy(d["rastrigin_f32_x"], weights=(-1.0,), gtype="f32")
    got = benchmarks.rastrigin(pop).cpu().numpy()[:, 0]
    assert _rel_close(got, d["rastrigin_f32_f"], 1e-12)


def test_eval_only_invalid_and_nevals(gpu):
    import torch
    from deap_amd import benchmarks
    x = np.random.default_rng(3).uniform(-5, 5, size=(1000, 64))
    pop = _dp().from_numpy(x, weights=(-1.0,), gtype="f64")
    pop.valid[::2] = 1
    pop.wvalues[::2] = 123.0
    nev = torch.zeros(1, dtype=torch.int64, device=gpu)
    benchmarks.sphere(pop, only_invalid=True, nevals=nev)
    assert int(nev.item()) == 500
    wv = pop.wvalues.cpu().numpy()[:, 0]
    assert np.all(wv[::2] == 123.0)
    assert _rel_close(wv[1::2], -(x[1::2] ** 2).sum(1), 1e-12)


def _decisions_from(d, k, gpu, aspirants=None):
    from deap_amd.decisions import Decisions
    return Decisions.from_numpy(gpu, aspirants=aspirants, cx_flag=d[k + "cx_flag"],
                                cx_raw=d[k + "cx_raw"], blend_u=d[k + "blend_u"],
                                mut_flag=d[k + "mut_flag"], mut_mask=d[k + "mask"],
                                gauss=d[k + "gauss"])


def test_var_and_matches_reference(gpu):
    from deap_amd import algorithms
    d = golden("varand.npz")
    j = 0
    while "va%d_genes" % j in d:
        k = "va%d_" % j
        gt, tc, cx, mut, cxpb, mutpb, indpb, alpha = d[k + "meta"]
        pop = _dp().from_numpy(d[k + "genes"], weights=(1.0,), gtype=gt, wvalues=d[k + "wv"],
                               valid=d[k + "valid"])
        tb = _toolbox(cx, mut, float(indpb), float(alpha))
        dec = _decisions_from(d, k, gpu)
        off = algorithms.varAnd(pop, tb, float(cxpb), float(mutpb), decisions=dec, mode="inject")
        g, wv, ok = off.to_numpy()
        assert np.array_equal(g, d[k + "out_genes"]), (j, gt, cx, mut)
        assert np.array_equal(ok, d[k + "out_valid"])
        assert np.array_equal(wv[ok], d[k + "out_wv"][ok])
        j += 1


def test_ea_generation_matches_reference(gpu):
    from deap_amd import algorithms
    d = golden("generation.npz")
    j = 0
    while "ea%d_genes" % j in d:
        k = "ea%d_" % j
        gt, tc, cx, mut, objective, t, cxpb, mutpb, indpb, alpha, w0 = d[k + "meta"]
        pop = _dp().from_numpy(d[k + "genes"], weights=(float(w0),), gtype=gt,
                               wvalues=d[k + "wv"], valid=d[k + "valid"])
        tb = _toolbox(cx, mut, float(indpb), float(alpha), evaluate=objective,
                      tournsize=int(t))
        dec = _decisions_from(d, k, gpu, aspirants=d[k + "asp"])
        pop, log = algorithms.eaSimple(pop, tb, float(cxpb), float(mutpb), 1, verbose=False,
                                       decisions=[dec], mode="inject")
        g, wv, ok = pop.to_numpy()
        assert np.array_equal(g, d[k + "out_genes"]), j
        assert ok.all()
        tol = 0 if objective == "onemax" else 1e-12
        assert _rel_close(wv, d[k + "out_wv"], tol), (j, np.max(np.abs(wv - d[k + "out_wv"])))
        assert log.select("nevals") == d[k + "nevals"].tolist()
        j += 1


def test_selection_matches_reference(gpu):
    from deap_amd import tools
    from deap_amd.decisions import Decisions
    d = golden("selection.npz")
    for j in range(3):
        k = "sel%d_" % j
        wv = d[k + "wv"]
        n, m = wv.shape
        pop = _dp().from_numpy(np.zeros((n, 3)), weights=tuple(d[k + "weights"]), gtype="f64",
                               wvalues=wv, valid=np.ones(n))
        asp = d[k + "asp"]
        dec = Decisions.from_numpy(gpu, aspirants=asp)
        got = tools.selTournament(pop, n, asp.shape[1], mode="inject", decisions=dec)
        assert got.cpu().numpy().tolist() == d[k + "out"].tolist()
        assert tools.selBest(pop, 10).cpu().numpy().tolist() == d[k + "best"].tolist()
        assert tools.selWorst(pop, 10).cpu().numpy().tolist() == d[k + "worst"].tolist()


def test_var_or_matches_reference(gpu):
    from deap_amd import algorithms
    from deap_amd.decisions import Decisions
    d = golden("varor.npz")
    for j in range(2):
        k = "vo%d_" % j
        gt, tc, cx, mut, lam, cxpb, mutpb, indpb, alpha = d[k + "meta"]
        pop = _dp().from_numpy(d[k + "genes"], weights=(-1.0, -1.0), gtype=gt,
                               wvalues=d[k + "wv"], valid=d[k + "valid"])
        tb = _toolbox(cx, mut, float(indpb), float(alpha))
        dec = Decisions.from_numpy(gpu, varor_op=d[k + "op"], varor_idx=d[k + "idx"],
                                   cx_raw=d[k + "cx_raw"], blend_u=d[k + "blend_u"],
                                   mut_mask=d[k + "mask"], gauss=d[k + "gauss"])
        off = algorithms.varOr(pop, tb, int(lam), float(cxpb), float(mutpb), decisions=dec,
                               mode="inject")
        g, wv, ok = off.to_numpy()
        assert np.array_equal(g, d[k + "out_genes"]), j
        assert np.array_equal(ok, d[k + "out_valid"])
        assert np.array_equal(wv[ok], d[k + "out_wv"][ok])


def test_nsga2_matches_reference(gpu):
    from deap_amd import tools
    from deap_amd.tools import emo
    d = golden("nsga2.npz")
    for j in range(6):
        k = "nd%d_" % j
        wv, weights, kk = d[k + "wv"], tuple(d[k + "weights"]), int(d[k + "k"])
        n = len(wv)
        pop = _dp().from_numpy(np.zeros((n, 2)), weights=weights, gtype="f64", wvalues=wv,
                               valid=np.ones(n))
        fronts = tools.sortNondominated(pop, kk)
        flat = np.concatenate([f.cpu().numpy() for f in fronts]).tolist()
        assert flat == d[k + "order"].tolist(), j
        assert np.cumsum([0] + [len(f) for f in fronts]).tolist() == d[k + "fstart"].tolist()
        crowd = emo.assignCrowdingDist(pop, fronts)
        got = crowd.cpu().numpy()[np.array(flat)]
        assert np.array_equal(got, d[k + "crowd"]), j
        chosen = tools.selNSGA2(pop, kk)
        assert chosen.cpu().numpy().tolist() == d[k + "chosen"].tolist(), j
        ff = tools.sortNondominated(pop, kk, first_front_only=True)
        assert len(ff) == 1 and len(ff[0]) == d[k + "first"][0]


def test_mig_ring_matches_reference(gpu):
    import torch
    from deap_amd import tools
    from deap_amd.tools import migration
    d = golden("migration.npz")
    for j in range(3):
        k = "mig%d_" % j
        nd, kk, repl = d[k + "meta"]
        nd, kk = int(nd), int(kk)
        demes = [_dp().from_numpy(d[k + "in_genes%d" % i], weights=(1.0,), gtype="f64",
                                  wvalues=d[k + "in_wv%d" % i],
                                  valid=np.ones(len(d[k + "in_wv%d" % i])))
                 for i in range(nd)]
        if repl == "None":
            tools.migRing(demes, kk, tools.selBest)
        else:
            # replacement=random.sample with the reference's drawn indices
            em = [migration.pack(demes[i], torch.tensor(d[k + "sel%d" % i], dtype=torch.int32,
                                                         device=gpu)) for i in range(nd)]
            im = [migration.pack(demes[i], torch.tensor(d[k + "repl%d" % i], dtype=torch.int32,
                                                         device=gpu)) for i in range(nd)]
            for frm, to in enumerate(list(range(1, nd)) + [0]):
                migration.place(demes[to], im[to], em[frm], kk)
        for i in range(nd):
            g, wv, _ = demes[i].to_numpy()
            assert np.array_equal(g, d[k + "out_genes%d" % i]), (j, i)
            assert np.array_equal(wv, d[k + "out_wv%d" % i]), (j, i)


def test_c1_trajectory_bit_exact(gpu):
    """README OneMax (examples/ga/onemax_short.py, seed 64): the reference's
    own 40 generations of decisions replayed on the GPU give its final
    population and logbook."""
    from deap_amd import algorithms
    from deap_amd.decisions import Decisions
    d = golden("c1_trajectory.npz")
    pop = _dp().from_numpy(d["c1_init"], weights=(1.0,), gtype="bits")
    decs = [Decisions.from_numpy(gpu, aspirants=d["c1_asp"][g], cx_flag=d["c1_cx_flag"][g],
                                 cx_raw=d["c1_cx_raw"][g], mut_flag=d["c1_mut_flag"][g],
                                 mut_mask=np.unpackbits(d["c1_mask"][g], axis=-1)[:, :100])
            for g in range(40)]
    tb = _toolbox("twopoint", "flipbit", 0.05, evaluate="onemax")
    pop, log = algorithms.eaSimple(pop, tb, 0.5, 0.2, 40, verbose=False, decisions=decs,
                                   mode="inject")
    g, wv, ok = pop.to_numpy()
    assert np.array_equal(g, d["c1_final"])
    assert np.array_equal(wv, d["c1_final_wv"])
    assert log.select("nevals") == d["c1_nevals"].tolist()


# ---------------------------------------------------------------------------
# Native (counter-based RNG) mode: the decisions the device drew are dumped
# and replayed into the oracle.
# ---------------------------------------------------------------------------
def _replay_native(gpu, gt, dim, n, cx, mut, objective, weights, seed):
    from deap_amd import algorithms, tools
    from deap_amd.ops import RandomStream
    stream = RandomStream(seed)
    low, high = (-5.12, 5.12) if gt != "bits" else (0, 1)
    pop = tools.initPopulation(n=n, dim=dim, low=low, high=high, gtype=gt, weights=weights,
                               stream=stream)
    tb = _toolbox(cx, mut, 0.05, 0.5, evaluate=objective)
    from deap_amd import benchmarks
    getattr(benchmarks, objective)(pop)
    g0, wv0, ok0 = pop.to_numpy()
    decs = []
    pop, log = algorithms.eaSimple(pop, tb, 0.5, 0.2, 1, verbose=False, decisions=decs,
                                   mode="dump", stream=stream)
    g1, wv1, ok1 = pop.to_numpy()
    dn = decs[0].numpy()
    dec = {"aspirants": dn["aspirants"], "cx_flag": dn["cx_flag"].astype(bool),
           "cx_raw": dn.get("cx_raw"), "blend_u": dn.get("blend_u"),
           "mut_flag": dn["mut_flag"].astype(bool),
           "mut_mask": ops.unpack_mask(dn["mut_mask"], dim), "gauss": dn.get("gauss")}
    og, owv, ook, nev = ops.ea_generation(g0, wv0, ok0, 0.5, 0.2, cx, mut, dec, objective,
                                          weights, 0.5)
    return g1, wv1, og, owv, nev, log, dn, stream


@pytest.mark.parametrize("gt,dim,n,cx,mut,objective,weights", [
    ("f64", 1000, 512, "blend", "gaussian", "rastrigin", (-1.0,)),
    ("f64", 1000, 256, "blend", "gaussian", "rosenbrock", (-1.0,)),
    ("f32", 200, 300, "blend", "gaussian", "rastrigin", (-1.0,)),
    ("f64", 77, 301, "twopoint", "gaussian", "sphere", (-1.0,)),
    ("bits", 4096, 512, "twopoint", "flipbit", "onemax", (1.0,)),
    ("bits", 100, 301, "twopoint", "flipbit", "onemax", (1.0,)),
])
def test_native_generation_replays_in_oracle(gpu, gt, dim, n, cx, mut, objective, weights):
    g1, wv1, og, owv, nev, log, dn, _ = _replay_native(gpu, gt, dim, n, cx, mut, objective,
                                                       weights, 1234)
    assert np.array_equal(g1, og)
    tol = 0 if objective == "onemax" else 1e-12
    assert _rel_close(wv1, owv, tol)
    assert log.select("nevals")[1] == nev


def test_native_decisions_follow_the_documented_stream(gpu):
    """Integer decisions of native mode recomputed from the Philox spec."""
    from deap_amd import algorithms, tools, benchmarks
    from deap_amd.ops import RandomStream
    n, dim, seed = 1000, 40, 99
    stream = RandomStream(seed, island=3)
    pop = tools.initPopulation(n=n, dim=dim, low=-1, high=1, gtype="f64", weights=(-1.0,),
                               stream=stream)
    benchmarks.sphere(pop)
    decs = []
    gen_counter = stream.counter
    algorithms.eaSimple(pop, _toolbox("twopoint", "gaussian", evaluate="sphere"), 0.5, 0.2, 1,
                        verbose=False, decisions=decs, mode="dump", stream=stream)
    dn = decs[0].numpy()
    r = philox.Rng(seed, island=3, gen=gen_counter)
    c = np.arange(n)
    w = r(philox.ST_SEL, c, 0)
    w1 = r(philox.ST_SEL, c, 1)
    asp = np.stack([philox.bounded64(w[:, 0], w[:, 1], n), philox.bounded64(w[:, 2], w[:, 3], n),
                    philox.bounded64(w1[:, 0], w1[:, 1], n)], 1)
    assert np.array_equal(dn["aspirants"], asp)
    p = np.arange(n // 2)
    wc = r(philox.ST_CX, p, 0)
    flags = wc[:, 0].astype(np.uint64) < philox.prob_threshold(0.5)
    assert np.array_equal(dn["cx_flag"].astype(bool), flags)
    wc2 = r(philox.ST_CX, p, 1)
    r1 = 1 + philox.bounded64(wc[:, 2], wc[:, 3], dim)
    r2 = 1 + philox.bounded64(wc2[:, 0], wc2[:, 1], dim - 1)
    assert np.array_equal(dn["cx_raw"][flags], np.stack([r1, r2], 1)[flags])
    wm = r(philox.ST_MUT, c, 0)
    mflags = wm[:, 0].astype(np.uint64) < philox.prob_threshold(0.2)
    assert np.array_equal(dn["mut_flag"].astype(bool), mflags)
    # per-gene masks of float genomes
    mask = np.zeros((n, dim), bool)
    for gi in range(dim):
        sub, word = philox.gene_slot(gi, 8)
        ww = r(philox.ST_MASK, c, int(sub))
        mask[:, gi] = ww[:, int(word)].astype(np.uint64) < philox.prob_threshold(0.05)
    got = ops.unpack_mask(dn["mut_mask"], dim)
    assert np.array_equal(got[mflags], mask[mflags])


def test_sort_nondominated_large_random(gpu):
    """Random 3-objective fronts at n=3000 vs the oracle (exact order)."""
    from deap_amd import tools
    rng = np.random.default_rng(5)
    for kind in ("cont", "ties"):
        n = 3000
        wv = (rng.uniform(0, 1, size=(n, 3)) if kind == "cont"
              else rng.integers(0, 12, size=(n, 3)).astype(np.float64))
        pop = _dp().from_numpy(np.zeros((n, 2)), weights=(1.0, 1.0, 1.0), gtype="f64",
                               wvalues=wv, valid=np.ones(n))
        fronts = tools.sortNondominated(pop, n // 2)
        want = ops.sort_nondominated(wv, n // 2)
        assert [f.cpu().numpy().tolist() for f in fronts] == want
        chosen = tools.selNSGA2(pop, n // 2).cpu().numpy().tolist()
        want_c, _ = ops.sel_nsga2(wv, (1.0, 1.0, 1.0), n // 2)
        assert chosen == want_c


def _near_clone_fitness(rng, m, nbase, long_mixed, ulp0=False):
    """Rows in runs of equal objective 0: exact clones, and near-clones a few
    ulps apart in the other objectives (what cxBlend of two clones leaves in
    C5's populations), in shuffled order; a run of 100 exact clones; with
    long_mixed a run of 90 rows equal in objective 0 and all different in the
    others (longer than the 64-row in-place run sort: the full sort).  ulp0:
    the near-clones and the 90-row run also a few ulps apart in objective 0
    (equal in the top 32 key bits the 4-pass objective-0 sort orders, so its
    fix-up sorts them; the 90-row run overflows it into the whole-key sort)."""
    base = rng.uniform(0, 1, size=(nbase, m))
    rows = []
    for b in base:
        for _ in range(int(rng.integers(1, 9))):
            r = b.copy()
            if rng.random() < 0.6:
                for o in range(0 if ulp0 else 1, m):
                    for _ in range(int(rng.integers(0, 3))):
                        r[o] = np.nextafter(r[o], 2.0 if rng.random() < 0.5 else -1.0)
            rows.append(r)
    rows += [base[0]] * 100
    if long_mixed:
        x0 = 0.25
        for _ in range(90):
            rows.append(np.concatenate([[x0], rng.uniform(0, 1, m - 1)]))
            if ulp0:
                x0 = np.nextafter(x0, 1.0)
    wv = np.array(rows)
    return wv[rng.permutation(len(wv))]


@pytest.mark.parametrize("m", [2, 3, 4, 5, 8])
@pytest.mark.parametrize("long_mixed", [False, True])
@pytest.mark.parametrize("ulp0", [False, True])
def test_near_clone_runs_lexicographic_order(gpu, m, long_mixed, ulp0):
    """The grouping sorts by objective 0 and then sorts, in place, only the
    runs of equal objective 0 that are out of order in the other objectives
    (nsga2.hip lex_bad_kernel / lex_run_sort_kernel), falling back to the full
    lexicographic sort for such a run over 64 rows: fronts and selNSGA2 equal
    the oracle (deap/tools/emo.py:15-50, 53-117) exactly on near-clone
    populations.  m = 5 and 8: rows tied in objectives 0-3 and out of order
    only in the later ones (the run sort keys objectives 1-3 only, so those
    objective counts take the full lexicographic sort)."""
    from deap_amd import tools
    rng = np.random.default_rng(70 + 10 * m + long_mixed + 100 * ulp0)
    wv = _near_clone_fitness(rng, m, 500, long_mixed, ulp0)
    if m > 4:  # near-clones that differ only in objectives 4..m-1
        tail = rng.choice(len(wv), len(wv) // 3, replace=False)
        wv[tail, 1:4] = wv[tail, 0:1]
        wv[tail[1::2]] = wv[tail[::2]][:len(tail[1::2])]
        wv[tail[1::2], 4:] = np.nextafter(wv[tail[1::2], 4:], -1.0)
    n = len(wv)
    w = (-1.0,) * m
    pop = _dp().from_numpy(np.zeros((n, 1)), weights=w, gtype="f64", wvalues=wv,
                           valid=np.ones(n))
    fronts = tools.sortNondominated(pop, n)
    assert [f.cpu().numpy().tolist() for f in fronts] == ops.sort_nondominated(wv, n)
    chosen = tools.selNSGA2(pop, n // 2).cpu().numpy().tolist()
    want_c, _ = ops.sel_nsga2(wv, w, n // 2)
    assert chosen == want_c


@pytest.mark.parametrize("m", [2, 3, 4])
def test_sort_nondominated_with_nan_fitness(gpu, m):
    """NaN objectives (e.g. ZDT1 of an out-of-range gene): Fitness.dominates
    (base.py:209-224) treats an objective with a NaN side as equal.  The NaN
    rows' other objectives are all -1, below every finite row, so every finite
    row dominates them, they never dominate one another and the relation stays
    acyclic (a cycle would hang the reference's peel loop too)."""
    from deap_amd import tools
    rng = np.random.default_rng(11 + m)
    n = 700
    wv = rng.uniform(0, 1, size=(n, m))
    rows = rng.choice(n, 40, replace=False)
    wv[rows] = -1.0
    wv[rows, rng.integers(0, m, 40)] = np.nan
    pop = _dp().from_numpy(np.zeros((n, 2)), weights=(1.0,) * m, gtype="f64", wvalues=wv,
                           valid=np.ones(n))
    fronts = tools.sortNondominated(pop, n)
    want = ops.sort_nondominated(wv, n)
    assert [f.cpu().numpy().tolist() for f in fronts] == want


@pytest.mark.parametrize("m", [2, 3, 4])
def test_dominance_paths_agree_large(gpu, m):
    """At sizes the oracle cannot finish: the default path (bitset tables +
    table peel for 2-3 objectives, integer compare kernel + D peel for 4) and
    the cross-check paths (dm_ctx_set_dom_path: integer compare kernel, bitset
    rows + D peel, fp64 ballot kernel, fp64 LDS kernel) give identical fronts
    and selNSGA2 choices."""
    from deap_amd import tools
    from deap_amd.device import dominance_path
    rng = np.random.default_rng(31 + m)
    n = 30011
    wv = np.round(rng.uniform(0, 1, size=(n, m)), 2)  # many equal fitnesses
    w = (1.0, -1.0, 1.0, -1.0)[:m]
    pop = _dp().from_numpy(np.zeros((n, 1)), weights=w, gtype="f64", wvalues=wv,
                           valid=np.ones(n))
    got = []
    for path in ("default", "compare", "ballot", "lds", "peel_d"):
        with dominance_path(path):
            fronts = tools.sortNondominated(pop, n)
            got.append(([f.cpu().numpy().tolist() for f in fronts],
                        tools.selNSGA2(pop, n // 2).cpu().numpy().tolist(),
                        [len(f) for f in tools.sortNondominated(pop, n // 3)]))
    assert got[0] == got[1] == got[2] == got[3] == got[4]
    assert sum(len(f) for f in got[0][0]) == n


def _tie_fitness(rng, n, m, kind):
    if kind == "cont":
        return rng.uniform(0, 1, size=(n, m))
    if kind == "ties":  # few values per objective: rank ties in every objective
        return rng.integers(0, 9, size=(n, m)).astype(np.float64)
    # objective 0 takes 3 values (tie groups span many 512-v chunks), the
    # others continuous, a tenth of the rows duplicated
    wv = np.concatenate([rng.integers(0, 3, size=(n, 1)).astype(np.float64),
                         rng.uniform(0, 1, size=(n, m - 1))], 1)
    wv[rng.integers(0, n, n // 10)] = wv[rng.integers(0, n, n // 10)]
    return wv


@pytest.mark.parametrize("m", [2, 3, 4])
@pytest.mark.parametrize("n", [1, 37, 511, 513, 1100, 2900, 9001])
def test_bitset_dominance_equals_compare_kernel(gpu, m, n):
    """The default dominance pass against independent cross-check paths and,
    up to n = 3,000, the oracle (deap/tools/emo.py:53-117): identical fronts,
    member for member and in order, on continuous fitnesses, ties in every
    objective, and objective-0 tie groups wider than a 512-v chunk (the
    prefix / suffix masks), at sizes around one chunk and with a partial last
    chunk.  Two and three objectives: the bitset-table pass with the
    table-fed peel (bitdom.hip) against the same pass writing D for the
    D-reading peel (DM_DOM_PEEL_D) and the integer compare kernel
    (DM_DOM_COMPARE).  Four objectives: the integer compare kernel + D peel,
    checked against the fp64 ballot and LDS kernels (the four-objective bitset
    path exists only in diagnostic builds)."""
    from deap_amd import _lib, tools
    from deap_amd.device import Context, dominance_path
    ctx = Context.get()
    bitset = m <= 3
    assert _lib.load().dm_ctx_dom_bitset(ctx.handle, m) == (1 if bitset else 0)
    paths = ("default", "compare", "peel_d") if bitset else ("default", "ballot", "lds")
    rng = np.random.default_rng(1000 * m + n)
    w = (1.0, -1.0, 1.0, -1.0)[:m]
    for kind in ("cont", "ties", "obj0"):
        wv = _tie_fitness(rng, n, m, kind)
        pop = _dp().from_numpy(np.zeros((n, 1)), weights=w, gtype="f64", wvalues=wv,
                               valid=np.ones(n))
        got = []
        for path in paths:
            with dominance_path(path):
                got.append([f.cpu().numpy().tolist() for f in tools.sortNondominated(pop, n)])
        assert got[0] == got[1] == got[2], kind
        assert sum(len(f) for f in got[0]) == n
        if n <= 3000:
            assert got[0] == ops.sort_nondominated(wv, n), kind


def test_front_larger_than_the_lds_sort(gpu):
    """A second front of 20,000 unique fitnesses (beyond the 16,384 the
    one-workgroup LDS sort orders) goes through the host's radix-sort
    fallback; fronts equal the fp64 LDS path."""
    from deap_amd import tools
    k = 20000
    i = np.arange(k, dtype=np.float64)
    front0 = np.stack([i, k - i], 1)
    front1 = np.stack([i - 0.5, k - i - 0.5], 1)  # each dominated by its front-0 twin
    wv = np.concatenate([front1, front0, front1[:7]])[np.random.default_rng(2).permutation(2 * k + 7)]
    pop = _dp().from_numpy(np.zeros((len(wv), 1)), weights=(1.0, 1.0), gtype="f64",
                           wvalues=wv, valid=np.ones(len(wv)))
    from deap_amd.device import dominance_path
    fast = [f.cpu().numpy().tolist() for f in tools.sortNondominated(pop, len(wv))]
    with dominance_path("lds"):
        ref = [f.cpu().numpy().tolist() for f in tools.sortNondominated(pop, len(wv))]
    assert [len(f) for f in fast] == [k, k + 7]
    assert fast == ref


def test_sel_best_large_ties(gpu):
    from deap_amd import tools
    rng = np.random.default_rng(6)
    n = 100000
    wv = rng.integers(0, 50, size=(n, 2)).astype(np.float64)
    wv[rng.integers(0, n, 100), 0] = -0.0
    pop = _dp().from_numpy(np.zeros((n, 1)), weights=(1.0, -1.0), gtype="f64", wvalues=wv,
                           valid=np.ones(n))
    got = tools.selBest(pop, 500).cpu().numpy().tolist()
    assert got == ops.sel_best(wv, 500).tolist()
    got = tools.selWorst(pop, 500).cpu().numpy().tolist()
    assert got == ops.sel_worst(wv, 500).tolist()


@pytest.mark.parametrize("gt,dim,n,cx,mut,objective,sel", [
    ("f64", 1000, 1000, "blend", "gaussian", "rastrigin", "tournament"),
    ("f64", 1000, 257, "blend", "gaussian", "rosenbrock", "tournament"),
    ("f64", 300, 400, "twopoint", "gaussian", "sphere", "tournament"),
    ("f32", 200, 300, "blend", "gaussian", "rastrigin", "tournament"),
    ("f64", 513, 64, "blend", "gaussian", "rastrigin", "random"),
    # more pairs than resident waves: every wave's row ring wraps several times
    ("f64", 130, 9001, "twopoint", "gaussian", "rastrigin", "tournament"),
    ("f32", 1000, 6001, "blend", "gaussian", "rastrigin", "tournament"),
    ("f64", 700, 5000, "blend", "gaussian", "rosenbrock", "random"),
    ("f64", 1000, 4099, "blend", "gaussian", "rastrigin", "tournament7"),
    # packed bits (C2 hot path): partial last wave of DM_BITS_PP pairs, odd n
    ("bits", 4096, 40001, "twopoint", "flipbit", "onemax", "tournament"),
    ("bits", 100, 3000, "twopoint", "flipbit", "onemax", "random"),
    ("bits", 1000, 999, "twopoint", "flipbit", "onemax", "tournament7"),
    # more than 8 aspirants: the plan kernel + burst kernel form
    ("bits", 500, 2001, "twopoint", "flipbit", "onemax", "tournament9"),
    # round 6: short float rows (generation_rows.hpp, lane groups of 4 / 8 / 16)
    ("f64", 30, 5001, "blend", "gaussian", "rastrigin", "tournament"),
    ("f32", 10, 3001, "twopoint", "gaussian", "rosenbrock", "tournament"),
    ("f64", 64, 2001, "blend", "gaussian", "sphere", "random"),
    ("f64", 3, 999, "twopoint", "gaussian", "rastrigin", "tournament7"),
    # round 6: rows past 1,024 genes (run-time chunk count) and the fp32 ring
    ("f64", 2000, 3001, "blend", "gaussian", "rastrigin", "tournament"),
    ("f32", 2500, 2001, "blend", "gaussian", "rosenbrock", "tournament"),
    ("f32", 300, 3001, "twopoint", "gaussian", "rastrigin", "tournament"),
    ("f64", 5000, 601, "twopoint", "gaussian", "sphere", "tournament7"),
    # round 6: packed rows of 65-256 words (the fused kernel's 64-word pieces)
    ("bits", 8192, 3001, "twopoint", "flipbit", "onemax", "tournament"),
    ("bits", 10000, 1001, "twopoint", "flipbit", "onemax", "random"),
    ("bits", 16384, 777, "twopoint", "flipbit", "onemax", "tournament7"),
])
def test_native_hot_kernel_equals_replay_kernel(gpu, gt, dim, n, cx, mut, objective, sel):
    """The hot path (per-pair plan kernel + rolling-pipeline kernel, native
    mode) draws the same decisions as the replay kernel's dump mode and
    produces the same genomes bit for bit (the dump mode is itself replayed in
    the oracle).  Fitness sums run in a different lane order (different
    cosine too, for Rastrigin), so wvalues agree to 1e-12 relative — the
    tolerance the north star sets for fp64 fitness."""
    from deap_amd import algorithms, benchmarks, tools
    from deap_amd.ops import RandomStream
    outs = []
    for mode in ("native", "dump"):
        stream = RandomStream(77)
        pop = tools.initPopulation(n=n, dim=dim, low=-3, high=3, gtype=gt, weights=(-1.0,),
                                   stream=stream)
        getattr(benchmarks, objective)(pop)
        tb = _toolbox(cx, mut, 0.05, 0.5, evaluate=objective,
                      tournsize=int(sel[10:] or 3) if sel.startswith("tournament") else 3)
        if sel == "random":
            tb.register("select", tools.selRandom)
        decs = [] if mode == "dump" else None
        pop, log = algorithms.eaSimple(pop, tb, 0.5, 0.2, 2, verbose=False, decisions=decs,
                                       mode=mode, stream=stream)
        outs.append((pop.to_numpy(), log.select("nevals")))
    (g1, wv1, ok1), nev1 = outs[0]
    (g2, wv2, ok2), nev2 = outs[1]
    assert np.array_equal(g1, g2)
    assert np.array_equal(ok1, ok2)
    assert _rel_close(wv1, wv2, 1e-12)
    assert nev1 == nev2


@pytest.mark.parametrize("gt,dim,objective,obj", [
    ("f64", 30, "zdt1", None), ("f32", 12, "dtlz2", 3), ("f64", 64, "zdt3", None),
    ("f64", 7, "dtlz1", 4),
    # ZDT1 / ZDT2 / ZDT4 take the light final formula (mo_finalize_light)
    ("f64", 20, "zdt2", None), ("f32", 10, "zdt4", None), ("f64", 40, "zdt6", None)])
def test_native_short_rows_multiobjective_equal_replay(gpu, gt, dim, objective, obj):
    """Multi-objective eaSimple on short rows (generation_rows.hpp): the
    lexicographic tournaments of the plan kernel (selection.py:55-70 through
    Fitness.__gt__) and the ZDT / DTLZ objectives (deap/benchmarks/__init__.py:
    391-521) in the lane-group kernel equal the replay kernel's dump mode --
    genomes bit for bit, fitness within 1e-12 relative."""
    from deap_amd import algorithms, base, benchmarks, tools
    from deap_amd.ops import RandomStream
    m = 2 if objective.startswith("zdt") else obj
    outs = []
    for mode in ("native", "dump"):
        stream = RandomStream(78)
        pop = tools.initPopulation(n=4001, dim=dim, low=0.2, high=0.8, gtype=gt,
                                   weights=(-1.0,) * m, stream=stream)
        kw = {"obj": obj} if obj else {}
        getattr(benchmarks, objective)(pop, **kw)
        tb = base.Toolbox()
        tb.register("mate", tools.cxTwoPoint)
        tb.register("mutate", tools.mutGaussian, mu=0, sigma=0.01, indpb=0.1)
        tb.register("evaluate", getattr(benchmarks, objective), **kw)
        tb.register("select", tools.selTournament, tournsize=3)
        decs = [] if mode == "dump" else None
        pop, log = algorithms.eaSimple(pop, tb, 0.6, 0.3, 2, verbose=False, decisions=decs,
                                       mode=mode, stream=stream)
        outs.append((pop.to_numpy(), log.select("nevals")))
    (g1, wv1, ok1), nev1 = outs[0]
    (g2, wv2, ok2), nev2 = outs[1]
    assert np.array_equal(g1, g2)
    assert np.array_equal(ok1, ok2)
    assert _rel_close(wv1, wv2, 1e-12)
    assert nev1 == nev2


def test_clones_keep_negative_zero_fitness(gpu):
    """Minimised OneMax: an all-zero genome has wvalues (-0.0,) (base.py:187-198,
    0 * -1.0).  The fused packed-bit kernel's tournaments read int16 fitness
    keys; a clone must still inherit -0.0 exactly as deepcopy does
    (base.py:252-261), so fitness.values stays 0.0 and not -0.0."""
    from deap_amd import algorithms, benchmarks, tools
    from deap_amd.ops import RandomStream
    n, dim = 4001, 256
    genes = np.zeros((n, dim), np.uint8)
    genes[1::2, :3] = 1  # half the rows count 3
    pop = _dp().from_numpy(genes, weights=(-1.0,), gtype="bits")
    benchmarks.onemax(pop)
    wv0 = pop.wvalues[:n, 0].cpu().numpy()
    assert np.signbit(wv0[0]) and wv0[0] == 0.0
    tb = _toolbox("twopoint", "flipbit", 0.05, 0.5, evaluate="onemax")
    pop, _ = algorithms.eaSimple(pop, tb, 0.0, 0.0, 1, verbose=False, stream=RandomStream(5))
    wv = pop.wvalues[:n, 0].cpu().numpy()
    zero = wv == 0.0
    assert zero.sum() > n // 4
    assert np.signbit(wv[zero]).all()


@pytest.mark.parametrize("maxsize,weights", [(1, (1.0,)), (5, (1.0,)), (12, (1.0, -1.0)),
                                             (40, (-1.0,))])
def test_hall_of_fame_device_equals_reference_loop(gpu, maxsize, weights):
    """HallOfFame.update on a DevicePopulation (candidate set on device) keeps
    exactly what the reference loop (support.py:528-548) keeps when it walks
    every individual on the host — duplicates, fitness ties, several updates."""
    from deap_amd import tools
    rng = np.random.default_rng(maxsize)
    hof_dev, hof_host = tools.HallOfFame(maxsize), tools.HallOfFame(maxsize)
    for gen in range(4):
        n = 3000
        genes = rng.integers(0, 4, size=(n, 6)).astype(np.float64)
        genes[rng.integers(0, n, 300)] = genes[rng.integers(0, n, 300)]  # duplicates
        wv = np.stack([genes.sum(1) // 2 + gen * 0.5] +
                      ([-genes[:, 0]] if len(weights) > 1 else []), 1) * np.array(weights)
        pop = _dp().from_numpy(genes, weights=weights, gtype="f64", wvalues=wv,
                               valid=np.ones(n))
        hof_dev.update(pop)
        hof_host.update(pop.to_individuals())
        assert [list(h) for h in hof_dev] == [list(h) for h in hof_host]
        assert [h.fitness.wvalues for h in hof_dev] == [h.fitness.wvalues for h in hof_host]


@pytest.mark.parametrize("comma", [False, True])
def test_mu_lambda_drivers_replay_in_oracle(gpu, comma):
    """eaMuCommaLambda / eaMuPlusLambda (algorithms.py:248-437) with selBest:
    one generation in dump mode replayed through the oracle's varOr,
    evaluation and selBest over offspring (comma) or parents + offspring."""
    from deap_amd import algorithms, benchmarks, tools
    from deap_amd.ops import RandomStream
    n, dim, mu, lam = 300, 40, 300, 500
    stream = RandomStream(5)
    pop = tools.initPopulation(n=n, dim=dim, low=-2, high=2, gtype="f64", weights=(-1.0,),
                               stream=stream)
    benchmarks.sphere(pop)
    g0, wv0, ok0 = pop.to_numpy()
    tb = _toolbox("blend", "gaussian", 0.1, 0.5, evaluate="sphere")
    tb.register("select", tools.selBest)
    decs = []
    drv = algorithms.eaMuCommaLambda if comma else algorithms.eaMuPlusLambda
    pop, log = drv(pop, tb, mu, lam, 0.5, 0.3, 1, verbose=False, decisions=decs, mode="dump",
                   stream=stream)
    dn = decs[0].numpy()
    dec = {"varor_op": dn["varor_op"], "varor_idx": dn["varor_idx"], "blend_u": dn["blend_u"],
           "mut_mask": ops.unpack_mask(dn["mut_mask"], dim), "gauss": dn["gauss"]}
    og, owv, ook = ops.var_or(g0, wv0, ok0, lam, 0.5, 0.3, "blend", "gaussian", dec)
    inv = ~ook
    for i in np.nonzero(inv)[0]:
        owv[i] = -ops.sphere(og[i].tolist())[0]
    assert log.select("nevals")[1] == int(inv.sum())
    pool_g = og if comma else np.concatenate([g0, og])
    pool_w = owv if comma else np.concatenate([wv0, owv])
    want = ops.sel_best(pool_w, mu)
    g1, wv1, _ = pop.to_numpy()
    assert np.array_equal(g1, pool_g[want])
    assert _rel_close(wv1, pool_w[want], 1e-12)


def test_checkpoint_resume_is_bit_exact(gpu, tmp_path):
    """Checkpoint after 2 of 4 eaSimple generations, reload, finish: the same
    population, hall of fame and logbook as the uninterrupted run
    (doc/tutorials/advanced/checkpoint.rst:21-65 pattern, no pickle)."""
    from deap_amd import algorithms, checkpoint, tools
    from deap_amd.ops import RandomStream

    def start():
        stream = RandomStream(42, island=2)
        pop = tools.initPopulation(n=1001, dim=300, low=-5.12, high=5.12, gtype="f64",
                                   weights=(-1.0,), stream=stream)
        return pop, stream

    tb = _toolbox("blend", "gaussian", 0.05, 0.5, evaluate="rastrigin")
    pop, stream = start()
    hof = tools.HallOfFame(7)
    pop, log = algorithms.eaSimple(pop, tb, 0.5, 0.2, 4, halloffame=hof, verbose=False,
                                   stream=stream)
    full = pop.to_numpy()

    pop2, stream2 = start()
    hof2 = tools.HallOfFame(7)
    pop2, log2 = algorithms.eaSimple(pop2, tb, 0.5, 0.2, 2, halloffame=hof2, verbose=False,
                                     stream=stream2)
    path = str(tmp_path / "ck.npz")
    checkpoint.save(path, pop2, stream2, generation=2, halloffame=hof2, logbook=log2)
    del pop2, stream2, hof2
    ck = checkpoint.load(path)
    assert ck["generation"] == 2
    pop3, log3 = algorithms.eaSimple(ck["population"], tb, 0.5, 0.2, 2,
                                     halloffame=ck["halloffame"], verbose=False,
                                     stream=ck["stream"])
    resumed = pop3.to_numpy()
    for a, b in zip(full, resumed):
        assert np.array_equal(a, b)
    assert [list(h) for h in hof] == [list(h) for h in ck["halloffame"]]
    assert log.select("nevals")[1:3] == ck["logbook"].select("nevals")[1:3]
    assert log.select("nevals")[3:] == log3.select("nevals")[1:]


def test_checkpoint_reference_dict_round_trip(gpu):
    """export_reference_dict writes the tutorial's checkpoint dict
    (doc/tutorials/advanced/checkpoint.rst:21-65: population, generation,
    halloffame, logbook, rndstate) with materialised individuals; pickled and
    reloaded (as the tutorial does), import_reference_dict rebuilds the device
    population bit for bit and the resumed run equals the uninterrupted one."""
    import pickle
    from deap_amd import algorithms, checkpoint, tools
    from deap_amd.ops import RandomStream

    def start():
        stream = RandomStream(7, island=1)
        pop = tools.initPopulation(n=513, dim=64, low=-5.12, high=5.12, gtype="f64",
                                   weights=(-1.0,), stream=stream)
        return pop, stream

    tb = _toolbox("blend", "gaussian", 0.05, 0.5, evaluate="rastrigin")
    pop, stream = start()
    pop, log = algorithms.eaSimple(pop, tb, 0.5, 0.2, 4, verbose=False, stream=stream)
    full = pop.to_numpy()
    pop2, stream2 = start()
    hof = tools.HallOfFame(5)
    pop2, log2 = algorithms.eaSimple(pop2, tb, 0.5, 0.2, 2, halloffame=hof, verbose=False,
                                     stream=stream2)
    before = pop2.to_numpy()
    cp = checkpoint.export_reference_dict(pop2, 2, hof, log2, stream2)
    assert set(cp) == {"population", "generation", "halloffame", "logbook", "rndstate",
                       "device_stream"}
    assert len(cp["population"]) == 513 and all(i.fitness.valid for i in cp["population"])
    cp = pickle.loads(pickle.dumps(cp))
    # the tutorial's resume line (checkpoint.rst:32) accepts rndstate
    import random
    state = random.getstate()
    random.setstate(cp["rndstate"])
    random.setstate(state)
    back = checkpoint.import_reference_dict(cp, device=pop2.device)
    for a, b in zip(before, back["population"].to_numpy()):
        assert np.array_equal(a, b)
    assert back["generation"] == 2 and len(back["halloffame"]) == 5
    pop3, _ = algorithms.eaSimple(back["population"], tb, 0.5, 0.2, 2, verbose=False,
                                  stream=back["stream"])
    for a, b in zip(full, pop3.to_numpy()):
        assert np.array_equal(a, b)


def _dcd_pop(wv, crowd):
    import torch
    n = len(wv)
    pop = _dp().from_numpy(np.zeros((n, 1)), weights=(1.0,) * wv.shape[1], gtype="f64",
                           wvalues=wv, valid=np.ones(n))
    pop.crowding_dist = torch.tensor(crowd, dtype=torch.float64, device=pop.device)
    return pop


def test_sel_tournament_dcd_matches_reference(gpu):
    """selTournamentDCD (emo.py:145-195), injected permutations and tie coins
    vs the reference's choices (golden)."""
    import torch
    from deap_amd import tools
    d = golden("dcd.npz")
    for j in range(5):
        key = "dcd%d_" % j
        pop = _dcd_pop(d[key + "wv"], d[key + "crowd"])
        dec = {name: torch.tensor(d[key + name], device=pop.device)
               for name in ("perm1", "perm2", "coin")}
        got = tools.selTournamentDCD(pop, int(d[key + "k"]), mode="inject", decisions=dec)
        assert got.cpu().numpy().tolist() == d[key + "chosen"].tolist(), j


def test_sel_tournament_dcd_native_replays_in_oracle(gpu):
    from deap_amd import tools
    from deap_amd.ops import RandomStream
    rng = np.random.default_rng(3)
    n, k = 50000, 30001
    wv = rng.integers(0, 6, size=(n, 2)).astype(np.float64)
    crowd = rng.choice([0.0, 1.0, np.inf], size=n)
    pop = _dcd_pop(wv, crowd)
    dec = {}
    got = tools.selTournamentDCD(pop, k, mode="dump", decisions=dec,
                                 stream=RandomStream(9)).cpu().numpy()
    p1, p2 = dec["perm1"].cpu().numpy(), dec["perm2"].cpu().numpy()
    assert np.array_equal(np.sort(p1), np.arange(n)) and np.array_equal(np.sort(p2), np.arange(n))
    assert not np.array_equal(p1, p2)
    want = ops.sel_tournament_dcd(wv, crowd, k, p1, p2, dec["coin"].cpu().numpy())
    assert got.tolist() == want
    assert len(got) == 30004
    # native mode draws the same stream as dump mode
    again = tools.selTournamentDCD(pop, k, stream=RandomStream(9)).cpu().numpy()
    assert np.array_equal(again, got)
    # each individual appears at most twice per permutation pass (4 per call)
    assert np.bincount(got, minlength=n).max() <= 4
    # the permutations (orders of Philox keys) carry no trace of the identity
    # or of each other
    idx = np.arange(n)
    for p in (p1, p2):
        assert abs(np.corrcoef(idx, p)[0, 1]) < 0.02
        assert (p == idx).sum() < 10
    assert abs(np.corrcoef(p1, p2)[0, 1]) < 0.02


@pytest.mark.parametrize("n", [5, 12, 33])
def test_sel_tournament_dcd_permutations_are_uniform(gpu, n):
    """random.sample(individuals, len(individuals)) draws uniform permutations
    (emo.py:186-187): over 3,000 streams the position-of-i histogram of both
    permutations passes a chi-square test against the uniform one, and every
    pair (i, j) comes in either order half of the time.  (Round 5's Feistel
    permutations failed this at p < 1e-12, tools_gpu/dcd_perm_sim.py.)"""
    from scipy.stats import chi2
    from deap_amd import tools
    from deap_amd.ops import RandomStream
    rng = np.random.default_rng(n)
    pop = _dcd_pop(rng.random((n, 2)), rng.random(n))
    S = 3000
    h = np.zeros((2, n, n))
    before = np.zeros((n, n))
    k = n - n % 4
    for s in range(S):
        dec = {}
        tools.selTournamentDCD(pop, k, mode="dump", decisions=dec, stream=RandomStream(1000 + s))
        for q, key in enumerate(("perm1", "perm2")):
            p = dec[key].cpu().numpy()
            h[q, np.arange(n), p] += 1
            if q == 0:
                inv = np.argsort(p)
                before += inv[:, None] < inv[None, :]
    e = S / n
    for q in range(2):
        stat = ((h[q] - e) ** 2 / e).sum()
        assert chi2.sf(stat, (n - 1) ** 2) > 1e-4, (q, stat)
    freq = before[np.triu_indices(n, 1)] / S
    assert np.all(np.abs(freq - 0.5) < 5 * np.sqrt(0.25 / S)), freq


def test_sel_tournament_dcd_permutations_small_sizes(gpu):
    """The cycle walk at every small size (domains of 2^2 .. 2^8 around n):
    both permutations are bijections of [0, n)."""
    from deap_amd import tools
    from deap_amd.ops import RandomStream
    rng = np.random.default_rng(5)
    for n in list(range(4, 70, 4)) + [100, 128, 200, 256, 260]:
        pop = _dcd_pop(rng.random((n, 2)), rng.random(n))
        dec = {}
        tools.selTournamentDCD(pop, n, mode="dump", decisions=dec, stream=RandomStream(n))
        for key in ("perm1", "perm2"):
            assert np.array_equal(np.sort(dec[key].cpu().numpy()), np.arange(n)), (n, key)


def test_sel_tournament_dcd_errors(gpu):
    from deap_amd import tools
    pop = _dcd_pop(np.zeros((10, 2)), np.zeros(10))
    with pytest.raises(ValueError):
        tools.selTournamentDCD(pop, 11)
    with pytest.raises(ValueError):
        tools.selTournamentDCD(pop, 10)
    with pytest.raises(IndexError):
        tools.selTournamentDCD(pop, 9)   # 4*ceil(9/4) = 12 > 10: the reference's IndexError


def _sbx_toolbox(low, up, eta_c, eta_m, indpb):
    from deap_amd import base, tools
    tb = base.Toolbox()
    tb.register("mate", tools.cxSimulatedBinaryBounded, low=low, up=up, eta=eta_c)
    tb.register("mutate", tools.mutPolynomialBounded, low=low, up=up, eta=eta_m, indpb=indpb)
    return tb


def _sbx_bounds(d, key):
    if int(d[key + "vec"]):
        return [float(v) for v in d[key + "low"]], [float(v) for v in d[key + "up"]]
    return float(d[key + "low"][0]), float(d[key + "up"][0])


SBX_TOL = 1e-12  # relative: Python `**` is glibc pow, the device ocml pow (both ~1 ulp)


def test_vary_bounded_matches_reference(gpu):
    """NSGA-II loop body (examples/ga/nsga2.py:96-105): cxSimulatedBinaryBounded +
    mutPolynomialBounded on injected random()s against DEAP's own output."""
    import torch
    from deap_amd import algorithms
    d = golden("sbx.npz")
    for j in range(4):
        key = "sbx%d_" % j
        cxpb, eta_c, eta_m, indpb = (float(v) for v in d[key + "meta"])
        genes = d[key + "genes"]
        n = len(genes)
        pop = _dp().from_numpy(genes, weights=(-1.0, -1.0), wvalues=np.zeros((n, 2)),
                               valid=np.ones(n, np.uint8))
        low, up = _sbx_bounds(d, key)
        tb = _sbx_toolbox(low, up, eta_c, eta_m, indpb)
        dec = {k: torch.from_numpy(np.ascontiguousarray(d[key + k])).cuda()
               for k in ("cx_u", "sbx_u", "mut_u")}
        idx = torch.from_numpy(d[key + "idx"]).cuda()
        off = algorithms.varBounded(pop, tb, cxpb, idx, mode="inject", decisions=dec)
        g, _wv, ok = off.to_numpy()
        assert _rel_close(g, d[key + "out"], SBX_TOL), j
        assert np.array_equal(ok.astype(bool), d[key + "valid"]), j


def test_vary_bounded_native_replays_in_oracle(gpu):
    """Native Philox decisions dumped by the kernel, replayed in the oracle
    (ZDT1-like [0,1]^30 population, 2^12 offspring from a random index)."""
    import torch
    from deap_amd import algorithms
    rng = np.random.default_rng(5)
    n, dim, k = 4096, 30, 4095
    genes = rng.uniform(0, 1, size=(n, dim))
    dup = np.arange(3, n - 1, 11)
    genes[dup] = genes[dup + 1]  # equal genes: the |x1 - x2| <= 1e-14 branch
    genes[rng.uniform(size=(n, dim)) < 0.02] = 0.0
    pop = _dp().from_numpy(genes, weights=(-1.0, -1.0), wvalues=rng.normal(size=(n, 2)),
                           valid=np.ones(n, np.uint8))
    idx_h = rng.integers(0, n, size=k).astype(np.int32)
    tb = _sbx_toolbox(0.0, 1.0, 20.0, 20.0, 1.0 / dim)
    dec = {}
    off = algorithms.varBounded(pop, tb, 0.9, torch.from_numpy(idx_h).cuda(), mode="dump",
                                decisions=dec)
    g, wv, ok = off.to_numpy()
    hd = {kk: v.cpu().numpy() for kk, v in dec.items()}
    lo, hi = np.zeros(dim), np.ones(dim)
    eg, _ewv, eok = ops.vary_bounded(genes, np.zeros((n, 2)), np.ones(n, bool), idx_h, 0.9, hd,
                                     (20.0, lo, hi), (20.0, lo, hi, 1.0 / dim))
    assert _rel_close(g, eg, SBX_TOL)
    assert np.array_equal(ok.astype(bool), eok)
    assert (g != genes[idx_h]).any(axis=1).mean() > 0.5  # the operators did act
    assert (g >= 0).all() and (g <= 1).all()
    # native == dump: the same stream state gives the same offspring
    from deap_amd.ops import RandomStream
    s1, s2 = RandomStream(9), RandomStream(9)
    a = algorithms.varBounded(pop, tb, 0.9, torch.from_numpy(idx_h).cuda(), stream=s1)
    b = algorithms.varBounded(pop, tb, 0.9, torch.from_numpy(idx_h).cuda(), stream=s2,
                              mode="dump", decisions={})
    assert np.array_equal(a.to_numpy()[0], b.to_numpy()[0])


def test_bounded_operators_batch_form(gpu):
    """cxSimulatedBinaryBounded / mutPolynomialBounded called on a population
    (every pair mated / every individual mutated, odd n) against the oracle;
    short bound sequences raise the reference's IndexError."""
    from deap_amd import tools
    rng = np.random.default_rng(8)
    n, dim = 257, 9
    low, up = [-1.0] * dim, [2.0] * dim
    genes = rng.uniform(-1, 2, size=(n, dim))
    pop = _dp().from_numpy(genes, weights=(1.0,), wvalues=np.zeros((n, 1)),
                           valid=np.ones(n, np.uint8))
    dec = {}
    off = tools.cxSimulatedBinaryBounded(pop, 15.0, low, up, mode="dump", decisions=dec)
    hd = {kk: v.cpu().numpy() for kk, v in dec.items()}
    lo, hi = np.array(low), np.array(up)
    eg, _w, eok = ops.vary_bounded(genes, np.zeros((n, 1)), np.ones(n, bool), None, 1.0, hd,
                                   (15.0, lo, hi), None)
    g, _wv, ok = off.to_numpy()
    assert _rel_close(g, eg, SBX_TOL) and np.array_equal(ok.astype(bool), eok)
    dec = {}
    off = tools.mutPolynomialBounded(pop, eta=3.0, low=low, up=up, indpb=0.4, mode="dump",
                                     decisions=dec)
    hd = {kk: v.cpu().numpy() for kk, v in dec.items()}
    eg, _w, eok = ops.vary_bounded(genes, np.zeros((n, 1)), np.ones(n, bool), None, 0.0, hd,
                                   None, (3.0, lo, hi, 0.4))
    g, _wv, ok = off.to_numpy()
    assert _rel_close(g, eg, SBX_TOL) and np.array_equal(ok.astype(bool), eok)
    assert not ok.any()
    with pytest.raises(IndexError):
        tools.mutPolynomialBounded(pop, 3.0, low[:-1], up, 0.4)
    with pytest.raises(IndexError):
        tools.cxSimulatedBinaryBounded(pop, 3.0, low, up[:2])


def test_vary_bounded_index_guard(gpu):
    """Host-side out-of-range indices raise IndexError; device-side ones are
    never dereferenced (their pair becomes NaN, invalid) and the rest match."""
    import torch
    from deap_amd import algorithms
    rng = np.random.default_rng(3)
    n, dim = 16, 5
    genes = rng.uniform(0, 1, size=(n, dim))
    pop = _dp().from_numpy(genes, weights=(-1.0,), wvalues=np.zeros((n, 1)),
                           valid=np.ones(n, np.uint8))
    tb = _sbx_toolbox(0.0, 1.0, 20.0, 20.0, 0.5)
    with pytest.raises(IndexError):
        algorithms.varBounded(pop, tb, 0.9, [0, 1, 2, n])
    idx = torch.tensor([0, 1, 2, n + 1000, 4, 5], dtype=torch.int32, device="cuda")
    dec = {}
    off = algorithms.varBounded(pop, tb, 0.9, idx, mode="dump", decisions=dec)
    g, _wv, ok = off.to_numpy()
    assert np.isnan(g[2:4]).all() and not ok[2:4].any()
    assert np.isfinite(g[[0, 1, 4, 5]]).all()


def test_sort_log_nondominated_matches_reference(gpu):
    """Device sortLogNondominated / selNSGA2(nd='log') against DEAP's output."""
    from deap_amd import tools
    d = golden("nsga2log.npz")
    for j in range(6):
        key = "log%d_" % j
        wv, k = d[key + "wv"], int(d[key + "k"])
        n, m = wv.shape
        weights = tuple([-1.0, 1.0, -1.0, 1.0][:m])
        pop = _dp().from_numpy(np.zeros((n, 2)), weights=weights, wvalues=wv,
                               valid=np.ones(n, np.uint8))
        fronts = tools.sortLogNondominated(pop, k)
        assert [len(f) for f in fronts] == d[key + "sizes"].tolist(), j
        assert np.concatenate([f.cpu().numpy() for f in fronts]).tolist() == \
            d[key + "order"].tolist(), j
        assert tools.selNSGA2(pop, k, nd="log").cpu().numpy().tolist() == \
            d[key + "chosen"].tolist(), j
    first = tools.sortLogNondominated(pop, 5, first_front_only=True)
    assert first.cpu().numpy().tolist() == d["log5_order"][: d["log5_sizes"][0]].tolist()


def test_nsga2_example_loop_steps_replay_in_oracle(gpu):
    """Three generations of DEAP's NSGA-II example loop (examples/ga/nsga2.py:94-114)
    on ZDT1, every stage checked against the oracle from the GPU's own state:
    selTournamentDCD (dumped permutations/coins, exact) -> varBounded (dumped
    random()s, 1e-12 rel) -> evaluate -> selNSGA2(pop + offspring) (exact)."""
    import torch
    from deap_amd import algorithms, benchmarks, tools
    from deap_amd.ops import RandomStream
    rng = np.random.default_rng(11)
    n, dim, w = 64, 30, (-1.0, -1.0)
    genes = rng.uniform(0, 1, size=(n, dim))
    pop = _dp().from_numpy(genes, weights=w)
    benchmarks.zdt1(pop)
    idx = tools.selNSGA2(pop, n)  # assigns crowding distances (nsga2.py:92)
    tb = _sbx_toolbox(0.0, 1.0, 20.0, 20.0, 1.0 / dim)
    stream = RandomStream(21)
    for _gen in range(3):
        g0, wv0, _ = pop.to_numpy()
        crowd = pop.crowding_dist[:n].cpu().numpy()
        dcd = {}
        sel = tools.selTournamentDCD(pop, n, mode="dump", decisions=dcd, stream=stream)
        want = ops.sel_tournament_dcd(wv0, crowd, n, dcd["perm1"].cpu().numpy(),
                                      dcd["perm2"].cpu().numpy(), dcd["coin"].cpu().numpy())
        assert sel.cpu().numpy().tolist() == want
        dec = {}
        off = algorithms.varBounded(pop, tb, 0.9, sel, mode="dump", decisions=dec, stream=stream)
        hd = {kk: v.cpu().numpy() for kk, v in dec.items()}
        lo, hi = np.zeros(dim), np.ones(dim)
        eg, _ewv, eok = ops.vary_bounded(g0, wv0, np.ones(n, bool), np.array(want), 0.9, hd,
                                         (20.0, lo, hi), (20.0, lo, hi, 1.0 / dim))
        og, _owv, ook = off.to_numpy()
        assert _rel_close(og, eg, SBX_TOL) and np.array_equal(ook, eok)
        benchmarks.zdt1(off)
        og, owv, _ = off.to_numpy()
        ewv = np.array([[f * x for f, x in zip(ops.zdt1(list(r)), w)] for r in og])
        assert _rel_close(owv, ewv, 1e-12)
        both = np.concatenate([g0, og])
        bwv = np.concatenate([wv0, owv])
        comb = _dp().from_numpy(both, weights=w, wvalues=bwv, valid=np.ones(2 * n, np.uint8))
        chosen = tools.selNSGA2(comb, n).cpu().numpy()
        echosen, ecrowd = ops.sel_nsga2(bwv, w, n)
        assert chosen.tolist() == echosen
        # pop[:] = chosen, carrying the crowding distances
        pop = _dp().from_numpy(both[chosen], weights=w, wvalues=bwv[chosen],
                               valid=np.ones(n, np.uint8))
        pop.crowding_dist = comb.crowding_dist[torch.from_numpy(chosen).long().cuda()].contiguous()
        assert np.allclose(pop.crowding_dist.cpu().numpy(), [ecrowd[i] for i in chosen])


@pytest.mark.parametrize("weight", [1.0, -2.5])
def test_bits_tournament_keys_fall_back_exactly(gpu, weight):
    """The C2 hot kernel reads parent fitness through int16 keys (exact
    multiples of |w0|, generation_pipe_bits.hip fit_key_kernel).  Parents
    whose wvalues are not such multiples (fractions, beyond int16, NaN, -0.0)
    or whose fitness is invalid take the wvalues / valid fallback: one
    generation of the native kernel must still equal the dump-mode replay
    kernel (which reads wvalues directly) bit for bit — genomes, fitness,
    validity of the clones."""
    import ctypes
    import torch
    from deap_amd import algorithms, benchmarks, tools
    from deap_amd.ops import RandomStream
    n, dim = 4099, 300
    sel = np.random.default_rng(5).permutation(n)
    outs = []
    for mode in ("native", "dump"):
        stream = RandomStream(91)
        pop = tools.initPopulation(n=n, dim=dim, low=0, high=1, gtype="bits", weights=(weight,),
                                   stream=stream)
        benchmarks.onemax(pop)
        wv = pop.wvalues[:n, 0].cpu().numpy().copy()
        wv[sel[:300]] += 0.25 * weight                    # not a multiple of |w0|
        wv[sel[300:320]] = 40000.0 * weight               # beyond int16
        wv[sel[320:330]] = np.nan
        wv[sel[330:400]] = -0.0
        valid = np.ones(n, np.uint8)
        valid[sel[400:500]] = 0                           # invalid parents
        pop.wvalues[:n, 0].copy_(torch.from_numpy(wv))
        pop.valid[:n].copy_(torch.from_numpy(valid))
        tb = _toolbox("twopoint", "flipbit", 0.05, 0.5, evaluate="onemax", tournsize=3)
        step = algorithms.GenerationStep(pop, tb, 0.5, 0.2)
        off = pop.like(n, capacity=n)
        nev = torch.zeros(1, dtype=torch.int64, device=pop.device)
        decs = [] if mode == "dump" else None
        step.step(pop, off, stream, ctypes.c_void_p(nev.data_ptr()), mode, decs, 0)
        outs.append((off.to_numpy(), int(nev.item())))
    (g1, wv1, ok1), n1 = outs[0]
    (g2, wv2, ok2), n2 = outs[1]
    assert np.array_equal(g1, g2)
    assert np.array_equal(ok1, ok2)
    assert np.array_equal(wv1, wv2, equal_nan=True)
    assert n1 == n2
